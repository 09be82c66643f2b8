// group_probe.hip -- timing probe: rocPRIM stable radix sort of (key id, arrival index) pairs for the
// device-side grouping of arrival-order batches (CEP_BATCH_ARRIVAL_ORDER), by batch size and key bits.
#include <hip/hip_runtime.h>
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/iterator/counting_iterator.hpp>
#include <cstdio>
#include <vector>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

using onesweep_cfg = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                                rocprim::default_config, 0>;

template <class Cfg>
float run(int n, int bits, int reps, hipStream_t st) {
  std::vector<int> h(n);
  uint32_t x = 12345;
  for (int i = 0; i < n; i++) { x = x * 1664525u + 1013904223u; h[i] = int(x >> (32 - bits)); }
  int *k, *ko, *vo;
  CK(hipMalloc(&k, n * 4)); CK(hipMalloc(&ko, n * 4)); CK(hipMalloc(&vo, n * 4));
  CK(hipMemcpy(k, h.data(), n * 4, hipMemcpyHostToDevice));
  size_t tb = 0;
  rocprim::counting_iterator<int> it(0);
  CK(rocprim::radix_sort_pairs<Cfg>(nullptr, tb, k, ko, it, vo, size_t(n), 0, bits, st));
  void* tmp; CK(hipMalloc(&tmp, tb + 16));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int w = 0; w < 3; w++) CK(rocprim::radix_sort_pairs<Cfg>(tmp, tb, k, ko, it, vo, size_t(n), 0, bits, st));
  CK(hipEventRecord(a, st));
  for (int r = 0; r < reps; r++) CK(rocprim::radix_sort_pairs<Cfg>(tmp, tb, k, ko, it, vo, size_t(n), 0, bits, st));
  CK(hipEventRecord(b, st));
  CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  std::vector<int> ho(n), hv(n);
  CK(hipMemcpy(ho.data(), ko, n * 4, hipMemcpyDeviceToHost)); CK(hipMemcpy(hv.data(), vo, n * 4, hipMemcpyDeviceToHost));
  for (int i = 1; i < n; i++) if (ho[i] < ho[i-1] || (ho[i] == ho[i-1] && hv[i] < hv[i-1])) { printf("NOT STABLE\n"); exit(1); }
  hipFree(k); hipFree(ko); hipFree(vo); hipFree(tmp);
  return ms * 1000.f / reps;
}

int main() {
  hipStream_t st; CK(hipStreamCreate(&st));
  for (int n : {4096, 16384, 65536, 262144, 1 << 20}) for (int bits : {16, 20})
    printf("n %7d bits %d  default %.1f us  onesweep %.1f us\n", n, bits, run<rocprim::default_config>(n, bits, 50, st),
           run<onesweep_cfg>(n, bits, 50, st));
  return 0;
}

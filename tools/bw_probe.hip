// bw_probe.hip — read-bandwidth ceiling for the stencil kernel's access pattern.
// 100M int32 keys + 100M int32 values (800 MB), streamed once per launch:
//   tiles   one 256-thread workgroup per 16K-record super-tile (the stencil grid)
//   persist a fixed grid that strides over super-tiles
//   nt      the same with non-temporal loads
// Prints GB/s (median of 20 launches, HIP events).  Build:
//   hipcc --offload-arch=gfx950 -O3 tools/bw_probe.hip -o tools/bw_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

typedef int v4i __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ v4i ld(const int* p) {
  if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const v4i*>(p));
  else return *reinterpret_cast<const v4i*>(p);
}

// one super-tile = 4 tiles x 4096 records; 16 records per thread per tile
template <bool NT>
__device__ __forceinline__ int tile_sum(const int* key, const int* val, long base, int tid) {
  int acc = 0;
#pragma unroll
  for (int j = 0; j < 4; j++) {
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const long g = base + j * 4096 + q * 1024 + tid * 4;
      const v4i k = ld<NT>(key + g), v = ld<NT>(val + g);
      acc += k.x ^ v.x ^ k.y ^ v.y ^ k.z ^ v.z ^ k.w ^ v.w;
    }
  }
  return acc;
}

template <bool NT>
__global__ __launch_bounds__(256) void tiles(const int* key, const int* val, long ntiles, int* out) {
  const int acc = tile_sum<NT>(key, val, long(blockIdx.x) * 16384, threadIdx.x);
  if (acc == 0x7FFFFFFF) out[threadIdx.x] = acc;
}

template <bool NT>
__global__ __launch_bounds__(256) void persist(const int* key, const int* val, long ntiles, int* out) {
  int acc = 0;
  for (long t = blockIdx.x; t < ntiles; t += gridDim.x) acc += tile_sum<NT>(key, val, t * 16384, threadIdx.x);
  if (acc == 0x7FFFFFFF) out[threadIdx.x] = acc;
}

template <class F>
float time_ms(F&& f) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  std::vector<float> ts;
  for (int i = 0; i < 23; i++) {
    hipEventRecord(a);
    f();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    if (i >= 3) ts.push_back(ms);
  }
  std::sort(ts.begin(), ts.end());
  return ts[ts.size() / 2];
}

int main() {
  const long n = 100000000L / 16384 * 16384;
  const long ntiles = n / 16384;
  int *key, *val, *out;
  hipMalloc(&key, n * 4);
  hipMalloc(&val, n * 4);
  hipMalloc(&out, 4096);
  hipMemset(key, 1, n * 4);
  hipMemset(val, 2, n * 4);
  const double gb = 8.0 * n / 1e9;
  auto rep = [&](const char* name, float ms) { printf("%-28s %8.4f ms  %7.0f GB/s\n", name, ms, gb / (ms * 1e-3)); };
  rep("tiles (stencil grid)", time_ms([&] { tiles<false><<<ntiles, 256>>>(key, val, ntiles, out); }));
  rep("tiles nt", time_ms([&] { tiles<true><<<ntiles, 256>>>(key, val, ntiles, out); }));
  for (int g : {1024, 2048, 3072, 4096})
    for (int nt = 0; nt < 2; nt++) {
      char nm[64];
      snprintf(nm, sizeof nm, "persist %d%s", g, nt ? " nt" : "");
      rep(nm, time_ms([&] {
        if (nt) persist<true><<<g, 256>>>(key, val, ntiles, out);
        else persist<false><<<g, 256>>>(key, val, ntiles, out);
      }));
    }
  hipDeviceSynchronize();
  return 0;
}

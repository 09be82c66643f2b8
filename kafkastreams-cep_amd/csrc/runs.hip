// runs.hip — deterministic strict runs (CEP_PATH_RUNS): one lane per start record.
//
// For the patterns compile.cpp analyse_runs accepts (strict contiguity
// everywhere, no stage whose TAKE and PROCEED edges can match together) the
// reference NFA never branches: each record its begin stage consumes starts one
// run, which either consumes every following record of its key (a BEGIN or
// TAKE edge, possibly after PROCEED / SKIP_PROCEED recursion into later stages,
// NFA.java:190-341) or dies.  A run owns a fresh run sequence, so its
// aggregates (AggregatesStoreImpl, States) are private registers here; its
// Dewey versions begin with a digit no other run has, so the shared buffer's
// first-compatible traversal (SharedVersionedBufferStoreImpl.java:176-201)
// returns exactly the records it consumed, final stage first.
//
// So instead of one lane per key walking a run queue, every record is a lane
// that simulates the run it may start, over consecutive records of its key:
//   runs_sim    find where each run completes (or the record whose predicate throws)
//   (sort)      order completed runs by (completing record, start): the queue is
//               oldest-first, so that is the order NFA.matchPattern emits them
//   runs_write  re-walk each completed run and write its traversal into the CSR
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string.h>

#include <rocprim/device/device_radix_sort.hpp>

#include "../../include/kcep.h"
#include "kcep_internal.h"
#include "interp.h"
#include "runs_dev.h"

namespace kcep {

namespace {

__global__ __launch_bounds__(RT) void runs_sim(RunsArgs A, int64_t* __restrict__ flag, int32_t* __restrict__ end_of) {
  runs_sim_body(InterpTab{A.P}, A, flag, end_of);
}

__global__ __launch_bounds__(RT) void runs_write(WriteArgs W) { runs_write_body(InterpTab{W.R.P}, W); }

// completed runs in start order: key (end << 31 | start); each workgroup's total of their lengths
// (entries of the CSR) into blk_len[blockIdx] (summed by a scan: no contended atomic)
__global__ __launch_bounds__(256) void runs_compact(const int64_t* __restrict__ flag, const int64_t* __restrict__ pos,
                                                    const int32_t* __restrict__ end_of, int64_t n,
                                                    unsigned long long* __restrict__ out, int64_t* __restrict__ blk_len) {
  __shared__ int64_t s_w[4];
  const int64_t j = int64_t(blockIdx.x) * 256 + threadIdx.x;
  int64_t len = 0;
  if (j < n && flag[j]) {
    out[pos[j]] = (unsigned long long)(int64_t(end_of[j]) << 31 | j);
    len = int64_t(end_of[j]) - j + 1;
  }
  for (int d = 32; d >= 1; d >>= 1) len += __shfl_xor(len, d, 64);
  if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = len;
  __syncthreads();
  if (threadIdx.x == 0) blk_len[blockIdx.x] = s_w[0] + s_w[1] + s_w[2] + s_w[3];
}

// the CSR of the sorted completed runs from their recorded stage segments (runs_sim with A.segs),
// entries final stage first (peek, SharedVersionedBufferStoreImpl.java:176-201).  A workgroup owns
// 256 consecutive matches and writes their entries as one contiguous range, thread-strided (coalesced
// stores); an entry finds its match by a binary search over the workgroup's entry offsets in LDS.
__global__ __launch_bounds__(256) void runs_expand(const DevProgram* __restrict__ P, const int32_t* __restrict__ key,
                                                   const uint32_t* __restrict__ segs,
                                                   const unsigned long long* __restrict__ sorted, int64_t nm,
                                                   const int64_t* __restrict__ ent_off, int64_t ne, int64_t base,
                                                   int64_t* __restrict__ match_record, int32_t* __restrict__ match_key,
                                                   int64_t* __restrict__ ent_off_out, int32_t* __restrict__ ent_name,
                                                   int64_t* __restrict__ ent_record) {
  __shared__ int64_t s_at[257];
  __shared__ int64_t s_j[256], s_e[256];
  __shared__ uint32_t s_seg[256][RUNS_MAX_SEGS];
  const int tid = threadIdx.x;
  const int64_t m0 = int64_t(blockIdx.x) * 256, m = m0 + tid;
  const int cnt = nm - m0 < 256 ? int(nm - m0) : 256;
  if (tid < cnt) {
    const unsigned long long kv = sorted[m];
    const int64_t j = int64_t(kv & 0x7FFFFFFFull), e = int64_t(kv >> 31);
    const int64_t at = ent_off[m];
    s_at[tid] = at;
    s_j[tid] = j;
    s_e[tid] = e;
    match_record[m] = base + e;
    match_key[m] = key[j];
    ent_off_out[m] = at;
#pragma unroll
    for (int i = 0; i < RUNS_MAX_SEGS; i++) s_seg[tid][i] = segs[j * RUNS_MAX_SEGS + i];
  }
  if (tid == 0) s_at[cnt] = m0 + cnt < nm ? ent_off[m0 + cnt] : ne;
  __syncthreads();
  const int64_t E0 = s_at[0], E1 = s_at[cnt];
  for (int64_t x = E0 + tid; x < E1; x += 256) {
    int lo = 0, hi = cnt - 1;                        // the last match whose range starts at or before x
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (s_at[mid] <= x) lo = mid; else hi = mid - 1;
    }
    const int64_t j = s_j[lo], e = s_e[lo];
    const int64_t o = (e - j) - (x - s_at[lo]);       // offset of the entry's record from the start
    uint32_t stage = 0;
#pragma unroll
    for (int i = 0; i < RUNS_MAX_SEGS; i++) {        // the segment holding offset o (segments ascend)
      const uint32_t w = s_seg[lo][i];
      if (w != ~0u && int64_t(w & 0xFFFFFFu) <= o) stage = w >> 24;
      if (w == ~0u) break;
    }
    ent_name[x] = P->st[stage].name;
    ent_record[x] = base + j + o;
  }
}

__global__ void runs_lengths(const unsigned long long* __restrict__ sorted, int64_t nm, int64_t* __restrict__ len) {
  const int64_t m = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (m < nm) len[m] = int64_t(sorted[m] >> 31) - int64_t(sorted[m] & 0x7FFFFFFFull) + 1;
}

}  // namespace

hipError_t exclusive_scan(const int64_t* in, int64_t n, int64_t* out, int64_t* total, int64_t* tmp, hipStream_t st);

static unsigned runs_blocks(int64_t items) {
  const int64_t waves = (items + RUNS_CHUNK - 1) / RUNS_CHUNK;
  return unsigned((waves * 64 + RT - 1) / RT);
}

// jf: the pattern's compiled runs_sim (jit.cpp), nullptr for the built-in interpreting kernel
hipError_t runs_sim_launch(const RunsArgs& A, int64_t* flag, int32_t* end_of, hipStream_t st, hipFunction_t jf) {
  if (A.n <= 0) return hipSuccess;
  if (jf) {
    RunsArgs a = A;
    void* args[] = {&a, &flag, &end_of};
    return hipModuleLaunchKernel(jf, runs_blocks(A.n), 1, 1, RT, 1, 1, 0, st, args, nullptr);
  }
  hipLaunchKernelGGL(runs_sim, dim3(runs_blocks(A.n)), dim3(RT), 0, st, A, flag, end_of);
  return hipGetLastError();
}

// blk_len: (n + 255) / 256 partial sums, then their exclusive scan in blk_pre with the total in *ent_total
hipError_t runs_compact_launch(const int64_t* flag, const int64_t* pos, const int32_t* end_of, int64_t n,
                               unsigned long long* out, int64_t* blk_len, int64_t* blk_pre, int64_t* ent_total,
                               int64_t* scan_tmp, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int64_t nb = (n + 255) / 256;
  hipLaunchKernelGGL(runs_compact, dim3(unsigned(nb)), dim3(256), 0, st, flag, pos, end_of, n, out, blk_len);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? exclusive_scan(blk_len, nb, blk_pre, ent_total, scan_tmp, st) : e;
}

// order of completed runs: (completing record, start record).  The compacted keys are already in
// start order and the radix sort is stable, so only the completing record's bits [31, 31 + bits)
// are sorted on.
hipError_t runs_sort(const unsigned long long* in, unsigned long long* out, int64_t nm, int bits, void* tmp,
                     size_t* tmp_bytes, hipStream_t st) {
  return rocprim::radix_sort_keys(tmp, *tmp_bytes, in, out, size_t(nm), 31, 31 + bits, st);
}

hipError_t runs_expand_launch(const RunsArgs& R, const unsigned long long* sorted, int64_t nm, const int64_t* ent_off,
                              int64_t ne, int64_t* match_record, int32_t* match_key, int64_t* ent_off_out, int32_t* ent_name,
                              int64_t* ent_record, hipStream_t st) {
  if (nm <= 0) return hipSuccess;
  hipLaunchKernelGGL(runs_expand, dim3(unsigned((nm + 255) / 256)), dim3(256), 0, st, R.P, R.key, R.segs, sorted, nm,
                     ent_off, ne, R.base, match_record, match_key, ent_off_out, ent_name, ent_record);
  return hipGetLastError();
}

hipError_t runs_write_launch(const RunsArgs& R, const unsigned long long* sorted, int64_t nm, int64_t* len,
                             int64_t* ent_off, int64_t* total, int64_t* scan_tmp, int64_t* match_record,
                             int32_t* match_key, int64_t* ent_off_out, int32_t* ent_name, int64_t* ent_record,
                             hipStream_t st, bool lengths_only, hipFunction_t jf) {
  if (nm <= 0) return hipMemsetAsync(total, 0, sizeof(int64_t), st);
  if (lengths_only) {
    hipLaunchKernelGGL(runs_lengths, dim3(unsigned((nm + 255) / 256)), dim3(256), 0, st, sorted, nm, len);
    return exclusive_scan(len, nm, ent_off, total, scan_tmp, st);
  }
  WriteArgs W{R, sorted, nm, ent_off, match_record, match_key, ent_off_out, ent_name, ent_record};
  if (jf) {
    void* args[] = {&W};
    return hipModuleLaunchKernel(jf, runs_blocks(nm), 1, 1, RT, 1, 1, 0, st, args, nullptr);
  }
  hipLaunchKernelGGL(runs_write, dim3(runs_blocks(nm)), dim3(RT), 0, st, W);
  return hipGetLastError();
}

}  // namespace kcep

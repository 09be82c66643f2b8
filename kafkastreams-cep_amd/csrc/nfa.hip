// nfa.hip — general NFA path: the full reference semantics on the GPU.
//
// One lane runs the NFA of one record key over that key's records in arrival
// order (per-key NFAs share nothing: buffer nodes are keyed by
// (stage, topic, partition, offset), aggregates by (key, state, run), the run
// counter is per key — SURVEY §8(e)).  Everything the reference keeps in its
// three state stores lives in a per-key workspace drawn from a batch-wide pool:
//
//   run queues   ComputationStage (nfa/ComputationStage.java:30-185), 4 words:
//                stage id | epsilon target | isBranching | isIgnored, Dewey
//                version handle, last event, run sequence
//   heap         immutable DeweyVersions [len, digits...] (nfa/DeweyVersion.java)
//                and predecessor pointers {version, slot, event, next, version
//                length, first digit} (state/internal/MatchedEvent.java:124-168)
//   nodes        dense [event][slot] -> {refs, first pred, last pred, flags}: the
//                shared versioned buffer (SharedVersionedBufferStoreImpl.java)
//                with slot = (stage name, stage type) as in Matched.java:31-35
//   aggregates   dense [run sequence][state] -> {boxed type, value}
//                (AggregatesStoreImpl.java:55-75)
//   output       per match: emitting stream position, traversal length, then
//                (stage name, stream position) triples, final stage first
//
// Events of a key are numbered locally: 0..C-1 are the events the key's carried
// state still references (previous batches, CEP_SESSION_CARRY), C..C+L-1 the
// key's records of this batch.
//
// The step follows NFA.matchPattern / evaluate (nfa/NFA.java:134-341) with the
// recursion on PROCEED/SKIP_PROCEED edges unrolled onto an explicit frame
// stack; the buffer operations follow put/branch/peek of
// SharedVersionedBufferStoreImpl.java:101-201 including the copy-on-read
// refcount semantics (decrements persist only at zero, deleted nodes can be
// resurrected).  Predicates and folds run the bytecode of compile.cpp; edge
// predicates that read only the current record are evaluated once per record
// for all runs (a uniform loop: every lane of the wave runs the same program).
//
// Arrays that outgrow their first allocation are re-allocated from the pool at
// twice the size; a lane that cannot allocate sets the overflow flag and the
// host re-runs the batch with a larger pool.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "../../include/kcep.h"
#include "kcep_internal.h"
#include "interp.h"
#include "nfa_dev.h"
#include "nfa_wave.h"
#include "jit.h"

namespace kcep {

__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) void nfa_kernel(NfaArgs A) {
  nfa_kernel_body(A);
}

// one key per wave, one queued run per lane (nfa_wave.h); AGG: patterns with aggregates or
// SequenceMatchers.  A persistent grid (nfa_wave_grid)
template <bool AGG>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(3))) void nfa_wave_kernel(NfaArgs A) {
  nfa_wave_body<AGG>(A);
}

// ---- segments, scans, output compaction, carry commit ----
// Key segments of a grouped batch in three passes over 1024-record blocks: boundaries per block, the
// blocks' exclusive prefix (scan_sums_reg), then every boundary's segment start.  flag / idx (optional:
// the runs carry build reads them) get the per-record boundary flag and its exclusive prefix.
__device__ __forceinline__ int64_t block_excl_256(int64_t v, int64_t* s, int64_t& total) {
  s[threadIdx.x] = v;
  __syncthreads();
  for (int d = 1; d < 256; d <<= 1) {
    const int64_t y = threadIdx.x >= unsigned(d) ? s[threadIdx.x - d] : 0;
    __syncthreads();
    s[threadIdx.x] += y;
    __syncthreads();
  }
  total = s[255];
  return s[threadIdx.x] - v;
}
__global__ void seg_count(const int32_t* __restrict__ key, int64_t n, int64_t* __restrict__ bsum) {
  __shared__ int64_t s[256];
  const int64_t b0 = int64_t(blockIdx.x) * 1024 + threadIdx.x * 4;
  int64_t acc = 0;
  for (int k = 0; k < 4; k++) {
    const int64_t i = b0 + k;
    if (i < n) acc += (i == 0 || key[i] != key[i - 1]) ? 1 : 0;
  }
  int64_t tot = 0;
  block_excl_256(acc, s, tot);
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}
__global__ void seg_write(const int32_t* __restrict__ key, int64_t n, const int64_t* __restrict__ boff,
                          const int64_t* __restrict__ nseg, int64_t* __restrict__ seg_start, int64_t* __restrict__ flag,
                          int64_t* __restrict__ idx) {
  __shared__ int64_t s[256];
  const int64_t b0 = int64_t(blockIdx.x) * 1024 + threadIdx.x * 4;
  int f[4], acc = 0;
  for (int k = 0; k < 4; k++) {
    const int64_t i = b0 + k;
    f[k] = i < n && (i == 0 || key[i] != key[i - 1]) ? 1 : 0;
    acc += f[k];
  }
  int64_t tot = 0;
  int64_t run = boff[blockIdx.x] + block_excl_256(acc, s, tot);
  for (int k = 0; k < 4; k++) {
    const int64_t i = b0 + k;
    if (i >= n) break;
    if (f[k]) seg_start[run] = i;
    if (flag) { flag[i] = f[k]; idx[i] = run; }
    run += f[k];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) seg_start[*nseg] = n;
}

// exclusive scans, 1024 elements per block: (1) block sums, (2) scan of block sums in one block,
// (3) per-block scan + offset.  Two arrays of one length at once (blockIdx.y / the block of pass 2
// picks the array; tmp holds 2 x the block count); n_dev (optional): the length on the device, at
// most n (the grid is sized by n).
struct ScanPair {
  const int64_t* in[2];
  int64_t* out[2];
  int64_t* total[2];
  int64_t n;
  const int64_t* n_dev;
  int64_t nb;                     // blocks of the grid (from n)
};
__device__ __forceinline__ int64_t scan_len(const ScanPair& S) {
  return S.n_dev ? (*S.n_dev < S.n ? *S.n_dev : S.n) : S.n;
}
__global__ void scan_blocks(ScanPair S, int64_t* __restrict__ bsum) {
  __shared__ int64_t s[256];
  const int64_t n = scan_len(S);
  const int64_t* __restrict__ in = S.in[blockIdx.y];
  const int64_t b0 = int64_t(blockIdx.x) * 1024;
  // loads at clamped indices, masked after (a load under `i < n` is a branch waited on inside it)
  const int64_t last = n > 0 ? n - 1 : 0;
  int64_t v[4], acc = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int64_t i = b0 + threadIdx.x * 4 + k;
    v[k] = in[i < n ? i : last];
  }
#pragma unroll
  for (int k = 0; k < 4; k++) acc += b0 + threadIdx.x * 4 + k < n ? v[k] : 0;
  s[threadIdx.x] = acc;
  __syncthreads();
  for (int d = 128; d > 0; d >>= 1) {
    if (threadIdx.x < unsigned(d)) s[threadIdx.x] += s[threadIdx.x + d];
    __syncthreads();
  }
  if (threadIdx.x == 0) bsum[blockIdx.y * S.nb + blockIdx.x] = s[0];
}
__global__ void scan_sums(int64_t* __restrict__ bsum, int64_t nb, int64_t* __restrict__ total) {
  __shared__ int64_t s[256];
  int64_t carry = 0;
  for (int64_t base = 0; base < nb; base += 256) {
    const int64_t i = base + threadIdx.x;
    const int64_t v = i < nb ? bsum[i] : 0;
    s[threadIdx.x] = v;
    __syncthreads();
    for (int d = 1; d < 256; d <<= 1) {
      const int64_t y = threadIdx.x >= unsigned(d) ? s[threadIdx.x - d] : 0;
      __syncthreads();
      s[threadIdx.x] += y;
      __syncthreads();
    }
    if (i < nb) bsum[i] = carry + s[threadIdx.x] - v;
    carry += s[255];
    __syncthreads();
  }
  if (threadIdx.x == 0) *total = carry;
}
// the same scan of up to 16 x 1024 block sums (batches of <= 16 M elements) in one pass: every
// thread holds its 16 consecutive sums in registers, one wave-level and one block-level scan (the loop
// above walks the sums 256 at a time, two barriers per step: 44 us for 10 M elements)
constexpr int SCAN_REG = 16;
__device__ __forceinline__ void scan_sums_reg_body(int64_t* __restrict__ bsum, int64_t nb, int64_t* __restrict__ total) {
  __shared__ int64_t s_w[16];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t per = (nb + 1023) / 1024, a = tid * per;
  int64_t v[SCAN_REG], sum = 0;
  const int64_t lastb = nb > 0 ? nb - 1 : 0;
#pragma unroll
  for (int i = 0; i < SCAN_REG; i++) v[i] = bsum[i < per && a + i < nb ? a + i : lastb];   // (clamped, masked below)
#pragma unroll
  for (int i = 0; i < SCAN_REG; i++) {
    if (!(i < per && a + i < nb)) v[i] = 0;
    sum += v[i];
  }
  int64_t incl = sum;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int64_t y = __shfl_up(incl, d, 64);
    if (lane >= d) incl += y;
  }
  if (lane == 63) s_w[wid] = incl;
  __syncthreads();
  int64_t run = incl - sum;
  for (int w = 0; w < wid; w++) run += s_w[w];
#pragma unroll
  for (int i = 0; i < SCAN_REG; i++)
    if (i < per && a + i < nb) { bsum[a + i] = run; run += v[i]; }
  if (tid == 1023) *total = run;
}
__global__ __launch_bounds__(1024) void scan_sums_reg(int64_t* __restrict__ bsum, int64_t nb, int64_t* __restrict__ total) {
  scan_sums_reg_body(bsum, nb, total);
}
__global__ __launch_bounds__(1024) void scan_sums_pair(ScanPair S, int64_t* __restrict__ bsum) {
  const int64_t nb = (scan_len(S) + 1023) / 1024;
  scan_sums_reg_body(bsum + blockIdx.x * S.nb, nb, S.total[blockIdx.x]);
}
__global__ void scan_final(ScanPair S, const int64_t* __restrict__ bsum) {
  __shared__ int64_t s[256];
  const int64_t n = scan_len(S);
  const int64_t* __restrict__ in = S.in[blockIdx.y];
  int64_t* __restrict__ out = S.out[blockIdx.y];
  const int64_t b0 = int64_t(blockIdx.x) * 1024;
  if (b0 >= n) return;                             // (whole block: the barriers below stay uniform)
  int64_t v[4], acc = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int64_t i = b0 + threadIdx.x * 4 + k;
    v[k] = in[i < n ? i : n - 1];                  // (clamped, masked below; n > b0 >= 0 here)
  }
#pragma unroll
  for (int k = 0; k < 4; k++) {
    if (b0 + threadIdx.x * 4 + k >= n) v[k] = 0;
    acc += v[k];
  }
  int64_t tot = 0;
  int64_t run = bsum[blockIdx.y * S.nb + blockIdx.x] + block_excl_256(acc, s, tot);
  for (int k = 0; k < 4; k++) {
    const int64_t i = b0 + threadIdx.x * 4 + k;
    if (i < n) out[i] = run;
    run += v[k];
  }
}

// jf: the pattern's compiled nfa kernel (jit.cpp), nullptr for the built-in interpreting one.
// One wave per workgroup, A.spread key segments per wave.
hipError_t nfa_launch(const NfaArgs& A, hipStream_t st, hipFunction_t jf) {
  if (A.nseg <= 0) return hipSuccess;
  const unsigned grid = unsigned((A.nseg + A.spread - 1) / A.spread);
  if (jf) {
    NfaArgs a = A;
    void* args[] = {&a};
    return hipModuleLaunchKernel(jf, grid, 1, 1, 64, 1, 1, 0, st, args, nullptr);
  }
  hipLaunchKernelGGL(nfa_kernel, dim3(grid), dim3(64), 0, st, A);
  return hipGetLastError();
}

// ---- the wave kernel's schedule (nfa_dev.h stage_may_take): heaviest estimated segments first ----
__global__ __launch_bounds__(256) void nfa_order_bits(NfaArgs A, uint8_t* bits) { nfa_order_bits_body(A, bits); }
// The per-wave bucket sizes of a 256-thread block into s_w[4][16] (no atomics: each wave its own row);
// returns the lane's rank among its wave's lanes of its bucket
__device__ __forceinline__ unsigned order_wave_counts(int b, unsigned (*s_w)[16]) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  unsigned rank = 0;
  for (int q = 0; q < 16; q++) {
    const uint64_t m = __builtin_amdgcn_ballot_w64(b == q);
    if (lane == 0) s_w[wv][q] = unsigned(__popcll(m));
    if (b == q) rank = __builtin_amdgcn_mbcnt_hi(uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0));
  }
  return rank;
}
// one thread per segment: its weight from its records' bits (walked backwards: sum over begin-matching
// records of 2^(later matching records)), log2-bucketed, buckets below lo merged into bucket 0 (their
// segments keep arrival order); each block's bucket sizes into bcnt[block][16]
__global__ __launch_bounds__(256) void nfa_order_count(const int64_t* __restrict__ seg_start,
                                                       const int64_t* __restrict__ nseg_dev, int64_t nseg_host,
                                                       const uint8_t* __restrict__ bits, uint8_t* __restrict__ bucket,
                                                       unsigned* __restrict__ bcnt, int lo) {
  __shared__ unsigned s_w[4][16];
  const int64_t nseg = nseg_dev ? *nseg_dev : nseg_host;
  if (int64_t(blockIdx.x) * blockDim.x >= nseg) return;   // (the grid is sized by a bound)
  const int64_t t = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  int b = -1;
  if (t < nseg) {
    float w = 0.f;
    int after = 0;
    for (int64_t g = seg_start[t + 1] - 1; g >= seg_start[t]; g--) {
      const uint32_t x = bits[g];
      if (x & 1) w += exp2f(float(after < 100 ? after : 100));
      after += (x >> 1) & 1;
    }
    const int lb = w < 2.f ? 0 : int(log2f(w));
    b = lb < 15 ? lb : 15;
    b = b < lo ? 0 : b;
    bucket[t] = uint8_t(b);
  }
  order_wave_counts(b, s_w);
  __syncthreads();
  if (threadIdx.x < 16) {
    const int q = threadIdx.x;
    bcnt[size_t(blockIdx.x) * 16 + q] = s_w[0][q] + s_w[1][q] + s_w[2][q] + s_w[3][q];
  }
}
// each segment's place: the buckets from the heaviest down, within a bucket by segment index (a
// deterministic schedule; the schedule only: every key's results land in its own segment's slots)
__global__ __launch_bounds__(256) void nfa_order_place(const int64_t* __restrict__ nseg_dev, int64_t nseg_host,
                                                       const uint8_t* __restrict__ bucket,
                                                       const unsigned* __restrict__ bcnt, int32_t* __restrict__ order) {
  __shared__ unsigned s_tot[16][17], s_bef[16][17], s_base[16], s_w[4][16];
  const int64_t nseg = nseg_dev ? *nseg_dev : nseg_host;
  if (int64_t(blockIdx.x) * blockDim.x >= nseg) return;
  const int64_t nblk = (nseg + 255) / 256;
  {                                                // bucket q over all blocks / the blocks before this one
    const int q = threadIdx.x & 15, part = threadIdx.x >> 4;
    unsigned tot = 0, bef = 0;
    for (int64_t k = part; k < nblk; k += 16) {
      const unsigned c = bcnt[size_t(k) * 16 + q];
      tot += c;
      bef += k < int64_t(blockIdx.x) ? c : 0u;
    }
    s_tot[q][part] = tot;
    s_bef[q][part] = bef;
  }
  const int64_t t = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const int b = t < nseg ? int(bucket[t]) : -1;
  const unsigned rank = order_wave_counts(b, s_w);
  __syncthreads();
  if (threadIdx.x < 16) {
    const int q = threadIdx.x;
    unsigned tot = 0, bef = 0;
    for (int k = 0; k < 16; k++) {
      tot += s_tot[q][k];
      bef += s_bef[q][k];
    }
    s_tot[q][16] = tot;
    s_bef[q][16] = bef;
  }
  __syncthreads();
  if (threadIdx.x < 16) {                          // heavier buckets first, then this bucket's earlier blocks
    const int q = threadIdx.x;
    unsigned base = s_bef[q][16];
    for (int r = q + 1; r < 16; r++) base += s_tot[r][16];
    s_base[q] = base;
  }
  __syncthreads();
  if (b < 0) return;
  const int wv = threadIdx.x >> 6;
  unsigned at = s_base[b] + rank;
  for (int k = 0; k < wv; k++) at += s_w[k][b];
  order[at] = int32_t(t);
}
// bits: A.n bytes; bcnt: 16 words per 256 segments; the segment grids over nseg (an upper bound with
// A.nseg_dev: their blocks past the real count return at once)
hipError_t nfa_order_launch(const NfaArgs& A, int64_t nseg, uint8_t* bits, unsigned* bcnt, int32_t* order,
                            hipStream_t st, const JitModule* j, int lo) {
  if (nseg <= 0 || A.n <= 0) return hipSuccess;
  const unsigned rblocks = unsigned((A.n + 255) / 256), sblocks = unsigned((nseg + 255) / 256);
  if (j && j->nfa_order) {
    NfaArgs a = A;
    void* args[] = {&a, &bits};
    hipError_t e = hipModuleLaunchKernel(j->nfa_order, rblocks, 1, 1, 256, 1, 1, 0, st, args, nullptr);
    if (e != hipSuccess) return e;
  } else {
    hipLaunchKernelGGL(nfa_order_bits, dim3(rblocks), dim3(256), 0, st, A, bits);
  }
  hipLaunchKernelGGL(nfa_order_count, dim3(sblocks), dim3(256), 0, st, A.seg_start, A.nseg_dev, nseg, bits, A.seg_bucket,
                     bcnt, lo);
  hipLaunchKernelGGL(nfa_order_place, dim3(sblocks), dim3(256), 0, st, A.nseg_dev, nseg, A.seg_bucket, bcnt, order);
  return hipGetLastError();
}

// The workgroups (one wave each) the wave kernel's persistent grid should have: as many as the chip
// holds at once (occupancy x compute units), at most one per segment.
int64_t nfa_wave_grid(int64_t nseg, bool agg, const JitModule* j) {
  int per_cu = 0, cus = 0, dev = 0;
  hipError_t e = j ? hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, j->nfa_wave, 64, 0)
                   : agg ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, nfa_wave_kernel<true>, 64, 0)
                         : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, nfa_wave_kernel<false>, 64, 0);
  if (e != hipSuccess || per_cu <= 0) per_cu = 12;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      cus <= 0)
    cus = 256;
  const int64_t g = int64_t(per_cu) * cus;
  return nseg < g ? nseg : g;
}

// The wave kernel over A.nseg key segments on `grid` persistent workgroups (A.seg_next zeroed by the
// caller; A.scratch holds grid x A.scratch_words words).  j: the pattern's compiled kernel (null: the
// built-in interpreting one).
hipError_t nfa_wave_launch(const NfaArgs& A, int64_t grid, hipStream_t st, const JitModule* j) {
  if (A.nseg <= 0 || grid <= 0) return hipSuccess;
  NfaArgs a = A;
  void* args[] = {&a};
  if (j) return hipModuleLaunchKernel(j->nfa_wave, unsigned(grid), 1, 1, 64, 1, 1, 0, st, args, nullptr);
  if (A.wave_agg) hipLaunchKernelGGL(nfa_wave_kernel<true>, dim3(unsigned(grid)), dim3(64), 0, st, A);
  else hipLaunchKernelGGL(nfa_wave_kernel<false>, dim3(unsigned(grid)), dim3(64), 0, st, A);
  return hipGetLastError();
}

hipError_t exclusive_scan(const int64_t* in, int64_t n, int64_t* out, int64_t* total, int64_t* tmp,
                          hipStream_t st) {
  if (n <= 0) return hipMemsetAsync(total, 0, sizeof(int64_t), st);
  const int64_t nb = (n + 1023) / 1024;
  const ScanPair S{{in, in}, {out, out}, {total, total}, n, nullptr, nb};
  hipLaunchKernelGGL(scan_blocks, dim3(unsigned(nb)), dim3(256), 0, st, S, tmp);
  if (nb <= int64_t(SCAN_REG) * 1024) hipLaunchKernelGGL(scan_sums_reg, dim3(1), dim3(1024), 0, st, tmp, nb, total);
  else hipLaunchKernelGGL(scan_sums, dim3(1), dim3(256), 0, st, tmp, nb, total);
  hipLaunchKernelGGL(scan_final, dim3(unsigned(nb)), dim3(256), 0, st, S, tmp);
  return hipGetLastError();
}

// w[0..n) = 0 except w[at] = v
__global__ void set_words(int64_t* __restrict__ w, int n, int at, int64_t v) {
  const int t = threadIdx.x;
  if (t < n) w[t] = t == at ? v : 0;
}
hipError_t set_words_launch(int64_t* w, int n, int at, int64_t v, hipStream_t st) {
  if (n > 64) return hipErrorInvalidValue;
  hipLaunchKernelGGL(set_words, dim3(1), dim3(64), 0, st, w, n, at, v);
  return hipGetLastError();
}
// a[0..na) then b[0..nb) into h (pinned host memory mapped for the device): the host's view of a batch
__global__ void gather_words(const int64_t* __restrict__ a, int na, const int64_t* __restrict__ b, int nb,
                             int64_t* __restrict__ h) {
  const int t = threadIdx.x;
  if (t < na) h[t] = a[t];
  else if (t < na + nb) h[t] = b[t - na];
}
hipError_t gather_words_launch(const int64_t* a, int na, const int64_t* b, int nb, int64_t* h, hipStream_t st) {
  if (na + nb > 64) return hipErrorInvalidValue;
  hipLaunchKernelGGL(gather_words, dim3(1), dim3(64), 0, st, a, na, b, nb, h);
  return hipGetLastError();
}

// Two exclusive scans of one length n (or *n_dev <= n, read on the device) in one set of launches;
// tmp: 2 x ceil(n / 1024) words.
hipError_t exclusive_scan_pair(const int64_t* in0, const int64_t* in1, int64_t n, const int64_t* n_dev, int64_t* out0,
                               int64_t* out1, int64_t* total0, int64_t* total1, int64_t* tmp, hipStream_t st) {
  const int64_t nb = (std::max<int64_t>(n, 1) + 1023) / 1024;
  const ScanPair S{{in0, in1}, {out0, out1}, {total0, total1}, std::max<int64_t>(n, 0), n_dev, nb};
  hipLaunchKernelGGL(scan_blocks, dim3(unsigned(nb), 2), dim3(256), 0, st, S, tmp);
  if (nb <= int64_t(SCAN_REG) * 1024) {
    hipLaunchKernelGGL(scan_sums_pair, dim3(2), dim3(1024), 0, st, S, tmp);
  } else {                                         // (blocks past *n_dev summed to 0 in scan_blocks)
    hipLaunchKernelGGL(scan_sums, dim3(1), dim3(256), 0, st, tmp, nb, total0);
    hipLaunchKernelGGL(scan_sums, dim3(1), dim3(256), 0, st, tmp + nb, nb, total1);
  }
  hipLaunchKernelGGL(scan_final, dim3(unsigned(nb), 2), dim3(256), 0, st, S, tmp);
  return hipGetLastError();
}

// The segments' matches into one CSR in segment (key) order: one thread per match and one per entry,
// each finding its segment by a binary search over the segments' exclusive prefixes (moff / eoff, in
// L2), so that a key with thousands of matches is copied as fast as one with a single match.  A key's
// match headers {pos lo, pos hi, entries, first entry} and entries {name, pos lo, pos hi} are each
// contiguous in the pool (nfa_dev.h emit_match, nfa_wave.h wave_emit_matches).
__device__ __forceinline__ int64_t seg_of(const int64_t* __restrict__ off, int64_t nseg, int64_t x) {
  int64_t lo = 0, hi = nseg - 1;                   // the last segment whose range starts at or before x
  while (lo < hi) {
    const int64_t mid = (lo + hi + 1) >> 1;
    if (off[mid] <= x) lo = mid; else hi = mid - 1;
  }
  return lo;
}
// tot_dev / nseg_dev (optional): the batch's match / entry totals and segment count on the device, the
// grid sized by an upper bound (a compaction enqueued before the host has read them)
__global__ void nfa_compact_matches(int64_t nseg, const int64_t* __restrict__ nseg_dev, int64_t nm,
                                    const int64_t* __restrict__ tot_dev, const int32_t* __restrict__ key,
                                    const int64_t* __restrict__ seg_start, const int64_t* __restrict__ res_out,
                                    const int64_t* __restrict__ moff, const int64_t* __restrict__ eoff,
                                    int64_t* __restrict__ match_record, int32_t* __restrict__ match_key,
                                    int64_t* __restrict__ ent_off) {
  const int64_t m = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (m >= (tot_dev && tot_dev[0] < nm ? tot_dev[0] : nm)) return;
  const int64_t s = seg_of(moff, nseg_dev ? *nseg_dev : nseg, m);
  const int4 h = reinterpret_cast<const int4*>(uintptr_t(res_out[s]))[m - moff[s]];
  match_record[m] = int64_t(uint64_t(uint32_t(h.x)) | (uint64_t(uint32_t(h.y)) << 32));
  match_key[m] = key[seg_start[s]];
  ent_off[m] = eoff[s] + h.w;
}
__global__ void nfa_compact_entries(int64_t nseg, const int64_t* __restrict__ nseg_dev, int64_t ne,
                                    const int64_t* __restrict__ tot_dev, const int64_t* __restrict__ res_ent,
                                    const int64_t* __restrict__ eoff, int32_t* __restrict__ ent_name,
                                    int64_t* __restrict__ ent_record) {
  const int64_t e = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (e >= (tot_dev && tot_dev[1] < ne ? tot_dev[1] : ne)) return;
  const int64_t s = seg_of(eoff, nseg_dev ? *nseg_dev : nseg, e);
  const int32_t* x = reinterpret_cast<const int32_t*>(uintptr_t(res_ent[s])) + 3 * (e - eoff[s]);
  ent_name[e] = x[0];
  ent_record[e] = cw64(x + 1);
}
// NFAStoreImpl.put of every key of the batch: the key's table entry points at its new blob
// (keys whose processing raised keep their previous state, like the failed task)
__global__ void carry_commit(int64_t nseg, const int32_t* __restrict__ key, const int64_t* __restrict__ seg_start,
                             const int64_t* __restrict__ res_carry, const int32_t* __restrict__ res_err,
                             int64_t* __restrict__ ctab) {
  const int64_t s = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (s >= nseg || res_err[s] || res_carry[s] < 0) return;
  ctab[key[seg_start[s]]] = res_carry[s];
}
// Carry sessions need each key in one contiguous segment (the batch contract of kcep.h): a key
// met in two segments would load its blob twice and lose one segment's update.  Every segment
// stamps its key with the batch number; a stamp that is already there means a second segment.
// flags: bit 0 a key id outside [0, max_keys), bit 1 a key owning two segments.
__global__ void carry_keycheck(const int64_t* __restrict__ nseg, const int32_t* __restrict__ key,
                               const int64_t* __restrict__ seg_start, int32_t max_keys, int32_t* __restrict__ stamp,
                               int32_t batch_no, unsigned long long* __restrict__ flags) {
  const int64_t s = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (s >= *nseg) return;
  const int32_t k = key[seg_start[s]];
  if (k < 0 || k >= max_keys) { atomicOr(flags, 1ull); return; }
  if (atomicExch(stamp + k, batch_no) == batch_no) atomicOr(flags, 2ull);
}
// carry-pool compaction: live blob sizes, then a copy to the fresh pool
__global__ void carry_sizes(const int64_t* __restrict__ ctab, int64_t nkeys, const int32_t* __restrict__ cpool,
                            int64_t* __restrict__ words) {
  const int64_t k = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (k < nkeys) words[k] = ctab[k] >= 0 ? cpool[ctab[k] + CB_WORDS] : 0;
}
__global__ void carry_move(int64_t* __restrict__ ctab, int64_t nkeys, const int32_t* __restrict__ src,
                           const int64_t* __restrict__ off, int32_t* __restrict__ dst) {
  const int64_t k = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (k >= nkeys || ctab[k] < 0) return;
  const int32_t* a = src + ctab[k];
  int32_t* b = dst + off[k];
  const int32_t w = a[CB_WORDS];
  for (int32_t i = 0; i < w; i++) b[i] = a[i];
  ctab[k] = off[k];
}

// flag / idx: nullptr, or n words each (the runs carry build's per-record boundary flags); tmp:
// ceil(n / 1024) + 1 words.  *nseg: the segment count (device).
hipError_t nfa_segments(const int32_t* key, int64_t n, int64_t* flag, int64_t* idx, int64_t* seg_start, int64_t* nseg,
                        int64_t* tmp, hipStream_t st) {
  if (n <= 0) return hipMemsetAsync(nseg, 0, sizeof(int64_t), st);
  const int64_t nb = (n + 1023) / 1024;
  hipLaunchKernelGGL(seg_count, dim3(unsigned(nb)), dim3(256), 0, st, key, n, tmp);
  if (nb <= int64_t(SCAN_REG) * 1024) hipLaunchKernelGGL(scan_sums_reg, dim3(1), dim3(1024), 0, st, tmp, nb, nseg);
  else hipLaunchKernelGGL(scan_sums, dim3(1), dim3(256), 0, st, tmp, nb, nseg);
  hipLaunchKernelGGL(seg_write, dim3(unsigned(nb)), dim3(256), 0, st, key, n, tmp, nseg, seg_start, flag, idx);
  return hipGetLastError();
}

hipError_t nfa_compact_launch(int64_t nseg, const int64_t* nseg_dev, int64_t nm, int64_t ne, const int64_t* tot_dev,
                              const int32_t* key, const int64_t* seg_start, const int64_t* res_out, const int64_t* res_ent,
                              const int64_t* moff, const int64_t* eoff, int64_t* match_record, int32_t* match_key,
                              int64_t* ent_off, int32_t* ent_name, int64_t* ent_record, hipStream_t st) {
  if (nseg <= 0) return hipSuccess;
  if (nm > 0)
    hipLaunchKernelGGL(nfa_compact_matches, dim3(unsigned((nm + 255) / 256)), dim3(256), 0, st, nseg, nseg_dev, nm, tot_dev,
                       key, seg_start, res_out, moff, eoff, match_record, match_key, ent_off);
  if (ne > 0)
    hipLaunchKernelGGL(nfa_compact_entries, dim3(unsigned((ne + 255) / 256)), dim3(256), 0, st, nseg, nseg_dev, ne, tot_dev,
                       res_ent, eoff, ent_name, ent_record);
  return hipGetLastError();
}

hipError_t carry_commit_launch(int64_t nseg, const int32_t* key, const int64_t* seg_start, const int64_t* res_carry,
                               const int32_t* res_err, int64_t* ctab, hipStream_t st) {
  if (nseg <= 0) return hipSuccess;
  hipLaunchKernelGGL(carry_commit, dim3(unsigned((nseg + 255) / 256)), dim3(256), 0, st, nseg, key, seg_start,
                     res_carry, res_err, ctab);
  return hipGetLastError();
}

// max_seg: a host bound on the segment count (the batch size); the count itself is on the device
hipError_t carry_keycheck_launch(int64_t max_seg, const int64_t* nseg, const int32_t* key, const int64_t* seg_start,
                                int32_t max_keys, int32_t* stamp, int32_t batch_no, unsigned long long* flags,
                                hipStream_t st) {
  if (max_seg <= 0) return hipSuccess;
  hipLaunchKernelGGL(carry_keycheck, dim3(unsigned((max_seg + 255) / 256)), dim3(256), 0, st, nseg, key, seg_start,
                     max_keys, stamp, batch_no, flags);
  return hipGetLastError();
}

hipError_t carry_sizes_launch(const int64_t* ctab, int64_t nkeys, const int32_t* cpool, int64_t* words,
                              hipStream_t st) {
  if (nkeys <= 0) return hipSuccess;
  hipLaunchKernelGGL(carry_sizes, dim3(unsigned((nkeys + 255) / 256)), dim3(256), 0, st, ctab, nkeys, cpool, words);
  return hipGetLastError();
}

hipError_t carry_move_launch(int64_t* ctab, int64_t nkeys, const int32_t* src, const int64_t* off, int32_t* dst,
                             hipStream_t st) {
  if (nkeys <= 0) return hipSuccess;
  hipLaunchKernelGGL(carry_move, dim3(unsigned((nkeys + 255) / 256)), dim3(256), 0, st, ctab, nkeys, src, off, dst);
  return hipGetLastError();
}

}  // namespace kcep

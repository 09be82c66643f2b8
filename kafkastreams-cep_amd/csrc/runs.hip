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

#include <stdlib.h>
#include <string.h>

#include <algorithm>

#include <rocprim/device/device_radix_sort.hpp>

#include "../../include/kcep.h"
#include "kcep_internal.h"
#include "interp.h"
#include "runs_dev.h"

namespace kcep {

namespace {

__global__ __launch_bounds__(RT) void runs_sim(RunsArgs A, int64_t* __restrict__ flag, int32_t* __restrict__ end_of) {
  runs_sim_body(InterpTab{A.P}, runs_args_dev(A), flag, end_of);
}

__global__ __launch_bounds__(RT) void runs_write(WriteArgs W) { runs_write_body(InterpTab{W.R.P}, W); }

// completed runs in start order, key (end << 31 | start): one workgroup per runs_sim chunk, placed at
// the exclusive scan of the chunks' counts (pre), each thread's items contiguous so that a block scan
// of the per-thread counts ranks them.  256 threads x up to 4 items: the chunk is a power of two of at
// most 1024 records (runs_compact_launch checks it)
static_assert(RUNS_CHUNK <= 1024 && (RUNS_CHUNK & (RUNS_CHUNK - 1)) == 0, "runs_compact covers chunks of <= 4 x 256");
__global__ __launch_bounds__(256) void runs_compact(const int32_t* __restrict__ end_of, int64_t n, int chunk,
                                                    const int64_t* __restrict__ pre, unsigned long long* __restrict__ out) {
  __shared__ int32_t s_w[4];
  const int ipt = chunk > 256 ? chunk >> 8 : 1;
  const int64_t c0 = int64_t(blockIdx.x) * chunk, c1 = c0 + chunk < n ? c0 + chunk : n;
  const int64_t a = c0 + int64_t(threadIdx.x) * ipt;
  int32_t e[4];
  int cnt = 0;
#pragma unroll
  for (int q = 0; q < 4; q++) {
    e[q] = -1;
    if (q < ipt && a + q < c1) e[q] = end_of[a + q];
    cnt += e[q] >= 0;
  }
  int inc = cnt;                                    // inclusive scan over the wave
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(inc, d, 64);
    if ((threadIdx.x & 63) >= d) inc += y;
  }
  if ((threadIdx.x & 63) == 63) s_w[threadIdx.x >> 6] = inc;
  __syncthreads();
  int64_t at = pre[blockIdx.x] + inc - cnt;
  for (int w = 0; w < int(threadIdx.x >> 6); w++) at += s_w[w];
#pragma unroll
  for (int q = 0; q < 4; q++)
    if (e[q] >= 0) out[at++] = (unsigned long long)(int64_t(e[q]) << 31 | (a + q));
}

// exclusive scans of the chunks' run counts and lengths (stat[w], stat[W + w]) in one workgroup:
// pre[w], pre[W + w]; the totals into *tot_cnt / *tot_len
// (each thread sums a contiguous run of chunks, one block scan of the thread sums, then the thread
// writes its run's prefixes: one pass, two barriers)
// by_end: the chunks' runs counted by the chunk they END in (runs_sim's stat[2W..6W): those ending in
// chunk w are chunk w's own plus chunk w - 1's that ran over)
template <bool by_end>
__device__ __forceinline__ int64_t chunk_stat(const int64_t* __restrict__ stat, int64_t W, int q, int64_t w) {
  if (!by_end) return stat[q * W + w];
  return stat[(2 + q) * W + w] + (w > 0 ? stat[(4 + q) * W + w - 1] : 0);
}
// n_dev (optional): the records on the device (the chunks past them hold no statistics)
template <bool by_end>
__global__ __launch_bounds__(1024) void runs_chunk_scan(const int64_t* __restrict__ stat, int64_t nw, int64_t W,
                                                        int64_t* __restrict__ pre, int64_t* __restrict__ tot_cnt,
                                                        int64_t* __restrict__ tot_len, const int64_t* __restrict__ n_dev,
                                                        int chunk) {
  __shared__ int64_t s_c[16], s_l[16];
  constexpr int REG = 16;                          // up to 16 K chunks: each thread's sums stay in registers
  if (n_dev && (*n_dev + chunk - 1) / chunk < nw) nw = (*n_dev + chunk - 1) / chunk;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t per = (nw + 1023) / 1024, w0 = int64_t(threadIdx.x) * per, w1 = w0 + per < nw ? w0 + per : nw;
  int64_t c = 0, l = 0;
  int64_t cc[REG], ll[REG];
  if (per <= REG) {                                // every load in flight at once
#pragma unroll
    for (int q = 0; q < REG; q++) {
      cc[q] = w0 + q < w1 ? chunk_stat<by_end>(stat, W, 0, w0 + q) : 0;
      ll[q] = w0 + q < w1 ? chunk_stat<by_end>(stat, W, 1, w0 + q) : 0;
    }
#pragma unroll
    for (int q = 0; q < REG; q++) { c += cc[q]; l += ll[q]; }
  } else {
    for (int64_t w = w0; w < w1; w++) {
      c += chunk_stat<by_end>(stat, W, 0, w);
      l += chunk_stat<by_end>(stat, W, 1, w);
    }
  }
  int64_t ic = c, il = l;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int64_t yc = __shfl_up(ic, d, 64), yl = __shfl_up(il, d, 64);
    if (lane >= d) { ic += yc; il += yl; }
  }
  if (lane == 63) { s_c[wv] = ic; s_l[wv] = il; }
  __syncthreads();
  int64_t oc = ic - c, ol = il - l;
  for (int q = 0; q < wv; q++) { oc += s_c[q]; ol += s_l[q]; }
  if (per <= REG) {
#pragma unroll
    for (int q = 0; q < REG; q++)
      if (w0 + q < w1) {
        pre[w0 + q] = oc;
        pre[W + w0 + q] = ol;
        oc += cc[q];
        ol += ll[q];
      }
  } else {
    for (int64_t w = w0; w < w1; w++) {
      pre[w] = oc;
      pre[W + w] = ol;
      oc += chunk_stat<by_end>(stat, W, 0, w);
      ol += chunk_stat<by_end>(stat, W, 1, w);
    }
  }
  if (threadIdx.x == 1023) {
    int64_t tc = 0, tl = 0;
    for (int q = 0; q < 16; q++) { tc += s_c[q]; tl += s_l[q]; }
    *tot_cnt = tc;
    *tot_len = tl;
  }
}

// Completed runs from start order into (completing record, start) order without a device-wide sort.
// Each start record begins at most one run, so the compacted runs have distinct, increasing starts.
// Run i's place in the stable order by end: i - #{j < i : e_j > e_i} + #{j > i : e_j < e_i}.  Such a j
// overlaps run i, so with every run's span e - s <= W: j < i has s_j >= s_i - W, j > i has s_j < e_i <=
// s_i + W, and (distinct starts) |i - j| <= W.  A workgroup ranks 256 runs against the window of runs
// [first - W, last + W] staged in LDS (W <= RUNS_ORDER_MAX_W; wider batches take the radix sort).
static_assert(RUNS_MAX_SEGS == 8, "a run's segments are at most one uint4 of 16-bit words");
constexpr int RUNS_ORDER_MAX_W = 1024;
constexpr int RUNS_ORDER_WIN = 256 + 2 * RUNS_ORDER_MAX_W;
// The backward count skips whole groups of 16 window entries whose latest end is <= e: no run there
// ends after run i.  Most runs are short (C3: mean span 5, p99 35, max 91), so only the few groups
// holding a long run are scanned; a plain scan over [i - W, i) took ~100 steps per run (131 us at C3).
__global__ __launch_bounds__(256) void runs_order(const unsigned long long* __restrict__ in, int64_t nm, int w,
                                                  unsigned long long* __restrict__ out, int64_t* __restrict__ len) {
  __shared__ unsigned long long s_r[RUNS_ORDER_WIN];
  __shared__ int32_t s_gm[RUNS_ORDER_WIN / 16 + 1];
  const int64_t b0 = int64_t(blockIdx.x) * 256;
  const int64_t lo = b0 - w > 0 ? b0 - w : 0, hi = b0 + 256 + w < nm ? b0 + 256 + w : nm;
  const int L = int(hi - lo);
  for (int x = threadIdx.x; x < L; x += 256) s_r[x] = in[lo + x];
  __syncthreads();
  for (int g = threadIdx.x; g < (L + 15) / 16; g += 256) {
    int32_t m = -1;
    const int x1 = g * 16 + 16 < L ? g * 16 + 16 : L;
    for (int x = g * 16; x < x1; x++) {
      const int32_t e = int32_t(s_r[x] >> 31);
      m = e > m ? e : m;
    }
    s_gm[g] = m;
  }
  __syncthreads();
  const int64_t i = b0 + threadIdx.x;
  if (i >= nm) return;
  const int il = int(i - lo);
  const unsigned long long me = s_r[il];
  const int32_t e = int32_t(me >> 31);
  int64_t p = i;
  int x = il - 1;                                  // earlier starts ending later
  for (; x >= 0 && (x & 15) != 15; x--) p -= int32_t(s_r[x] >> 31) > e;
  for (; x >= 0; x -= 16) {
    if (s_gm[x >> 4] <= e) continue;
#pragma unroll
    for (int q = 0; q < 16; q++) p -= int32_t(s_r[x - q] >> 31) > e;
  }
  for (int y = il + 1; y < L; y++) {               // later starts ending earlier
    const unsigned long long r = s_r[y];
    if (int64_t(r & 0x7FFFFFFFull) >= int64_t(e)) break;
    p += int32_t(r >> 31) < e;
  }
  out[p] = me;
  len[p] = int64_t(e) - int64_t(me & 0x7FFFFFFFull) + 1;     // its entries (runs_lengths, fused)
}


// the CSR of the sorted completed runs from their recorded stage segments (runs_sim with A.segs),
// entries final stage first (peek, SharedVersionedBufferStoreImpl.java:176-201).  A workgroup owns
// 256 consecutive matches and writes their entries as one contiguous range, thread-strided (coalesced
// stores); an entry finds its match by a binary search over the workgroup's entry offsets in LDS.
// the stage of the record `o` records after the run's start, from its packed segments (runs_sim)
__device__ __forceinline__ uint32_t seg_word(const uint4& v, int i) {
  const uint32_t w = i < 2 ? v.x : i < 4 ? v.y : i < 6 ? v.z : v.w;
  return (i & 1) ? w >> 16 : w & 0xFFFF;
}
__device__ __forceinline__ int seg_stage(const uint4& v, int segn, int64_t o) {
  int stage = 0;
#pragma unroll
  for (int i = 0; i < RUNS_MAX_SEGS; i++) {        // the segment holding offset o (segments ascend)
    if (i >= segn) break;
    const uint32_t w = seg_word(v, i);
    if (w == 0xFFFF) break;
    if (int64_t(w & 0xFFF) <= o) stage = int(w >> 12);
  }
  return stage;
}
__device__ __forceinline__ uint4 seg_load(const uint16_t* __restrict__ segs, int segn, int64_t j) {
  if (segn == 4) {
    const uint2 a = *reinterpret_cast<const uint2*>(segs + j * 4);
    return make_uint4(a.x, a.y, 0xFFFFFFFFu, 0xFFFFFFFFu);
  }
  return *reinterpret_cast<const uint4*>(segs + j * 8);
}
__global__ __launch_bounds__(256) void runs_expand(const DevProgram* __restrict__ P, const int32_t* __restrict__ key,
                                                   const int64_t* __restrict__ pos, const uint16_t* __restrict__ segs, int segn,
                                                   const unsigned long long* __restrict__ sorted, int64_t nm,
                                                   const int64_t* __restrict__ ent_off, int64_t ne, int64_t base,
                                                   int64_t* __restrict__ match_record, int32_t* __restrict__ match_key,
                                                   int64_t* ent_off_out, int32_t* __restrict__ ent_name,
                                                   int64_t* __restrict__ ent_record) {
  __shared__ int64_t s_at[257];
  __shared__ int64_t s_j[256], s_e[256];
  __shared__ uint4 s_seg[256];
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
    match_record[m] = pos ? pos[e] : base + e;
    match_key[m] = key[j];
    if (ent_off_out != ent_off) ent_off_out[m] = at;
    s_seg[tid] = seg_load(segs, segn, j);
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
    ent_name[x] = P->st[seg_stage(s_seg[lo], segn, o)].name;
    ent_record[x] = pos ? pos[j + o] : base + j + o;
  }
}

// The CSR straight from runs_sim's results when every completed run spans fewer records than a chunk
// (so a run ends in its start's chunk or the next): one workgroup per chunk of END records [c0, c1).
// Its runs start in [c0 - span, c1); they are bucketed by end record in LDS (counting sort, each
// bucket then ordered by start), which is (completing record, start) order -- NFA.matchPattern's --
// and placed at the chunk's prefix of the end-chunk counts / entry counts (runs_chunk_scan<true>).
// Match headers, then the entries (final stage first, peek :176-201) thread-strided over the chunk's
// contiguous entry range, each entry's stage from its run's packed segments.  Replaces runs_compact +
// runs_order + the entry-offset scan + runs_expand (one pass over end_of and the segments instead of a
// start-ordered list, a sorted copy, a length array and gathers at start positions).
#ifndef RUNS_EMIT_PROBE
#define RUNS_EMIT_PROBE 0                          // timing probes (A/B builds only): 1 no output, 2 headers only
#endif
constexpr int RUNS_EMIT_MAX = 2 * RUNS_CHUNK;      // window of starts: chunk + span < 2 chunks
constexpr int EMIT_T = 2048;                       // entries per pass of the entry phase (8 per thread)
static_assert(RUNS_EMIT_MAX <= 65536, "run indices are 16-bit in the entry phase");
// SEG4: 4-word segment records (staged in LDS); POS: stream positions from pos[] (else base + record).
// Template flags, not run-time branches: a branch that may load from global memory makes the compiler
// wait for every outstanding memory operation -- this loop's own stores included -- before the merged
// value is used, one store round trip per entry pass
template <bool SEG4, bool POS>
__global__ __launch_bounds__(256) void runs_emit(const DevProgram* __restrict__ P, const int32_t* __restrict__ key,
                                                 const int64_t* __restrict__ pos, int64_t base,
                                                 const uint16_t* __restrict__ segs, int segn,
                                                 const int32_t* __restrict__ end_of, int64_t n, int chunk, int span,
                                                 const int64_t* __restrict__ pre, int64_t W,
                                                 int64_t* __restrict__ match_record, int32_t* __restrict__ match_key,
                                                 int64_t* __restrict__ ent_off, int32_t* __restrict__ ent_name,
                                                 int64_t* __restrict__ ent_record) {
  // dynamic LDS sized by the window (runs_emit_lds): at most chunk + span runs end in the chunk
  extern __shared__ __attribute__((aligned(16))) unsigned char emit_lds[];
  const int WN = chunk + span + 1;
  uint2* const s_seg = reinterpret_cast<uint2*>(emit_lds);   // the runs' packed segments (segn == 4)
  int32_t* const s_run = reinterpret_cast<int32_t*>(s_seg + WN);   // window offset of the start | end slot << 11
  int32_t* const s_at = s_run + WN;                // the runs' entry offsets in the chunk (WN + 1) ...
  int32_t* const s_fill = s_at;                    // ... and, before them, the end slots' fill cursors
  // end slot counts, then their prefix (chunk + 1 <= WN words): in s_seg's space, which is written only
  // after the runs are sorted (one 4 KB array less: 8 workgroups per CU instead of 7 at C3's span)
  int32_t* const s_cnt = reinterpret_cast<int32_t*>(s_seg);
  __shared__ int32_t s_w[4];
  __shared__ int32_t s_name[16];
  __shared__ __attribute__((aligned(16))) uint16_t s_of[EMIT_T];   // per entry of the pass: its run
  const int tid = threadIdx.x;
  const int64_t c = blockIdx.x, c0 = c * chunk, c1 = c0 + chunk < n ? c0 + chunk : n;
  if (tid < 16) s_name[tid] = tid < P->nstages ? P->st[tid].name : 0;
  const int E = int(c1 - c0);
  const int64_t lo = c0 - span > 0 ? c0 - span : 0;
  const int L = int(c1 - lo);                      // <= chunk + span < RUNS_EMIT_MAX
  for (int x = tid; x < E; x += 256) { s_cnt[x] = 0; s_fill[x] = 0; }
  __syncthreads();
  int32_t my[RUNS_EMIT_MAX / 256];                 // this thread's window entries: end slot, or -1
  // the loads at clamped (always valid) addresses, all in flight together: a load under `x < L` was a
  // branch each, waited on inside it -- eight memory round trips in a row
#pragma unroll
  for (int q = 0; q < RUNS_EMIT_MAX / 256; q++) {
    const int x = tid + 256 * q;
    my[q] = end_of[lo + (x < L ? x : L - 1)];
  }
#pragma unroll
  for (int q = 0; q < RUNS_EMIT_MAX / 256; q++) {
    const int x = tid + 256 * q;
    const int64_t e = x < L ? int64_t(my[q]) : -1;
    my[q] = e >= c0 && e < c1 ? int32_t(e - c0) : -1;
  }
#pragma unroll
  for (int q = 0; q < RUNS_EMIT_MAX / 256; q++)
    if (my[q] >= 0) atomicAdd(&s_cnt[my[q]], 1);
  __syncthreads();
  // exclusive scan of the end slots' counts (up to 4 per thread)
  int v[4], acc = 0;
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const int x = 4 * tid + q;
    v[q] = x < E ? s_cnt[x] : 0;
    acc += v[q];
  }
  int inc = acc;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(inc, d, 64);
    if ((tid & 63) >= d) inc += y;
  }
  if ((tid & 63) == 63) s_w[tid >> 6] = inc;
  __syncthreads();
  int run = inc - acc;
  for (int w = 0; w < (tid >> 6); w++) run += s_w[w];
  const int M = s_w[0] + s_w[1] + s_w[2] + s_w[3];  // the chunk's runs
#pragma unroll
  for (int q = 0; q < 4; q++) {                    // (each thread rewrites only the counts it read)
    const int x = 4 * tid + q;
    if (x < E) s_cnt[x] = run;
    run += v[q];
  }
  if (tid == 0) s_cnt[E] = M;
  __syncthreads();
#pragma unroll
  for (int q = 0; q < RUNS_EMIT_MAX / 256; q++)
    if (my[q] >= 0) s_run[s_cnt[my[q]] + atomicAdd(&s_fill[my[q]], 1)] = (tid + 256 * q) | my[q] << 11;
  __syncthreads();
  // each end record's runs by start (insertion sort: buckets hold a few runs)
  for (int x = tid; x < E; x += 256) {
    const int b0 = s_cnt[x], b1 = s_cnt[x + 1];
    for (int i = b0 + 1; i < b1; i++) {
      const int32_t t = s_run[i];
      int k = i - 1;
      while (k >= b0 && s_run[k] > t) { s_run[k + 1] = s_run[k]; k--; }
      s_run[k + 1] = t;
    }
  }
  __syncthreads();
  // the runs' entry offsets: thread tid owns runs [R tid, R tid + R)
  const int R = (M + 255) / 256;
  int lens = 0;
  for (int i = R * tid; i < R * tid + R && i < M; i++) {
    const int32_t r = s_run[i];
    lens += int(c0 - lo) + (r >> 11) - (r & 2047) + 1;
  }
  inc = lens;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(inc, d, 64);
    if ((tid & 63) >= d) inc += y;
  }
  if ((tid & 63) == 63) s_w[tid >> 6] = inc;     // (s_w's first use was read before the last barrier)
  __syncthreads();
  run = inc - lens;
  for (int w = 0; w < (tid >> 6); w++) run += s_w[w];
  const int NE = s_w[0] + s_w[1] + s_w[2] + s_w[3];
  for (int i = R * tid; i < R * tid + R && i < M; i++) {
    s_at[i] = run;
    const int32_t r = s_run[i];
    run += int(c0 - lo) + (r >> 11) - (r & 2047) + 1;
  }
  if (tid == 0) s_at[M] = NE;
  __syncthreads();
  if (RUNS_EMIT_PROBE == 1) return;                // timing probes only (tools/variants.sh): no output
  // match headers, and every run's segments into LDS (all loads of the pass in flight together)
  const int64_t mb = pre[c], eb = pre[W + c];
  if (M > 0) {                                     // (uniform) loads at clamped indices first, then the stores
    uint2 sv[RUNS_EMIT_MAX / 256];
    int32_t kv[RUNS_EMIT_MAX / 256];
    int64_t pv[POS ? RUNS_EMIT_MAX / 256 : 1];
#pragma unroll
    for (int q = 0; q < RUNS_EMIT_MAX / 256; q++) {
      const int i = tid + 256 * q;
      const int32_t r = s_run[i < M ? i : M - 1];
      const int64_t e = c0 + (r >> 11);
      if (SEG4) sv[q] = *reinterpret_cast<const uint2*>(segs + (lo + (r & 2047)) * 4);
      kv[q] = key[e];
      if constexpr (POS) pv[q] = pos[e];
    }
#pragma unroll
    for (int q = 0; q < RUNS_EMIT_MAX / 256; q++) {
      const int i = tid + 256 * q;
      if (i < M) {
        const int64_t e = c0 + (s_run[i] >> 11);
        if (SEG4) s_seg[i] = sv[q];
        if constexpr (POS) match_record[mb + i] = pv[q];
        else match_record[mb + i] = base + e;
        match_key[mb + i] = kv[q];
        ent_off[mb + i] = eb + s_at[i];
      }
    }
  }
  __syncthreads();
  if (RUNS_EMIT_PROBE == 2) return;
  // the entries, EMIT_T at a time: each run's index scattered at its first entry's offset in the window
  // (and the run going on from the previous window at offset 0), an inclusive max-scan over the window
  // gives every entry its run, then each thread writes entries tid, tid + 256, ... (coalesced stores, the
  // window's LDS reads independent of each other).  (Was: per wave, 64 entries at a time, their runs from
  // a bit mask of the run starts built by LDS atomics -- a chain of dependent LDS round trips and two wave
  // barriers per 64 entries: 133 of runs_emit's 206 us on C3.  Before that: a binary search per entry,
  // 222 us; one thread walking each of its runs' entries, 714 us.)
  int carry = 0;                                   // the run holding the window's first entry (or 0)
  for (int w0 = 0; w0 < NE; w0 += EMIT_T) {
#pragma unroll
    for (int q = 0; q < EMIT_T / 256 / 8; q++) reinterpret_cast<uint4*>(s_of)[q * 256 + tid] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    for (int i = tid; i < M; i += 256) {
      const int p = s_at[i] - w0;
      if (p >= 0 && p < EMIT_T) s_of[p] = uint16_t(i);
    }
    __syncthreads();
    // inclusive max-scan, seeded with the run going on (its index is below every run starting in the
    // window: runs are numbered by first entry): 8 consecutive per thread, the wave by shuffles, the
    // waves by s_w
    uint4 v8 = reinterpret_cast<const uint4*>(s_of)[tid];
    uint32_t h[8] = {v8.x & 0xFFFFu, v8.x >> 16, v8.y & 0xFFFFu, v8.y >> 16,
                     v8.z & 0xFFFFu, v8.z >> 16, v8.w & 0xFFFFu, v8.w >> 16};
#pragma unroll
    for (int q = 1; q < 8; q++) h[q] = h[q] > h[q - 1] ? h[q] : h[q - 1];
    uint32_t m = h[7];
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(m, d, 64);
      if ((tid & 63) >= d) m = y > m ? y : m;
    }
    if ((tid & 63) == 63) s_w[tid >> 6] = int(m);
    uint32_t ex = __shfl_up(m, 1, 64);
    if ((tid & 63) == 0) ex = 0;
    ex = ex > uint32_t(carry) ? ex : uint32_t(carry);
    __syncthreads();
    for (int w = 0; w < (tid >> 6); w++) ex = uint32_t(s_w[w]) > ex ? uint32_t(s_w[w]) : ex;
#pragma unroll
    for (int q = 0; q < 8; q++) h[q] = h[q] > ex ? h[q] : ex;
    reinterpret_cast<uint4*>(s_of)[tid] = make_uint4(h[0] | h[1] << 16, h[2] | h[3] << 16, h[4] | h[5] << 16,
                                                     h[6] | h[7] << 16);
    __syncthreads();
    carry = s_of[EMIT_T - 1];
#pragma unroll 4
    for (int q = 0; q < EMIT_T / 256; q++) {
      const int x = w0 + q * 256 + tid;
      if (x < NE) {
        const int a = s_of[q * 256 + tid];
        const int32_t r = s_run[a];
        const int jo = r & 2047;                   // the start, from lo
        const int o = int(c0 - lo) + (r >> 11) - jo - (x - s_at[a]);   // the entry's record, from the start
        const uint4 sg = SEG4 ? make_uint4(s_seg[a].x, s_seg[a].y, 0xFFFFFFFFu, 0xFFFFFFFFu)
                              : seg_load(segs, segn, lo + jo);
        const int64_t rec = lo + jo + o;
        ent_name[eb + x] = s_name[seg_stage(sg, segn, o)];
        ent_record[eb + x] = POS ? pos[rec] : base + rec;
      }
    }
    __syncthreads();                               // (s_of is rewritten by the next window)
  }
}

__global__ void runs_lengths(const unsigned long long* __restrict__ sorted, int64_t nm, int64_t* __restrict__ len) {
  const int64_t m = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (m < nm) len[m] = int64_t(sorted[m] >> 31) - int64_t(sorted[m] & 0x7FFFFFFFull) + 1;
}

// ---- carried tails (CEP_SESSION_CARRY on the runs path) ----
// A run here is a function of its start record and the key's following records, so a key's open
// runs are carried as the key's records from its oldest open run's start on (its "tail", stream
// positions and every field a predicate or fold can read): the next batch of the key is prefixed
// with them and every run is simulated again from its start, which reproduces its stage and fold
// registers exactly.  Runs that end or fail inside the tail were emitted / raised by the earlier
// batch (RunsArgs.emit_from).  Tail records are int64 words: pos, offset, ts, key | topic << 32,
// partition, then the columns' bits.
__device__ __forceinline__ int64_t col_bits(const void* c, int type, int64_t i) {
  return type == T_I32 ? int64_t(static_cast<const int32_t*>(c)[i]) : static_cast<const int64_t*>(c)[i];
}
__device__ __forceinline__ void col_put(void* c, int type, int64_t i, int64_t v) {
  if (type == T_I32) static_cast<int32_t*>(c)[i] = int32_t(v);
  else static_cast<int64_t*>(c)[i] = v;
}

// per batch segment: its key's carried tail length (0 beyond the segment count)
// (a key id outside [0, max_keys) gets none: carry_keycheck flags the batch, which then fails)
__global__ void rc_tail_len(const int64_t* __restrict__ nseg, const int64_t* __restrict__ seg_start,
                            const int32_t* __restrict__ key, const int64_t* __restrict__ rtab, int64_t nmax,
                            int64_t* __restrict__ tlen, int32_t max_keys) {
  const int64_t sg = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (sg >= nmax) return;
  const int32_t k = sg < *nseg ? key[seg_start[sg]] : -1;
  tlen[sg] = k >= 0 && k < max_keys ? rtab[2 * int64_t(k) + 1] : 0;
}

// the batch's records into the extended batch, after their key's tail
__global__ void rc_build_new(RcExt X, int64_t n, const int64_t* __restrict__ seg_flag, const int64_t* __restrict__ seg_idx,
                             const int64_t* __restrict__ toff, const int64_t* __restrict__ tlen, int64_t base,
                             RcIn B) {
  const int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (i >= n) return;
  const int64_t sg = seg_idx[i] + seg_flag[i] - 1;
  const int64_t e = i + toff[sg] + tlen[sg];
  if (e >= X.cap) return;                          // (only a batch the key check rejects gets here)
  X.key[e] = B.key[i];
  X.topic[e] = B.topic ? B.topic[i] : 0;
  X.partition[e] = B.partition ? B.partition[i] : 0;
  const int64_t p = B.pos ? B.pos[i] : base + i;
  X.pos[e] = p;
  X.offset[e] = B.offset ? B.offset[i] : p;
  X.ts[e] = B.ts ? B.ts[i] : p;
  X.seg[e] = int32_t(sg);
  for (int c = 0; c < X.ncols; c++) col_put(X.cols[c], X.coltype[c], e, col_bits(B.cols[c], X.coltype[c], i));
}

// the carried tails into the extended batch (one thread per segment: tails are short)
__global__ void rc_build_tail(RcExt X, int64_t nmax, const int64_t* __restrict__ nseg, const int64_t* __restrict__ seg_start,
                              const int32_t* __restrict__ key, const int64_t* __restrict__ rtab,
                              const int64_t* __restrict__ rpool, const int64_t* __restrict__ toff,
                              const int64_t* __restrict__ tlen) {
  const int64_t sg = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (sg >= nmax || sg >= *nseg) return;
  const int64_t T = tlen[sg];
  if (!T) return;
  const int RW = 5 + X.ncols;
  const int32_t k = key[seg_start[sg]];
  const int64_t* src = rpool + rtab[2 * int64_t(k)] * RW;
  const int64_t e0 = seg_start[sg] + toff[sg];
  for (int64_t t = 0; t < T && e0 + t < X.cap; t++, src += RW) {
    const int64_t e = e0 + t;
    X.pos[e] = src[0];
    X.offset[e] = src[1];
    X.ts[e] = src[2];
    X.key[e] = k;                                  // the key's current id (a spilled key may come back under another)
    X.topic[e] = int32_t(uint64_t(src[3]) >> 32);
    X.partition[e] = int32_t(src[4]);
    X.seg[e] = int32_t(sg);
    for (int c = 0; c < X.ncols; c++) col_put(X.cols[c], X.coltype[c], e, src[5 + c]);
  }
}

// per segment: the first start whose run is still open (runs_sim's end_of == -2)
__global__ void rc_open_min(const int32_t* __restrict__ end_of, const int32_t* __restrict__ seg, int64_t n,
                            unsigned long long* __restrict__ tstart, const int64_t* __restrict__ n_dev) {
  const int64_t j = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (j < n && (!n_dev || j < *n_dev) && end_of[j] == -2) atomicMin(&tstart[seg[j]], (unsigned long long)j);
}

__global__ void rc_new_len(int64_t nmax, const int64_t* __restrict__ nseg, const int64_t* __restrict__ seg_start,
                           const int64_t* __restrict__ toff, const unsigned long long* __restrict__ tstart,
                           int64_t* __restrict__ newlen) {
  const int64_t sg = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (sg >= nmax) return;
  int64_t L = 0;
  if (sg < *nseg) {
    const int64_t end = seg_start[sg + 1] + toff[sg + 1];          // the segment's end in the extended batch
    const unsigned long long t = tstart[sg];
    if (int64_t(t) >= 0 && int64_t(t) < end) L = end - int64_t(t);
  }
  newlen[sg] = L;
}

// the new tails appended to the pool (at *top + noff): the key table per segment, then the records one
// thread each (a thread walking its segment's whole tail took 97 us per 1 M-record C3 batch)
// bad: the batch's key-check flags -- a failing batch leaves the tail pool and table as they were
__global__ void rc_tail_table(int64_t nmax, const int64_t* __restrict__ nseg, const int64_t* __restrict__ seg_start,
                              const int32_t* __restrict__ key, const int64_t* __restrict__ newlen,
                              const int64_t* __restrict__ noff, const int64_t* __restrict__ top,
                              int64_t* __restrict__ rtab, const int64_t* __restrict__ bad) {
  const int64_t sg = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (sg >= nmax || sg >= *nseg || *bad) return;
  const int64_t k = key[seg_start[sg]];
  const int64_t L = newlen[sg];
  if (L) rtab[2 * k] = *top + noff[sg];
  rtab[2 * k + 1] = L;
}
__global__ void rc_tail_write(RcExt X, int64_t nrec, const int64_t* __restrict__ nseg,
                              const unsigned long long* __restrict__ tstart, const int64_t* __restrict__ noff,
                              const int64_t* __restrict__ new_total, const int64_t* __restrict__ top,
                              int64_t* __restrict__ rpool, const int64_t* __restrict__ bad) {
  const int64_t x = int64_t(blockIdx.x) * 256 + threadIdx.x;   // the x-th new tail record of the batch
  if (x >= nrec || x >= *new_total || *bad) return;
  int64_t lo = 0, hi = *nseg - 1;                  // its segment: the last whose tail starts at or before x
  while (lo < hi) {
    const int64_t mid = (lo + hi + 1) >> 1;
    if (noff[mid] <= x) lo = mid; else hi = mid - 1;
  }
  const int RW = 5 + X.ncols;
  const int64_t e = int64_t(tstart[lo]) + (x - noff[lo]);
  int64_t* d = rpool + (*top + x) * RW;
  d[0] = X.pos[e];
  d[1] = X.offset[e];
  d[2] = X.ts[e];
  d[3] = int64_t(uint64_t(uint32_t(X.key[e])) | (uint64_t(uint32_t(X.topic[e])) << 32));
  d[4] = X.partition[e];
  for (int c = 0; c < X.ncols; c++) d[5 + c] = col_bits(X.cols[c], X.coltype[c], e);
}

__global__ void rc_top_add(int64_t* __restrict__ top, const int64_t* __restrict__ add, const int64_t* __restrict__ bad) {
  if (!*bad) *top += *add;
}
// *out = min(a + *b, cap) (the extended batch's record count on the device; over cap only for a batch
// with a key in two segments, which the key check rejects)
__global__ void rc_count(int64_t* __restrict__ out, int64_t a, const int64_t* __restrict__ b, int64_t cap) {
  *out = a + *b < cap ? a + *b : cap;
}

// compaction of the tail pool: every key's tail copied to `dst` at the exclusive prefix of the lengths
__global__ void rc_gc_len(const int64_t* __restrict__ rtab, int64_t nkeys, int64_t* __restrict__ len) {
  const int64_t k = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (k < nkeys) len[k] = rtab[2 * k + 1];
}
__global__ void rc_gc_copy(int64_t* __restrict__ rtab, int64_t nkeys, const int64_t* __restrict__ off, int RW,
                           const int64_t* __restrict__ src, int64_t* __restrict__ dst) {
  const int64_t k = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (k >= nkeys) return;
  const int64_t L = rtab[2 * k + 1];
  if (!L) return;
  const int64_t* a = src + rtab[2 * k] * RW;
  int64_t* b = dst + off[k] * RW;
  for (int64_t w = 0; w < L * RW; w++) b[w] = a[w];
  rtab[2 * k] = off[k];
}

}  // namespace

hipError_t exclusive_scan(const int64_t* in, int64_t n, int64_t* out, int64_t* total, int64_t* tmp, hipStream_t st);

static unsigned runs_blocks(int64_t items, int32_t chunk) {
  const int64_t waves = (items + chunk - 1) / chunk;
  return unsigned((waves * 64 + RT - 1) / RT);
}

// jf: the pattern's compiled runs_sim (jit.cpp), nullptr for the built-in interpreting kernel
hipError_t runs_sim_launch(const RunsArgs& A, int64_t* flag, int32_t* end_of, hipStream_t st, hipFunction_t jf) {
  if (A.n <= 0) return hipSuccess;
  if (jf) {
    RunsArgs a = A;
    void* args[] = {&a, &flag, &end_of};
    return hipModuleLaunchKernel(jf, runs_blocks(A.n, A.chunk), 1, 1, RT, 1, 1, 0, st, args, nullptr);
  }
  hipLaunchKernelGGL(runs_sim, dim3(runs_blocks(A.n, A.chunk)), dim3(RT), 0, st, A, flag, end_of);
  return hipGetLastError();
}

// stat: runs_sim's per-chunk counts / lengths (W = the sim launch's waves); pre: 2 W entries of scratch;
// the completed runs into out in start order, their count into *tot_cnt, their total length *tot_len
// n_grid: the record count runs_sim's grid was sized by (its statistics' layout), >= n
hipError_t runs_compact_launch(const int64_t* stat, const int32_t* end_of, int64_t n, int32_t chunk, int64_t* pre,
                               unsigned long long* out, int64_t* tot_cnt, int64_t* tot_len, int64_t* scan_tmp,
                               hipStream_t st, int64_t n_grid) {
  if (n <= 0) return hipSuccess;
  const int64_t nw = (n + chunk - 1) / chunk, W = int64_t(runs_blocks(n_grid, chunk)) * (RT / 64);
  if (chunk > RUNS_CHUNK || chunk < 64 || (chunk & (chunk - 1))) return hipErrorInvalidValue;
  if (nw <= (int64_t(1) << 16)) {
    hipLaunchKernelGGL(runs_chunk_scan<false>, dim3(1), dim3(1024), 0, st, stat, nw, W, pre, tot_cnt, tot_len, nullptr,
                       chunk);
  } else {
    hipError_t e = exclusive_scan(stat, nw, pre, tot_cnt, scan_tmp, st);
    if (e == hipSuccess) e = exclusive_scan(stat + W, nw, pre + W, tot_len, scan_tmp, st);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(runs_compact, dim3(unsigned(nw)), dim3(256), 0, st, end_of, n, chunk, pre, out);
  return hipGetLastError();
}

// the host's view of a runs batch, into pinned host memory h: {completed runs, first exception, entries,
// segment overflow, longest span, failing runs, tail pool top}
// ... and, for a carry batch, h[7] its key-check flags and h[8] its carried tail records (x: scal)
__global__ void runs_results(const unsigned long long* __restrict__ ctl, const int64_t* __restrict__ nm,
                             const int64_t* __restrict__ top, int64_t* __restrict__ h, const int64_t* __restrict__ x) {
  const int t = threadIdx.x;
  if (t < 7) h[t] = t == 0 ? *nm : t == 6 ? (top ? *top : 0) : int64_t(ctl[t]);
  else if (t == 7) h[t] = x ? x[1] : 0;
  else if (t == 8) h[t] = x ? x[5] : 0;
}
hipError_t runs_results_launch(const unsigned long long* ctl, const int64_t* nm, const int64_t* top, int64_t* h,
                               hipStream_t st, const int64_t* x) {
  hipLaunchKernelGGL(runs_results, dim3(1), dim3(64), 0, st, ctl, nm, top, h, x);
  return hipGetLastError();
}

int64_t runs_sim_waves(int64_t n, int32_t chunk) { return n <= 0 ? 0 : int64_t(runs_blocks(n, chunk)) * (RT / 64); }

// len: each sorted run's entry count (what runs_lengths computes)
hipError_t runs_order_launch(const unsigned long long* in, int64_t nm, int w, unsigned long long* out, int64_t* len,
                             hipStream_t st) {
  if (nm <= 0) return hipSuccess;
  if (w < 0 || w > RUNS_ORDER_MAX_W) return hipErrorInvalidValue;
  hipLaunchKernelGGL(runs_order, dim3(unsigned((nm + 255) / 256)), dim3(256), 0, st, in, nm, w, out, len);
  return hipGetLastError();
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
  hipLaunchKernelGGL(runs_expand, dim3(unsigned((nm + 255) / 256)), dim3(256), 0, st, R.P, R.key, R.pos, R.segs, R.segn, sorted, nm,
                     ent_off, ne, R.base, match_record, match_key, ent_off_out, ent_name, ent_record);
  return hipGetLastError();
}

// runs_emit's chunk prefixes: the runs and entries ending in each chunk, scanned (pre: 2 W entries),
// with the batch's totals into *tot_cnt / *tot_len.  False when the chunks are too many for one
// scanning workgroup (then the batch takes runs_compact + runs_order / the sort instead).
bool runs_emit_scan(const int64_t* stat, int64_t n, int32_t chunk, int64_t* pre, int64_t* tot_cnt, int64_t* tot_len,
                    hipStream_t st, const int64_t* n_dev) {
  const int64_t nw = (n + chunk - 1) / chunk, W = int64_t(runs_blocks(n, chunk)) * (RT / 64);
  if (n <= 0 || nw > (int64_t(1) << 16) || chunk > RUNS_CHUNK) return false;
  hipLaunchKernelGGL(runs_chunk_scan<true>, dim3(1), dim3(1024), 0, st, stat, nw, W, pre, tot_cnt, tot_len, n_dev, chunk);
  return true;
}
// the CSR from runs_sim's results (runs_emit_scan's pre); span: the longest completed span (< chunk)
// n_grid: the record count runs_sim's grid was sized by (its statistics' layout), >= R.n
hipError_t runs_emit_launch(const RunsArgs& R, const int32_t* end_of, const int64_t* pre, int span, int64_t* match_record,
                            int32_t* match_key, int64_t* ent_off, int32_t* ent_name, int64_t* ent_record, hipStream_t st,
                            int64_t n_grid) {
  const int64_t nw = (R.n + R.chunk - 1) / R.chunk, W = int64_t(runs_blocks(n_grid, R.chunk)) * (RT / 64);
  if (R.n <= 0) return hipSuccess;
  if (span < 0 || span >= R.chunk || R.chunk > RUNS_CHUNK || !R.segs) return hipErrorInvalidValue;
  const size_t lds = size_t(R.chunk + span + 1) * 16 + 4;   // s_seg (and s_cnt) 8, s_run 4, s_at 4 per slot
  auto k = R.segn == 4 ? (R.pos ? runs_emit<true, true> : runs_emit<true, false>)
                       : (R.pos ? runs_emit<false, true> : runs_emit<false, false>);
  hipLaunchKernelGGL(k, dim3(unsigned(nw)), dim3(256), lds, st, R.P, R.key, R.pos, R.base, R.segs, R.segn, end_of, R.n,
                     R.chunk, span, pre, W, match_record, match_key, ent_off, ent_name, ent_record);
  return hipGetLastError();
}

static unsigned blocks256(int64_t n) { return unsigned((std::max<int64_t>(n, 1) + 255) / 256); }

// the extended batch of a runs carry session: every batch segment prefixed by its key's tail.
// seg_flag / seg_idx / seg_start / nseg: nfa_segments of the batch; nmax >= segment count (the batch
// size); tlen / toff: n + 1 entries of scratch; total: the tails' record count (device)
hipError_t runs_carry_build(const RcIn& B, int64_t n, int64_t base, const int64_t* seg_flag, const int64_t* seg_idx,
                            const int64_t* seg_start, const int64_t* nseg, const int64_t* rtab, const int64_t* rpool,
                            int64_t* tlen, int64_t* toff, int64_t* total, int64_t* scan_tmp, const RcExt& X,
                            hipStream_t st, bool lens_only, int32_t max_keys) {
  if (lens_only) {
    hipLaunchKernelGGL(rc_tail_len, dim3(blocks256(n + 1)), dim3(256), 0, st, nseg, seg_start, B.key, rtab, n + 1, tlen,
                       max_keys);
    return exclusive_scan(tlen, n + 1, toff, total, scan_tmp, st);
  }
  hipLaunchKernelGGL(rc_build_new, dim3(blocks256(n)), dim3(256), 0, st, X, n, seg_flag, seg_idx, toff, tlen, base, B);
  hipLaunchKernelGGL(rc_build_tail, dim3(blocks256(n)), dim3(256), 0, st, X, n, nseg, seg_start, B.key, rtab, rpool, toff,
                     tlen);
  return hipGetLastError();
}

// after runs_sim over the extended batch (ext_n records): the keys' new tails
hipError_t runs_carry_tails(const RcExt& X, int64_t ext_n, int64_t n, const int64_t* nseg, const int64_t* seg_start,
                            const int32_t* key, const int64_t* toff, const int32_t* end_of, unsigned long long* tstart,
                            int64_t* newlen, int64_t* noff, int64_t* new_total, int64_t* scan_tmp, int64_t* top,
                            int64_t* rpool, int64_t* rtab, hipStream_t st, const int64_t* ext_n_dev, const int64_t* bad) {
  hipError_t e = hipMemsetAsync(tstart, 0x7F, size_t(n + 1) * 8, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(rc_open_min, dim3(blocks256(ext_n)), dim3(256), 0, st, end_of, X.seg, ext_n, tstart, ext_n_dev);
  hipLaunchKernelGGL(rc_new_len, dim3(blocks256(n + 1)), dim3(256), 0, st, n + 1, nseg, seg_start, toff, tstart, newlen);
  if ((e = exclusive_scan(newlen, n + 1, noff, new_total, scan_tmp, st)) != hipSuccess) return e;
  hipLaunchKernelGGL(rc_tail_table, dim3(blocks256(n)), dim3(256), 0, st, n, nseg, seg_start, key, newlen, noff, top, rtab,
                     bad);
  hipLaunchKernelGGL(rc_tail_write, dim3(blocks256(ext_n)), dim3(256), 0, st, X, ext_n, nseg, tstart, noff, new_total, top,
                     rpool, bad);
  hipLaunchKernelGGL(rc_top_add, dim3(1), dim3(1), 0, st, top, new_total, bad);
  return hipGetLastError();
}

// *out = min(nb + *tails, cap): the extended batch's records, for the launches sized by a bound (cap)
hipError_t runs_carry_count(int64_t* out, int64_t nb, const int64_t* tails, int64_t cap, hipStream_t st) {
  hipLaunchKernelGGL(rc_count, dim3(1), dim3(1), 0, st, out, nb, tails, cap);
  return hipGetLastError();
}

// compaction of the tail pool into dst (len / off: nkeys + 1 entries of scratch; *total: live records)
hipError_t runs_carry_gc(int64_t* rtab, int64_t nkeys, int RW, const int64_t* src, int64_t* dst, int64_t* len,
                         int64_t* off, int64_t* total, int64_t* scan_tmp, hipStream_t st) {
  hipLaunchKernelGGL(rc_gc_len, dim3(blocks256(nkeys)), dim3(256), 0, st, rtab, nkeys, len);
  hipError_t e = exclusive_scan(len, nkeys, off, total, scan_tmp, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(rc_gc_copy, dim3(blocks256(nkeys)), dim3(256), 0, st, rtab, nkeys, off, RW, src, dst);
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
  W.R.chunk = runs_chunk(nm);
  if (jf) {
    void* args[] = {&W};
    return hipModuleLaunchKernel(jf, runs_blocks(nm, W.R.chunk), 1, 1, RT, 1, 1, 0, st, args, nullptr);
  }
  hipLaunchKernelGGL(runs_write, dim3(runs_blocks(nm, W.R.chunk)), dim3(RT), 0, st, W);
  return hipGetLastError();
}

}  // namespace kcep

// stencil.hip -- scan, gather and post-processing of the stencil / chain path; the kernel itself is
// in stencil_kernel.h, instantiated per K in stencil_k<N>.hip.
#include "stencil_kernel.h"

namespace kcep {

hipError_t stencil_count_k1(const StencilLaunch& L, hipStream_t st);
hipError_t stencil_count_k2(const StencilLaunch& L, hipStream_t st);
hipError_t stencil_count_k3(const StencilLaunch& L, hipStream_t st);
hipError_t stencil_count_k4(const StencilLaunch& L, hipStream_t st);
hipError_t stencil_count_k5(const StencilLaunch& L, hipStream_t st);
hipError_t stencil_count_k6(const StencilLaunch& L, hipStream_t st);
hipError_t stencil_count_k7(const StencilLaunch& L, hipStream_t st);
hipError_t stencil_count_k8(const StencilLaunch& L, hipStream_t st);

// Tiles' match slots -> one contiguous output in record order (the order
// context.forward sees them, CEPProcessor.java:148): tile t's matches start at
// the exclusive prefix of the tile counts.  One workgroup per tile.
// The slot of super-tile t holds one int per match -- the plain kernel: its first record (the
// stages are consecutive records); the keyed kernel: its completing record, with an aux byte per
// match after the super-tile's sub x 4096 ints (stencil_row) -- written out as k-int rows.
struct SlotFormat {
  int k, plain, chain, carry, dense, kdense;
  int64_t nsuper;
  int sub;
  // match m of super-tile t (c matches): its slot word and aux byte, then stage s of its row from them
  __device__ __forceinline__ void load(const int32_t* slots, int64_t t, int64_t c, int64_t m, int32_t& v,
                                       uint32_t& a) const {
    a = 0;
    if (dense) {
      v = m < ST_DENSE ? slots[t * ST_DENSE + m] : slots[nsuper * ST_DENSE + t * int64_t(sub) * ST_TILE + m];
      return;
    }
    if (kdense && c <= ST_DENSE_KEYED) {
      const int64_t i = t * ST_DENSE_KEYED + m;
      v = slots[i];
      a = reinterpret_cast<const uint8_t*>(slots + nsuper * ST_DENSE_KEYED)[i];
      return;
    }
    const int32_t* src = slots + (kdense ? nsuper * (ST_DENSE_KEYED + ST_DENSE_KEYED / 4) : 0) +
                         t * int64_t(sub) * ST_TILE * k;
    const uint8_t* aux = reinterpret_cast<const uint8_t*>(src + int64_t(sub) * ST_TILE);
    v = src[m];
    if (plain ? (carry && v < 0) : k > 1) a = aux[m];
  }
  __device__ __forceinline__ int32_t value(int32_t v, uint32_t a, int s) const {
    if (dense) return v + s;
    if (plain) {                                 // first record; carry boundary: -(1 + completing record)
      if (!carry || v >= 0) return v + s;
      const int need = int(a);
      return s < need ? -(1 + (need - s)) : -(1 + v) - (k - 1) + s;
    }
    return stencil_row(v, a, s, k, chain, carry);
  }
  // match m of super-tile t (c matches), stage s
  __device__ __forceinline__ int32_t entry(const int32_t* slots, int64_t t, int64_t c, int64_t m, int s) const {
    if (dense)                                   // the plain kernel without carry (kcep_internal.h ST_DENSE)
      return (m < ST_DENSE ? slots[t * ST_DENSE + m] : slots[nsuper * ST_DENSE + t * int64_t(sub) * ST_TILE + m]) + s;
    if (kdense && c <= ST_DENSE_KEYED) {         // the keyed kernel without carry (kcep_internal.h)
      const int64_t i = t * ST_DENSE_KEYED + m;
      return stencil_row(slots[i], reinterpret_cast<const uint8_t*>(slots + nsuper * ST_DENSE_KEYED)[i], s, k, chain,
                         carry);
    }
    const int32_t* src = slots + (kdense ? nsuper * (ST_DENSE_KEYED + ST_DENSE_KEYED / 4) : 0) +
                         t * int64_t(sub) * ST_TILE * k;
    const uint8_t* aux = reinterpret_cast<const uint8_t*>(src + int64_t(sub) * ST_TILE);
    const int32_t v = src[m];
    if (plain) {                                 // first record; carry boundary: -(1 + completing record)
      if (!carry || v >= 0) return v + s;
      const int need = aux[m];
      return s < need ? -(1 + (need - s)) : -(1 + v) - (k - 1) + s;
    }
    return stencil_row(v, k > 1 ? aux[m] : 0u, s, k, chain, carry);
  }
};
// One thread per match: its slot word (and aux byte) loaded once, its k row entries stored (a wave's
// stores of one stage k ints apart, the k stores together filling the wave's rows).  (Was one thread
// per output word: a divide by k and the slot loads repeated k times per match.)
// The plain kernel's dense slots (the headline path), K a template parameter: a thread's first
// GATHER_B slot words are loaded at clamped addresses before any row is stored, so the loads are one
// memory round trip, not one per match each behind the stores before it (a load under a branch or a
// loop over a run-time k makes the compiler wait for every outstanding memory operation, stores
// included); the rest, if a super-tile has more matches, one at a time
constexpr int GATHER_B = 4;
template <int K>
__global__ __launch_bounds__(256) void stencil_gather_dense(const int32_t* __restrict__ slots,
                                                            const int64_t* __restrict__ cnt,
                                                            const int64_t* __restrict__ pre, int32_t* __restrict__ out,
                                                            int64_t out_cap, int64_t nsuper, int sub) {
  const int64_t t = blockIdx.x;                  // super-tile
  const int64_t c = cnt[t], p = pre[t];
  if (p + c > out_cap || c <= 0) return;
  int32_t* const dst = out + p * K;
  const int32_t* const dense = slots + t * ST_DENSE;
  const int32_t* const over = slots + nsuper * ST_DENSE + t * int64_t(sub) * ST_TILE;
  const int64_t cb = c < int64_t(GATHER_B) * blockDim.x ? c : int64_t(GATHER_B) * blockDim.x;
  int32_t v[GATHER_B];
#pragma unroll
  for (int q = 0; q < GATHER_B; q++) {
    const int64_t m = threadIdx.x + int64_t(q) * blockDim.x;
    const int64_t mm = m < cb ? m : 0;
    v[q] = (mm < ST_DENSE ? dense : over)[mm];
  }
#pragma unroll
  for (int q = 0; q < GATHER_B; q++) {
    const int64_t m = threadIdx.x + int64_t(q) * blockDim.x;
    if (m < cb) {
#pragma unroll
      for (int s = 0; s < K; s++) dst[m * K + s] = v[q] + s;
    }
  }
  for (int64_t m = cb + threadIdx.x; m < c; m += blockDim.x) {
    const int32_t w = (m < ST_DENSE ? dense : over)[m];
#pragma unroll
    for (int s = 0; s < K; s++) dst[m * K + s] = w + s;
  }
}

// Every other slot format (keyed / chain / carry), K a template parameter, the same batching: a
// thread's first GATHER_B matches' slot words and aux bytes loaded before any row is stored.  The
// format's branches are taken once per workgroup (uniform) around loads of one shape each: a value
// loaded in either arm of a branch is merged after it, and that merge waits for every outstanding
// memory operation
template <int K, class Ld>
__device__ __forceinline__ void gather_rows(int32_t* __restrict__ dst, int64_t c, const SlotFormat& F, Ld&& ld) {
  const int64_t cb = c < int64_t(GATHER_B) * blockDim.x ? c : int64_t(GATHER_B) * blockDim.x;
  int32_t v[GATHER_B];
  uint32_t a[GATHER_B];
#pragma unroll
  for (int q = 0; q < GATHER_B; q++) {
    const int64_t m = threadIdx.x + int64_t(q) * blockDim.x;
    ld(m < cb ? m : 0, v[q], a[q]);
  }
#pragma unroll
  for (int q = 0; q < GATHER_B; q++) {
    const int64_t m = threadIdx.x + int64_t(q) * blockDim.x;
    if (m < cb) {
#pragma unroll
      for (int s = 0; s < K; s++) dst[m * K + s] = F.value(v[q], a[q], s);
    }
  }
  for (int64_t m = cb + threadIdx.x; m < c; m += blockDim.x) {
    int32_t w;
    uint32_t b;
    ld(m, w, b);
#pragma unroll
    for (int s = 0; s < K; s++) dst[m * K + s] = F.value(w, b, s);
  }
}
template <int K>
__global__ __launch_bounds__(256) void stencil_gather_k(const int32_t* __restrict__ slots, const int64_t* __restrict__ cnt,
                                                        const int64_t* __restrict__ pre, int32_t* __restrict__ out,
                                                        int64_t out_cap, SlotFormat F) {
  const int64_t t = blockIdx.x;                  // super-tile
  const int64_t c = cnt[t], p = pre[t];
  if (p + c > out_cap || c <= 0) return;
  int32_t* const dst = out + p * K;
  if (F.kdense && c <= ST_DENSE_KEYED) {         // the keyed kernel's dense region (no carry)
    const int32_t* const w0 = slots + t * ST_DENSE_KEYED;
    const uint8_t* const a0 = reinterpret_cast<const uint8_t*>(slots + F.nsuper * ST_DENSE_KEYED) + t * ST_DENSE_KEYED;
    gather_rows<K>(dst, c, F, [&](int64_t m, int32_t& v, uint32_t& a) { v = w0[m]; a = a0[m]; });
    return;
  }
  const int32_t* const src = slots + (F.kdense ? F.nsuper * (ST_DENSE_KEYED + ST_DENSE_KEYED / 4) : 0) +
                             t * int64_t(F.sub) * ST_TILE * K;
  const uint8_t* const aux = reinterpret_cast<const uint8_t*>(src + int64_t(F.sub) * ST_TILE);
  // the aux byte: keyed rows always (k > 1); plain rows only for a carry boundary match (v < 0) -- loaded
  // whenever the format has it (K > 1: inside the slot) and used only then
  const bool has_aux = K > 1 && (!F.plain || F.carry);
  if (has_aux)
    gather_rows<K>(dst, c, F, [&](int64_t m, int32_t& v, uint32_t& a) { v = src[m]; a = aux[m]; });
  else
    gather_rows<K>(dst, c, F, [&](int64_t m, int32_t& v, uint32_t& a) { v = src[m]; a = 0; });
}

__global__ __launch_bounds__(256) void stencil_gather(const int32_t* __restrict__ slots, const int64_t* __restrict__ cnt,
                                                      const int64_t* __restrict__ pre, int32_t* __restrict__ out,
                                                      int64_t out_cap, int sub, SlotFormat F) {
  const int64_t t = blockIdx.x;                  // super-tile
  const int k = F.k;
  const int64_t c = cnt[t], p = pre[t];
  if (p + c > out_cap) return;
  int32_t* const dst = out + p * k;
  for (int64_t m = threadIdx.x; m < c; m += blockDim.x) {
    int32_t v;
    uint32_t a;
    F.load(slots, t, c, m, v, a);
    for (int s = 0; s < k; s++) dst[m * k + s] = F.value(v, a, s);
  }
}

// ---- launcher ------------------------------------------------------------

int64_t stencil_tiles(int64_t n) { return (n + ST_TILE - 1) / ST_TILE; }

// exclusive prefix of the super-tile counts in one 1024-thread workgroup, plus
// the total (a batch has at most 2^31 / 16384 super-tiles: <= 128 per thread;
// the loads go out 8 at a time)
__global__ __launch_bounds__(1024) void tile_scan(const int64_t* __restrict__ cnt, int64_t nt, int64_t* __restrict__ pre,
                                                  int64_t* __restrict__ total, unsigned long long* __restrict__ clear_flag) {
  __shared__ int64_t s_w[16];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t per = (nt + 1023) / 1024, a = tid * per, b = a + per < nt ? a + per : nt;
  int64_t sum = 0;
  int64_t r8[8];                                  // per <= 8 (<= 8192 super-tiles): one pass over global memory
  const bool one_pass = per <= 8;
  if (one_pass) {
#pragma unroll
    for (int i = 0; i < 8; i++) { r8[i] = a + i < b ? cnt[a + i] : 0; sum += r8[i]; }
  } else {
    for (int64_t c = a; c < b; c += 8) {
      int64_t v[8];
#pragma unroll
      for (int i = 0; i < 8; i++) v[i] = c + i < b ? cnt[c + i] : 0;
#pragma unroll
      for (int i = 0; i < 8; i++) sum += v[i];
    }
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
  if (one_pass) {
#pragma unroll
    for (int i = 0; i < 8; i++)
      if (a + i < b) { pre[a + i] = run; run += r8[i]; }
  } else {
    for (int64_t c = a; c < b; c += 8) {
      int64_t v[8];
#pragma unroll
      for (int i = 0; i < 8; i++) v[i] = c + i < b ? cnt[c + i] : 0;
#pragma unroll
      for (int i = 0; i < 8; i++) {
        if (c + i < b) pre[c + i] = run;
        run += v[i];
      }
    }
  }
  if (tid == 1023) *total = run;
  if (tid == 0 && clear_flag) *clear_flag = 0;    // carry: the next batch's error-flag word (the kernel is done)
}

// small batches (processor flushes): the scan and the gather in one workgroup, one launch instead of
// two -- the prefix of <= 1024 super-tile counts in LDS, then each wave copies super-tiles' slots
constexpr int SMALL_FINISH = 1024;
__global__ __launch_bounds__(1024) void stencil_finish_small(const int32_t* __restrict__ slots,
                                                             const int64_t* __restrict__ cnt, int64_t nt, int k,
                                                             int32_t* __restrict__ out, int64_t out_cap, int sub,
                                                             int64_t* __restrict__ total,
                                                             unsigned long long* __restrict__ clear_flag,
                                                             SlotFormat F) {
  __shared__ int64_t s_pre[SMALL_FINISH + 1];
  __shared__ int64_t s_w[16];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t c = tid < nt ? cnt[tid] : 0;
  int64_t incl = c;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int64_t y = __shfl_up(incl, d, 64);
    if (lane >= d) incl += y;
  }
  if (lane == 63) s_w[wid] = incl;
  __syncthreads();
  int64_t run = incl - c;
  for (int w = 0; w < wid; w++) run += s_w[w];
  s_pre[tid] = run;
  if (tid == 1023) { s_pre[SMALL_FINISH] = run + c; *total = run + c; }
  if (tid == 0 && clear_flag) *clear_flag = 0;    // carry: the next batch's error-flag word (the kernel is done)
  __syncthreads();
  for (int64_t t = wid; t < nt; t += 16) {                 // one wave per super-tile
    const int64_t pre = s_pre[t], m = s_pre[t + 1] - pre;
    if (pre + m > out_cap) continue;
    int32_t* dst = out + pre * k;
    for (int64_t q = lane; q < m; q += 64) {               // a match's slot word (and aux byte) loaded once
      int32_t v;
      uint32_t a;
      F.load(slots, t, m, q, v, a);
      for (int s2 = 0; s2 < k; s2++) dst[q * k + s2] = F.value(v, a, s2);
    }
  }
}

// The end of a delivered batch: the last workgroup to finish (a ticket in device memory) stamps the host
// header, after every workgroup's writes were made visible to the host -- cep_collect spins on that word
// instead of waiting for the stream (one wake-up latency fewer per flush).
__device__ __forceinline__ void deliver_done(unsigned* ticket, unsigned nblocks, int64_t* hdr, int64_t stamp) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence_system();
    const unsigned prev = atomicAdd(ticket, 1u);
    if (prev == nblocks - 1) {
      __threadfence_system();
      *ticket = 0;                                   // ready for the next batch
      *reinterpret_cast<volatile int64_t*>(hdr + 2) = stamp;
    }
  }
}

// Small carry batches collected at once (CEP_BATCH_DELIVER: a processor flush, <= 1024 super-tiles):
// scan, rows and delivery in one launch, one workgroup per super-tile.  Each workgroup sums the counts
// before its super-tile itself (<= 1024 of them: no separate scan launch), then one thread per match
// expands the slot into the k-int row (kept on the device for cep_checksum) and hands the row's stream
// positions and the match's key to pinned host memory.
__global__ __launch_bounds__(256) void stencil_finish_deliver(const int32_t* __restrict__ slots,
                                                              const int64_t* __restrict__ cnt, int64_t nt, int k,
                                                              int32_t* __restrict__ out, int64_t out_cap, int sub,
                                                              int64_t* __restrict__ total,
                                                              unsigned long long* __restrict__ clear_flag,
                                                              SlotFormat F, const int32_t* __restrict__ key,
                                                              StencilCarry C, int64_t host_cap, int64_t* __restrict__ hdr,
                                                              int32_t* __restrict__ hkey, int64_t* __restrict__ hpos,
                                                              int32_t* __restrict__ dkey, int64_t* __restrict__ dpos,
                                                              unsigned* ticket, int64_t stamp) {
  __shared__ int64_t s_red[2][4];
  const int64_t t = blockIdx.x;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int64_t before = 0, all = 0;
  for (int64_t i = threadIdx.x; i < nt; i += 256) {
    const int64_t c = cnt[i];
    all += c;
    if (i < t) before += c;
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    before += __shfl_xor(before, d, 64);
    all += __shfl_xor(all, d, 64);
  }
  if (lane == 0) { s_red[0][wid] = before; s_red[1][wid] = all; }
  __syncthreads();
  const int64_t pre = s_red[0][0] + s_red[0][1] + s_red[0][2] + s_red[0][3];
  const int64_t tot = s_red[1][0] + s_red[1][1] + s_red[1][2] + s_red[1][3];
  if (t == 0 && threadIdx.x == 0) {
    *total = tot;
    hdr[0] = tot;
    hdr[1] = int64_t(*C.flags);                    // this batch's error flags (the count kernel is done)
    if (clear_flag) *clear_flag = 0;               // the next batch's error-flag word
  }
  const int64_t m = cnt[t];
  if (pre + m <= out_cap) {
    for (int64_t q = threadIdx.x; q < m; q += 256) {
      const int64_t i = pre + q;
      int32_t row[STENCIL_MAX_K], last = 0, v;
      uint32_t av;
      F.load(slots, t, m, q, v, av);                 // (once per match, not once per stage)
#pragma unroll
      for (int s = 0; s < STENCIL_MAX_K; s++)
        if (s < k) {
          row[s] = F.value(v, av, s);
          out[i * k + s] = row[s];
          last = row[s];
        }
      const int32_t kk = key[last];
      // a key id outside [0, max_keys) (error flag bit 0, the host fails the batch): no halo lookup
      const bool kok = kk >= 0 && kk < C.max_keys;
      const HaloHdr* h = kok ? C.hdr + kk : nullptr;
      const int old = kok ? halo_old(*h, C.stamp) : 0;
      const int64_t* hp = kok ? C.pos + (2 * int64_t(kk) + old) * C.km1 : nullptr;
      const bool host = i < host_cap;
      int64_t* p = host ? hpos + i * k : dpos + i * k;
#pragma unroll
      for (int s = 0; s < STENCIL_MAX_K; s++)
        if (s < k) {
          const int32_t r = row[s];
          p[s] = r >= 0 ? halo_gpos(C, r) : (r == -1 || !kok ? -1 : hp[h->cnt[old] - (-r - 1)]);
        }
      if (host) hkey[i] = kk;
      else dkey[i] = kk;
    }
  }
  deliver_done(ticket, unsigned(gridDim.x), hdr, stamp);
}

// Small arrival-order carry flushes (CEP_BATCH_ARRIVAL_ORDER, <= ARR_SMALL records, <= SMALL_FINISH
// super-tiles): the rows, their order by the arrival of the completing record and the delivery in one
// workgroup, one launch (was: the rows, a count, a three-kernel scan over the batch and the delivery).
// Per arrival record a byte of LDS counts its matches (a strict fixed-length pattern completes at most
// one run per record, a chain pattern at most K); match i of completing record a goes to
// (matches of the records before a) + (its rank among a's matches, which are consecutive in the grouped
// order: same key, same record).
constexpr int ARR_SMALL = 65536;
__global__ __launch_bounds__(1024) void stencil_finish_deliver_arrival(
    const int32_t* __restrict__ slots, const int64_t* __restrict__ cnt, int64_t nt, int k, int32_t* __restrict__ out,
    int64_t out_cap, int sub, int64_t* __restrict__ total, unsigned long long* __restrict__ clear_flag, SlotFormat F,
    const int32_t* __restrict__ key, StencilCarry C, int64_t n, int64_t host_cap, int64_t* __restrict__ hdr,
    int32_t* __restrict__ hkey, int64_t* __restrict__ hpos, int32_t* __restrict__ dkey, int64_t* __restrict__ dpos,
    unsigned* ticket, int64_t stamp) {
  __shared__ int64_t s_pre[SMALL_FINISH + 1];
  __shared__ int64_t s_w[16];
  __shared__ uint32_t s_cnt[ARR_SMALL / 4];      // byte a & 3 of word a >> 2: matches completing at record a
  __shared__ uint32_t s_tpre[1024];              // matches completing at records before thread t's 64
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t c0 = tid < nt ? cnt[tid] : 0;
  int64_t incl = c0;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int64_t y = __shfl_up(incl, d, 64);
    if (lane >= d) incl += y;
  }
  if (lane == 63) s_w[wid] = incl;
  for (int i = tid; i < ARR_SMALL / 4; i += 1024) s_cnt[i] = 0;
  __syncthreads();
  int64_t run = incl - c0;
  for (int w = 0; w < wid; w++) run += s_w[w];
  s_pre[tid] = run;
  if (tid == 1023) s_pre[SMALL_FINISH] = run + c0;
  __syncthreads();
  const int64_t tot = s_pre[SMALL_FINISH];
  if (tid == 0) {
    *total = tot;
    hdr[0] = tot;
    hdr[1] = int64_t(*C.flags);                    // this batch's error flags (the count kernel is done)
    if (clear_flag) *clear_flag = 0;
  }
  const bool fits = tot <= out_cap;
  // pass A: every match's completing record, counted by its arrival index.  A thread's first FA_KEEP
  // matches keep their slot word, aux byte, arrival index and key for pass B (loaded once, the key with
  // the arrival index: pass B's chain of dependent loads is then the halo's alone)
  constexpr int FA_KEEP = 2;
  int32_t kv[FA_KEEP], kk_[FA_KEEP];
  uint32_t ka[FA_KEEP];
  int64_t karr[FA_KEEP];
  {
    int it = 0;
    for (int64_t t = wid; t < nt && fits; t += 16) {
      const int64_t m = s_pre[t + 1] - s_pre[t];
      for (int64_t q = lane; q < m; q += 64, it++) {
        int32_t v;
        uint32_t a;
        F.load(slots, t, m, q, v, a);
        const int32_t last = F.value(v, a, k - 1);
        const int64_t arr = C.gpos[last] - C.base;
        const int32_t kk = key[last];
        atomicAdd(&s_cnt[arr >> 2], 1u << (8 * (arr & 3)));
#pragma unroll
        for (int u = 0; u < FA_KEEP; u++)
          if (u == it) { kv[u] = v; ka[u] = a; karr[u] = arr; kk_[u] = kk; }
      }
    }
  }
  __syncthreads();
  {                                                // per thread 64 records: the byte sum, then a block scan
    uint32_t sum = 0;
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const uint32_t w = s_cnt[tid * 16 + j];
      sum += (w & 0xFF) + ((w >> 8) & 0xFF) + ((w >> 16) & 0xFF) + (w >> 24);
    }
    uint32_t x = sum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(x, d, 64);
      if (lane >= d) x += y;
    }
    __syncthreads();                               // (s_w reused)
    if (lane == 63) s_w[wid] = x;
    __syncthreads();
    uint32_t before = x - sum;
    for (int w = 0; w < wid; w++) before += uint32_t(s_w[w]);
    s_tpre[tid] = before;
  }
  __syncthreads();
  // pass B: the rows (kept on the device for cep_checksum) and their delivery at the arrival rank
  int it = 0;
  for (int64_t t = wid; t < nt && fits; t += 16) {
    const int64_t m = s_pre[t + 1] - s_pre[t];
    for (int64_t q = lane; q < m; q += 64, it++) {
      const int64_t i = s_pre[t] + q;
      int32_t v = 0, kk = 0;
      uint32_t av = 0;
      int64_t a = 0;
#pragma unroll
      for (int u = 0; u < FA_KEEP; u++)
        if (u == it) { v = kv[u]; av = ka[u]; a = karr[u]; kk = kk_[u]; }
      if (it >= FA_KEEP) F.load(slots, t, m, q, v, av);
      int32_t row[STENCIL_MAX_K], last = 0;
#pragma unroll
      for (int s2 = 0; s2 < STENCIL_MAX_K; s2++)
        if (s2 < k) {
          row[s2] = F.value(v, av, s2);
          out[i * k + s2] = row[s2];
          last = row[s2];
        }
      if (it >= FA_KEEP) {
        a = C.gpos[last] - C.base;
        kk = key[last];
      }
      int64_t j = s_tpre[a >> 6];
      for (int64_t b = (a & ~int64_t(63)) >> 2; b < (a >> 2); b++) {   // whole words before a's, then a's bytes
        const uint32_t w = s_cnt[b];
        j += (w & 0xFF) + ((w >> 8) & 0xFF) + ((w >> 16) & 0xFF) + (w >> 24);
      }
      for (int64_t b = a & ~int64_t(3); b < a; b++) j += (s_cnt[b >> 2] >> (8 * (b & 3))) & 0xFF;
      if (F.chain)                                 // (a strict fixed-length pattern: one match per record)
        for (int64_t p = q - 1; p >= 0 && F.entry(slots, t, m, p, k - 1) == last; p--) j++;   // same record, earlier
      const bool kok = kk >= 0 && kk < C.max_keys;
      const HaloHdr* h = kok ? C.hdr + kk : nullptr;
      const int old = kok ? halo_old(*h, C.stamp) : 0;
      const int64_t* hp = kok ? C.pos + (2 * int64_t(kk) + old) * C.km1 : nullptr;
      const bool host = j < host_cap;
      int64_t* pp = host ? hpos + j * k : dpos + j * k;
#pragma unroll
      for (int s2 = 0; s2 < STENCIL_MAX_K; s2++)
        if (s2 < k) {
          const int32_t r = row[s2];
          pp[s2] = r >= 0 ? halo_gpos(C, r) : (r == -1 || !kok ? -1 : hp[h->cnt[old] - (-r - 1)]);
        }
      if (host) hkey[j] = kk;
      else dkey[j] = kk;
    }
  }
  (void)n;
  deliver_done(ticket, 1u, hdr, stamp);
}

static hipError_t stencil_count(const StencilLaunch& L, hipStream_t st) {
  if (L.chain && L.k != 3 && L.k != 4) return hipErrorInvalidValue;   // an optional stage needs k >= 3; chain k <= 4
  switch (L.k) {
    case 1: return stencil_count_k1(L, st);
    case 2: return stencil_count_k2(L, st);
    case 3: return stencil_count_k3(L, st);
    case 4: return stencil_count_k4(L, st);
    case 5: return stencil_count_k5(L, st);
    case 6: return stencil_count_k6(L, st);
    case 7: return stencil_count_k7(L, st);
    case 8: return stencil_count_k8(L, st);
  }
  return hipErrorInvalidValue;
}

hipError_t exclusive_scan(const int64_t* in, int64_t n, int64_t* out, int64_t* total, int64_t* tmp, hipStream_t st);
hipError_t stencil_deliver_launch(const int32_t* key, const int32_t* out, int k, const int64_t* total, int64_t out_cap,
                                  const StencilCarry& C, const DeliverArgs& D, hipStream_t st);

// stencil_kernel (timed as the dominant kernel between ev0 and ev1), then the
// tile-count scan and the gather into the contiguous output
hipError_t stencil_launch(const StencilLaunch& L, hipEvent_t ev0, hipEvent_t ev1, hipStream_t st) {
  // null events: timing off (cep_session_set_timing), no event packets in the stream
  const DeliverArgs& D = L.deliver;
  if (L.n <= 0) {
    hipError_t e = ev0 ? hipEventRecord(ev0, st) : hipSuccess;
    if (e == hipSuccess && L.clear_flag) e = hipMemsetAsync(L.clear_flag, 0, 8, st);
    if (e == hipSuccess && ev1) e = hipEventRecord(ev1, st);
    if (e == hipSuccess) e = hipMemsetAsync(L.total, 0, sizeof(int64_t), st);
    if (e == hipSuccess && D.hdr)                  // an empty delivery: the header only
      e = stencil_deliver_launch(L.key, L.out, L.k, L.total, 0, L.carry, D, st);
    return e;
  }
  const int64_t ntiles = (L.n + ST_TILE - 1) / ST_TILE;
  const int sub = stencil_sub(ntiles);
  const int64_t nsuper = (ntiles + sub - 1) / sub;
  hipError_t e = ev0 ? hipEventRecord(ev0, st) : hipSuccess;
  if (e == hipSuccess) e = stencil_count(L, st);
  if (e == hipSuccess && ev1) e = hipEventRecord(ev1, st);
  if (e != hipSuccess) return e;
  // the kernel that ran (stencil_kernel.h launch_kts) and its slot format
  const bool plain = L.plain && !L.chain && L.k <= 7;
  const SlotFormat F{L.k, plain, L.chain, L.carry.hdr != nullptr, plain && !L.carry.hdr && ST_PLAIN_STAGE,
                     !plain && !L.carry.hdr && ST_KEYED_DENSE, nsuper, sub};
  if (nsuper <= SMALL_FINISH && D.hdr && L.carry.hdr && D.a_moff && L.n <= ARR_SMALL) {   // a small arrival-order flush
    hipLaunchKernelGGL(stencil_finish_deliver_arrival, dim3(1), dim3(1024), 0, st, L.slots, L.tile_count, nsuper, L.k,
                       L.out, L.out_cap, sub, L.total, L.clear_flag, F, L.key, L.carry, L.n, D.host_cap, D.hdr, D.hkey,
                       D.hpos, D.dkey, D.dpos, D.ticket, D.stamp);
    return hipGetLastError();
  }
  if (nsuper <= SMALL_FINISH && D.hdr && L.carry.hdr && !D.a_moff) {   // a small carry flush: scan, rows and delivery at once
    hipLaunchKernelGGL(stencil_finish_deliver, dim3(unsigned(nsuper)), dim3(256), 0, st, L.slots, L.tile_count, nsuper,
                       L.k, L.out, L.out_cap, sub, L.total, L.clear_flag, F, L.key, L.carry, D.host_cap, D.hdr, D.hkey,
                       D.hpos, D.dkey, D.dpos, D.ticket, D.stamp);
    return hipGetLastError();
  }
  if (nsuper <= SMALL_FINISH) {
    hipLaunchKernelGGL(stencil_finish_small, dim3(1), dim3(1024), 0, st, L.slots, L.tile_count, nsuper, L.k, L.out,
                       L.out_cap, sub, L.total, L.clear_flag, F);
  } else {
    if (nsuper <= 8 * 1024) {
      hipLaunchKernelGGL(tile_scan, dim3(1), dim3(1024), 0, st, L.tile_count, nsuper, L.tile_pre, L.total, L.clear_flag);
    } else {
      // past 8 counts per thread tile_scan walks each thread's range twice, uncoalesced (C5, 61 k
      // super-tiles: 101 us); the multi-workgroup scan takes a few microseconds per pass
      hipError_t e = exclusive_scan(L.tile_count, nsuper, L.tile_pre, L.total, L.scan_tmp, st);
      if (e == hipSuccess && L.clear_flag) e = hipMemsetAsync(L.clear_flag, 0, 8, st);
      if (e != hipSuccess) return e;
    }
    if (F.dense) {
      decltype(&stencil_gather_dense<1>) g = nullptr;
      switch (L.k) {
        case 1: g = stencil_gather_dense<1>; break;
        case 2: g = stencil_gather_dense<2>; break;
        case 3: g = stencil_gather_dense<3>; break;
        case 4: g = stencil_gather_dense<4>; break;
        case 5: g = stencil_gather_dense<5>; break;
        case 6: g = stencil_gather_dense<6>; break;
        case 7: g = stencil_gather_dense<7>; break;
        default: return hipErrorInvalidValue;     // (the plain kernel: k <= 7)
      }
      hipLaunchKernelGGL(g, dim3(unsigned(nsuper)), dim3(128), 0, st, L.slots, L.tile_count, L.tile_pre, L.out,
                         L.out_cap, nsuper, sub);
    } else {
      decltype(&stencil_gather_k<1>) g = nullptr;
      switch (L.k) {
        case 1: g = stencil_gather_k<1>; break;
        case 2: g = stencil_gather_k<2>; break;
        case 3: g = stencil_gather_k<3>; break;
        case 4: g = stencil_gather_k<4>; break;
        case 5: g = stencil_gather_k<5>; break;
        case 6: g = stencil_gather_k<6>; break;
        case 7: g = stencil_gather_k<7>; break;
        case 8: g = stencil_gather_k<8>; break;
        default: break;
      }
      if (g) {
        hipLaunchKernelGGL(g, dim3(unsigned(nsuper)), dim3(128), 0, st, L.slots, L.tile_count, L.tile_pre, L.out,
                           L.out_cap, F);
      } else {
        hipLaunchKernelGGL(stencil_gather, dim3(unsigned(nsuper)), dim3(128), 0, st, L.slots, L.tile_count, L.tile_pre,
                           L.out, L.out_cap, sub, F);
      }
    }
  }
  if (D.hdr) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return stencil_deliver_launch(L.key, L.out, L.k, L.total, L.out_cap, L.carry, D, st);
  }
  return hipGetLastError();
}

// ---- post-processing helpers (not on the timed path) ----
__global__ void stencil_gather_keys(const int32_t* __restrict__ key, const int32_t* __restrict__ out, int k,
                                    int64_t nm, int32_t* __restrict__ mkey) {
  const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < nm) mkey[i] = key[out[i * k + k - 1]];
}

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
  return x;
}

// checksum identical to oracle/cep_oracle.c shard_main: per match
//   h = mix64(record * golden); for each traversal entry (final -> begin)
//   h = mix64(h ^ (record << 8) ^ name); sum of h over matches (mod 2^64)
__global__ void stencil_checksum(const int32_t* __restrict__ out, int k, int64_t nm,
                                 const StencilProgram* __restrict__ P, unsigned long long* __restrict__ sum) {
  const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  uint64_t h = 0;
  if (i < nm) {
    const int64_t j = out[i * k + k - 1];
    h = mix64(uint64_t(j) * 0x9e3779b97f4a7c15ULL);
    for (int s = k - 1; s >= 0; s--) {
      const int32_t r = out[i * k + s];
      if (r >= 0) h = mix64(h ^ (uint64_t(r) << 8) ^ uint64_t(P->name[s]));   // -1: skipped optional stage
    }
  }
  for (int d = 32; d >= 1; d >>= 1) h += __shfl_xor(h, d, 64);
  if ((threadIdx.x & 63) == 0 && h) atomicAdd(sum, (unsigned long long)h);
}

// carry sessions: every entry as a stream position (int64), halo entries looked up in the key's
// halo slot the batch read (kcep_internal.h halo_old); -1 stays (a skipped optional stage)
__global__ void stencil_resolve(const int32_t* __restrict__ key, const int32_t* __restrict__ out, int k, int64_t nm,
                                StencilCarry C, int64_t* __restrict__ pos) {
  const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= nm) return;
  const int32_t last = out[i * k + k - 1];
  const int32_t kk = key[last];
  const HaloHdr& h = C.hdr[kk];
  const int old = halo_old(h, C.stamp);
  const int64_t* hp = C.pos + (2 * int64_t(kk) + old) * C.km1;
  for (int s = 0; s < k; s++) {
    const int32_t r = out[i * k + s];
    pos[i * k + s] = r >= 0 ? halo_gpos(C, r) : (r == -1 ? -1 : hp[h.cnt[old] - (-r - 1)]);
  }
}
// CEP_BATCH_DELIVER (a carry session's flush, GpuCEPProcessor): the batch's matches handed to pinned host
// memory by the device itself, right after the scan -- the header {match count, this batch's error
// flags}, then per match its key id and its k entries as stream positions (stencil_resolve's rule) --
// so that cep_collect is one wait instead of one host round trip per post-processing step.  Matches
// past host_cap go to the device arrays (dkey / dpos), which cep_collect copies.  The match count is
// read on the device: the grid strides over the session's capacity.
// CEP_BATCH_ARRIVAL_ORDER (moff != null): match i goes to moff[a] + (i - head[a]), a = the arrival index of its
// completing record (group.hip stencil_arrival_ranks)
__global__ __launch_bounds__(256) void stencil_deliver(const int32_t* __restrict__ key, const int32_t* __restrict__ out,
                                                       int k, const int64_t* __restrict__ total, int64_t out_cap,
                                                       StencilCarry C, int64_t host_cap, int64_t* __restrict__ hdr,
                                                       int32_t* __restrict__ hkey, int64_t* __restrict__ hpos,
                                                       int32_t* __restrict__ dkey, int64_t* __restrict__ dpos,
                                                       unsigned* ticket, int64_t stamp, const int64_t* __restrict__ moff,
                                                       const int32_t* __restrict__ head) {
  const int64_t t = *total, nm = t < out_cap ? t : out_cap;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    hdr[0] = t;
    hdr[1] = int64_t(*C.flags);
  }
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < nm; i += int64_t(gridDim.x) * blockDim.x) {
    const int32_t last = out[i * k + k - 1];
    const int32_t kk = key[last];
    const bool kok = kk >= 0 && kk < C.max_keys;   // else error flag bit 0: the host fails the batch
    const HaloHdr* h = kok ? C.hdr + kk : nullptr;
    const int old = kok ? halo_old(*h, C.stamp) : 0;
    const int64_t* hp = kok ? C.pos + (2 * int64_t(kk) + old) * C.km1 : nullptr;
    int64_t j = i;
    if (moff) {
      const int64_t a = C.gpos[last] - C.base;
      j = moff[a] + (i - head[a]);
    }
    const bool host = j < host_cap;
    int64_t* p = host ? hpos + j * k : dpos + j * k;
    for (int s = 0; s < k; s++) {
      const int32_t r = out[i * k + s];
      p[s] = r >= 0 ? halo_gpos(C, r) : (r == -1 || !kok ? -1 : hp[h->cnt[old] - (-r - 1)]);
    }
    if (host) hkey[j] = kk;
    else dkey[j] = kk;
  }
  deliver_done(ticket, unsigned(gridDim.x), hdr, stamp);
}
hipError_t stencil_deliver_launch(const int32_t* key, const int32_t* out, int k, const int64_t* total, int64_t out_cap,
                                  const StencilCarry& C, const DeliverArgs& D, hipStream_t st) {
  const int64_t blocks = std::min<int64_t>((out_cap + 255) / 256, 1024);
  if (D.a_moff) {                                  // arrival order: the matches' ranks first
    hipError_t e = stencil_arrival_ranks(out, k, total, out_cap, C.gpos, C.base, D.a_n, D.a_cnt, D.a_head, D.a_moff,
                                         D.a_tot, D.a_tmp, st);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(stencil_deliver, dim3(unsigned(std::max<int64_t>(blocks, 1))), dim3(256), 0, st, key, out, k, total,
                     out_cap, C, D.host_cap, D.hdr, D.hkey, D.hpos, D.dkey, D.dpos, D.ticket, D.stamp, D.a_moff, D.a_head);
  return hipGetLastError();
}

__global__ void stencil_checksum_pos(const int64_t* __restrict__ pos, int k, int64_t nm,
                                     const StencilProgram* __restrict__ P, unsigned long long* __restrict__ sum) {
  const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  uint64_t h = 0;
  if (i < nm) {
    h = mix64(uint64_t(pos[i * k + k - 1]) * 0x9e3779b97f4a7c15ULL);
    for (int s = k - 1; s >= 0; s--) {
      const int64_t r = pos[i * k + s];
      if (r >= 0) h = mix64(h ^ (uint64_t(r) << 8) ^ uint64_t(P->name[s]));
    }
  }
  for (int d = 32; d >= 1; d >>= 1) h += __shfl_xor(h, d, 64);
  if ((threadIdx.x & 63) == 0 && h) atomicAdd(sum, (unsigned long long)h);
}
hipError_t stencil_resolve_launch(const int32_t* key, const int32_t* out, int k, int64_t nm, const StencilCarry& C,
                                  int64_t* pos, const StencilProgram* P, unsigned long long* sum, hipStream_t st) {
  if (nm <= 0) return hipSuccess;
  const unsigned blocks = unsigned((nm + 255) / 256);
  hipLaunchKernelGGL(stencil_resolve, dim3(blocks), dim3(256), 0, st, key, out, k, nm, C, pos);
  if (sum) hipLaunchKernelGGL(stencil_checksum_pos, dim3(blocks), dim3(256), 0, st, pos, k, nm, P, sum);
  return hipGetLastError();
}

hipError_t stencil_post(const int32_t* key, const int32_t* out, int k, int64_t nm, int32_t* mkey,
                        const StencilProgram* P, unsigned long long* sum, hipStream_t st) {
  if (nm <= 0) return hipSuccess;
  const unsigned blocks = unsigned((nm + 255) / 256);
  if (mkey) hipLaunchKernelGGL(stencil_gather_keys, dim3(blocks), dim3(256), 0, st, key, out, k, nm, mkey);
  if (sum) hipLaunchKernelGGL(stencil_checksum, dim3(blocks), dim3(256), 0, st, out, k, nm, P, sum);
  return hipGetLastError();
}

}  // namespace kcep

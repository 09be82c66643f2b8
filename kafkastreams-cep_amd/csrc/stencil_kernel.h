// stencil_kernel.h -- the streaming stencil / chain kernel and its per-K launchers, shared by
// stencil.hip (scan, gather, post-processing) and the per-K instantiation units stencil_k<N>.hip
// (one translation unit per K, so the variants compile in parallel).
#pragma once
// stencil.hip — strict-contiguity, single-cardinality fast path.
//
// For a pattern P1 -> ... -> Pk whose stages are all strict, cardinality ONE,
// not optional, fold-free and distinctly named, the reference NFA
// (nfa/NFA.java:134-341) keeps at most one run waiting per stage and every
// shared-buffer node has exactly one predecessor, so per key it emits exactly
// one match at record j iff the k consecutive same-key records j-k+1..j satisfy
// P1..Pk (the traversal is final -> begin, one event per stage).
//
// HBM-bound integer streaming: 4 B key + 4/8 B value per record in, 4*k B per
// match out, one pass, ordered output:
//   * 256-thread workgroups each own a super-tile of ST_SUB x 4096 records;
//     no workgroup ever waits on another (no dequeue atomic, no look-back: a
//     returning atomic per workgroup cost ~20% of the kernel, measured);
//   * count phase, per 4096-record tile: lane-contiguous 16-B non-temporal
//     loads (the next tile is in flight while this one is scanned), stage
//     bitmask per record from an interval table, keys + masks staged in LDS
//     with a halo carried over from the previous tile, 16 consecutive records
//     per thread tested in registers, block scan;
//   * write phase: each tile's matches compacted in LDS and written as one
//     coalesced run into the super-tile's own slot (at s * 16384 * k ints),
//     with the super-tile's count;
//   * then an exclusive scan of those counts and stencil_gather move the
//     slots into one contiguous output in record order (matches are sparse:
//     ~2% of records in C2, so this touches ~2 x 18 MB against 800 MB read).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "kcep_internal.h"

namespace kcep {

constexpr int ST_THREADS = 256;
constexpr int ST_EPT = 16;                        // records per thread per tile
constexpr int ST_TILE = ST_THREADS * ST_EPT;      // 4096
constexpr int ST_SUB = 4;                         // tiles per workgroup (large batches)
// Super-tile size per launch: 4 tiles per workgroup once the grid fills the chip several times over
// (>= 2048 workgroups); smaller batches (e.g. one carry batch of a stream) take one tile per workgroup,
// so that more workgroups run their latency-bound tile pipelines side by side.
inline int stencil_sub(int64_t ntiles) { return ntiles >= int64_t(ST_SUB) * 2048 ? ST_SUB : 1; }

typedef int v4i __attribute__((ext_vector_type(4)));
typedef long long v2l __attribute__((ext_vector_type(2)));
// streamed once: non-temporal 16-B loads
__device__ __forceinline__ v4i ld_nt4(const void* p) { return __builtin_nontemporal_load(reinterpret_cast<const v4i*>(p)); }
__device__ __forceinline__ v2l ld_nt2(const void* p) { return __builtin_nontemporal_load(reinterpret_cast<const v2l*>(p)); }

// LDS image of a tile: record r of the tile sits at r' = r + 16 (the 8 halo
// records before the tile at r' = 8..15); keys are padded by 4 words per 16 so
// that both the lane-striped int4 writes of the load and the thread-blocked
// int4 reads of the scan are bank-conflict free.
__device__ __forceinline__ int kpos(int rp) { return rp + 4 * (rp >> 4); }
constexpr int ST_KWORDS = (ST_TILE + 16) + 4 * ((ST_TILE + 16) >> 4) + 16;

// ---- one tile of records in registers (16-B vectors, compile-time indices) ----
template <class VT>
struct VVec;
template <>
struct VVec<int32_t> { v4i a; };
template <>
struct VVec<int64_t> { v2l a, b; };
template <>
struct VVec<double> { v2l a, b; };

// the element is copied out before __builtin_bit_cast: bit-casting a
// vector-element lvalue directly reads element 0 with this clang
template <class VT>
__device__ __forceinline__ VT vget(const VVec<VT>& x, int i) {
  if constexpr (sizeof(VT) == 4) {
    const int32_t e = x.a[i];
    return __builtin_bit_cast(VT, e);
  } else {
    const long long e = i < 2 ? x.a[i] : x.b[i - 2];
    return __builtin_bit_cast(VT, e);
  }
}

template <class VT, bool TOPIC>
struct Chunk {
  v4i k[ST_EPT / 4];
  VVec<VT> v[ST_EPT / 4];
  v4i t[TOPIC ? ST_EPT / 4 : 1];
};

// q-th 16-B vector of thread tid at base + q * STRIDE + 4 * tid (STRIDE: 4 x the threads sharing a tile)
template <class VT, bool TOPIC, int STRIDE = ST_THREADS * 4>
__device__ __forceinline__ void load_chunk(Chunk<VT, TOPIC>& c, const int32_t* __restrict__ key,
                                           const VT* __restrict__ val, const int32_t* __restrict__ topic,
                                           int64_t base, int64_t n, int tid) {
#pragma unroll
  for (int q = 0; q < ST_EPT / 4; q++) {
    const int64_t g = base + q * STRIDE + tid * 4;
    if (g + 3 < n) {
      c.k[q] = ld_nt4(key + g);
      if constexpr (sizeof(VT) == 4) {
        c.v[q].a = ld_nt4(val + g);
      } else {
        c.v[q].a = ld_nt2(val + g);
        c.v[q].b = ld_nt2(val + g + 2);
      }
      if constexpr (TOPIC) c.t[q] = ld_nt4(topic + g);
    } else {
      // tail of the stream: clamped element loads; records >= n get an empty mask
      const int64_t g0 = g < n ? g : n - 1, g1 = g + 1 < n ? g + 1 : n - 1;
      const int64_t g2 = g + 2 < n ? g + 2 : n - 1, g3 = g + 3 < n ? g + 3 : n - 1;
      c.k[q] = v4i{key[g0], key[g1], key[g2], key[g3]};
      if constexpr (sizeof(VT) == 4) {
        c.v[q].a = v4i{__builtin_bit_cast(int32_t, val[g0]), __builtin_bit_cast(int32_t, val[g1]),
                       __builtin_bit_cast(int32_t, val[g2]), __builtin_bit_cast(int32_t, val[g3])};
      } else {
        c.v[q].a = v2l{__builtin_bit_cast(long long, val[g0]), __builtin_bit_cast(long long, val[g1])};
        c.v[q].b = v2l{__builtin_bit_cast(long long, val[g2]), __builtin_bit_cast(long long, val[g3])};
      }
      if constexpr (TOPIC) c.t[q] = v4i{topic[g0], topic[g1], topic[g2], topic[g3]};
    }
  }
}

// interval index of a value: number of breakpoints <= v (breakpoints uniform, in SGPRs)
template <class VT>
__device__ __forceinline__ VT bp_at(const StencilProgram* __restrict__ P, int b) {
  if constexpr (std::is_same<VT, double>::value) return P->bpf[b];
  else return VT(P->bpi[b]);
}

template <class VT, bool TOPIC>
__device__ __forceinline__ void masks_of_chunk(const Chunk<VT, TOPIC>& c, const StencilProgram* __restrict__ P,
                                               const uint8_t* s_tab, const uint8_t* s_nan, uint32_t (&packed)[4],
                                               const uint8_t* s_lut) {
  if constexpr (!TOPIC && !std::is_same<VT, double>::value) {
    const int32_t lut_n = P->lut_n;
    if (lut_n > 0) {                               // dense table: one LDS byte per record (uniform branch)
      const int64_t lo = P->lut_lo;
      const uint32_t below = s_tab[0], above = s_tab[P->nbp];
#pragma unroll
      for (int q = 0; q < 4; q++) {
        uint32_t w = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const int64_t dv = int64_t(vget<VT>(c.v[q], i)) - lo;
          const uint32_t m = dv < 0 ? below : dv >= lut_n ? above : uint32_t(s_lut[dv]);
          w |= m << (8 * i);
        }
        packed[q] = w;
      }
      return;
    }
  }
  int iv[ST_EPT], it[ST_EPT];
#pragma unroll
  for (int e = 0; e < ST_EPT; e++) { iv[e] = 0; it[e] = 0; }
  const int nbp = P->nbp;
  for (int b = 0; b < nbp; b++) {                 // scalar loop: breakpoint in an SGPR, 16 records per step
    const VT bp = bp_at<VT>(P, b);
#pragma unroll
    for (int e = 0; e < ST_EPT; e++) iv[e] += bp <= vget<VT>(c.v[e >> 2], e & 3) ? 1 : 0;
  }
  if constexpr (TOPIC) {
    const int ntbp = P->ntbp;
    for (int b = 0; b < ntbp; b++) {
      const int32_t tb = P->tbp[b];
#pragma unroll
      for (int e = 0; e < ST_EPT; e++) {
        const int32_t tv = c.t[e >> 2][e & 3];
        it[e] += tb <= tv ? 1 : 0;
      }
    }
  }
#pragma unroll
  for (int q = 0; q < 4; q++) {
    uint32_t w = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int e = 4 * q + i;
      uint32_t m = s_tab[it[e] * 16 + iv[e]];
      if constexpr (std::is_same<VT, double>::value) {
        const double v = vget<VT>(c.v[q], i);
        if (v != v) m = s_nan[it[e]];
      }
      w |= m << (8 * i);
    }
    packed[q] = w;
  }
}

template <class VT, bool TOPIC>
__device__ __forceinline__ uint32_t mask_of(const StencilProgram* __restrict__ P, const uint8_t* s_tab,
                                            const uint8_t* s_nan, VT v, int32_t t) {
  int iv = 0, it = 0;
  for (int b = 0; b < P->nbp; b++) iv += bp_at<VT>(P, b) <= v ? 1 : 0;
  if constexpr (TOPIC)
    for (int b = 0; b < P->ntbp; b++) it += P->tbp[b] <= t ? 1 : 0;
  if constexpr (std::is_same<VT, double>::value)
    if (v != v) return s_nan[it];
  return s_tab[it * 16 + iv];
}

// Chain patterns (strict, optional() stages, K <= 4; compile.cpp analyse_stencil),
// evaluated bit-parallel over the thread's 24-record window (bit w = window
// position w).  A run started at record a (stage 0 consumes a) is deterministic:
// at stage i on record r, BEGIN (slot i) consumes r; else the SKIP_PROCEED edge
// of an optional stage i (slot 4+i, and not slot i) moves on to stage i+1 on the
// same record; else the run dies (NFA.java:190-341 without TAKE/IGNORE edges).
// X[i] after d steps = runs started d records before bit p that consumed p and
// wait at stage i; each start is one run, so the bits never merge.
template <int K>
struct ChainWin {
  uint32_t b[K];      // slot i (BEGIN edge of stage i) per record
  uint32_t s[K];      // slot 4+i (SKIP_PROCEED of optional stage i), 0 for mandatory stages
  uint32_t same;      // record w has the key of record w-1
};

// bit i of each of the 8 bytes of m -> 8 contiguous bits (byte b -> bit b): the
// byte-LSB gather by one multiply (0x0102040810204080 lands byte b's bit at 56+b;
// the cross terms stay below bit 56 or overflow past 63)
__device__ __forceinline__ uint32_t byte_bits(uint64_t m, int i) {
  return uint32_t((((m >> i) & 0x0101010101010101ull) * 0x0102040810204080ull) >> 56);
}

template <int K>
__device__ __forceinline__ ChainWin<K> chain_window(const int32_t (&wk)[24], const uint64_t (&m8)[3], uint32_t opt) {
  ChainWin<K> c;
#pragma unroll
  for (int i = 0; i < K; i++) { c.b[i] = 0; c.s[i] = 0; }
  c.same = 0;
#pragma unroll
  for (int q = 0; q < 3; q++) {
#pragma unroll
    for (int i = 0; i < K; i++) {
      c.b[i] |= byte_bits(m8[q], i) << (8 * q);
      c.s[i] |= byte_bits(m8[q], CHAIN_MAX_K + i) << (8 * q);
    }
  }
#pragma unroll
  for (int w = 1; w < 24; w++) c.same |= uint32_t(wk[w] == wk[w - 1]) << w;
#pragma unroll
  for (int i = 0; i < K; i++)
    if (!((opt >> i) & 1)) c.s[i] = 0;
  return c;
}

// e[d]: bit p set iff the run started at p-d completes (consumes stage K-1) at p.
// consumed(d, p): the stages the run started at p-d consumed (records p-d..p in order).
template <int K>
struct ChainEnds {
  uint32_t e[K];
  __device__ __forceinline__ void run(const ChainWin<K>& c, int want_d, int want_p, uint32_t* cm) {
    uint32_t x[K + 1];
#pragma unroll
    for (int i = 0; i <= K; i++) x[i] = 0;
    x[1] = c.b[0];
    e[0] = 0;
    if (cm) *cm = 1;
#pragma unroll
    for (int d = 1; d < K; d++) {
      uint32_t y[K + 1];
#pragma unroll
      for (int i = 0; i <= K; i++) y[i] = 0;
#pragma unroll
      for (int i = 1; i < K; i++) {
        uint32_t pass = (x[i] << 1) & c.same;       // the run's next record, same key
#pragma unroll
        for (int j = i; j < K; j++) {
          const uint32_t take = pass & c.b[j];
          y[j + 1] |= take;
          if (cm && d <= want_d && ((take >> (want_p - want_d + d)) & 1)) *cm |= 1u << j;
          pass &= c.s[j] & ~c.b[j];                   // skipped on this record
        }
      }
#pragma unroll
      for (int i = 0; i <= K; i++) x[i] = y[i];
      e[d] = x[K];
    }
  }
};

// Carry sessions (CARRY): record j is a "boundary" record when fewer than K-1 records of its key
// precede it in the batch -- the key's earlier records are in its halo (kcep_internal.h HaloHdr,
// written by the previous batch that had the key).  The match test then takes the first stages
// from the halo; the entries of those stages are written as -(1 + d), d = records before the
// segment's first record (cep_collect resolves them to stream positions).  The thread holding a
// segment's last record writes the key's new halo into the key's other slot.  Chain patterns replay
// the runs that started in the halo at each boundary record (chain_halo_ends).
//
// A thread reads the halos of the first and last key it visits in one round of independent loads
// (HaloHead: both slots' headers, then the slot the batch reads is picked) and claims the keys whose
// segments start in its records (C.claim, one returning atomic each, issued with those loads), so a
// tile costs one dependent global round trip per thread, not several per boundary record.  The new
// slot's stamp is written with its contents: readers of the same batch ignore a slot stamped with
// the batch (halo_old), so they keep reading the old one.
struct HaloHead {
  int32_t key = INT32_MIN;           // cached key (INT32_MIN: none)
  int32_t old = 0;                   // slot the batch reads (halo_old); the batch writes 1 - old
  int32_t stamp = 0, cnt = 0;        // of the read slot
  uint64_t masks = 0;
};
struct HaloRaw {
  v4i w;                             // stamp[0], stamp[1], claim, cnt[0] | cnt[1] << 8
  v2l m;                             // masks[0], masks[1]
};
__device__ __forceinline__ HaloRaw halo_load(const StencilCarry& C, int32_t k) {
  const HaloHdr* h = C.hdr + k;
  return HaloRaw{*reinterpret_cast<const v4i*>(h), *reinterpret_cast<const v2l*>(&h->masks[0])};
}
__device__ __forceinline__ void halo_pick(const StencilCarry& C, int32_t k, const HaloRaw& r, HaloHead& H) {
  const int32_t sa = r.w[0] < C.stamp ? r.w[0] : -1, sb = r.w[1] < C.stamp ? r.w[1] : -1;   // as halo_old
  H.key = k;
  H.old = sa >= sb ? 0 : 1;
  H.stamp = H.old ? r.w[1] : r.w[0];
  H.cnt = H.old ? (r.w[3] >> 8) & 0xFF : r.w[3] & 0xFF;
  const long long m0 = r.m[0], m1 = r.m[1];
  H.masks = uint64_t(H.old ? m1 : m0);
}
__device__ __forceinline__ bool key_ok(const StencilCarry& C, int32_t k) {
  if (k >= 0 && k < C.max_keys) return true;
  atomicOr(C.flags, 1ull);
  return false;
}
__device__ __forceinline__ bool halo_head(const StencilCarry& C, int32_t k, HaloHead& H) {
  if (k == H.key && k >= 0) return true;
  if (!key_ok(C, k)) return false;
  halo_pick(C, k, halo_load(C, k), H);
  return true;
}

template <int K>
__device__ __forceinline__ bool halo_match(const HaloHead& H, int need) {
  if (H.stamp <= 0 || H.cnt < need) return false;
  bool ok = true;
#pragma unroll
  for (int t = 0; t < K - 1; t++)
    if (t < need) ok = ok && ((H.masks >> (8 * (H.cnt - need + t) + t)) & 1);
  return ok;
}

// the key's halo after this batch: its last K-1 records (older ones from the previous halo when the
// segment is shorter); seg = segment records j-seg+1..j (<= K-1), wmk: their stage masks, oldest first
template <int K>
__device__ __forceinline__ void halo_write(const StencilCarry& C, const HaloHead& H, int seg, uint64_t wmk, int64_t gj) {
  HaloHdr* h = C.hdr + H.key;
  const int nw = 1 - H.old;
  const int64_t* op = C.pos + (2 * int64_t(H.key) + H.old) * (K - 1);
  int64_t* np = C.pos + (2 * int64_t(H.key) + nw) * (K - 1);
  const int keep = H.stamp > 0 ? (K - 1 - seg < H.cnt ? K - 1 - seg : H.cnt) : 0;
  uint64_t masks = 0;
  int c = 0;
  for (int t = H.cnt - keep; t < H.cnt; t++, c++) {
    masks |= ((H.masks >> (8 * t)) & 0xFFull) << (8 * c);
    np[c] = op[t];
  }
  for (int t = 0; t < seg; t++, c++) {
    masks |= ((wmk >> (8 * t)) & 0xFFull) << (8 * c);
    np[c] = halo_gpos(C, gj - (seg - 1) + t);
  }
  h->masks[nw] = masks;
  h->cnt[nw] = uint8_t(c);
  h->stamp[nw] = C.stamp;
}

// Chain carry sessions: the runs a boundary record j can complete that started in the key's halo
// (its last K-1 records of earlier batches).  Each start is one deterministic run (analyse_stencil):
// replayed over the halo records then the segment's records up to j (seg[0..o], oldest first), it
// completes at j or not.  Returns bit d set when the run started d records before j completes at j,
// with its consumed stages in cms[d]; d > o always (the start lies before the segment).
template <int K>
__device__ __forceinline__ uint32_t chain_halo_ends(const HaloHead& H, int o, uint32_t seg, uint32_t opt,
                                                    uint32_t (&cms)[K]) {
  if (H.stamp <= 0) return 0;
  const int cnt = H.cnt;
  const uint64_t hm = H.masks;
  uint32_t res = 0;
  const int t0 = cnt - (K - 1 - o) > 0 ? cnt - (K - 1 - o) : 0;
  for (int t = t0; t < cnt; t++) {
    const int d = (cnt - t) + o;
    int stage = 0;
    uint32_t cm = 0;
    bool done = false;
    for (int v = 0; v <= d; v++) {
      const uint32_t m = v < cnt - t ? uint32_t((hm >> (8 * (t + v))) & 0xFFull) : (seg >> (8 * (v - (cnt - t)))) & 0xFFu;
      bool alive = false;
      while (stage < K) {                          // BEGIN consumes; else SKIP_PROCEED of an optional stage
        if ((m >> stage) & 1) { cm |= 1u << stage; stage++; alive = true; break; }
        if (((opt >> stage) & 1) && ((m >> (CHAIN_MAX_K + stage)) & 1)) { stage++; continue; }
        break;
      }
      if (!alive) break;
      if (stage == K) { done = v == d; break; }
    }
    if (done) { res |= 1u << d; cms[d] = cm; }
  }
  return res;
}

// stage s's entry of a keyed-kernel match (completing record rj, aux byte a; see the write phase):
// the record, -1 for a skipped optional stage, -(1 + d) for a halo record d records before the segment
__device__ __forceinline__ int32_t stencil_row(int32_t rj, uint32_t a, int s, int k, bool chain, bool carry) {
  if (chain) {
    const uint32_t d = a & 3u, cm = (a >> 2) & 15u;
    const int ho = int(a >> 6);
    const int rel = -int32_t(d) + __popc(cm & ((1u << s) - 1));
    if (!((cm >> s) & 1)) return -1;
    if (carry && ho != 3 && rel < -ho) return -(1 + (-ho - rel));
    return rj + rel;
  }
  const int need = carry ? int(a) : 0;
  return s < need ? -(1 + (need - s)) : rj - (k - 1) + s;
}

template <int K, class VT, bool TOPIC, bool CHAIN, bool CARRY, int SUB>
__global__ __launch_bounds__(ST_THREADS) void stencil_kernel(
    const int32_t* __restrict__ key, const VT* __restrict__ val, const int32_t* __restrict__ topic, int64_t n,
    const StencilProgram* __restrict__ P, int32_t* __restrict__ out, int64_t* __restrict__ tile_count,
    int64_t ntiles, StencilCarry C) {
  __shared__ __attribute__((aligned(16))) int32_t s_key[ST_KWORDS];   // keys; then the match list
  __shared__ __attribute__((aligned(16))) uint8_t s_mask[ST_TILE + 16];
  __shared__ int32_t s_wsum[SUB][ST_THREADS / 64];
  __shared__ uint8_t s_tab[64];
  __shared__ uint8_t s_lut[256];
  __shared__ uint8_t s_nan[4];
  __shared__ uint32_t s_super;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  if (tid == 0) s_super = blockIdx.x;             // no ordering between workgroups is needed
  if (tid < 64) s_tab[tid] = P->table[tid];
  s_lut[tid] = P->lut[tid];                       // (ST_THREADS == 256 entries)
  if (tid < 4) s_nan[tid] = P->nan_mask[tid];
  __syncthreads();
  const int64_t tile0 = int64_t(s_super) * SUB;
  const int ntl = int(ntiles - tile0 < SUB ? ntiles - tile0 : SUB);   // tiles of this workgroup

  Chunk<VT, TOPIC> cur;
  load_chunk<VT, TOPIC>(cur, key, val, topic, tile0 * ST_TILE, n, tid);
  // halo of the first tile (the K-1 records before it), fetched with the tile;
  // later tiles take theirs from the previous tile's LDS image
  int32_t h_key = INT32_MIN;
  uint32_t h_mask = 0;
  VT h_val{};
  int32_t h_top = 0;
  const bool halo_lane = tid >= 16 - (K - 1) && tid < 16;
  const bool h_first = halo_lane && tile0 * ST_TILE - 16 + tid >= 0;   // a record exists before the batch start?
  if (h_first) {
    const int64_t g = tile0 * ST_TILE - 16 + tid;
    h_key = key[g];
    h_val = val[g];
    if constexpr (TOPIC) h_top = topic[g];
  }

  uint32_t hits[SUB];
  uint64_t bneed[CARRY ? SUB : 1];              // carry: halo records of each hit (4 bits per record)
  int excl[SUB], total[SUB];
  uint32_t wpk[CHAIN ? SUB : 1][2 * K], wsame[CHAIN ? SUB : 1];   // chain: the window bits, kept for the write phase
  uint32_t hb[CHAIN && CARRY ? SUB : 1];        // chain carry: own records completing runs started in the halo
  const uint32_t opt = CHAIN ? uint32_t(P->optmask) : 0u;

  // ================= count phase =================
#pragma unroll
  for (int j = 0; j < SUB; j++) {
    hits[j] = 0; excl[j] = 0; total[j] = 0;
    if (j < ntl) {                                // uniform
      const int64_t tile = tile0 + j;
      const int64_t base = tile * ST_TILE;
      const int lb = ST_EPT * tid + 8;            // 16 records of this thread + 8 of history
      // carry: the keys go to LDS first, so that each thread finds its segment starts and ends and
      // issues its halo loads and claims before the stage masks are computed (their latency hides
      // behind that work)
      uint32_t bnd = 0, endm = 0, todo = 0;
      int32_t ka = 0, kb = 0;
      bool oka = false, okb = false, twice = false;
      HaloRaw ra{}, rb{};
      if constexpr (CARRY) {
#pragma unroll
        for (int q = 0; q < ST_EPT / 4; q++)
          *reinterpret_cast<v4i*>(&s_key[kpos(16 + q * (ST_THREADS * 4) + tid * 4)]) = cur.k[q];
        if (tid < 16) s_key[kpos(tid)] = halo_lane ? h_key : INT32_MIN;
        __syncthreads();
        int32_t ck[25];
#pragma unroll
        for (int q = 0; q < 6; q++) {
          const v4i k4 = *reinterpret_cast<const v4i*>(&s_key[kpos(lb + 4 * q)]);
          ck[4 * q] = k4[0]; ck[4 * q + 1] = k4[1]; ck[4 * q + 2] = k4[2]; ck[4 * q + 3] = k4[3];
        }
        ck[24] = tid + 1 < ST_THREADS ? s_key[kpos(lb + 24)] : (base + ST_TILE < n ? key[base + ST_TILE] : INT32_MIN);
        const int64_t g0 = base + tid * ST_EPT;            // batch index of own record 0
        uint32_t starts = 0;
#pragma unroll
        for (int i = 0; i < ST_EPT; i++) {
          const int32_t kj = ck[8 + i];
          bool full = true;
#pragma unroll
          for (int t = 1; t < K; t++) full = full && ck[8 + i - t] == kj;
          const bool live = g0 + i < n;
          bnd |= uint32_t(live && !full) << i;
          endm |= uint32_t(live && (ck[9 + i] != kj || g0 + i + 1 >= n)) << i;
          starts |= uint32_t(ck[7 + i] != kj) << i;
        }
        starts &= bnd;
        todo = bnd | endm;
        if (todo) {
          ka = ck[8 + __ffs(todo) - 1];
          kb = ck[8 + 31 - __clz(todo)];
          oka = key_ok(C, ka);
          okb = kb != ka && key_ok(C, kb);
          ra = halo_load(C, oka ? ka : 0);
          rb = halo_load(C, okb ? kb : 0);
          if (C.grouped) starts = 0;
          while (starts) {                                 // claims, checked after the visits
            const int i = __ffs(starts) - 1;
            starts &= starts - 1;
            const int32_t ks = s_key[kpos(lb + 8 + i)];
            if (ks >= 0 && ks < C.max_keys) twice |= atomicMax(&C.hdr[ks].claim, C.stamp) == C.stamp;
          }
        }
      }
      uint32_t packed[4];
      masks_of_chunk<VT, TOPIC>(cur, P, s_tab, s_nan, packed, s_lut);
#pragma unroll
      for (int q = 0; q < ST_EPT / 4; q++) {
        const int local = q * (ST_THREADS * 4) + tid * 4;
        uint32_t w = packed[q];
        const int64_t left = n - (base + local);  // records >= n match nothing
        if (left < 4) w &= left <= 0 ? 0u : (0xFFFFFFFFu >> (8 * (4 - left)));
        if constexpr (!CARRY) *reinterpret_cast<v4i*>(&s_key[kpos(16 + local)]) = cur.k[q];
        *reinterpret_cast<uint32_t*>(&s_mask[16 + local]) = w;
      }
      if (tid < 16) {                             // halo: the records before the tile (r' = 0..15)
        if (j == 0 && h_first) h_mask = mask_of<VT, TOPIC>(P, s_tab, s_nan, h_val, h_top);
        if constexpr (!CARRY) s_key[kpos(tid)] = halo_lane ? h_key : INT32_MIN;
        s_mask[tid] = halo_lane ? uint8_t(h_mask) : 0;
      }
      __syncthreads();
      if (j + 1 < ntl) load_chunk<VT, TOPIC>(cur, key, val, topic, base + ST_TILE, n, tid);   // prefetch

      int32_t wk[24];
      uint8_t wm[24];
      uint64_t m8s[3];
#pragma unroll
      for (int q = 0; q < 6; q++) {
        const v4i k4 = *reinterpret_cast<const v4i*>(&s_key[kpos(lb + 4 * q)]);
        wk[4 * q] = k4[0]; wk[4 * q + 1] = k4[1]; wk[4 * q + 2] = k4[2]; wk[4 * q + 3] = k4[3];
      }
#pragma unroll
      for (int q = 0; q < 3; q++) {
        const uint64_t m8 = *reinterpret_cast<const uint64_t*>(&s_mask[lb + 8 * q]);
        m8s[q] = m8;
#pragma unroll
        for (int b = 0; b < 8; b++) wm[8 * q + b] = uint8_t(m8 >> (8 * b));
      }
      uint32_t hit = 0;
      int cnt = 0;
      if constexpr (CHAIN) {
        const ChainWin<K> cw = chain_window<K>(wk, m8s, opt);
        ChainEnds<K> ce;
        ce.run(cw, 0, 0, nullptr);
#pragma unroll
        for (int d = 1; d < K; d++) cnt += __popc(ce.e[d] & 0xFFFF00u);   // ends at own records 8..23
#pragma unroll
        for (int i = 0; i < K; i++) { wpk[j][i] = cw.b[i]; wpk[j][K + i] = cw.s[i]; }
        wsame[j] = cw.same;
      } else {
#pragma unroll
        for (int i = 0; i < ST_EPT; i++) {
          bool ok = true;
#pragma unroll
          for (int s = 0; s < K; s++) {
            const int w = 8 + i - (K - 1) + s;
            ok = ok && ((wm[w] >> s) & 1) && wk[w] == wk[8 + i];
          }
          hit |= uint32_t(ok) << i;
        }
      }
      if constexpr (CARRY) {
        // boundary records (fewer than K-1 same-key records before them in the batch) and segment
        // ends (bit masks over the thread's 16 records, found before the masks): only those records
        // are visited, with keys and masks read back from the tile's LDS image (dynamic index, no
        // register arrays)
        const int64_t g0 = base + tid * ST_EPT;            // batch index of own record 0
        if constexpr (CHAIN) hb[j] = 0;
        else { bnd &= ~hit; bneed[j] = 0; todo = bnd | endm; }
        HaloHead H0, H1;                                   // the first and the last visited key
        if (oka) halo_pick(C, ka, ra, H0);
        if (okb) halo_pick(C, kb, rb, H1);
        while (todo) {
          const int i = __ffs(todo) - 1;
          todo &= todo - 1;
          const int32_t kj = s_key[kpos(lb + 8 + i)];
          int o = 0;                                       // same-key records before it in the batch
#pragma unroll
          for (int t = 1; t < K; t++)
            if (o == t - 1 && s_key[kpos(lb + 8 + i - t)] == kj) o = t;
          HaloHead H = kj == H0.key ? H0 : H1;
          if (!halo_head(C, kj, H)) continue;
          if ((bnd >> i) & 1) {
            if constexpr (CHAIN) {                         // runs started in the halo may end here
              uint32_t seg = 0, cms[K];
              for (int t = 0; t <= o; t++) seg |= uint32_t(s_mask[lb + 8 + i - o + t]) << (8 * t);
              const uint32_t ends = chain_halo_ends<K>(H, o, seg, opt, cms);
              if (ends) { cnt += __popc(ends); hb[j] |= 1u << i; }
            } else {                                       // the first stages in the halo
              const int need = K - 1 - o;
              bool inb = true;
              for (int t = 0; t <= o; t++) inb = inb && ((s_mask[lb + 8 + i - o + t] >> (need + t)) & 1);
              if (inb && halo_match<K>(H, need)) {
                hit |= 1u << i;
                bneed[j] |= uint64_t(need) << (4 * i);
              }
            }
          }
          if ((endm >> i) & 1) {                           // the segment's last record: the new halo
            const int sg = o + 1 < K - 1 ? o + 1 : K - 1;
            uint64_t wmk = 0;
            for (int t = 0; t < sg; t++) wmk |= uint64_t(s_mask[lb + 8 + i - (sg - 1) + t]) << (8 * t);
            halo_write<K>(C, H, sg, wmk, g0 + i);
          }
        }
        if (twice) atomicOr(C.flags, 2ull);               // a key in two segments of the batch
      }
      if constexpr (!CHAIN) cnt = __popc(hit);
      int incl = cnt;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int y = __shfl_up(incl, d, 64);
        if (lane >= d) incl += y;
      }
      if (lane == 63) s_wsum[j][wid] = incl;
      if (halo_lane) {                            // the next tile's halo: this tile's last records
        h_key = s_key[kpos(ST_TILE + tid)];
        h_mask = s_mask[ST_TILE + tid];
      }
      __syncthreads();                            // LDS tile free for the next tile; wave sums visible
      int woff = 0, tot = 0;
#pragma unroll
      for (int w = 0; w < ST_THREADS / 64; w++) {
        const int x = s_wsum[j][w];
        woff += w < wid ? x : 0;
        tot += x;
      }
      hits[j] = hit;
      excl[j] = woff + incl - cnt;
      total[j] = tot;

    }
  }

  // ================= write phase: the super-tile's matches into its slot =================
  // each thread stores its own matches at their place in the tile's run (record order; per record
  // oldest start first): no compaction through LDS, no barrier.  One int per match (its completing
  // record) plus one aux byte (chain: start distance | consumed stages << 2 | halo records << 6;
  // carry: the stages taken from the halo) after the super-tile's SUB x 4096 ints; stencil_gather
  // writes the K-int rows (stencil_row)
  // without carry, a super-tile of at most ST_DENSE_KEYED matches writes them to the dense regions
  // (kcep_internal.h; uniform per workgroup), a larger one to its own region after them
  constexpr bool KD = !CARRY && ST_KEYED_DENSE;
  const int64_t nsup = gridDim.x;
  int64_t stot = 0;
#pragma unroll
  for (int j = 0; j < SUB; j++) stot += total[j];
  const bool dense = KD && stot <= ST_DENSE_KEYED;
  int32_t* const own = out + (KD ? nsup * (ST_DENSE_KEYED + ST_DENSE_KEYED / 4) : 0) + tile0 * int64_t(ST_TILE) * K;
  int32_t* const slot = dense ? out + int64_t(s_super) * ST_DENSE_KEYED : own;
  uint8_t* const aux = dense ? reinterpret_cast<uint8_t*>(out + nsup * ST_DENSE_KEYED) + int64_t(s_super) * ST_DENSE_KEYED
                             : reinterpret_cast<uint8_t*>(own + SUB * ST_TILE);
  auto store_match = [&](int64_t m, int32_t v, uint8_t a) {
    slot[m] = v;
    if constexpr (K > 1) aux[m] = a;             // (k = 1: the own region has no room after the ints; never read)
  };
  int64_t mbase = 0;                               // matches of the super-tile's earlier tiles
  if constexpr (CHAIN && CARRY) {                  // halo runs can exceed a tile's match space: fail the batch
    int64_t sum = 0;
    bool over = false;
#pragma unroll
    for (int j = 0; j < SUB; j++) { sum += total[j]; over = over || total[j] > ST_TILE + 16; }
    if (over || sum > int64_t(ntl) * ST_TILE) {          // (the slot holds ntl tiles); uniform over the workgroup
      if (tid == 0) { tile_count[s_super] = 0; atomicOr(C.flags, 4ull); }
      return;
    }
  }
  if (tid == 0) {
    int64_t sum = 0;
#pragma unroll
    for (int j = 0; j < SUB; j++) sum += total[j];
    tile_count[s_super] = sum;
  }
#pragma unroll
  for (int j = 0; j < SUB; j++) {
    if (j < ntl) {
      const int64_t base = (tile0 + j) * ST_TILE;
      int o = excl[j];
      if constexpr (CHAIN) {
        ChainWin<K> cw;
#pragma unroll
        for (int i = 0; i < K; i++) { cw.b[i] = wpk[j][i]; cw.s[i] = wpk[j][K + i]; }
        cw.same = wsame[j];
        ChainEnds<K> ce;
        ce.run(cw, 0, 0, nullptr);
        uint32_t any = 0;
#pragma unroll
        for (int d = 1; d < K; d++) any |= ce.e[d];
        any &= 0xFFFF00u;
        if constexpr (CARRY) any |= hb[j] << 8;
        // one match: completing record rj, started d records before, consumed-stage mask cm; ho: the
        // segment's records before rj when the run started in the halo (3: it did not)
        auto put = [&](int32_t rj, uint32_t d, uint32_t cm, int ho) {
          store_match(mbase + o, rj, uint8_t(d | (cm << 2) | (uint32_t(ho) << 6)));
          o++;
        };
        while (any) {                                // record order; per record oldest start first
          const int p = __ffs(any) - 1;
          any &= any - 1;
          uint32_t hends = 0, hcms[K], ho = 3;        // halo starts (older than any start in the segment)
          if constexpr (CARRY) {
            if ((hb[j] >> (p - 8)) & 1) {
              uint32_t so = 0, seg = 0;
#pragma unroll
              for (int t = 1; t < K; t++)
                if (so == uint32_t(t - 1) && ((cw.same >> (p - t + 1)) & 1)) so = t;
              for (uint32_t t = 0; t <= so; t++) {    // mask bytes of the segment's records p-so..p
                const int w = p - int(so) + int(t);
                uint32_t mb = 0;
#pragma unroll
                for (int i = 0; i < K; i++)
                  mb |= (((cw.b[i] >> w) & 1u) << i) | (((cw.s[i] >> w) & 1u) << (CHAIN_MAX_K + i));
                seg |= mb << (8 * t);
              }
              HaloHead H;
              if (halo_head(C, key[base + tid * ST_EPT + (p - 8)], H)) hends = chain_halo_ends<K>(H, int(so), seg, opt, hcms);
              ho = so;
            }
          }
          const int32_t rj = int32_t(base + tid * ST_EPT + (p - 8));
          for (int d = K - 1; d >= 1; d--) {
            if ((hends >> d) & 1) {
              put(rj, uint32_t(d), hcms[d], int(ho));
            } else if ((ce.e[d] >> p) & 1) {
              uint32_t cm;
              ChainEnds<K> one;
              one.run(cw, d, p, &cm);
              put(rj, uint32_t(d), cm, 3);
            }
          }
        }
      } else {
        uint32_t h = hits[j];
        while (h) {
          const int i = __ffs(h) - 1;
          h &= h - 1;
          // record index < 2^31 (checked by the launcher); aux: carry: the stages taken from the halo
          store_match(mbase + o, int32_t(base + tid * ST_EPT + i),
                      CARRY && K > 1 ? uint8_t((bneed[j] >> (4 * i)) & 0xF) : uint8_t(0));
          o++;
        }
      }
      mbase += total[j];
    }
  }
}


// ---- the plain stencil (no carry, no optional stage, K <= 7): no keys in LDS ----
// A match needs the K-1 records before record j to have j's key, i.e. the chain of "same key as the
// record before" bits over j-K+2..j.  So the LDS image of a tile holds ONE byte per record: the
// stage bits (bits 0..K-1) with the same-key bit in bit 7, computed by the loading thread (the key
// of the record before its first one comes from the lane below by a shuffle).  Only records at a
// multiple of 256 in the tile have their predecessor in another wave: their bit is resolved by the
// reader from two 17-entry LDS key tables.  The window test is bit-parallel over the thread's 24
// window records (8 of history + its 16): hit(p) = AND_s B_s(p-K+1+s) AND_d same(p-d), d < K-1.
// Against the keyed kernel: 4 B instead of 5 B of LDS traffic per record written and 3 instead of
// 9 LDS reads per window, ~5 KB of LDS per workgroup instead of 25 KB, no 24-key register window;
// each thread stores its own matches (no compaction through LDS).

// load_chunk for a tile that lies wholly inside the batch (uniform branch): uniform tile base
// pointers and 32-bit lane offsets, so every load is one saddr + voffset instruction
template <class VT, bool TOPIC>
__device__ __forceinline__ void load_tile(Chunk<VT, TOPIC>& c, const int32_t* __restrict__ key,
                                          const VT* __restrict__ val, const int32_t* __restrict__ topic,
                                          int64_t base, int64_t n, int tid) {
  if (base + ST_TILE > n) {
    load_chunk<VT, TOPIC>(c, key, val, topic, base, n, tid);
    return;
  }
  const int32_t* kb = key + base;
  const VT* vb = val + base;
  const int32_t* tb = TOPIC ? topic + base : nullptr;
#pragma unroll
  for (int q = 0; q < ST_EPT / 4; q++) {
    const uint32_t o = uint32_t(q * (ST_THREADS * 4) + tid * 4);
    c.k[q] = ld_nt4(kb + o);
    if constexpr (sizeof(VT) == 4) {
      c.v[q].a = ld_nt4(vb + o);
    } else {
      c.v[q].a = ld_nt2(vb + o);
      c.v[q].b = ld_nt2(vb + o + 2);
    }
    if constexpr (TOPIC) c.t[q] = ld_nt4(tb + o);
  }
}

#ifndef ST_PLAIN_EARLY
#define ST_PLAIN_EARLY 1                          // next tile's loads issued before the image barrier (A/B knob)
#endif
#ifndef ST_PLAIN_WAVES
#define ST_PLAIN_WAVES 6                          // waves per SIMD the register budget is cut for (A/B knob)
#endif
// Carry sessions (CARRY): the same window test finds the records with K-1 same-key records before
// them in the batch; the boundary records (the segment's first K-1) and the segments' ends are
// visited as in stencil_kernel<CARRY> (halo reads, claims, halo writes), with their keys from a
// sparse LDS key image: the loader stores the key of each record that starts or ends a segment
// (and of every record whose neighbour lies in another lane), the only keys a visit reads.  A
// boundary match is stored as -(1 + completing record) with its halo record count in the slot's
// aux byte (stencil_gather writes the -(1 + d) halo entries); an interior one as its first record.
#ifndef ST_PLAIN_STAGE
#define ST_PLAIN_STAGE 1                          // the super-tile's matches staged in LDS, one store run (A/B knob)
#endif
#ifndef ST_PLAIN_NTSTORE
#define ST_PLAIN_NTSTORE 1                        // the staged run stored non-temporally (A/B knob)
#endif
#ifndef ST_PLAIN_PROBE
#define ST_PLAIN_PROBE 0                          // timing probes (A/B builds only): 1 no match stores, 2 per-wave runs,
                                                  // 3 no match stores with barrier (B) kept
#endif
#ifndef ST_CARRY_WAVES
#define ST_CARRY_WAVES 4                          // waves per SIMD the carry variant's registers are cut for
#endif
template <int K, class VT, bool TOPIC, int SUB, bool CARRY>
__global__ __launch_bounds__(ST_THREADS, CARRY ? ST_CARRY_WAVES : ST_PLAIN_WAVES) void stencil_plain_kernel(
    const int32_t* __restrict__ key, const VT* __restrict__ val, const int32_t* __restrict__ topic, int64_t n,
    const StencilProgram* __restrict__ P, int32_t* __restrict__ out, int64_t* __restrict__ tile_count,
    int64_t ntiles, StencilCarry C) {
  static_assert(K >= 1 && K <= 7, "bit 7 of a record's byte is its same-key bit");
  __shared__ __attribute__((aligned(16))) uint8_t s_mask[ST_TILE + 16];   // record r at r + 16
  __shared__ int32_t s_bk[CARRY ? ST_TILE + 16 : 1];   // carry: keys of segment starts/ends, record r at r + 16
  __shared__ int32_t s_lastk[2][17];   // [tile & 1][m]: key of tile record 256m - 1 (m >= 1); [0][0]: before tile 0
  __shared__ int32_t s_firstk[16];     // key of tile record 256m
  __shared__ int32_t s_wsum[2][ST_THREADS / 64];
  __shared__ uint8_t s_tab[64];
  __shared__ uint8_t s_lut[256];
  __shared__ uint8_t s_nan[4];
  constexpr bool STAGE = !CARRY && ST_PLAIN_STAGE;
  __shared__ int32_t s_out[STAGE ? ST_TILE : 1];   // staged matches of the super-tile (see the tile loop's end)

  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  if (tid < 64) s_tab[tid] = P->table[tid];
  s_lut[tid] = P->lut[tid];                       // (ST_THREADS == 256 entries)
  if (tid < 4) s_nan[tid] = P->nan_mask[tid];
  const int64_t tile0 = int64_t(blockIdx.x) * SUB;
  const int ntl = int(ntiles - tile0 < SUB ? ntiles - tile0 : SUB);

  Chunk<VT, TOPIC> cur;
  load_tile<VT, TOPIC>(cur, key, val, topic, tile0 * ST_TILE, n, tid);
  // the first tile's halo (its K-1 records before; later tiles take the previous tile's LDS bytes)
  const bool halo_lane = tid >= 16 - (K - 1) && tid < 16;
  const int64_t hg = tile0 * ST_TILE - 16 + tid;
  int32_t h_key = INT32_MIN, h_prev = INT32_MIN, h_top = 0;
  VT h_val{};
  if (halo_lane && hg >= 0) {
    h_key = key[hg];
    h_val = val[hg];
    if constexpr (TOPIC) h_top = topic[hg];
    if (hg > 0) h_prev = key[hg - 1];
  }
  int32_t before0 = INT32_MIN;                    // key of the record before the workgroup's first tile
  if (tid == 0 && tile0 > 0) before0 = key[tile0 * ST_TILE - 1];
  __syncthreads();                                // the tables
  uint32_t h_mask = 0;
  if (halo_lane && hg >= 0)
    h_mask = mask_of<VT, TOPIC>(P, s_tab, s_nan, h_val, h_top) | (uint32_t(hg > 0 && h_prev == h_key) << 7);
  int32_t h_bk = h_key;                           // carry: the history records' keys
  bool twice = false;                             // carry: a key claimed twice in this batch

  // per tile: count, then its matches written as one run into the super-tile's slot right away (the
  // next tile's loads are in flight meanwhile)
  int32_t* slot = out + tile0 * int64_t(ST_TILE) * K;
  uint8_t* const aux = reinterpret_cast<uint8_t*>(slot + SUB * ST_TILE);   // carry: per match, after the ints
  int64_t sum = 0;
  int nbuf = 0;                                   // STAGE: the first nbuf matches are staged in s_out (uniform)
  // STAGE: the slot layout of kcep_internal.h ST_DENSE (the first matches in the dense region)
  int32_t* const dense = out + int64_t(blockIdx.x) * ST_DENSE;
  int32_t* const over = out + int64_t(gridDim.x) * ST_DENSE + tile0 * ST_TILE;
  for (int j = 0; j < ntl; j++) {                 // uniform
    const int64_t base = (tile0 + j) * ST_TILE;
    int32_t nk = INT32_MIN;                       // carry: the key after the tile (thread 255)
    if constexpr (CARRY)
      if (tid == ST_THREADS - 1 && base + ST_TILE < n) nk = key[base + ST_TILE];
    uint32_t packed[4];
    masks_of_chunk<VT, TOPIC>(cur, P, s_tab, s_nan, packed, s_lut);
#pragma unroll
    for (int q = 0; q < ST_EPT / 4; q++) {
      const int local = q * (ST_THREADS * 4) + tid * 4;
      const v4i k = cur.k[q];
      // the record before this lane's first: lane - 1's last (DPP wave_shr:1; lane 0: resolved by readers)
      const int32_t kp = __builtin_amdgcn_update_dpp(INT32_MIN, k[3], 0x138, 0xF, 0xF, false);
      const uint32_t same = uint32_t(lane > 0 && kp == k[0]) | (uint32_t(k[1] == k[0]) << 8) |
                            (uint32_t(k[2] == k[1]) << 16) | (uint32_t(k[3] == k[2]) << 24);
      uint32_t w = packed[q] | (same << 7);
      const int64_t left = n - (base + local);    // records >= n match nothing
      if (left < 4) w &= left <= 0 ? 0u : (0xFFFFFFFFu >> (8 * (4 - left)));
      *reinterpret_cast<uint32_t*>(&s_mask[16 + local]) = w;
      if (lane == 0) s_firstk[4 * q + wid] = k[0];
      if (lane == 63) s_lastk[j & 1][4 * q + wid + 1] = k[3];
      if constexpr (CARRY) {                      // the keys a visit may read (see above)
        const int32_t kn = __builtin_amdgcn_update_dpp(INT32_MIN, k[0], 0x130, 0xF, 0xF, false);   // wave_shl:1
        // c_e: record e differs from the one before, or lies past the batch end (unloaded key)
        const bool c1 = k[1] != k[0] || left <= 1, c2 = k[2] != k[1] || left <= 2, c3 = k[3] != k[2] || left <= 3;
        if (lane == 0 || kp != k[0] || c1) s_bk[16 + local] = k[0];
        if (c1 || c2) s_bk[16 + local + 1] = k[1];
        if (c2 || c3) s_bk[16 + local + 2] = k[2];
        if (c3 || lane == 63 || kn != k[3] || left <= 4) s_bk[16 + local + 3] = k[3];
      }
    }
    if (tid < 16) s_mask[tid] = halo_lane ? uint8_t(h_mask) : 0;
    if constexpr (CARRY)
      if (tid < 16) s_bk[tid] = h_bk;
    if (j == 0 && tid == 0) s_lastk[0][0] = before0;
    // the chunk is consumed: the next tile's loads go out before the barrier, so a wave whose data
    // came early does not hold its refill back until the slowest wave's has arrived
#if ST_PLAIN_EARLY
    if (j + 1 < ntl) load_tile<VT, TOPIC>(cur, key, val, topic, base + ST_TILE, n, tid);
#endif
    __syncthreads();                              // (A) the tile's image
#if !ST_PLAIN_EARLY
    if (j + 1 < ntl) load_tile<VT, TOPIC>(cur, key, val, topic, base + ST_TILE, n, tid);   // prefetch
#endif

    const int lb = ST_EPT * tid + 8;              // LDS byte of window record 0 (tile record 16 tid - 8)
    uint64_t m8[3];
#pragma unroll
    for (int q = 0; q < 3; q++) m8[q] = *reinterpret_cast<const uint64_t*>(&s_mask[lb + 8 * q]);
    uint32_t S = 0;
#pragma unroll
    for (int q = 0; q < 3; q++) S |= byte_bits(m8[q], 7) << (8 * q);
    // the window's record at a multiple of 256 (if any): its same-key bit from the key tables
    const int rb = ((ST_EPT * tid + 15) >> 8) << 8;
    const int pb = rb - (ST_EPT * tid - 8);
    if (pb >= 0 && pb < 24) {
      const int m = rb >> 8;
      const int32_t kb = m == 0 ? (j == 0 ? s_lastk[0][0] : s_lastk[(j - 1) & 1][16]) : s_lastk[j & 1][m];
      S = (S & ~(1u << pb)) | (uint32_t(kb == s_firstk[m]) << pb);
    }
    uint32_t h = 0xFFFFFFFFu;
    uint32_t Bs[K];
#pragma unroll
    for (int s = 0; s < K; s++) {
      uint32_t B = 0;
#pragma unroll
      for (int q = 0; q < 3; q++) B |= byte_bits(m8[q], s) << (8 * q);
      Bs[s] = B;
      h &= B << (K - 1 - s);
    }
#pragma unroll
    for (int d = 0; d < K - 1; d++) h &= S << d;
    uint32_t hit = (h >> 8) & 0xFFFFu;
    uint64_t bneed = 0;                           // carry: halo records of each boundary hit (4 bits each)
    if constexpr (CARRY) {
      // same-key bit of the record after the thread's last (the next thread's first; thread 255: the
      // next tile's first, from the key read at the tile's start)
      const int rn = ST_EPT * tid + 16;
      uint32_t sn = 0;
      if ((rn & 255) == 0) {
        const int m = rn >> 8;
        sn = m < 16 ? uint32_t(s_lastk[j & 1][m] == s_firstk[m]) : uint32_t(base + ST_TILE < n && nk == s_lastk[j & 1][16]);
      } else {
        sn = s_mask[16 + rn] >> 7;
      }
      const int64_t g0 = base + ST_EPT * tid;     // batch index of own record 0 (window record 8)
      if (g0 + ST_EPT >= n) sn = 0;               // the batch's last record ends its segment
      const int64_t left = n - g0;
      const uint32_t live = left >= 16 ? 0xFFFFu : left <= 0 ? 0u : (1u << left) - 1u;
      S &= (live << 8) | 0xFFu;                   // a record past the batch end (table-resolved bit) starts nothing
      const uint32_t Sown = (S >> 8) & 0xFFFFu;
      const uint32_t starts = ~Sown & live;
      const uint32_t ends = ~((S >> 9) | (sn << 15)) & live;
      // boundary candidates: o < K-1 same-key records before the record in the batch (a segment
      // start o records back) and stages K-1-o..K-1 on the segment's records; stages 0..K-2-o must
      // come from the halo
      uint32_t cand = 0;
#pragma unroll
      for (int o = 0; o < K - 1; o++) {
        uint32_t c = ~S << o;
#pragma unroll
        for (int t = 0; t < o; t++) c &= S << t;
#pragma unroll
        for (int t = 0; t <= o; t++) c &= Bs[K - 1 - o + t] << (o - t);
        cand |= c;
      }
      cand = (cand >> 8) & live;
      uint32_t todo = cand | ends | starts;
      if (todo) {
        const int lb16 = 16 + ST_EPT * tid;       // s_bk index of own record 0
        // same-key records before own record i in the batch (capped at K-1)
        auto before_of = [&](int i) {
          int o = 0;
#pragma unroll
          for (int t = 1; t < K; t++)
            if (o == t - 1 && ((S >> (8 + i - t + 1)) & 1)) o = t;
          return o;
        };
        auto key_of = [&](int i) {                // a start or end: its own entry; a candidate: its start's
          const bool own = ((starts | ends) >> i) & 1;
          return s_bk[lb16 + i - (own ? 0 : before_of(i))];
        };
        const int32_t ka = key_of(__ffs(todo) - 1), kb = key_of(31 - __clz(todo));
        const bool oka = key_ok(C, ka), okb = kb != ka && key_ok(C, kb);
        const HaloRaw ra = halo_load(C, oka ? ka : 0), rb = halo_load(C, okb ? kb : 0);
        uint32_t st = C.grouped ? 0u : starts;
        while (st) {                              // claims
          const int i = __ffs(st) - 1;
          st &= st - 1;
          const int32_t ks = s_bk[lb16 + i];
          if (ks >= 0 && ks < C.max_keys) twice |= atomicMax(&C.hdr[ks].claim, C.stamp) == C.stamp;
        }
        HaloHead H0, H1;
        if (oka) halo_pick(C, ka, ra, H0);
        if (okb) halo_pick(C, kb, rb, H1);
        todo = cand | ends;
        while (todo) {
          const int i = __ffs(todo) - 1;
          todo &= todo - 1;
          const int o = before_of(i);
          const int32_t kj = key_of(i);
          HaloHead H = kj == H0.key ? H0 : H1;
          if (!halo_head(C, kj, H)) continue;
          if ((cand >> i) & 1) {                  // the first stages in the halo
            const int need = K - 1 - o;
            if (halo_match<K>(H, need)) {
              hit |= 1u << i;
              bneed |= uint64_t(need) << (4 * i);
            }
          }
          if ((ends >> i) & 1) {                  // the segment's last record: the new halo
            const int sg = o + 1 < K - 1 ? o + 1 : K - 1;
            uint64_t wmk = 0;
            for (int t = 0; t < sg; t++) wmk |= uint64_t(s_mask[lb + 8 + i - (sg - 1) + t] & 0x7Fu) << (8 * t);
            halo_write<K>(C, H, sg, wmk, g0 + i);
          }
        }
      }
    }
    const int cnt = __popc(hit);
    // the wave's exclusive prefix of the counts (<= 16: five bits) by ballots, no shuffle table
    int before = 0, wtot = 0;
#pragma unroll
    for (int b = 0; b < 5; b++) {
      const uint64_t m = __ballot((cnt >> b) & 1);
      before += int(__builtin_amdgcn_mbcnt_hi(uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u))) << b;
      wtot += __popcll(m) << b;
    }
#if ST_PLAIN_PROBE == 1 || ST_PLAIN_PROBE == 2
    if constexpr (!CARRY) {                       // timing probes only (wrong output order / no output)
      if (halo_lane) h_mask = s_mask[ST_TILE + tid];
      if (ST_PLAIN_PROBE == 2) {
        int32_t* ws = out + tile0 * int64_t(ST_TILE) * K + j * ST_TILE + wid * 1024 + before;
        const int32_t b32 = int32_t(base) - (K - 1);
        while (hit) {
          const int i = __ffs(hit) - 1;
          hit &= hit - 1;
          *ws++ = b32 + tid * ST_EPT + i;
        }
      }
      sum += wtot;
      continue;
    }
#endif
    if (lane == 0) s_wsum[j & 1][wid] = wtot;
    if (halo_lane) h_mask = s_mask[ST_TILE + tid];   // the next tile's halo: this tile's last records
    if constexpr (CARRY)
      if (halo_lane) h_bk = s_bk[ST_TILE + tid];
    __syncthreads();                              // (B) wave sums
    int o = before, tot = 0;
#pragma unroll
    for (int w = 0; w < ST_THREADS / 64; w++) {
      const int x = s_wsum[j & 1][w];
      o += w < wid ? x : 0;
      tot += x;
    }
    tot = __builtin_amdgcn_readfirstlane(tot);
    const int32_t b32 = int32_t(base) - (K - 1);  // record index < 2^31 (checked by the launcher)
    if constexpr (STAGE) {
      // the super-tile's matches are staged in LDS and stored once, as one run into the dense region
      // (kcep_internal.h ST_DENSE): C2 kernel 139 -> 131 us; storing each tile's run into the
      // super-tile's own region (196 KB apart) cost 16 us over no stores at all, with or without the
      // LDS staging (profiles/r04_ab_stencil_stores.txt)
      // A tile whose matches no longer fit (over a quarter of the super-tile's records matching)
      // stores them straight to their place, and so do the later ones (sum only grows).
      const int p0 = int(sum) + o;
      if (ST_PLAIN_PROBE == 3) {                  // timing probe: barrier (B) kept, no stores
        sum += tot;
        continue;
      }
      if (sum + tot <= ST_TILE) {                 // uniform
        for (int q = 0; hit; q++) {
          const int i = __ffs(hit) - 1;
          hit &= hit - 1;
          s_out[p0 + q] = b32 + tid * ST_EPT + i;
        }
        nbuf = int(sum) + tot;
      } else {
        for (int q = 0; hit; q++) {
          const int i = __ffs(hit) - 1;
          hit &= hit - 1;
          const int p = p0 + q;
          (p < ST_DENSE ? dense : over)[p] = b32 + tid * ST_EPT + i;
        }
      }
      sum += tot;
      continue;
    }
    // each thread stores its own matches at their place in the tile's run of the slot (no LDS
    // compaction and no third barrier: L2 merges the run's lines; 147.7-150.2 vs 150.8-152.1 us,
    // profiles/r03_ab_stencil_direct_store.jsonl).  ONE int per match -- its first record: the
    // stages' records are consecutive here, so stencil_gather expands them to the K-int output
    while (hit) {
      const int i = __ffs(hit) - 1;
      hit &= hit - 1;
      if constexpr (CARRY) {
        const uint32_t need = uint32_t(bneed >> (4 * i)) & 0xFu;
        if (need) {                               // a boundary match: -(1 + completing record), halo count in aux
          slot[o] = -(1 + int32_t(base) + tid * ST_EPT + i);
          aux[sum + o] = uint8_t(need);
          o++;
          continue;
        }
      }
      slot[o++] = b32 + tid * ST_EPT + i;
    }
    slot += tot;
    sum += tot;
  }
  if constexpr (STAGE) {
    __syncthreads();                              // the last tile's staged matches
#if ST_PLAIN_NTSTORE
    for (int i = tid; i < nbuf; i += ST_THREADS) __builtin_nontemporal_store(s_out[i], &(i < ST_DENSE ? dense : over)[i]);
#else
    for (int i = tid; i < nbuf; i += ST_THREADS) (i < ST_DENSE ? dense : over)[i] = s_out[i];
#endif
  }
#if ST_PLAIN_PROBE == 1 || ST_PLAIN_PROBE == 2
  if constexpr (!CARRY) {
    if (lane == 0) s_wsum[0][wid] = int(sum);
    __syncthreads();
    if (tid == 0) tile_count[blockIdx.x] = s_wsum[0][0] + s_wsum[0][1] + s_wsum[0][2] + s_wsum[0][3];
    return;
  }
#endif
  if (tid == 0) tile_count[blockIdx.x] = sum;
  if constexpr (CARRY)
    if (twice) atomicOr(C.flags, 2ull);           // a key in two segments of the batch
}

template <int K, class VT, bool TP, bool CH, int SUB>
inline void launch_kts(const StencilLaunch& L, int64_t ntiles, hipStream_t st) {
  const int64_t nsuper = (ntiles + SUB - 1) / SUB;
  if constexpr (!CH && K <= 7) {
    if (L.plain) {
      if (L.carry.hdr)
        hipLaunchKernelGGL((stencil_plain_kernel<K, VT, TP, SUB, true>), dim3(unsigned(nsuper)), dim3(ST_THREADS), 0, st,
                           L.key, static_cast<const VT*>(L.val), L.topic, L.n, L.prog_dev, L.slots, L.tile_count,
                           ntiles, L.carry);
      else
        hipLaunchKernelGGL((stencil_plain_kernel<K, VT, TP, SUB, false>), dim3(unsigned(nsuper)), dim3(ST_THREADS), 0, st,
                           L.key, static_cast<const VT*>(L.val), L.topic, L.n, L.prog_dev, L.slots, L.tile_count,
                           ntiles, L.carry);
      return;
    }
  }
  if (L.carry.hdr)
    hipLaunchKernelGGL((stencil_kernel<K, VT, TP, CH, true, SUB>), dim3(unsigned(nsuper)), dim3(ST_THREADS), 0, st,
                       L.key, static_cast<const VT*>(L.val), L.topic, L.n, L.prog_dev, L.slots, L.tile_count, ntiles,
                       L.carry);
  else
    hipLaunchKernelGGL((stencil_kernel<K, VT, TP, CH, false, SUB>), dim3(unsigned(nsuper)), dim3(ST_THREADS), 0, st,
                       L.key, static_cast<const VT*>(L.val), L.topic, L.n, L.prog_dev, L.slots, L.tile_count, ntiles,
                       L.carry);
}

template <int K, class VT, bool TP, bool CH>
inline hipError_t launch_kt(const StencilLaunch& L, hipStream_t st) {
  const int64_t ntiles = (L.n + ST_TILE - 1) / ST_TILE;
  if (stencil_sub(ntiles) == ST_SUB) launch_kts<K, VT, TP, CH, ST_SUB>(L, ntiles, st);
  else launch_kts<K, VT, TP, CH, 1>(L, ntiles, st);
  return hipGetLastError();
}

template <int K, bool CH = false>
inline hipError_t launch_k(const StencilLaunch& L, hipStream_t st) {
  if (L.coltype == T_I32)
    return L.use_topic ? launch_kt<K, int32_t, true, CH>(L, st) : launch_kt<K, int32_t, false, CH>(L, st);
  if (L.coltype == T_I64)
    return L.use_topic ? launch_kt<K, int64_t, true, CH>(L, st) : launch_kt<K, int64_t, false, CH>(L, st);
  return L.use_topic ? launch_kt<K, double, true, CH>(L, st) : launch_kt<K, double, false, CH>(L, st);
}

}  // namespace kcep

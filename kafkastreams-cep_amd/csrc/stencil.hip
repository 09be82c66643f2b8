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
// match out.  One pass, ordered output:
//   * 256-thread workgroups, 4096 records per tile, tile ids drawn in launch
//     order from an atomic counter (so every predecessor tile is resident:
//     the look-back never waits on an unscheduled tile);
//   * coalesced 16-B loads of key/value (lane-contiguous), predicate bitmask
//     per record computed in registers, staged to LDS with a (k-1) halo;
//   * each thread then scans 16 consecutive records from LDS, block scan of
//     match counts, decoupled look-back over 8-byte {epoch, flag, count}
//     granules (agent-scope relaxed atomics, no fences: the granule is the
//     flag, MI355X_MICROARCH.md "R2"), matches staged in LDS and written as
//     one contiguous, coalesced run per tile.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "kcep_internal.h"

namespace kcep {

constexpr int ST_THREADS = 256;
constexpr int ST_EPT = 16;                        // records per thread
constexpr int ST_TILE = ST_THREADS * ST_EPT;      // 4096

// look-back granule: [63:48] epoch, [47:46] flag, [45:0] value
constexpr uint64_t LB_AGG = 1, LB_INC = 2;
__device__ __forceinline__ uint64_t lb_pack(uint32_t epoch, uint64_t flag, uint64_t v) {
  return (uint64_t(epoch) << 48) | (flag << 46) | (v & ((1ull << 46) - 1));
}

template <class VT>
__device__ __forceinline__ uint32_t stage_mask(const StencilProgram* __restrict__ P, int k, VT v, int32_t topic,
                                               bool use_topic) {
  uint32_t m = 0;
#pragma unroll
  for (int s = 0; s < STENCIL_MAX_K; s++) {
    if (s >= k) break;
    const int nt = P->nterms[s];
    bool any = false;
    for (int t = 0; t < nt; t++) {
      bool ok;
      if (!P->hasv[s][t]) ok = true;
      else if constexpr (std::is_same<VT, double>::value) ok = P->vf[s][t].lo <= double(v) && double(v) <= P->vf[s][t].hi;
      else ok = P->vi[s][t].lo <= int64_t(v) && int64_t(v) <= P->vi[s][t].hi;
      if (use_topic) ok = ok && P->tp[s][t].lo <= int64_t(topic) && int64_t(topic) <= P->tp[s][t].hi;
      any |= ok;
    }
    m |= uint32_t(any) << s;
  }
  return m;
}

// LDS image of the tile: record r of the tile sits at r' = r + 16 (the 8
// halo records before the tile at r' = 8..15); keys are padded by 4 words
// per 16 so that both the lane-striped int4 writes of phase 1 and the
// thread-blocked int4 reads of phase 2 are bank-conflict free.
__device__ __forceinline__ int kpos(int rp) { return rp + 4 * (rp >> 4); }
constexpr int ST_KWORDS = (ST_TILE + 16) + 4 * ((ST_TILE + 16) >> 4) + 16;

template <int K, class VT, bool TOPIC>
__global__ __launch_bounds__(ST_THREADS) void stencil_kernel(
    const int32_t* __restrict__ key, const VT* __restrict__ val, const int32_t* __restrict__ topic, int64_t n,
    const StencilProgram* __restrict__ P, int32_t* __restrict__ out, int64_t out_cap,
    uint64_t* __restrict__ status, uint32_t* __restrict__ tile_counter, int64_t* __restrict__ total_out,
    uint32_t epoch, int64_t ntiles) {
  __shared__ __attribute__((aligned(16))) int32_t s_key[ST_KWORDS];   // reused for the match list
  __shared__ __attribute__((aligned(16))) uint8_t s_mask[ST_TILE + 16];
  __shared__ int32_t s_wsum[ST_THREADS / 64];
  __shared__ int64_t s_prefix;
  __shared__ uint32_t s_tile;

  const int tid = threadIdx.x;
  if (tid == 0) s_tile = atomicAdd(tile_counter, 1u);
  __syncthreads();
  const int64_t tile = s_tile;
  const int64_t base = tile * ST_TILE;

  // ---- phase 1: coalesced lane-striped loads, predicate masks -> LDS ----
#pragma unroll
  for (int c = 0; c < ST_EPT / 4; c++) {
    const int local = c * (ST_THREADS * 4) + tid * 4;
    const int64_t g = base + local;
    int32_t kk[4];
    VT vv[4];
    int32_t tt[4] = {0, 0, 0, 0};
    if (g + 3 < n) {
      const int4 k4 = *reinterpret_cast<const int4*>(key + g);
      kk[0] = k4.x; kk[1] = k4.y; kk[2] = k4.z; kk[3] = k4.w;
      if constexpr (sizeof(VT) == 4) {
        const int4 v4 = *reinterpret_cast<const int4*>(val + g);
        vv[0] = __builtin_bit_cast(VT, v4.x); vv[1] = __builtin_bit_cast(VT, v4.y);
        vv[2] = __builtin_bit_cast(VT, v4.z); vv[3] = __builtin_bit_cast(VT, v4.w);
      } else {
        const longlong2 a = *reinterpret_cast<const longlong2*>(val + g);
        const longlong2 b = *reinterpret_cast<const longlong2*>(val + g + 2);
        vv[0] = __builtin_bit_cast(VT, a.x); vv[1] = __builtin_bit_cast(VT, a.y);
        vv[2] = __builtin_bit_cast(VT, b.x); vv[3] = __builtin_bit_cast(VT, b.y);
      }
      if constexpr (TOPIC) {
        const int4 t4 = *reinterpret_cast<const int4*>(topic + g);
        tt[0] = t4.x; tt[1] = t4.y; tt[2] = t4.z; tt[3] = t4.w;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const bool in = g + i < n;
        kk[i] = in ? key[g + i] : INT32_MIN;
        vv[i] = in ? val[g + i] : VT(0);
        if constexpr (TOPIC) tt[i] = in ? topic[g + i] : 0;
      }
    }
    uint32_t packed = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const bool in = g + i < n;
      const uint32_t m = in ? stage_mask<VT>(P, K, vv[i], tt[i], TOPIC) : 0u;
      packed |= m << (8 * i);
    }
    *reinterpret_cast<int4*>(&s_key[kpos(16 + local)]) = make_int4(kk[0], kk[1], kk[2], kk[3]);
    *reinterpret_cast<uint32_t*>(&s_mask[16 + local]) = packed;
  }
  if (tid < 16) {                               // halo: the 8 records before the tile (r' = 8..15)
    const int64_t g = base - 16 + tid;
    int32_t kk = INT32_MIN;
    uint32_t m = 0;
    if (tid >= 16 - (K - 1) && g >= 0) {
      kk = key[g];
      m = stage_mask<VT>(P, K, val[g], TOPIC ? topic[g] : 0, TOPIC);
    }
    s_key[kpos(tid)] = kk;
    s_mask[tid] = uint8_t(m);
  }
  __syncthreads();

  // ---- phase 2: 16 consecutive records per thread (+ 8 of history) ----
  const int lb = ST_EPT * tid + 8;
  int32_t wk[24];
  uint8_t wm[24];
#pragma unroll
  for (int q = 0; q < 6; q++) {
    const int4 k4 = *reinterpret_cast<const int4*>(&s_key[kpos(lb + 4 * q)]);
    wk[4 * q] = k4.x; wk[4 * q + 1] = k4.y; wk[4 * q + 2] = k4.z; wk[4 * q + 3] = k4.w;
  }
#pragma unroll
  for (int q = 0; q < 3; q++) {
    const uint64_t m8 = *reinterpret_cast<const uint64_t*>(&s_mask[lb + 8 * q]);
#pragma unroll
    for (int b = 0; b < 8; b++) wm[8 * q + b] = uint8_t(m8 >> (8 * b));
  }
  uint32_t hit = 0;
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
  const int cnt = __popc(hit);

  // ---- block exclusive scan of per-thread counts ----
  const int lane = tid & 63, wid = tid >> 6;
  int incl = cnt;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(incl, d, 64);
    if (lane >= d) incl += y;
  }
  if (lane == 63) s_wsum[wid] = incl;
  __syncthreads();                               // also: every thread has read s_key/s_mask
  int woff = 0, tile_total = 0;
#pragma unroll
  for (int w = 0; w < ST_THREADS / 64; w++) {
    const int x = s_wsum[w];
    woff += w < wid ? x : 0;
    tile_total += x;
  }
  const int excl = woff + incl - cnt;

  // ---- decoupled look-back (wave 0) ----
  if (wid == 0) {
    int64_t prefix = 0;
    if (tile == 0) {
      if (lane == 0) __hip_atomic_store(&status[0], lb_pack(epoch, LB_INC, uint64_t(tile_total)), __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT);
    } else {
      if (lane == 0) __hip_atomic_store(&status[tile], lb_pack(epoch, LB_AGG, uint64_t(tile_total)), __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT);
      int64_t idx = tile - 1;
      for (;;) {
        const int64_t p = idx - lane;
        uint64_t w = 0;
        uint32_t flag;
        for (;;) {
          if (p >= 0) w = __hip_atomic_load(&status[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          flag = p < 0 ? uint32_t(LB_INC) : ((w >> 48) == epoch ? uint32_t((w >> 46) & 3) : 0u);
          const uint64_t inc_mask = __ballot(flag == LB_INC);
          const uint64_t bad_mask = __ballot(flag == 0);
          // lanes nearer than the first inclusive predecessor must all be ready
          const uint64_t first_inc = inc_mask ? (inc_mask & (~inc_mask + 1)) : 0;
          const uint64_t need = first_inc ? (first_inc - 1) | first_inc : ~0ull;
          if ((bad_mask & need) == 0) break;
          __builtin_amdgcn_s_sleep(1);
        }
        const uint64_t inc_mask = __ballot(flag == LB_INC);
        const int stop = inc_mask ? __ffsll((unsigned long long)inc_mask) - 1 : 64;
        int64_t v = (p >= 0 && lane <= stop) ? int64_t(w & ((1ull << 46) - 1)) : 0;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
        prefix += v;
        if (inc_mask) break;
        idx -= 64;
      }
      if (lane == 0) __hip_atomic_store(&status[tile], lb_pack(epoch, LB_INC, uint64_t(prefix + tile_total)),
                                        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane == 0) {
      s_prefix = prefix;
      if (tile == ntiles - 1) {
        *total_out = prefix + tile_total;
        *tile_counter = 0;                        // every tile id has been drawn: reset for the next launch
      }
    }
  }

  // ---- stage the tile's matches (final record index) in LDS ----
  int32_t* s_match = s_key;                       // safe: the barrier above ordered all key reads
  {
    int o = excl;
    uint32_t h = hit;
    while (h) {
      const int i = __ffs(h) - 1;
      h &= h - 1;
      s_match[o++] = int32_t(base + tid * ST_EPT + i);   // record index < 2^31 (checked by the launcher)
    }
  }
  __syncthreads();
  const int64_t pre = s_prefix;
  // coalesced write-out: K ints per match, contiguous across the tile
  const int words = tile_total * K;
  for (int w = tid; w < words; w += ST_THREADS) {
    const int m = w / K, s = w - m * K;
    const int64_t gm = pre + m;
    if (gm < out_cap) out[gm * K + s] = s_match[m] - (K - 1) + s;
  }
}

// ---- launcher ------------------------------------------------------------
struct StencilLaunch {
  const int32_t* key;
  const void* val;
  const int32_t* topic;
  int64_t n;
  const StencilProgram* prog_dev;
  int k, coltype, use_topic;
  int32_t* out;
  int64_t out_cap;
  uint64_t* status;
  uint32_t* counter;
  int64_t* total;
  uint32_t epoch;
};

template <int K, class VT, bool TP>
static hipError_t launch_kt(const StencilLaunch& L, hipStream_t st) {
  const int64_t ntiles = (L.n + ST_TILE - 1) / ST_TILE;
  hipLaunchKernelGGL((stencil_kernel<K, VT, TP>), dim3(unsigned(ntiles)), dim3(ST_THREADS), 0, st, L.key,
                     static_cast<const VT*>(L.val), L.topic, L.n, L.prog_dev, L.out, L.out_cap, L.status, L.counter,
                     L.total, L.epoch, ntiles);
  return hipGetLastError();
}

template <int K>
static hipError_t launch_k(const StencilLaunch& L, hipStream_t st) {
  if (L.coltype == T_I32) return L.use_topic ? launch_kt<K, int32_t, true>(L, st) : launch_kt<K, int32_t, false>(L, st);
  if (L.coltype == T_I64) return L.use_topic ? launch_kt<K, int64_t, true>(L, st) : launch_kt<K, int64_t, false>(L, st);
  return L.use_topic ? launch_kt<K, double, true>(L, st) : launch_kt<K, double, false>(L, st);
}

int64_t stencil_tiles(int64_t n) { return (n + ST_TILE - 1) / ST_TILE; }

hipError_t stencil_launch(const StencilLaunch& L, hipStream_t st) {
  if (L.n <= 0) return hipMemsetAsync(L.total, 0, sizeof(int64_t), st);
  switch (L.k) {
    case 1: return launch_k<1>(L, st);
    case 2: return launch_k<2>(L, st);
    case 3: return launch_k<3>(L, st);
    case 4: return launch_k<4>(L, st);
    case 5: return launch_k<5>(L, st);
    case 6: return launch_k<6>(L, st);
    case 7: return launch_k<7>(L, st);
    case 8: return launch_k<8>(L, st);
  }
  return hipErrorInvalidValue;
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
    for (int s = k - 1; s >= 0; s--) h = mix64(h ^ (uint64_t(out[i * k + s]) << 8) ^ uint64_t(P->name[s]));
  }
  for (int d = 32; d >= 1; d >>= 1) h += __shfl_xor(h, d, 64);
  if ((threadIdx.x & 63) == 0 && h) atomicAdd(sum, (unsigned long long)h);
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

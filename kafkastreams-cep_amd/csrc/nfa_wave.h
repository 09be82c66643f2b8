// nfa_wave.h — the general NFA path with one key per wave and one queued run per lane.
//
// NFA.matchPattern (nfa/NFA.java:134-149) polls the key's run queue in order and evaluates
// each run (NFA.evaluate :190-341).  For a pattern without aggregates (no folds, no state reads,
// no SequenceMatcher -- DevProgram.wave_ok) an evaluation reads nothing another run of the same
// record writes: edge predicates depend on the record only, Dewey versions are immutable values,
// and the shared buffer is only written.  The runs of a record are therefore evaluated in rounds
// of 64, one per lane, and their side effects are committed afterwards in queue order:
//
//   * new runs: each lane's results go to a private list; a wave prefix scan gives every lane its
//     place in the next queue (and in the final-run list, matchConstruction :151-158), so the
//     queue order is the reference's;
//   * NFA.runs++ (:297, :331): placeholders, numbered in queue order by a prefix scan;
//   * buffer puts / branches (SharedVersionedBufferStoreImpl.java:101-157): logged per lane.  If no
//     run of the round died and none raised, they commute except for the predecessor order of the
//     current record's nodes: branch walks only touch earlier records' nodes (refs++, atomically;
//     their predecessor lists cannot change without a remove), and a node of the current record
//     ends as "the last 3-arg put, then every later 5-arg put, in queue order" -- a contiguous
//     block of predecessor entries placed by per-node prefix counts.  Otherwise (a dead run's
//     removePattern :160-163, or an exception) lane 0 replays the round's operations in queue
//     order with the sequential buffer code, stopping where the reference throws.
//   * matchConstruction after the last round: the final runs' buffer walks, 64 at a time, stepped
//     event by event (wave_emit_matches).
//
// The key's workspace is the lane kernel's (nfa_dev.h): nodes, queues and heap in the pool, with
// the heap allocated by an LDS atomic; a round that outgrows the heap is re-run after the wave has
// doubled it.
#pragma once
#include "nfa_dev.h"

namespace kcep {

constexpr int WAVE = 64;
// LDS per key-wave: WAVE_ARENA words of workspace + 64 x WAVE_PRIV words of private run lists and
// operation logs, sized together for 3 waves per SIMD.  C4 sweep (profiles/r04_c4_lds_sweep.log,
// ms per step): arena 2048 + lists in the pool 8.43; 1024 + 16 7.78; 1024 + 12 8.02; 1024 + 20 8.23;
// 1280 + 16 8.22; 768 + 16 9.75; 512 + 32 10.9; 4 waves per SIMD 11.2
#ifndef WAVE_ARENA
#define WAVE_ARENA 1024                    // LDS words per key workspace (KCEP_WAVE_ARENA A/B: 0 = pool only)
#endif
#ifndef WAVE_PRIV
#define WAVE_PRIV 16                       // LDS words per lane for its private run list + operation log
#endif                                     // (KCEP_WAVE_PRIV A/B; 0 = in the pool)
#ifndef GROUP_LANES
#define GROUP_LANES 16                     // lanes per key of the grouped kernel (4 keys per wave)
#endif
#ifndef GROUP_ARENA
#define GROUP_ARENA 1024                   // LDS words per key workspace of the grouped kernel (KCEP_GROUP_ARENA A/B)
#endif
#ifndef GROUP_RUNS
#define GROUP_RUNS 32                      // a key of the grouped kernel with more live runs moves to a whole wave
#endif

// The lanes of one key: GL consecutive lanes of the wave (GL = 64: the whole wave, one key per
// workgroup; GL = 16: four keys per wave).  Ballots, broadcasts and scans stay inside the group, so
// the keys of one wave never exchange anything; their lanes merely share the instruction stream,
// which is what a latency-bound key leaves idle.
template <int GL>
struct Grp {
  int gl;                                  // lane within the group
  int base;                                // the group's first lane in the wave
  __device__ __forceinline__ uint64_t ballot(bool x) const {
    const uint64_t b = __ballot(x);
    if constexpr (GL == 64) return b;
    else return (b >> base) & ((1ull << GL) - 1);
  }
  template <class T>
  __device__ __forceinline__ T bcast(T v, int src = 0) const { return __shfl(v, src, GL); }
  // exclusive prefix of v over the group's lanes, and the group total
  __device__ __forceinline__ int excl_scan(int v, int& total) const {
    int x = v;
    for (int d = 1; d < GL; d <<= 1) {
      const int y = __shfl_up(x, d, GL);
      if (gl >= d) x += y;
    }
    total = __shfl(x, GL - 1, GL);
    return x - v;
  }
  __device__ __forceinline__ int max_all(int v) const {
    for (int d = GL / 2; d > 0; d >>= 1) { const int o = __shfl_xor(v, d, GL); v = o > v ? o : v; }
    return v;
  }
};

// A hand-off between lanes of the wave (the workgroup is one wave): a wavefront performs its
// memory operations in program order, so only the compiler must not move them across it.  No
// s_barrier, which the grouped kernel could not take anyway: its keys leave loops at different
// times.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

#define KCEP_LDSM 0
#include "nfa_wave_body.h"
#undef KCEP_LDSM

}  // namespace kcep

// Whole-wave keys first in the LDS mode (KCEP_WAVE_LDSM=1).  Off by default: on C4 about half the keys
// outgrow the arena and pay for a wasted first attempt -- 8.95 vs 7.63 ms, and 9.7-10.5 ms with a
// 1536-3072-word arena (profiles/r04_c4_ldsm_ab.log)
#ifndef WAVE_LDSM
#define WAVE_LDSM 0
#endif

// the LDS-pointer mode of the engine (nfa_dev.h): a key whose workspace fits the arena runs on ds
// instructions; one that outgrows it is re-run in the generic mode above
namespace kcep {
#if WAVE_LDSM
namespace ldsm {
typedef lds_i32* kp_t;
typedef const lds_i32* kcp_t;
typedef i4v __attribute__((address_space(3)))* kp4_t;
typedef const i4v __attribute__((address_space(3)))* kcp4_t;
#define KCEP_LDSM 1
#define KCEP_NS kcep::ldsm
#include "nfa_dev_body.h"
#include "nfa_wave_body.h"
#undef KCEP_NS
#undef KCEP_LDSM
}  // namespace ldsm
#endif



// the key descriptor of either mode (one lives at a time)
template <int GL>
union WaveSharedU {
  WaveShared<GL> g;
#if WAVE_LDSM
  ldsm::WaveShared<GL> l;
#endif
};

// One whole-wave key: in the LDS mode while its workspace fits the arena, else (re-run from the
// batch start of the key: nothing of the first attempt was committed) in the generic mode
template <bool AGG>
__device__ __forceinline__ int wave_key_any(const NfaArgs& A, int seg, const Grp<WAVE>& gp, WaveSharedU<WAVE>& w,
                                            int32_t* s_arena, int arena_words, int32_t*& s_priv) {
#if WAVE_LDSM
  const int r = ldsm::wave_key<AGG, WAVE>(A, seg, gp, w.l, s_arena, arena_words, s_priv);
  if (r != 2) return r;
  wave_sync();
#endif
  return wave_key<AGG, WAVE>(A, seg, gp, w.g, s_arena, arena_words, s_priv);
}

// The key segments of a batch, GL lanes per key: workgroup b takes segments b * (64 / GL) ... (one
// per group).  GL < 64 (light keys): a key whose live runs outgrow its group is appended to the
// heavy list (A.heavy / A.heavy_n) for nfa_wave_heavy.
template <bool AGG, int GL>
__device__ __forceinline__ void nfa_wave_body(const NfaArgs& A) {
  constexpr int NG = WAVE / GL;
  constexpr int ARENA = (GL == WAVE ? WAVE_ARENA : GROUP_ARENA) & ~3;   // LDS words of each key's hot workspace
  __shared__ WaveSharedU<GL> ws[NG];
  // (+4 words: the LDS mode's arena and private slices never start at LDS offset 0, which an LDS pointer
  // test would take for null)
  __shared__ __attribute__((aligned(16))) int32_t s_arena[NG * ARENA + 8];
  __shared__ int32_t* s_priv[NG];
  const Grp<GL> gp{int(threadIdx.x) & (GL - 1), int(threadIdx.x) & ~(GL - 1)};
  const int grp = int(threadIdx.x) / GL;
  const int seg = int(blockIdx.x) * NG + grp;
  if (seg >= A.nseg) return;
#if WAVE_PRIV > 0
  __shared__ __attribute__((aligned(16))) int32_t s_priv_lds[WAVE * WAVE_PRIV + 4];
  if (gp.gl == 0) s_priv[grp] = s_priv_lds + 4 + gp.base * WAVE_PRIV;
#endif
  int r;
  if constexpr (GL == WAVE) r = wave_key_any<AGG>(A, seg, gp, ws[grp], s_arena + 4, ARENA, s_priv[grp]);
  else r = wave_key<AGG, GL>(A, seg, gp, ws[grp].g, s_arena + grp * ARENA, ARENA, s_priv[grp]);
  if (r == 0 && gp.gl == 0) A.heavy[atomicAdd(A.heavy_n, 1)] = seg;
}

// The heavy list of a grouped launch, one key per workgroup-wave (persistent over the list).
template <bool AGG>
__device__ __forceinline__ void nfa_wave_heavy(const NfaArgs& A) {
  __shared__ WaveSharedU<WAVE> w;
  __shared__ __attribute__((aligned(16))) int32_t s_arena[WAVE_ARENA];
  __shared__ int32_t* s_priv;
#if WAVE_PRIV > 0
  __shared__ __attribute__((aligned(16))) int32_t s_priv_lds[WAVE * WAVE_PRIV];
  s_priv = s_priv_lds;
#endif
  const Grp<WAVE> gp{int(threadIdx.x), 0};
  const int nh = *A.heavy_n;
  for (int i = blockIdx.x; i < nh; i += gridDim.x) {
    wave_key<AGG, WAVE>(A, A.heavy[i], gp, w.g, s_arena, WAVE_ARENA, s_priv);   // (generic: keys that grew)
    wave_sync();
  }
}

}  // namespace kcep

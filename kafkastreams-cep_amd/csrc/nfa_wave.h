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
// The key's workspace is the lane kernel's (nfa_dev.h): nodes, queues and heap in the key's LDS arena
// while they fit, then in the wave's recycled scratch region, then in the batch pool, with the heap
// allocated by an LDS atomic; a round that outgrows the heap is re-run after the wave has doubled it.
// The grid is persistent: each workgroup (one wave) takes key segments from a counter until none is
// left, and hands its scratch region to every key it takes (nfa_dev.h KeyAlloc).
#pragma once
#include "nfa_dev.h"

namespace kcep {

constexpr int WAVE = 64;
// LDS per key-wave: WAVE_ARENA words of workspace + 64 x WAVE_PRIV words of private run lists and
// operation logs, sized together for 3 waves per SIMD.  C4 sweep (profiles/r04_c4_lds_sweep.log,
// ms per step): arena 2048 + lists in the pool 8.43; 1024 + 16 7.78; 1024 + 12 8.02; 1024 + 20 8.23;
// 1280 + 16 8.22; 768 + 16 9.75; 512 + 32 10.9; 4 waves per SIMD 11.2
#ifndef WAVE_ARENA
#define WAVE_ARENA 1664                    // LDS words per key workspace (jit.cpp: the sizes measured)
#endif
#ifndef WAVE_PRIV
#define WAVE_PRIV 16                       // LDS words per lane for its private run list + operation log
#endif

// The lanes of one key: GL consecutive lanes of the wave (GL = 64: the whole wave, one key per
// workgroup).  Ballots, broadcasts and scans stay inside the group.  (A grouped build -- four keys per
// wave, 16 lanes each, outgrown keys re-run on whole waves -- was measured slower in rounds 3 and 4,
// DESIGN.md 4.4, and removed; the helpers keep the group width as a parameter.)
template <int GL>
struct Grp {
  static_assert(GL == 64, "the wave kernel runs one key per wave");
  int gl;                                  // lane within the group
  int base;                                // the group's first lane in the wave
  __device__ __forceinline__ uint64_t ballot(bool x) const { return __ballot(x); }
  // lane src's value in every lane (v_readlane: a scalar result, no LDS round trip; src is uniform)
  template <class T>
  __device__ __forceinline__ T bcast(T v, int src = 0) const {
    static_assert(sizeof(T) == 4 || sizeof(T) == 8, "bcast: 4- or 8-byte values");
    if constexpr (sizeof(T) == 4) {
      return __builtin_bit_cast(T, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), src));
    } else {
      const uint64_t u = __builtin_bit_cast(uint64_t, v);
      const uint32_t lo = __builtin_amdgcn_readlane(int(uint32_t(u)), src);
      const uint32_t hi = __builtin_amdgcn_readlane(int(uint32_t(u >> 32)), src);
      return __builtin_bit_cast(T, uint64_t(lo) | (uint64_t(hi) << 32));
    }
  }
  // exclusive prefix of v over the wave, and the total: DPP row shifts and row broadcasts (VALU
  // lane moves, rocPRIM's warp_scan_dpp pattern) instead of six LDS-crossbar permutes.  Every lane of
  // the wave must be active (the callers are wave-uniform points); a shifted-in lane outside the row
  // reads 0 (update_dpp's old value)
  __device__ __forceinline__ int excl_scan(int v, int& total) const {
    int x = v;
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);   // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);   // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);   // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);   // row_shr:8
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);   // row_bcast:15 into rows 1, 3
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);   // row_bcast:31 into rows 2, 3
    total = __builtin_amdgcn_readlane(x, 63);
    return x - v;
  }
  __device__ __forceinline__ int max_all(int v) const {
    for (int d = GL / 2; d > 0; d >>= 1) { const int o = __shfl_xor(v, d, GL); v = o > v ? o : v; }
    return v;
  }
};

// A hand-off between lanes of the wave (the workgroup is one wave): a wavefront performs its
// memory operations in program order, so only the compiler must not move them across it.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// the key's shared workspace descriptor (LDS); lanes keep register copies in their Lane
template <int GL>
struct WaveShared {
  int32_t *nodes, *heap, *qa, *qb, *fq, *out, *hwm, *aggs;
  int32_t heapcap, heap_top, qa_cap, qb_cap, fq_cap, qlen, outcap, out_top, nhwm, runs, seqcap;
  int32_t* oent;                   // the match entries (headers in out)
  int32_t ecap, etop;
  int64_t nmatch;
  KeyAlloc ka;                     // the key's allocator: its words, the wave's scratch region
  int32_t err, overflow, cap_hit;
  int32_t* grown;                  // a shared array lane 0 re-allocated (pool), for the copy ...
  int64_t grown_n;                 // ... and its capacity
  int32_t *arena, arena_used, arena_cap;   // the key's LDS arena, its bump pointer (re-allocations go there first), size
  // scratch of one phase of a record at a time (the phases never overlap): ~2.3 KB less LDS per wave
  union {
    struct { int32_t* logp[GL]; int32_t logn[GL], errc[GL]; } sq;   // the sequential commit's operation logs
    struct { int32_t lastp3[NFA_MAX_SLOTS], scnt[NFA_MAX_SLOTS], sblk[NFA_MAX_SLOTS]; } pc;   // parallel commit
    // matchConstruction: the walks waiting at a node the walks change (wave_emit_matches)
    struct { int32_t slot[GL], e[GL], pv[GL], cnt[GL], done[GL], err[GL]; } ms;
    int32_t conf[2 * GL];          // stateful rounds: each lane's run sequence, whether it wrote it
  } u;
};

template <class W>
__device__ __forceinline__ void ws_to_lane(Lane& l, const W& w) {
  l.nodes = w.nodes; l.heap = w.heap; l.qa = w.qa; l.qb = w.qb; l.fq = w.fq; l.out = w.out; l.hwm = w.hwm;
  l.aggs = w.aggs; l.seqcap = w.seqcap;
  l.heapcap = w.heapcap; l.heap_top = w.heap_top; l.qa_cap = w.qa_cap; l.qb_cap = w.qb_cap; l.fq_cap = w.fq_cap;
  l.qlen = w.qlen; l.outcap = w.outcap; l.out_top = w.out_top; l.nhwm = w.nhwm; l.runs = w.runs;
  l.oent = w.oent; l.ecap = w.ecap; l.etop = w.etop;
  l.nmatch = w.nmatch; l.err = w.err; l.overflow = w.overflow; l.cap_hit = w.cap_hit;
}
template <class W>
__device__ __forceinline__ void lane_to_ws(W& w, const Lane& l) {
  w.nodes = l.nodes; w.heap = l.heap; w.qa = l.qa; w.qb = l.qb; w.fq = l.fq; w.out = l.out; w.hwm = l.hwm;
  w.aggs = l.aggs; w.seqcap = l.seqcap;
  w.heapcap = l.heapcap; w.heap_top = l.heap_top; w.qa_cap = l.qa_cap; w.qb_cap = l.qb_cap; w.fq_cap = l.fq_cap;
  w.qlen = l.qlen; w.outcap = l.outcap; w.out_top = l.out_top; w.nhwm = l.nhwm; w.runs = l.runs;
  w.oent = l.oent; w.ecap = l.ecap; w.etop = l.etop;
  w.nmatch = l.nmatch; w.err = l.err; w.overflow = l.overflow; w.cap_hit = l.cap_hit;
}

// A shared array of `cap` words (used up to `used`) re-allocated at >= need words: lane 0 draws it
// from the pool, the group copies.  Returns the new array (nullptr: pool exhausted -> w.overflow).
// lds_ok: the array may move into the key's LDS arena (not the match output, read after the kernel)
template <int GL>
__device__ __forceinline__ int32_t* wave_regrow(Lane& l, WaveShared<GL>& w, int32_t* a, int32_t& cap, int64_t used,
                                                int64_t need, const Grp<GL>& g, int kind, bool lds_ok = true) {
  int64_t nc = int64_t(cap) * 2;
  if (nc < need) nc = need;
  wave_sync();
  if (g.gl == 0) {
    if (lds_ok && w.arena_used + nc <= w.arena_cap) {   // room left in the LDS arena
      w.grown = w.arena + w.arena_used;
      w.arena_used += int32_t((nc + 3) & ~int64_t(3));
    } else {
      // past the arena: 16x while the wave's scratch region has room for it (words never touched cost
      // no traffic, and every regrow copies the array: fewer copies, fewer bytes), else 2x.  C4 HBM
      // bytes per launch at 2x / 4x / 8x / 16x: 232 / 210 / 176 / 171 MB (profiles/r05_c4_arena.txt)
      const int64_t n4 = int64_t(cap) * 16 > need ? int64_t(cap) * 16 : need;
      w.grown = nullptr;
      // Not under a per-key cap (cep_opts.max_key_words counts reserved words: the headroom would hand
      // keys back early -- C4's capped hand-off leg: 832 keys at 16x against 126 at 2x)
      if (lds_ok && w.ka.scr && int64_t(w.ka.scr_top) + ((n4 + 3) & ~int64_t(3)) <= w.ka.scr_cap &&
          n4 <= (int64_t(1) << 30) && l.A->max_key_words <= 0) {
        w.grown = pool_alloc(l, n4, kind);
        if (w.grown) nc = n4;
      }
      if (!w.grown) w.grown = nc > (int64_t(1) << 30) ? nullptr : pool_alloc(l, nc, kind, !lds_ok);
    }
    w.grown_n = nc;
    if (!w.grown) { w.overflow = 1; w.cap_hit |= l.cap_hit; }
  }
  wave_sync();
  int32_t* na = w.grown;
  if (!na) return nullptr;
  nc = w.grown_n;
  for (int64_t i = g.gl; i < used; i += GL) na[i] = a[i];
  cap = int32_t(nc);
  wave_sync();
  return na;
}

template <int GL>
__device__ __forceinline__ bool wave_heap_reserve(Lane& l, WaveShared<GL>& w, int64_t need_top, const Grp<GL>& g) {
  if (need_top <= w.heapcap) return true;
  int32_t cap = w.heapcap;
  int32_t* na = wave_regrow(l, w, w.heap, cap, w.heap_top, need_top, g, AK_HEAP);
  if (!na) return false;
  if (g.gl == 0) { w.heap = na; w.heapcap = cap; }
  wave_sync();
  return true;
}

// the round's buffer operations, none of which can see another's effect (see the header): branch
// walks with atomic refcounts and the existence checks, then the current record's nodes.  Returns
// the reference exception of the first failing operation in queue order (CEP_OK if none).
template <int GL>
__device__ __forceinline__ int wave_commit_parallel(Lane& l, WaveShared<GL>& w, const Grp<GL>& g, int r) {
  const auto& P = KCEP_PROG(l);
  const int ns = P.nslots;
  // (1) existence of every 5-arg put's predecessor node; branch walks (refs++)
  int my_err = 0;
  for (int k = 0; k < l.log_n && !my_err; k++) {
    const int32_t* o = l.log + k * WL;
    const int kind = o[0] & 0xFF, sid = (o[0] >> 8) & 0xFF;
    if (kind == WOP_PUT5) {
      const int psid = (o[0] >> 16) & 0xFF;
      if (!exists(node(l, slot_of(l, psid), o[2]))) my_err = CEP_E_ILLEGAL_STATE;
    } else if (kind == WOP_BRANCH) {                        // branch (:132-142)
      int slot = slot_of(l, sid), e = o[1], pv = o[3];
      for (;;) {
        int32_t* nd = node(l, slot, e);
        if (!exists(nd)) { my_err = CEP_E_NPE; break; }
        atomicAdd(nd, 1);
        const int p = first_compatible(l, nd, pv, nullptr);
        if (p < 0 || l.heap[p + 1] < 0) break;
        pv = l.heap[p]; slot = l.heap[p + 1]; e = l.heap[p + 2];
      }
    }
  }
  const uint64_t em = g.ballot(my_err != 0);
  if (em) return g.bcast(my_err, __builtin_ctzll(em));
  // (2) the current record's nodes: the last 3-arg put of a node overwrites, later 5-arg puts append
  int before = 0, total = 0;
  before = g.excl_scan(l.log_n, total);
  for (int s = g.gl; s < ns; s += GL) { w.u.pc.lastp3[s] = -1; w.u.pc.scnt[s] = 0; }
  wave_sync();
  for (int k = 0; k < l.log_n; k++) {
    const int32_t* o = l.log + k * WL;
    if ((o[0] & 0xFF) == WOP_PUT3) atomicMax(&w.u.pc.lastp3[slot_of(l, (o[0] >> 8) & 0xFF)], before + k);
  }
  wave_sync();
  auto survives = [&](const int32_t* o, int gi) {
    const int kind = o[0] & 0xFF;
    if (kind == WOP_BRANCH || kind == WOP_AGG) return false;
    const int lp = w.u.pc.lastp3[slot_of(l, (o[0] >> 8) & 0xFF)];
    return kind == WOP_PUT3 ? gi == lp : gi > lp;
  };
  int npred = 0;
  for (int k = 0; k < l.log_n; k++) {
    const int32_t* o = l.log + k * WL;
    if (survives(o, before + k)) { atomicAdd(&w.u.pc.scnt[slot_of(l, (o[0] >> 8) & 0xFF)], 1); npred++; }
  }
  int all = 0;
  g.excl_scan(npred, all);
  wave_sync();
  if (!wave_heap_reserve(l, w, int64_t(w.heap_top) + int64_t(PW) * all, g)) return CEP_OK;   // w.overflow
  if (g.gl == 0) {
    int top = w.heap_top;
    for (int s = 0; s < ns; s++)
      if (w.u.pc.scnt[s]) { w.u.pc.sblk[s] = top; top += PW * w.u.pc.scnt[s]; }
    w.heap_top = top;
  }
  wave_sync();
  l.heap = w.heap;
  l.heapcap = w.heapcap;
  for (int s = 0; s < ns; s++) {                             // uniform loop over the record's slots
    const int cnt = w.u.pc.scnt[s];
    if (!cnt) continue;
    int mine = 0;
    for (int k = 0; k < l.log_n; k++) {
      const int32_t* o = l.log + k * WL;
      if (survives(o, before + k) && slot_of(l, (o[0] >> 8) & 0xFF) == s) mine++;
    }
    int tot = 0;
    const int ex = g.excl_scan(mine, tot);
    int j = 0;
    for (int k = 0; k < l.log_n; k++) {
      const int32_t* o = l.log + k * WL;
      if (!survives(o, before + k) || slot_of(l, (o[0] >> 8) & 0xFF) != s) continue;
      const int idx = ex + j++;
      const int p = w.u.pc.sblk[s] + PW * idx;
      const int ver = o[3];
      const bool p3 = (o[0] & 0xFF) == WOP_PUT3;
      l.heap[p] = ver;                                       // MatchedEvent.addPredecessor
      l.heap[p + 1] = p3 ? -1 : slot_of(l, (o[0] >> 16) & 0xFF);
      l.heap[p + 2] = p3 ? 0 : o[2];
      l.heap[p + 3] = idx + 1 < cnt ? p + PW : -1;
      l.heap[p + 4] = l.heap[ver];
      l.heap[p + 5] = l.heap[ver + 1];
    }
    if (g.gl == 0) {
      int32_t* nd = node(l, s, r);
      const int last = w.u.pc.sblk[s] + PW * (cnt - 1);
      if (w.u.pc.lastp3[s] >= 0 || !exists(nd)) {                 // overwritten by a 3-arg put, or created: refs 1
        nd[0] = 1; nd[1] = w.u.pc.sblk[s]; nd[2] = last; nd[3] = NF_EXISTS;
      } else {                                               // made by an earlier round: appended to
        if (nd[1] < 0) nd[1] = w.u.pc.sblk[s];
        else l.heap[nd[2] + 3] = w.u.pc.sblk[s];
        nd[2] = last;
      }
    }
  }
  return CEP_OK;
}

// matchConstruction (NFA.java:151-158) of the record's final runs, 64 walks at a time in final-run
// order.  A walk (SharedVersionedBufferStoreImpl.remove -> peek :176-201) persists a change only at
// a node whose refs are <= 1 (the decrement of a copy is written back only at 0, Q4); nodes with
// refs >= 2 stay so for the whole construction and are read-only.  Walks step to strictly earlier
// events, so the walks are advanced event by event from the latest one (the frontier): at a
// read-only node each lane picks its predecessor in parallel; the walks standing at a changing node
// are stepped by lane 0 in final-run order -- every walk that will ever reach that node is there,
// since none is left above the frontier.  The result is the sequential construction's.
template <int GL>
__device__ __forceinline__ bool wave_emit_matches(Lane& l, WaveShared<GL>& w, const Grp<GL>& g, int flen) {
  const int lane = g.gl;
  const int64_t pos = a_pos(*l.A, l.g);
  const int maxp = l.nev + 1;                                  // one node per event at most
  for (int base = 0; base < flen; base += GL) {
    const int nact = flen - base < GL ? flen - base : GL;
    const bool act = lane < nact;
    if (!wave_heap_reserve(l, w, int64_t(w.heap_top) + int64_t(GL) * 2 * maxp, g)) return false;
    l.heap = w.heap;
    l.heapcap = w.heapcap;
    int32_t* paths = w.heap + w.heap_top;                      // scratch above the heap top
    int32_t* path = paths + lane * 2 * maxp;
    int slot = 0, e = -1, pv = 0, cnt = 0, my_err = 0;
    bool done = !act;
    if (act) {
      const int4 y = reinterpret_cast<const int4*>(w.fq)[base + lane];
      slot = slot_of(l, y.x & 0xFF); e = y.z; pv = y.y;
      if (e < 0) my_err = CEP_E_NPE;
    }
    for (;;) {
      const bool live = !done && !my_err;
      const int fr = g.max_all(live ? e : -1);
      if (fr < 0) break;
      const bool at = live && e == fr;
      bool mut = false;
      if (at) {
        int32_t* nd = node(l, slot, e);
        if (!exists(nd)) my_err = CEP_E_NPE;
        else mut = nd[0] <= 1;
        if (!my_err && !mut) {                                 // read-only node: a parallel step
          path[2 * cnt] = slot; path[2 * cnt + 1] = e; cnt++;
          const int p = first_compatible(l, nd, pv, nullptr);
          if (p < 0 || l.heap[p + 1] < 0) done = true;
          else { pv = l.heap[p]; slot = l.heap[p + 1]; e = l.heap[p + 2]; }
        }
      }
      const uint64_t mm = g.ballot(at && !my_err && mut);
      if (mm) {                                                // changing nodes: lane 0, in walk order
        w.u.ms.slot[lane] = slot; w.u.ms.e[lane] = e; w.u.ms.pv[lane] = pv; w.u.ms.cnt[lane] = cnt; w.u.ms.done[lane] = done;
        w.u.ms.err[lane] = my_err;
        wave_sync();
        if (lane == 0) {
          for (uint64_t m = mm; m; m &= m - 1) {
            const int j = __builtin_ctzll(m);
            const int sj = w.u.ms.slot[j], ej = w.u.ms.e[j], c = w.u.ms.cnt[j];
            int32_t* nd = node(l, sj, ej);
            if (!exists(nd)) { w.u.ms.err[j] = CEP_E_NPE; continue; }
            int32_t* pj = paths + j * 2 * maxp;
            pj[2 * c] = sj; pj[2 * c + 1] = ej;
            w.u.ms.cnt[j] = c + 1;
            const bool single = nd[1] < 0 || l.heap[nd[1] + 3] < 0;
            int pp = -1;
            const int p = first_compatible(l, nd, w.u.ms.pv[j], &pp);
            if (p >= 0) {                                      // refs_left == 0: removePredecessor + put
              nd[0] = 0;
              const int nx = l.heap[p + 3];
              if (pp < 0) nd[1] = nx; else l.heap[pp + 3] = nx;
              if (nd[2] == p) nd[2] = pp;
              nd[3] |= NF_EXISTS;
            } else if (single) {
              nd[3] &= ~NF_EXISTS;                             // delete
            }
            if (p < 0 || l.heap[p + 1] < 0) w.u.ms.done[j] = 1;
            else { w.u.ms.pv[j] = l.heap[p]; w.u.ms.slot[j] = l.heap[p + 1]; w.u.ms.e[j] = l.heap[p + 2]; }
          }
        }
        wave_sync();
        if ((mm >> lane) & 1) {
          slot = w.u.ms.slot[lane]; e = w.u.ms.e[lane]; pv = w.u.ms.pv[lane]; cnt = w.u.ms.cnt[lane];
          done = w.u.ms.done[lane]; my_err = w.u.ms.err[lane];
        }
      }
    }
    const uint64_t em = g.ballot(my_err != 0);
    if (em) {                                                  // the reference throws at the first failing walk
      const int code = g.bcast(my_err, __builtin_ctzll(em));
      if (lane == 0) w.err = code;
      wave_sync();
      return true;
    }
    // the matches, in final-run order: a header per match {pos lo, pos hi, entries, first entry} (lane i's
    // is the i-th), then the entries {name, pos lo, pos hi} of all of them, contiguous
    int total = 0;
    const int off = g.excl_scan(act ? cnt : 0, total);
    if (w.out_top + 4 * nact > w.outcap) {
      int32_t cap = w.outcap;
      int32_t* na = wave_regrow(l, w, w.out, cap, w.out_top, int64_t(w.out_top) + 4 * nact, g, AK_OUT, false);
      if (!na) return false;
      if (lane == 0) { w.out = na; w.outcap = cap; }
      wave_sync();
    }
    if (3 * (w.etop + total) > w.ecap) {
      int32_t cap = w.ecap;
      int32_t* na = wave_regrow(l, w, w.oent, cap, int64_t(3) * w.etop, int64_t(3) * (w.etop + total), g, AK_OUT, false);
      if (!na) return false;
      if (lane == 0) { w.oent = na; w.ecap = cap; }
      wave_sync();
    }
    if (act) {
      const int first = w.etop + off;
      const int4 h = make_int4(int32_t(uint32_t(uint64_t(pos))), int32_t(uint32_t(uint64_t(pos) >> 32)), cnt, first);
      *reinterpret_cast<int4*>(w.out + w.out_top + 4 * lane) = h;
      int32_t* en = w.oent + int64_t(3) * first;
      for (int i = 0; i < cnt; i++) {
        const int64_t q = ev_pos(l, path[2 * i + 1]);
        en[3 * i] = SLOT_NAME(l, path[2 * i]);
        en[3 * i + 1] = int32_t(uint32_t(uint64_t(q)));
        en[3 * i + 2] = int32_t(uint32_t(uint64_t(q) >> 32));
      }
    }
    wave_sync();
    if (lane == 0) { w.out_top += 4 * nact; w.etop += total; w.nmatch += nact; }
    wave_sync();
  }
  return true;
}

// Stateful patterns: the round's aggregate writes (WOP_AGG log entries; wave_agg bit 0) in queue
// order.  Without a conflict (wave_round_conflict) no two lanes write one (sequence, state) -- a lane
// writes its own run's sequence and sequences it created -- so every lane applies its own entries,
// placeholders numbered as the run words are (rb).  The table first grows to the largest sequence.
template <int GL>
__device__ __forceinline__ bool wave_apply_aggs(Lane& l, WaveShared<GL>& w, const Grp<GL>& g, int rb) {
  const int ns = KCEP_PROG(l).nstates;
  auto real = [&](int sq) { return sq < -1 ? rb + (-sq - 2) + 1 : sq; };
  int need = -1;
  for (int k = 0; k < l.log_n; k++) {
    const int32_t* o = l.log + k * WL;
    if ((o[0] & 0xFF) == WOP_AGG) { const int sq = real(o[1]); need = sq > need ? sq : need; }
  }
  need = g.max_all(need);
  if (need < 0) return true;
  if (need >= w.seqcap) {
    int32_t capw = w.seqcap * ns * 3;
    const int64_t used = int64_t(capw);
    int32_t* na = wave_regrow(l, w, w.aggs, capw, used, (int64_t(need) + 1) * ns * 3, g, AK_AGG);
    if (!na) return false;
    for (int64_t i = used + g.gl; i < capw; i += GL) na[i] = 0;       // the new rows: every state null
    wave_sync();
    if (g.gl == 0) { w.aggs = na; w.seqcap = capw / (ns * 3); }
    wave_sync();
  }
  l.aggs = w.aggs;
  l.seqcap = w.seqcap;
  for (int k = 0; k < l.log_n; k++) {
    const int32_t* o = l.log + k * WL;
    if ((o[0] & 0xFF) != WOP_AGG) continue;
    int32_t* e = l.aggs + (int64_t(real(o[1])) * ns + ((o[0] >> 8) & 0xFF)) * 3;
    e[0] = (o[0] >> 16) & 0xFF; e[1] = o[2]; e[2] = o[3];
  }
  wave_sync();
  return true;
}

// A round whose parallel evaluation may differ from the reference's queue-order one: two runs of the
// round share a run sequence (AggregatesStore rows are per sequence, AggregatesStoreImpl.java:55-75)
// and one of them wrote it -- the later run would have read the earlier one's fold (NFA.java:319-321,
// 362-369) -- or, with SequenceMatchers, a run died before others read partial sequences (its
// removePattern, NFA.java:142-143, changes the buffer they walk).
// conf: 2 x GL words of LDS (each lane's run sequence, whether it wrote it)
template <int GL>
__device__ __forceinline__ bool wave_round_conflict(const Lane& l, int32_t* conf, const Grp<GL>& g, bool act, int seq,
                                                    uint64_t dmask) {
  if ((l.A->wave_agg & 2) && dmask) return true;
  if (!(l.A->wave_agg & 1)) return false;
  const int lane = g.gl;
  conf[lane] = act ? seq : INT32_MIN;
  conf[GL + lane] = act && l.ov_own;
  wave_sync();
  bool c = false;
  for (int j = 0; j < lane && act; j++) c = c || (conf[j] == seq && (conf[GL + j] || l.ov_own));
  wave_sync();
  return g.ballot(c) != 0;
}

// profiling kernels (KCEP_PHASES): lane 0's clocks per phase of the record loop -- record setup,
// evaluation rounds, buffer commit, run numbering + queue placement, matchConstruction
#ifdef KCEP_PHASES
#define KWP_MARK(t) const uint64_t t = clock64()
#define KWP_ADD(i, t) do { if (lane == 0) w.ka.ph[i] += clock64() - t; } while (0)
#else
#define KWP_MARK(t)
#define KWP_ADD(i, t)
#endif

// AGG: the pattern reads or writes aggregates / reads partial sequences (DevProgram, abi.cpp
// wave_stateful): the round machinery for them (conflict checks, the sequential re-evaluation,
// applying the logged aggregate writes) is compiled in only then.
// One key (segment `seg`) on the GL lanes of group gp (w, s_arena, s_priv: the group's LDS; scr: the
// wave's scratch region of A.scratch_words words, or nullptr).
template <bool AGG, int GL>
__device__ __forceinline__ void wave_key(const NfaArgs& A, int seg, const Grp<GL>& gp, WaveShared<GL>& w,
                                         int32_t* s_arena, int arena_words, int32_t* s_priv, int32_t* scr) {
  const int lane = gp.gl;
  Lane l;
  int ok = 1;
  if (lane == 0) {
    w.ka.pool_words = 0;
    w.ka.scr_top = 0;
    w.ka.scr = scr;
    w.ka.scr_cap = scr ? A.scratch_words : 0;
#ifdef KCEP_PHASES
    for (int i = 0; i <= AK_N; i++) w.ka.kw[i] = 0;
#endif
    ok = key_begin(l, A, seg, s_arena, arena_words, &w.ka) ? 1 : 0;
    if (ok) {
      lane_to_ws(w, l);
      w.arena = s_arena;
      w.arena_cap = arena_words;
      w.arena_used = l.arena_used >= 0 ? (l.arena_used + 3) & ~3 : arena_words;
    }
  }
  ok = gp.bcast(ok);
  if (!ok) return;
  wave_sync();
  if (lane != 0) {
    l.A = &A; l.P = A.P;
    l.seg0 = A.seg_start[seg];
    l.L = int32_t(A.seg_start[seg + 1] - l.seg0);
    l.cap_hit = 0;
  }
  l.wpool = &w.ka;
  // every lane: the key's fixed shape (lane 0's key_begin set it), as wave-uniform values
  l.seg0 = gp.bcast(l.seg0);
  l.L = gp.bcast(l.L);
  l.C = gp.bcast(l.C);
  l.nev = gp.bcast(l.nev);
  l.evw = gp.bcast(l.evw);
  l.cev = reinterpret_cast<const int32_t*>(gp.bcast(reinterpret_cast<uintptr_t>(l.cev)));
  l.tq = reinterpret_cast<int32_t*>(gp.bcast(reinterpret_cast<uintptr_t>(l.tq)));
  l.tq_cap = gp.bcast(l.tq_cap);
  l.runs_delta = gp.bcast(l.runs_delta);
  l.pool_words = 0;
  l.rec_etop = 0; l.rec_nmatch = 0;
  l.slm = 0; l.sle = 0; l.flen = 0; l.tlen = 0;
  ws_to_lane(l, w);
  // private run lists and operation logs: written by every evaluation and read back by the commit
  // and the queue placement.  A slice of LDS per lane (WAVE_PRIV words: 2 runs + 2 log entries, growing
  // into the scratch region on demand).  Next to the full 2048-word arena it cost occupancy (C4 9.39 vs
  // 8.34 ms, profiles/r03_ab_s5.jsonl); with the arena halved it is the faster build (7.78 vs 8.43 ms, r04)
  const int q0 = 2;
  constexpr int priv_stride = WAVE_PRIV, log0 = (WAVE_PRIV - 4 * q0) / WL;
  static_assert(WAVE_PRIV % 4 == 0 && log0 >= 1, "WAVE_PRIV: room for the run list and one log entry");
  wave_sync();
  const auto& P = KCEP_PROG(l);
  const int ns = P.nslots;
  Frame fr[MAXD];
  int64_t err_rec = -1;
  const bool proc = A.mode == CEP_MODE_PROCESSOR;
#ifdef KCEP_PHASES
  if (lane == 0)
    for (int i = 0; i < 11; i++) w.ka.ph[i] = 0;
#endif
  int32_t live_max = w.qlen;
  int64_t evals = 0;
  const uint64_t t0 = A.profile ? wall_clock64() : 0;
  if (!w.overflow) {
    int32_t* pv = s_priv + int64_t(lane) * priv_stride;
    l.tq = pv;
    l.tq_cap = q0;
    l.log = pv + 4 * q0;
    l.log_cap = log0;
  }
  l.wtop = &w.heap_top;
  for (int i = 0; i < l.L && !w.err && !w.overflow; i++) {
    const int r = l.C + i;
    const int64_t g = l.seg0 + i;
    l.r = r;
    l.g = g;
    KWP_MARK(t_rec);
    ws_to_lane(l, w);
    for (int x = lane; x < ns * NW; x += GL) {                   // the record's buffer nodes: none yet
      const int k = x & (NW - 1);
      l.nodes[(int64_t(r) * ns) * NW + x] = (k == 1 || k == 2) ? -1 : 0;
    }
    KWP_ADD(0, t_rec);
    KWP_MARK(t_adm);
    if (proc) {
      if (!record_admitted(l, g)) { wave_sync(); continue; }
      for (int k = lane; k < w.qlen; k += GL) l.qa[4 * k] &= ~(1 << 17);   // isIgnored not serialised (Q3)
    }
    wave_sync();
    KWP_ADD(5, t_adm);
    KWP_MARK(t_eo);
    eval_event_only(l);
    const int n = w.qlen;
    evals += n;
    if (lane == 0) { l.rec_etop = w.etop; l.rec_nmatch = w.nmatch; }
    int qn = 0, flen = 0;
    KWP_ADD(6, t_eo);
    for (int base = 0; base < n && !w.err && !w.overflow; base += GL) {
      KWP_MARK(t_rp);
      const int my = base + lane;
      const bool act = my < n;
      Run run{0, 0, 0, 0};
      if (act) {
        const int4 x = reinterpret_cast<const int4*>(l.qa)[my];
        run = Run{x.x, x.y, x.z, x.w};
      }
      const int top0 = w.heap_top;
      const int nact = n - base < GL ? n - base : GL;
      bool good = true, seqd = false;
      int jj = 0;                                              // sequential mode: the lane evaluating
      uint64_t emask = 0, dmask = 0;
      bool err_lane = false;
      KWP_ADD(7, t_rp);
      KWP_MARK(t_ev2);
      for (;;) {
        // one evaluation pass: every lane its run with logged side effects (parallel), or -- for a
        // stateful round that conflicts (wave_round_conflict) -- lane jj alone with the lane kernel's
        // immediate ones, on the key's shared state, lanes in queue order (one call site of evaluate)
        const bool me = seqd ? lane == jj : act;
        if (seqd) {
          wave_sync();
          if (me) ws_to_lane(l, w);
        } else {
          l.heap = w.heap; l.heapcap = w.heapcap;
        }
        if (me || !seqd) { l.tlen = 0; l.log_n = 0; l.nph = 0; l.err = 0; l.overflow = 0; l.wgrow = 0; l.ov_own = 0; }
        good = true;
        if (me) good = seqd ? evaluate<false>(l, run, fr) : evaluate<true>(l, run, fr);
        if (seqd) {
          if (me) {
            if (good && l.tlen == 0) buf_peek(l, r_sid(run), run.ev, run.ver, true, nullptr, 0);   // removePattern
            const int e = l.err, o = l.overflow;
            lane_to_ws(w, l);
            if (e) w.err = e;
            if (o) { w.overflow = 1; w.cap_hit |= l.cap_hit; }
          }
          wave_sync();
          if (w.err || w.overflow || ++jj >= nact) break;
          continue;
        }
        const bool grow = gp.ballot(l.wgrow) != 0;
        const bool pool_out = gp.ballot(l.overflow && !l.wgrow) != 0;
        if (pool_out) {                                        // a private list could not grow
          if (lane == 0) w.overflow = 1;
          const uint64_t ch = gp.ballot(l.cap_hit);
          if (lane == 0 && ch) w.cap_hit = 1;
          break;
        }
        if (grow) {
          wave_sync();
          if (lane == 0) w.heap_top = top0;
          wave_sync();
          if (!wave_heap_reserve(l, w, int64_t(w.heapcap) * 2, gp)) break;
          continue;
        }
        err_lane = act && !good && l.err;
        const bool dead = act && good && l.tlen == 0;
        emask = gp.ballot(err_lane);
        dmask = gp.ballot(dead);
        // a conflict is checked before the errors: a run may throw on a state an earlier run of the
        // round would have folded first
        if (AGG && A.wave_agg && wave_round_conflict(l, w.u.conf, gp, act, run.seq, dmask)) {
          seqd = true;
          l.tlen = 0; l.log_n = 0; l.nph = 0;                  // the parallel pass is discarded
          continue;
        }
        break;
      }
      wave_sync();
      KWP_ADD(1, t_ev2);
      if (w.overflow) break;
      // commit in queue order
      KWP_MARK(t_cm);
      if (seqd) {                                              // (committed as evaluated)
        ws_to_lane(l, w);
        if (w.err) { KWP_ADD(2, t_cm); break; }
      } else if (!emask && !dmask) {
        const int e = wave_commit_parallel(l, w, gp, r);
        if (lane == 0 && e) w.err = e;
        wave_sync();
      } else {
        w.u.sq.logp[lane] = l.log;
        w.u.sq.logn[lane] = l.log_n;
        w.u.sq.errc[lane] = err_lane ? l.err : 0;
        wave_sync();
        if (lane == 0) {                                       // the reference's order, sequentially
          ws_to_lane(l, w);
          l.err = 0; l.overflow = 0;
          for (int j = 0; j < nact && !l.err && !l.overflow; j++) {
            const int32_t* lg = w.u.sq.logp[j];
            for (int k = 0; k < w.u.sq.logn[j] && !l.err && !l.overflow; k++) {
              const int32_t* o = lg + k * WL;
              const int kind = o[0] & 0xFF, sid = (o[0] >> 8) & 0xFF, psid = (o[0] >> 16) & 0xFF;
              if (kind == WOP_PUT5) buf_put5(l, sid, o[1], psid, o[2], o[3]);
              else if (kind == WOP_PUT3) buf_put3(l, sid, o[1], o[3]);
              else if (kind == WOP_BRANCH) buf_branch(l, sid, o[1], o[3]);
            }
            if (l.err || l.overflow) break;
            if ((emask >> j) & 1) { l.err = w.u.sq.errc[j]; break; }
            if ((dmask >> j) & 1) {                            // removePattern (:160-163)
              const int4 x = reinterpret_cast<const int4*>(l.qa)[base + j];
              buf_peek(l, x.x & 0xFF, x.z, x.y, true, nullptr, 0);
            }
          }
          lane_to_ws(w, l);
        }
        wave_sync();
        ws_to_lane(l, w);
      }
      KWP_ADD(2, t_cm);
      if (w.err || w.overflow) break;
      // NFA.runs: the round's placeholders in queue order
      KWP_MARK(t_pl);
      int nrun = 0;
      const int rb = w.runs + gp.excl_scan(l.nph, nrun);
      if (AGG && (A.wave_agg & 1) && !seqd && !wave_apply_aggs(l, w, gp, rb)) {   // the round's folds and copies
        if (lane == 0) w.overflow = 1;
        break;
      }
      int nf = 0, nq = 0;
      for (int t = 0; t < l.tlen; t++) {
        int4* y = reinterpret_cast<int4*>(l.tq) + t;
        if (y->w < -1) y->w = rb + (-y->w - 2) + 1;
        if (is_fwd_final(l, y->x & 0xFF, (y->x >> 8) & 0xFF)) nf++; else nq++;
      }
      int tf = 0, tq = 0;
      const int ef = gp.excl_scan(nf, tf), eq = gp.excl_scan(nq, tq);
      wave_sync();
      KWP_ADD(3, t_pl);
      KWP_MARK(t_pl2);
      if (lane == 0) w.runs += nrun;
      // room in the next queue and the final list
      if (qn + tq > w.qb_cap) {
        int32_t capw = w.qb_cap * 4;
        int32_t* na = wave_regrow(l, w, w.qb, capw, int64_t(qn) * 4, int64_t(qn + tq) * 4, gp, AK_QUEUE);
        if (!na) break;
        if (lane == 0) { w.qb = na; w.qb_cap = capw / 4; }
      }
      if (flen + tf > w.fq_cap) {
        int32_t capw = w.fq_cap * 4;
        int32_t* na = wave_regrow(l, w, w.fq, capw, int64_t(flen) * 4, int64_t(flen + tf) * 4, gp, AK_QUEUE);
        if (!na) break;
        if (lane == 0) { w.fq = na; w.fq_cap = capw / 4; }
      }
      wave_sync();
      int a = qn + eq, b = flen + ef;
      for (int t = 0; t < l.tlen; t++) {
        const int4 y = reinterpret_cast<const int4*>(l.tq)[t];
        if (is_fwd_final(l, y.x & 0xFF, (y.x >> 8) & 0xFF)) reinterpret_cast<int4*>(w.fq)[b++] = y;
        else reinterpret_cast<int4*>(w.qb)[a++] = y;
      }
      qn += tq;
      flen += tf;
      wave_sync();
      KWP_ADD(10, t_pl2);
    }
    if (w.err) { err_rec = a_pos(A, g); break; }
    if (w.overflow) break;
    KWP_MARK(t_end);
    // swap the queues; matchConstruction (:151-158); the high-water mark on lane 0
    if (lane == 0) {
      int32_t* t = w.qa; w.qa = w.qb; w.qb = t;
      const int32_t c = w.qa_cap; w.qa_cap = w.qb_cap; w.qb_cap = c;
      w.qlen = qn;
    }
    wave_sync();
    KWP_MARK(t_mc);
    if (flen && !wave_emit_matches(l, w, gp, flen)) {
      if (lane == 0) w.overflow = 1;
    }
    wave_sync();
    KWP_ADD(4, t_mc);
    if (lane == 0 && !w.err && !w.overflow) {
      ws_to_lane(l, w);
      if (proc && !record_hwm(l, g)) l.overflow = 1;
      lane_to_ws(w, l);
    }
    wave_sync();
    KWP_ADD(8, t_end);
    if (w.err) { err_rec = a_pos(A, g); break; }
    live_max = w.qlen > live_max ? w.qlen : live_max;
  }
  wave_sync();
  if (lane == 0) {
    ws_to_lane(l, w);
    l.pool_words = int64_t(w.ka.pool_words);
    l.wpool = nullptr;
    key_end(l, A, seg, err_rec, live_max, evals, t0, &w.ka);
  }
}

// The key segments of a batch, one key per wave at a time.  The grid is persistent (the host sizes it
// to the waves the chip holds at once, or the segment count if smaller): each workgroup takes the next
// segment from A.seg_next until none is left, and every key it takes works in the workgroup's own
// scratch region (recycled, so L2-resident, instead of a fresh stretch of the pool per key).
template <bool AGG>
__device__ __forceinline__ void nfa_wave_body(const NfaArgs& A) {
  constexpr int ARENA = WAVE_ARENA & ~3;   // LDS words of the key's hot workspace
  __shared__ WaveShared<WAVE> ws;
  __shared__ __attribute__((aligned(16))) int32_t s_arena[ARENA + 4];
  __shared__ __attribute__((aligned(16))) int32_t s_priv[WAVE * WAVE_PRIV];
  const Grp<WAVE> gp{int(threadIdx.x), 0};
  int32_t* scr = A.scratch_words > 0 ? A.scratch + int64_t(blockIdx.x) * A.scratch_words : nullptr;
  const int32_t nseg = A.nseg_dev ? int32_t(*A.nseg_dev) : A.nseg;   // (counted on the device: no host round trip)
  for (;;) {
    int seg = 0;
    if (gp.gl == 0) seg = atomicAdd(A.seg_next, 1);
    seg = gp.bcast(seg);
    if (seg >= nseg) break;                        // every wave of the grid reaches this
    if (A.seg_order) seg = A.seg_order[seg];
    wave_key<AGG, WAVE>(A, seg, gp, ws, s_arena, ARENA, s_priv, scr);
    wave_sync();
  }
}

}  // namespace kcep

// nfa_dev.h — device engine of the general NFA path (see nfa.hip for the
// algorithm and the reference mapping).  Compiled twice: into libkcep.so's
// nfa_kernel, reading the pattern's DevProgram from device memory and
// interpreting predicates (interp.h), and per pattern by jit.cpp with
// KCEP_JIT defined, where KCEP_PROG is the constexpr program table and
// jit_eval the pattern's straight-line predicates.
#pragma once
#include "interp.h"

#ifdef KCEP_JIT
#define KCEP_PROG(l) (::kcep::kcep_prog)
#ifndef KCEP_UNROLL
#define KCEP_UNROLL _Pragma("unroll")
#endif
#else
#define KCEP_PROG(l) (*(l).P)
#ifndef KCEP_UNROLL
#define KCEP_UNROLL
#endif
#endif

namespace kcep {


constexpr int32_t EPS_NONE = 0xFF;
// PROCEED/SKIP_PROCEED recursion depth (checked by the compiler).  The per-pattern kernels size the
// suspended-frame stack (scratch memory) by the pattern's own depth (+1 spare): C4 88 B per lane
// instead of 704
#ifdef KCEP_JIT
constexpr int MAXD = ::kcep::kcep_prog.maxdepth + 1 < NFA_MAX_FRAMES ? ::kcep::kcep_prog.maxdepth + 1 : NFA_MAX_FRAMES;
#else
constexpr int MAXD = NFA_MAX_FRAMES;
#endif
constexpr int NW = 4;                      // node words: refs, first pred, last pred, flags
constexpr int32_t NF_EXISTS = 1, NF_MARK = 2, NF_NEED = 4;
constexpr int PW = 6;                      // pred words: version, prev slot, prev event, next, |version|, version[0]
constexpr int HWM_MAX = 16;

struct Run {
  int32_t w0, ver, ev, seq;     // w0: sid | eps << 8 | branching << 16 | ignored << 17
};
__device__ __forceinline__ int r_sid(const Run& r) { return r.w0 & 0xFF; }
__device__ __forceinline__ int r_eps(const Run& r) { return (r.w0 >> 8) & 0xFF; }
__device__ __forceinline__ bool r_br(const Run& r) { return (r.w0 >> 16) & 1; }
__device__ __forceinline__ bool r_ig(const Run& r) { return (r.w0 >> 17) & 1; }
__device__ __forceinline__ Run mk_run(int sid, int eps, int ver, int ev, int seq, bool br, bool ig) {
  return Run{sid | (eps << 8) | (int(br) << 16) | (int(ig) << 17), ver, ev, seq};
}

enum { ST_BEGIN_ = 0, ST_NORMAL_ = 1, ST_FINAL_ = 2 };

// What a workspace allocation is for (profiling builds count the words per kind, cep_key_profile)
enum : int { AK_WS = 0, AK_OUT, AK_HEAP, AK_QUEUE, AK_PRIV, AK_AGG, AK_OTHER, AK_N };

// The wave kernel's allocator state of the key on the wave (LDS, nfa_wave.h): its words so far (the
// per-key cap) and the wave's recycled scratch region.  A key's workspace dies with the key, so the
// persistent wave hands the same region to every key it takes: the region's lines stay in the XCD's
// L2 from one key to the next instead of a fresh stretch of the batch pool being dirtied (and
// written back to HBM) per key.  Only what outlives the kernel -- the match output -- and what does
// not fit the region come from the batch pool.
struct KeyAlloc {
  unsigned long long pool_words;   // every word the key took (scratch + pool): max_key_words
  unsigned long long scr_top;      // scratch words handed out (may pass scr_cap: then the pool)
  int32_t* scr;                    // the wave's region (nullptr: none)
  int64_t scr_cap;
#ifdef KCEP_PHASES
  unsigned long long kw[AK_N + 1]; // profiling kernels only: words allocated per kind (AK_*), then the pool's share
  uint64_t ph[11];                 // profiling kernels only: lane 0's clocks per record-loop phase (nfa_wave.h KWP_*)
#endif
};

struct Lane {
  const NfaArgs* A;
  const DevProgram* P;
  int64_t seg0;
  int32_t L, C, nev;           // batch records, carried events, all local events
  const int32_t* cev;          // carried events (blob section)
  int32_t evw;
  int32_t* hwm;
  int32_t nhwm;
  int32_t* nodes;
  int32_t *qa, *qb, *tq, *fq;
  int32_t qa_cap, qb_cap, tq_cap, fq_cap;
  int32_t* aggs;
  int32_t seqcap;
  int32_t* heap;
  int32_t heapcap, heap_top;
  int32_t* out;
  int32_t outcap, out_top;     // match headers: 4 words each {stream position lo, hi, entries, first entry}
  int32_t* oent;               // their entries: 3 words each {stage name, stream position lo, hi}
  int32_t ecap, etop;          // (words / entries)
  int32_t qlen, tlen, flen;
  int32_t runs;                // internal run counter; NFAStates.runs = runs + runs_delta
  int64_t runs_delta;
  int32_t err;
  int32_t overflow;
  int32_t cap_hit;             // the key went over NfaArgs.max_key_words
  int32_t rec_etop;            // entries / matches before the current record (capacity rollback)
  int64_t rec_nmatch;
  int32_t r;                   // current local event
  int64_t g;                   // its batch record index
  int64_t nmatch;
  uint64_t slm, sle;           // event-only edge predicates on record r: values / deferred errors
  int64_t pool_words;          // taken from the pool (profile)
  // ---- wave mode (nfa_wave.h: one key per wave, one queued run per lane) ----
  int32_t* wtop;               // wave: the key's heap top, in LDS
  int32_t* log;                // wave: this lane's run's deferred buffer operations, WL words each
  int32_t log_cap, log_n;
  int32_t arena_used;             // wave kernel: LDS arena words key_begin took (-1: workspace in the pool)
  int32_t nph;                 // wave: run-counter increments of this lane's run (seq placeholders)
  int32_t wgrow;               // wave: the shared heap was too small (grow it and re-run the round)
  int32_t ov_own;              // wave: this evaluation wrote an aggregate of its run's own sequence
  KeyAlloc* wpool;             // wave: the key's allocator, in LDS (every lane allocates for the key)
#ifdef KCEP_PHASES_LANE
  uint64_t ph[11];             // lane-engine profiling builds only: clocks in evaluate / predicates / buffer
                               // puts+branch / removePattern / matchConstruction / first_compatible / add_pred /
                               // versions, then counts: first_compatible calls / entries examined / digit checks
#endif
};

// phase timers of the lane engine (KCEP_PHASES_LANE builds only: they share Lane.ph with the wave
// kernel's record-loop timers, nfa_wave.h KWP_*, which the CEP_SESSION_PROFILE kernels keep)
#ifdef KCEP_PHASES_LANE
#define KPH_BEGIN(l, i) const uint64_t kph_t##i = clock64()
#define KPH_END(l, i) const_cast<Lane&>(l).ph[i] += clock64() - kph_t##i
#define KPH_COUNT(l, i, n) const_cast<Lane&>(l).ph[i] += (n)
#else
#define KPH_BEGIN(l, i)
#define KPH_END(l, i)
#define KPH_COUNT(l, i, n)
#endif

// ---- pool ----
// every allocation is a multiple of 16 bytes (queues are read as int4)
// the wave kernel's per-key counters live in LDS (WaveShared): LDS atomics, not flat ones (a flat atomic
// waits on both the vector-memory and the LDS counters)
typedef int32_t __attribute__((address_space(3))) lds_i32;
typedef unsigned long long __attribute__((address_space(3))) lds_u64;
__device__ __forceinline__ int32_t lds_add(int32_t* p, int32_t v) {
  return __hip_atomic_fetch_add((lds_i32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ unsigned long long lds_add(unsigned long long* p, unsigned long long v) {
  return __hip_atomic_fetch_add((lds_u64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// persist: the words must outlive the kernel (the match output): never from the wave's scratch
__device__ __forceinline__ int32_t* pool_alloc(Lane& l, int64_t words, int kind, bool persist = false) {
  const int64_t w = (words + 3) & ~int64_t(3);
  if (l.wpool) {
#ifdef KCEP_PHASES
    lds_add(&l.wpool->kw[kind], (unsigned long long)w);
#endif                                   // wave mode: one allocator for the key
    const int64_t was = int64_t(lds_add(&l.wpool->pool_words, (unsigned long long)w));
    if (l.A->max_key_words > 0 && was + w > l.A->max_key_words) { l.overflow = 1; l.cap_hit = 1; return nullptr; }
    if (!persist && l.wpool->scr && w <= l.wpool->scr_cap) {
      const int64_t at = int64_t(lds_add(&l.wpool->scr_top, (unsigned long long)w));
      if (at <= l.wpool->scr_cap - w) { l.pool_words += w; return l.wpool->scr + at; }
    }
  } else if (l.A->max_key_words > 0 && l.pool_words + w > l.A->max_key_words) {
    l.overflow = 1; l.cap_hit = 1; return nullptr;
  }
  const unsigned long long at = atomicAdd(l.A->pool_top, (unsigned long long)w);
  if (at + (unsigned long long)w > (unsigned long long)l.A->pool_cap) { l.overflow = 1; return nullptr; }
  l.pool_words += w;
#ifdef KCEP_PHASES
  if (l.wpool) lds_add(&l.wpool->kw[AK_N], (unsigned long long)w);
#endif
  return l.A->pool + at;
}
// re-allocate `*a` (cap words used up to `used`) at >= need words
__device__ __forceinline__ bool regrow(Lane& l, int32_t*& a, int32_t& cap, int64_t used, int64_t need, int kind,
                                       int32_t fill = 0, bool zero = false) {
  int64_t nc = int64_t(cap) * 2;
  if (nc < need) nc = need;
  if (nc > (int64_t(1) << 30)) { l.overflow = 1; return false; }
  int32_t* na = pool_alloc(l, nc, kind);
  if (!na) return false;
  for (int64_t i = 0; i < used; i++) na[i] = a[i];
  if (zero)
    for (int64_t i = used; i < nc; i++) na[i] = fill;
  a = na;
  cap = int32_t(nc);
  return true;
}

// ---- stage references (real stage or Stage.newEpsilonState(src, target), Stage.java:247-251) ----
__device__ __forceinline__ const DevStage& stg(const Lane& l, int sid) { return KCEP_PROG(l).st[sid]; }
// the stage table's small fields by a lane's own stage id: in the per-pattern kernels computed from
// immediates (jit.cpp gen_packed), not loaded from the program table (a divergent constant-memory load
// on every evaluation's dependency chain); the built-in kernels read the DevProgram
#ifdef KCEP_JIT
#define ST_TYPE(l, s) ::kcep::jst_type(s)
#define ST_NAME(l, s) ::kcep::jst_name(s)
#define ST_SLOT(l, s) ::kcep::jst_slot(s)
#define ST_NEDGES(l, s) ::kcep::jst_nedges(s)
#define ST_NFOLDS(l, s) ::kcep::jst_nfolds(s)
#define ST_OP(l, s, e) ::kcep::jst_op((s) * NFA_MAX_EDGES + (e))
#define ST_TARGET(l, s, e) ::kcep::jst_target((s) * NFA_MAX_EDGES + (e))
#define ST_PRED(l, s, e) ::kcep::jst_pred((s) * NFA_MAX_EDGES + (e))
#define ST_SL(l, s, e) ::kcep::jst_sl((s) * NFA_MAX_EDGES + (e))
#define SLOT_NAME(l, x) ::kcep::jst_slot_name(x)
#else
#define ST_TYPE(l, s) stg(l, s).type
#define ST_NAME(l, s) stg(l, s).name
#define ST_SLOT(l, s) stg(l, s).slot
#define ST_NEDGES(l, s) stg(l, s).nedges
#define ST_NFOLDS(l, s) stg(l, s).nfolds
#define ST_OP(l, s, e) stg(l, s).op[e]
#define ST_TARGET(l, s, e) stg(l, s).target[e]
#define ST_PRED(l, s, e) stg(l, s).pred[e]
#define ST_SL(l, s, e) stg(l, s).sl[e]
#define SLOT_NAME(l, x) (l).P->slot_name[x]
#endif
__device__ __forceinline__ bool is_begin(const Lane& l, int sid) { return ST_TYPE(l, sid) == ST_BEGIN_; }
__device__ __forceinline__ bool is_forwarding(const Lane& l, int sid, int eps) {   // ComputationStage.java:134-137
  if (eps != EPS_NONE) return true;
  return ST_NEDGES(l, sid) == 1 && ST_OP(l, sid, 0) == E_PROCEED;
}
__device__ __forceinline__ bool is_fwd_final(const Lane& l, int sid, int eps) {    // :143-147
  if (!is_forwarding(l, sid, eps)) return false;
  const int tgt = eps != EPS_NONE ? eps : ST_TARGET(l, sid, 0);
  return ST_TYPE(l, tgt) == ST_FINAL_;
}

// ---- heap: versions and predecessor pointers ----
// W: the wave kernel's parallel evaluation (nfa_wave.h) -- shared allocations and logged buffer
// operations; a compile-time mode, so that the wave's workspace pointers stay wave-uniform (scalar
// registers) through an evaluation instead of merging with the lane path's re-allocations
template <bool W = false>
__device__ __forceinline__ int heap_alloc(Lane& l, int words) {
  if constexpr (W) {                                    // versions are immutable: any allocation order will do
    const int at = lds_add(l.wtop, words);
    if (at + words > l.heapcap) { l.wgrow = 1; l.overflow = 1; return -1; }
    return at;
  }
  if (l.heap_top + words > l.heapcap && !regrow(l, l.heap, l.heapcap, l.heap_top, int64_t(l.heap_top) + words, AK_HEAP))
    return -1;
  const int at = l.heap_top;
  l.heap_top += words;
  return at;
}
// a version's digits copied to a fresh allocation: 4 loads issued before their 4 stores (the compiler
// cannot tell the two ranges apart, so a load-store-load chain would pay one memory latency per digit)
__device__ __forceinline__ void dw_copy(int32_t* h, int dst, int src, int len) {
  int i = 0;
  for (; i + 4 <= len; i += 4) {
    const int32_t a = h[src + i], b = h[src + i + 1], c = h[src + i + 2], d = h[src + i + 3];
    h[dst + i] = a; h[dst + i + 1] = b; h[dst + i + 2] = c; h[dst + i + 3] = d;
  }
  for (; i < len; i++) h[dst + i] = h[src + i];
}
template <bool W>
__device__ __forceinline__ int dw_add_stage_(Lane& l, int v) {            // DeweyVersion.addStage :95-97
  const int len = l.heap[v];
  const int n = heap_alloc<W>(l, len + 2);
  if (n < 0) return -1;
  l.heap[n] = len + 1;
  dw_copy(l.heap, n + 1, v + 1, len);
  l.heap[n + 1 + len] = 0;
  return n;
}
template <bool W>
__device__ __forceinline__ int dw_add_run_(Lane& l, int v, int off) {     // DeweyVersion.addRun :62-67
  const int len = l.heap[v];
  const int idx = len - off;
  if (idx < 0 || idx >= len) { l.err = CEP_E_INDEX; return -1; }
  const int n = heap_alloc<W>(l, len + 1);
  if (n < 0) return -1;
  const int32_t bumped = int32_t(uint32_t(l.heap[v + 1 + idx]) + 1u);
  l.heap[n] = len;
  dw_copy(l.heap, n + 1, v + 1, len);
  l.heap[n + 1 + idx] = bumped;
  return n;
}
template <bool W = false>
__device__ __forceinline__ int dw_add_stage(Lane& l, int v) {
  KPH_BEGIN(l, 7);
  const int n = dw_add_stage_<W>(l, v);
  KPH_END(l, 7);
  return n;
}
template <bool W = false>
__device__ __forceinline__ int dw_add_run(Lane& l, int v, int off) {
  KPH_BEGIN(l, 7);
  const int n = dw_add_run_<W>(l, v, off);
  KPH_END(l, 7);
  return n;
}

// a.isCompatible(b) (:73-93), with b's length and first digit known up front
__device__ __forceinline__ bool dw_compatible(const Lane& l, int a, int b, int lb, int b0) {
  const int la = l.heap[a];
  if (la < lb) return false;
  if (la == lb && la == 1) return l.heap[a + 1] >= b0;
  if (l.heap[a + 1] != b0) return false;               // every other case compares the first digit
  if (la > lb) {
    for (int i = 1; i < lb; i++)
      if (l.heap[a + 1 + i] != l.heap[b + 1 + i]) return false;
    return true;
  }
  for (int i = 1; i < la - 1; i++)
    if (l.heap[a + 1 + i] != l.heap[b + 1 + i]) return false;
  return l.heap[a + la] >= l.heap[b + lb];
}

// ---- shared versioned buffer ----
__device__ __forceinline__ int32_t* node(Lane& l, int slot, int ev) {
  return l.nodes + (int64_t(ev) * KCEP_PROG(l).nslots + slot) * NW;
}
__device__ __forceinline__ int slot_of(const Lane& l, int sid) { return ST_SLOT(l, sid); }
__device__ __forceinline__ bool exists(const int32_t* nd) { return nd[3] & NF_EXISTS; }

__device__ __forceinline__ bool add_pred_(Lane& l, int32_t* nd, int ver, int pslot, int pev) {   // MatchedEvent.addPredecessor
  const int p = heap_alloc(l, PW);
  if (p < 0) return false;
  l.heap[p] = ver; l.heap[p + 1] = pslot; l.heap[p + 2] = pev; l.heap[p + 3] = -1;
  l.heap[p + 4] = l.heap[ver]; l.heap[p + 5] = l.heap[ver + 1];
  if (nd[1] < 0) nd[1] = p;
  else l.heap[nd[2] + 3] = p;
  nd[2] = p;
  return true;
}
__device__ __forceinline__ bool add_pred(Lane& l, int32_t* nd, int ver, int pslot, int pev) {
  KPH_BEGIN(l, 6);
  const bool ok = add_pred_(l, nd, ver, pslot, pev);
  KPH_END(l, 6);
  return ok;
}
// wave mode: a buffer operation is logged (WL words: kind | cur sid << 8 | prev sid << 16, event, prev
// event, version) and applied in queue order after the round (nfa_wave.h)
constexpr int WL = 4;
enum : int32_t { WOP_PUT5 = 1, WOP_PUT3 = 2, WOP_BRANCH = 3, WOP_AGG = 4 };
__device__ __forceinline__ void wlog(Lane& l, int kind, int sid, int psid, int ev, int pev, int ver) {
  if (l.log_n >= l.log_cap) {
    int32_t capw = l.log_cap * WL;
    if (!regrow(l, l.log, capw, int64_t(l.log_n) * WL, int64_t(l.log_n + 1) * WL * 2, AK_PRIV)) return;
    l.log_cap = capw / WL;
  }
  int32_t* o = l.log + l.log_n * WL;
  o[0] = kind | (sid << 8) | ((psid & 0xFF) << 16);
  o[1] = ev; o[2] = pev; o[3] = ver;
  l.log_n++;
}
// put 5-arg (SharedVersionedBufferStoreImpl.java:101-126)
template <bool W = false>
__device__ __forceinline__ void buf_put5(Lane& l, int cur_sid, int ev, int prev_sid, int pev, int ver) {
  if (pev < 0) { l.err = CEP_E_NPE; return; }
  if constexpr (W) { wlog(l, WOP_PUT5, cur_sid, prev_sid, ev, pev, ver); return; }
  const int ps = slot_of(l, prev_sid);
  if (!exists(node(l, ps, pev))) { l.err = CEP_E_ILLEGAL_STATE; return; }
  int32_t* c = node(l, slot_of(l, cur_sid), ev);
  if (!exists(c)) { c[0] = 1; c[1] = -1; c[2] = -1; c[3] = NF_EXISTS; }
  add_pred(l, c, ver, ps, pev);
}
// put 3-arg (:149-157): a fresh node overwrites
template <bool W = false>
__device__ __forceinline__ void buf_put3(Lane& l, int cur_sid, int ev, int ver) {
  if constexpr (W) { wlog(l, WOP_PUT3, cur_sid, 0xFF, ev, -1, ver); return; }
  int32_t* c = node(l, slot_of(l, cur_sid), ev);
  c[0] = 1; c[1] = -1; c[2] = -1; c[3] = NF_EXISTS;
  add_pred(l, c, ver, -1, 0);
}
__device__ __forceinline__ int first_compatible_(const Lane& l, const int32_t* nd, int ver, int* prevp) {   // getPointerByVersion
  int pp = -1;
  for (int p = nd[1]; p >= 0; p = l.heap[p + 3]) {
    KPH_COUNT(l, 9, 1);
    if (dw_compatible(l, ver, l.heap[p], l.heap[p + 4], l.heap[p + 5])) { if (prevp) *prevp = pp; return p; }
    pp = p;
  }
  return -1;
}
__device__ __forceinline__ int first_compatible(const Lane& l, const int32_t* nd, int ver, int* prevp) {
  KPH_BEGIN(l, 5);
  const int p = first_compatible_(l, nd, ver, prevp);
  KPH_END(l, 5);
  KPH_COUNT(l, 8, 1);
  return p;
}
// branch (:132-142)
template <bool W = false>
__device__ __forceinline__ void buf_branch(Lane& l, int sid, int ev, int ver) {
  if (ev < 0) { l.err = CEP_E_NPE; return; }
  if constexpr (W) { wlog(l, WOP_BRANCH, sid, 0xFF, ev, ev, ver); return; }
  int slot = slot_of(l, sid), e = ev, pv = ver;
  for (;;) {
    int32_t* nd = node(l, slot, e);
    if (!exists(nd)) { l.err = CEP_E_NPE; return; }
    nd[0]++;
    const int p = first_compatible(l, nd, pv, nullptr);
    if (p < 0 || l.heap[p + 1] < 0) return;
    pv = l.heap[p]; slot = l.heap[p + 1]; e = l.heap[p + 2];
  }
}
// peek (:176-201).  emit: traversal (slot, event) pairs into dst; returns the count or -1.
__device__ __forceinline__ int buf_peek(Lane& l, int sid, int ev, int ver, bool remove, int32_t* dst, int dst_cap) {
  if (ev < 0) { l.err = CEP_E_NPE; return -1; }
  int slot = slot_of(l, sid), e = ev, pv = ver, cnt = 0;
  for (;;) {
    int32_t* nd = node(l, slot, e);
    if (!exists(nd)) { l.err = CEP_E_NPE; return -1; }
    const int refs_left = nd[0] == 0 ? 0 : nd[0] - 1;     // decremented on a copy
    const bool single = nd[1] < 0 || l.heap[nd[1] + 3] < 0;
    if (dst) {
      if (cnt + 1 > dst_cap) { l.overflow = 1; return -1; }   // callers reserve one entry per event
      dst[2 * cnt] = slot;
      dst[2 * cnt + 1] = e;
    }
    cnt++;
    int pp = -1;
    const int p = first_compatible(l, nd, pv, &pp);
    if (remove && p >= 0 && refs_left == 0) {
      nd[0] = 0;                                            // removePredecessor + put(copy)
      const int nx = l.heap[p + 3];
      if (pp < 0) nd[1] = nx; else l.heap[pp + 3] = nx;
      if (nd[2] == p) nd[2] = pp;
      nd[3] |= NF_EXISTS;
    } else if (remove && refs_left == 0 && single) {
      nd[3] &= ~NF_EXISTS;                                  // delete
    }
    if (p < 0 || l.heap[p + 1] < 0) return cnt;
    pv = l.heap[p]; slot = l.heap[p + 1]; e = l.heap[p + 2];
  }
}

// ---- aggregates: row per run sequence ----
__device__ __forceinline__ int32_t* agg(Lane& l, int state, int seq) {
  const int ns = KCEP_PROG(l).nstates;
  if (seq < 0) { l.overflow = 1; return nullptr; }
  if (seq >= l.seqcap) {
    int32_t cap = l.seqcap * ns * 3;
    int32_t* a = l.aggs;
    const int64_t need = (int64_t(seq) + 1) * ns * 3;
    if (!regrow(l, a, cap, int64_t(l.seqcap) * ns * 3, need, AK_AGG, 0, true)) return nullptr;
    l.aggs = a;
    l.seqcap = cap / (ns * 3);
  }
  return l.aggs + (int64_t(seq) * ns + state) * 3;
}

// AggregatesStore.find / put (AggregatesStoreImpl.java:55-75) for the evaluating run.  Wave mode: the
// round evaluates against the aggregates as they were before it; a lane's writes are logged (WOP_AGG:
// state, boxed type, sequence -- a placeholder for a sequence created in the round -- and the value)
// and read back by the same lane first, then applied in queue order after the round (nfa_wave.h).
template <bool W = false>
__device__ __forceinline__ bool agg_read(Lane& l, int state, int seq, int32_t& tag, int64_t& v) {
  if constexpr (W) {
    for (int k = l.log_n - 1; k >= 0; k--) {
      const int32_t* o = l.log + k * WL;
      if ((o[0] & 0xFF) == WOP_AGG && ((o[0] >> 8) & 0xFF) == state && o[1] == seq) {
        tag = (o[0] >> 16) & 0xFF;
        v = int64_t(uint32_t(o[2])) | (int64_t(o[3]) << 32);
        return true;
      }
    }
    if (seq < 0 || seq >= l.seqcap) { tag = 0; v = 0; return true; }   // a row not grown yet: every state null
    const int32_t* e = l.aggs + (int64_t(seq) * KCEP_PROG(l).nstates + state) * 3;
    tag = e[0];
    v = int64_t(uint32_t(e[1])) | (int64_t(e[2]) << 32);
    return true;
  }
  const int32_t* e = agg(l, state, seq);
  if (!e) return false;
  tag = e[0];
  v = int64_t(uint32_t(e[1])) | (int64_t(e[2]) << 32);
  return true;
}
template <bool W = false>
__device__ __forceinline__ bool agg_write(Lane& l, int state, int seq, int32_t tag, int64_t v) {
  const int32_t lo = int32_t(uint32_t(uint64_t(v))), hi = int32_t(uint32_t(uint64_t(v) >> 32));
  if constexpr (W) {
    const int n0 = l.log_n;
    wlog(l, WOP_AGG, state, tag, seq, lo, hi);
    return l.log_n > n0;
  }
  int32_t* e = agg(l, state, seq);
  if (!e) return false;
  e[0] = tag; e[1] = lo; e[2] = hi;
  return true;
}

// ---- event fields: local event e (carried below C) ----
__device__ __forceinline__ int64_t cw64(const int32_t* p) { return int64_t(uint32_t(p[0])) | (int64_t(p[1]) << 32); }
__device__ __forceinline__ const int32_t* cev_of(const Lane& l, int e) { return l.cev + int64_t(e) * l.evw; }
__device__ __forceinline__ int64_t gidx(const Lane& l, int e) { return l.seg0 + (e - l.C); }
__device__ __forceinline__ int64_t ev_pos(const Lane& l, int e) {
  return e < l.C ? cw64(cev_of(l, e)) : a_pos(*l.A, gidx(l, e));
}
__device__ __forceinline__ int32_t b_topic(const Lane& l, int64_t g) { return l.A->topic ? l.A->topic[g] : 0; }
__device__ __forceinline__ int32_t b_part(const Lane& l, int64_t g) { return l.A->partition ? l.A->partition[g] : 0; }
__device__ __forceinline__ int64_t b_off(const Lane& l, int64_t g) { return l.A->offset ? l.A->offset[g] : a_pos(*l.A, g); }
__device__ __forceinline__ int64_t b_ts(const Lane& l, int64_t g) { return l.A->ts ? l.A->ts[g] : a_pos(*l.A, g); }
__device__ __forceinline__ int64_t b_field(const Lane& l, int col, int t, int64_t g) {
  const void* c = l.A->cols[col];
  if (t == T_I32) return static_cast<const int32_t*>(c)[g];
  return static_cast<const int64_t*>(c)[g];            // i64, or f64 bits
}
__device__ __forceinline__ int32_t ev_topic(const Lane& l, int e) { return e < l.C ? cev_of(l, e)[2] : b_topic(l, gidx(l, e)); }
__device__ __forceinline__ int32_t ev_part(const Lane& l, int e) { return e < l.C ? cev_of(l, e)[3] : b_part(l, gidx(l, e)); }
__device__ __forceinline__ int64_t ev_off(const Lane& l, int e) { return e < l.C ? cw64(cev_of(l, e) + 4) : b_off(l, gidx(l, e)); }
__device__ __forceinline__ int64_t ev_ts(const Lane& l, int e) { return e < l.C ? cw64(cev_of(l, e) + 6) : b_ts(l, gidx(l, e)); }
__device__ __forceinline__ int64_t ev_field(const Lane& l, int col, int t, int e) {
  return e < l.C ? cw64(cev_of(l, e) + 8 + 2 * col) : b_field(l, col, t, gidx(l, e));
}

__device__ __forceinline__ double as_f(int64_t b) { return __builtin_bit_cast(double, b); }
__device__ __forceinline__ int64_t as_b(double d) { return __builtin_bit_cast(int64_t, d); }

// Event.compareTo (Event.java:118-122) == 0, for TreeSet de-duplication
__device__ __forceinline__ bool ev_same(const Lane& l, int a, int b) {
  if (ev_topic(l, a) != ev_topic(l, b) || ev_part(l, a) != ev_part(l, b)) return ev_ts(l, a) == ev_ts(l, b);
  return ev_off(l, a) == ev_off(l, b);
}

struct Ctx {
  int seq, prev_sid, pev, ver;   // prev_sid < 0: null previous stage
  bool in_fold;
  int32_t curr_tag;
  int64_t curr;
};

// scratch for a partial sequence's walk: above the heap top (wave mode: drawn from the shared heap,
// since the other lanes allocate concurrently)
template <bool W = false>
__device__ __forceinline__ int32_t* seq_scratch(Lane& l) {
  const int need = 2 * l.nev + 2;
  if constexpr (W) {
    const int at = heap_alloc<W>(l, need);
    return at < 0 ? nullptr : l.heap + at;
  }
  if (l.heap_top + need > l.heapcap && !regrow(l, l.heap, l.heapcap, l.heap_top, int64_t(l.heap_top) + need, AK_HEAP))
    return nullptr;
  return l.heap + l.heap_top;
}

// Java 8's compensated double summation (Collectors.sumWithCompensation / computeFinalSum, used by
// DoubleStream.sum / average and DoubleSummaryStatistics): Kahan sum + simple sum, finished as
// sum + compensation (JDK 8), or the simple sum when that is NaN and the simple sum infinite.  The
// build has -ffp-contract=off, so no step is fused.
struct JSum {
  double s = 0, c = 0, simple = 0;
  __device__ __forceinline__ void add(double d) {
    const double tmp = d - c;
    const double velvel = s + tmp;
    c = (velvel - s) - tmp;
    s = velvel;
    simple += d;
  }
  __device__ __forceinline__ double final_sum() const {
    const double tmp = s + c;
    return (tmp != tmp && __builtin_isinf(simple)) ? simple : tmp;
  }
};
__device__ __forceinline__ int ev_cmp(const Lane& l, int a, int b);
// the partial sequence's events in Sequence order -- what a stream over it visits (Sequence.java
// build(true) :210-223: stages in reverse first-seen order of the walk, each stage's events a TreeSet
// ascending by Event.compareTo, duplicates dropped); stage != SEQ_ANY_STAGE: that stage's only.
// tmp: the walk's (slot, event) pairs.  Only the compensated double sums depend on this order.
template <class F>
__device__ __forceinline__ void seq_visit(const Lane& l, const int32_t* tmp, int cnt, int stage, F&& f) {
  const auto& P = KCEP_PROG(l);
  for (int gi = cnt - 1; gi >= 0; gi--) {
    const int nm = P.slot_name[tmp[2 * gi]];
    bool first = true;
    for (int j = 0; j < gi && first; j++) first = P.slot_name[tmp[2 * j]] != nm;
    if (!first || (stage != SEQ_ANY_STAGE && nm != stage)) continue;
    int last = -1;
    for (;;) {                                     // the next event of the stage's TreeSet
      int pick = -1;
      for (int i = 0; i < cnt; i++) {
        if (P.slot_name[tmp[2 * i]] != nm) continue;
        const int e = tmp[2 * i + 1];
        if (last >= 0 && ev_cmp(l, e, last) <= 0) continue;
        if (pick < 0 || ev_cmp(l, e, pick) < 0) pick = e;
      }
      if (pick < 0) break;
      f(pick);
      last = pick;
    }
  }
}

// SequenceMatcher: average of a column over buffer.get(Matched(prev, prevEvent), version)
// (SequenceMatcher.java:21-26), with Sequence's per-stage TreeSet de-duplication.
template <bool W = false>
__device__ __forceinline__ bool seq_avg(Lane& l, const Ctx& c, int col, int64_t& out) {
  if (c.prev_sid < 0 || c.pev < 0) { l.err = CEP_E_NPE; return false; }
  int32_t* tmp = seq_scratch<W>(l);                     // the walk visits at most one node per event
  if (!tmp) return false;
  const int cnt = buf_peek(l, c.prev_sid, c.pev, c.ver, false, tmp, l.nev + 1);
  if (cnt < 0) return false;
  const int t = KCEP_PROG(l).coltype[col];
  int64_t isum = 0;
  JSum js;
  int64_t n = 0;
  if (t == T_F64) {                                // DoubleStream.average: compensated, in Sequence order
    seq_visit(l, tmp, cnt, SEQ_ANY_STAGE, [&](int e) { js.add(as_f(ev_field(l, col, t, e))); n++; });
  } else {
    for (int i = 0; i < cnt; i++) {
      bool dup = false;
      for (int j = 0; j < i && !dup; j++)
        dup = KCEP_PROG(l).slot_name[tmp[2 * j]] == KCEP_PROG(l).slot_name[tmp[2 * i]] && ev_same(l, tmp[2 * j + 1], tmp[2 * i + 1]);
      if (dup) continue;
      isum += ev_field(l, col, t, tmp[2 * i + 1]);
      n++;
    }
  }
  const double avg = n ? (t == T_F64 ? js.final_sum() : double(isum)) / double(n) : 0.0;
  out = as_b(avg);
  return true;
}

// Other SequenceMatcher reductions over the same partial sequence (Sequence.java:57-60, 116-167):
// every event (stage == SEQ_ANY_STAGE) or one stage's (getByName(stage).getEvents(), null -> NPE),
// each stage's events a TreeSet (Event.compareTo, Event.java:118-122: duplicates dropped, first /
// last are its ends).  SUM and COUNT are Java longs (mapToLong(...).sum(), count()); MIN / MAX /
// FIRST / LAST keep the column's type.
__device__ __forceinline__ int ev_cmp(const Lane& l, int a, int b) {
  int64_t x, y;
  if (ev_topic(l, a) != ev_topic(l, b) || ev_part(l, a) != ev_part(l, b)) { x = ev_ts(l, a); y = ev_ts(l, b); }
  else { x = ev_off(l, a); y = ev_off(l, b); }
  return x < y ? -1 : x > y ? 1 : 0;
}
template <bool W = false>
__device__ __forceinline__ bool seq_agg(Lane& l, const Ctx& c, int kind, int col, int stage, int64_t& out) {
  if (c.prev_sid < 0 || c.pev < 0) { l.err = CEP_E_NPE; return false; }
  int32_t* tmp = seq_scratch<W>(l);
  if (!tmp) return false;
  const int cnt = buf_peek(l, c.prev_sid, c.pev, c.ver, false, tmp, l.nev + 1);
  if (cnt < 0) return false;
  const auto& P = KCEP_PROG(l);
  const int t = P.coltype[col];
  if (kind == SEQ_SUM && t == T_F64) {             // DoubleStream.sum: compensated, in Sequence order
    JSum js;
    int64_t m = 0;
    seq_visit(l, tmp, cnt, stage, [&](int e) { js.add(as_f(ev_field(l, col, t, e))); m++; });
    if (m == 0 && stage != SEQ_ANY_STAGE) { l.err = CEP_E_NPE; return false; }
    out = as_b(js.final_sum());
    return true;
  }
  int64_t n = 0, acc = 0;
  int pick = -1;                                   // FIRST / LAST: the event chosen so far
  for (int i = 0; i < cnt; i++) {
    const int nm = P.slot_name[tmp[2 * i]];
    if (stage != SEQ_ANY_STAGE && nm != stage) continue;
    bool dup = false;
    for (int j = 0; j < i && !dup; j++)
      dup = P.slot_name[tmp[2 * j]] == nm && ev_same(l, tmp[2 * j + 1], tmp[2 * i + 1]);
    if (dup) continue;
    const int ev = tmp[2 * i + 1];
    if (kind == SEQ_FIRST || kind == SEQ_LAST) {
      if (pick < 0 || (kind == SEQ_FIRST ? ev_cmp(l, ev, pick) < 0 : ev_cmp(l, ev, pick) > 0)) pick = ev;
    } else if (kind != SEQ_COUNT) {
      const int64_t v = ev_field(l, col, t, ev);
      if (kind == SEQ_SUM) acc += v;
      else if (n == 0) acc = v;
      else if (t == T_F64) {                       // Math.min / max on doubles: NaN wins, -0.0 < 0.0
        const double a = as_f(acc), b = as_f(v);
        const bool take = a != a ? false : b != b ? true
                        : kind == SEQ_MIN ? (b < a || (b == 0 && a == 0 && __builtin_signbit(b) && !__builtin_signbit(a)))
                                          : (b > a || (b == 0 && a == 0 && !__builtin_signbit(b) && __builtin_signbit(a)));
        if (take) acc = v;
      } else if (kind == SEQ_MIN ? v < acc : v > acc) {
        acc = v;
      }
    }
    n++;
  }
  if (n == 0) {                                     // no such stage in the sequence: getByName -> null
    if (stage != SEQ_ANY_STAGE || kind == SEQ_MIN || kind == SEQ_MAX) { l.err = CEP_E_NPE; return false; }
  }
  if (kind == SEQ_COUNT) out = n;
  else if (kind == SEQ_FIRST || kind == SEQ_LAST) out = ev_field(l, col, t, pick);
  else out = acc;
  return true;
}

// interpreter environment of the general kernel: the lane's current record,
// the evaluating run's aggregates and partial sequence
template <bool W = false>
struct LaneEnv {
  Lane& l;
  const Ctx& c;
  bool in_fold;
  int32_t curr_tag;
  int64_t curr;
  __device__ __forceinline__ int64_t field(int col, int t) { return b_field(l, col, t, l.g); }
  __device__ __forceinline__ int64_t key() { return l.A->key[l.g]; }
  __device__ __forceinline__ int64_t ts() { return b_ts(l, l.g); }
  __device__ __forceinline__ int64_t off() { return b_off(l, l.g); }
  __device__ __forceinline__ int64_t part() { return b_part(l, l.g); }
  __device__ __forceinline__ int32_t topic() { return b_topic(l, l.g); }
  __device__ __forceinline__ bool state(int idx, int32_t& tag, int64_t& v) { return agg_read<W>(l, idx, c.seq, tag, v); }
  __device__ __forceinline__ bool seq_avg(int col, int64_t& v) { return kcep::seq_avg<W>(l, c, col, v); }
  __device__ __forceinline__ bool seq_agg(int kind, int col, int stage, int64_t& v) {
    return kcep::seq_agg<W>(l, c, kind, col, stage, v);
  }
  __device__ __forceinline__ void fail(int code) { l.err = code; }
};

// bytecode interpreter over the current record; returns false on error (l.err / l.overflow set)
template <bool W = false>
__device__ __forceinline__ bool run_code(Lane& l, int pc, const Ctx& c, int64_t& result) {
  LaneEnv<W> env{l, c, c.in_fold, c.curr_tag, c.curr};
#ifdef KCEP_JIT
  return jit_eval(pc, env, result);
#else
  return interp(l.P->code, pc, env, result);
#endif
}

// event-only edge predicates of the current record, once for every run: all
// lanes walk the same programs in the same order.  A predicate that throws is
// left to per-run evaluation so the exception surfaces exactly where the
// reference evaluates it (NFA.java:371-384).
__device__ __forceinline__ void eval_event_only(Lane& l) {
  l.slm = 0;
  l.sle = 0;
  const int nsl = KCEP_PROG(l).nsl;
  KCEP_UNROLL
  for (int i = 0; i < nsl; i++) {                  // uniform: lock-step interpreter, scalar code fetches
    const Ctx c{0, -1, -1, -1, false, 0, 0};
    LaneEnv<false> env{l, c, false, 0, 0};
    int64_t v = 0;
    const int e0 = l.err, o0 = l.overflow;
#ifdef KCEP_JIT
    if (jit_eval(KCEP_PROG(l).sl_pc[i], env, v)) {
#else
    if (interp_ls(l.P->code, l.P->sl_pc[i], env, true, v)) {
#endif
      if (v) l.slm |= 1ull << i;
    } else {
      l.sle |= 1ull << i;
      l.err = e0;
      l.overflow = o0;
    }
  }
}

// ---- the wave kernel's schedule: heaviest keys first ----
// A key's cost is unknown until it runs (C4: a key's live runs multiply with every matching record),
// and keys that happen to be heavy and come last leave the chip idle behind them (C4, one batch:
// 81 % of wave slots busy on average, the last 0.9 ms of 5.4 at < 90 %).  An estimate from the
// event-only edge predicates: each record that a begin-stage consuming edge may take opens runs that
// every later record a consuming edge of another stage may take can double, so a segment weighs
// sum over its begin-matching records of 2^(later matching records) -- bucketed by log2 (16 buckets).
// On C4's per-key times this order gives a list-schedule makespan within 1 % of the true-cost order
// (4479 / 4452 us against 5275 us as the keys come; tools/c4_profile.py --save).
__device__ __forceinline__ bool stage_may_take(const Lane& l, int s) {
  const int ne = ST_NEDGES(l, s);
  for (int e = 0; e < ne; e++) {
    const int op = ST_OP(l, s, e);
    if (op != E_BEGIN && op != E_TAKE) continue;
    const int sl = ST_SL(l, s, e);
    if (ST_PRED(l, s, e) < 0 || sl < 0 || ((l.slm | l.sle) >> sl) & 1) return true;   // (not event-only: may)
  }
  return false;
}
// one thread per batch record: bit 0 a begin-stage consuming edge may take it, bit 1 one of another stage
__device__ __forceinline__ void nfa_order_bits_body(const NfaArgs& A, uint8_t* bits) {
  const int64_t g = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (g >= A.n) return;
  Lane l{};
  l.A = &A;
  l.P = A.P;
  l.g = g;
  eval_event_only(l);
  const int ns = KCEP_PROG(l).nstages, b = KCEP_PROG(l).begin;
  bool other = false;
  for (int s = 1; s < ns; s++)
    if (s != b && stage_may_take(l, s)) { other = true; break; }
  bits[g] = uint8_t((stage_may_take(l, b) ? 1 : 0) | (other ? 2 : 0));
}

// NFA.runs++ (NFA.java:297, :331).  Wave mode: a placeholder -(2 + k) for the lane's k-th increment;
// the wave numbers them in queue order after the round (nfa_wave.h wave_fix_seq)
template <bool W = false>
__device__ __forceinline__ int next_seq(Lane& l) {
  if constexpr (W) return -(2 + l.nph++);
  return ++l.runs;
}

// queues keep their capacity in runs; regrow works in words
__device__ __forceinline__ bool push_run(Lane& l, int32_t*& q, int32_t& cap_runs, int32_t& len, const Run& x) {
  if (len >= cap_runs) {
    int32_t capw = cap_runs * 4;
    if (!regrow(l, q, capw, int64_t(len) * 4, (int64_t(len) + 1) * 4, q == l.tq ? AK_PRIV : AK_QUEUE)) return false;
    cap_runs = capw / 4;
  }
  reinterpret_cast<int4*>(q)[len++] = make_int4(x.w0, x.ver, x.ev, x.seq);
  return true;
}
__device__ __forceinline__ bool push_t(Lane& l, const Run& x) { return push_run(l, l.tq, l.tq_cap, l.tlen, x); }

// One level of NFA.evaluate's PROCEED/SKIP_PROCEED recursion (ComputationContext).  16 bytes: the
// suspended parents sit in private memory (fr[], scratch), so their size is the kernel's scratch
// footprint (with a 44-byte frame C4's wave kernel wrote ~0.4-2.8 GB of scratch lines back to HBM per
// launch, depending on occupancy).  A context's stage, event and sequence are always the run's own
// (NFA.java:222-237 only sets the version), so a frame keeps the version and two flags of it.
constexpr uint32_t FR_NONE = 0xFF;     // prev stage: none (Stage.newEpsilonState(null, ...))
struct Frame {
  int32_t ver;                 // the context's ComputationStage version
  uint32_t st;                 // cur stage | cur epsilon target << 8 | prev stage << 16 | prev epsilon << 24
  uint32_t fl;                 // bits 0-3 matched edges not taken yet, 4 branching, 5 ignored, 6 consumed,
                               // 7 proceed, 8 / 9 the context stage's isBranching / isIgnored, 10-31 nbase
  int32_t before;              // tq length when the child context was entered
  __device__ __forceinline__ int cur_sid() const { return int(st & 0xFF); }
  __device__ __forceinline__ int cur_eps() const { return int((st >> 8) & 0xFF); }
  __device__ __forceinline__ int prev_sid() const { const uint32_t p = (st >> 16) & 0xFF; return p == FR_NONE ? -1 : int(p); }
  __device__ __forceinline__ int prev_eps() const { return int(st >> 24); }
  __device__ __forceinline__ bool flag(int b) const { return (fl >> b) & 1u; }
  __device__ __forceinline__ void set(int b) { fl |= 1u << b; }
  __device__ __forceinline__ int nbase() const { return int(fl >> 10); }
};
enum { FB_BRANCHING = 4, FB_IGNORED = 5, FB_CONSUMED = 6, FB_PROCEED = 7, FB_CBR = 8, FB_CIG = 9 };
constexpr int FR_MAX_NBASE = 1 << 22;
__device__ __forceinline__ uint32_t fr_st(int cur, int eps, int prev, int peps) {
  return uint32_t(cur) | (uint32_t(eps) << 8) | (uint32_t(prev < 0 ? FR_NONE : uint32_t(prev)) << 16) | (uint32_t(peps) << 24);
}
// the context's ComputationStage: the run's stage, epsilon target, event and sequence, the frame's version
__device__ __forceinline__ Run fr_cs(const Frame& f, const Run& run) {
  return mk_run(r_sid(run), r_eps(run), f.ver, run.ev, run.seq, f.flag(FB_CBR), f.flag(FB_CIG));
}

// frame entry: matchEdgesAndGet (NFA.java:371-384) + isBranching (:392-397); keeps f's stage, version
// and context flags, resets the rest
template <bool W>
__device__ __forceinline__ bool frame_enter(Lane& l, Frame& f, const Run& run) {
  if (l.tlen >= FR_MAX_NBASE) { l.overflow = 1; return false; }
  f.fl = (f.fl & ((1u << FB_CBR) | (1u << FB_CIG))) | (uint32_t(l.tlen) << 10);
  uint32_t has = 0, rem = 0;
  const int cur = f.cur_sid(), ceps = f.cur_eps();
  const bool eps = ceps != EPS_NONE;
  const int ne = eps ? 1 : ST_NEDGES(l, cur);
  for (int e = 0; e < ne; e++) {
    const int op = eps ? E_PROCEED : ST_OP(l, cur, e);
    const int pc = eps ? -1 : ST_PRED(l, cur, e);
    bool ok = true;
    if (pc >= 0) {
      const int sl = ST_SL(l, cur, e);
      if (sl >= 0 && !((l.sle >> sl) & 1)) {
        ok = (l.slm >> sl) & 1;
      } else {
        Ctx c{run.seq, f.prev_sid(), run.ev, f.ver, false, 0, 0};
        int64_t v;
        KPH_BEGIN(l, 1);
        const bool good = run_code<W>(l, pc, c, v);
        KPH_END(l, 1);
        if (!good) return false;
        ok = v != 0;
      }
    }
    if (ok) { rem |= 1u << e; has |= 1u << op; }
  }
  auto H = [&](int o) { return (has >> o) & 1u; };
  const bool branching = (H(E_PROCEED) && H(E_TAKE)) || (H(E_IGNORE) && H(E_TAKE)) || (H(E_IGNORE) && H(E_BEGIN)) ||
                         (H(E_IGNORE) && H(E_PROCEED));
  f.fl |= rem | (uint32_t(branching) << FB_BRANCHING) | (uint32_t(H(E_IGNORE)) << FB_IGNORED);
  return true;
}

// NFA.evaluate (NFA.java:190-341) for one run; results appended to tq.  W: the wave kernel's parallel
// pass (logged buffer operations, shared heap, run-counter placeholders)
template <bool W = false>
__device__ __forceinline__ bool evaluate(Lane& l, const Run& run, Frame* fr) {
  // the current frame lives in registers; fr[] (scratch) holds only the suspended parents
  int d = 0;
  Frame f;
  f.ver = run.ver;
  f.st = fr_st(r_sid(run), r_eps(run), -1, EPS_NONE);
  f.fl = (uint32_t(r_br(run)) << FB_CBR) | (uint32_t(r_ig(run)) << FB_CIG);
  f.before = 0;
  if (!frame_enter<W>(l, f, run)) return false;
  for (;;) {
    if (f.fl & 0xFu) {                                               // the next matched edge, in edge order
      const int e = __builtin_ctz(f.fl & 0xFu);
      f.fl &= ~(1u << e);
      const int cur = f.cur_sid(), ceps = f.cur_eps();
      const bool eps = ceps != EPS_NONE;
      const int op = eps ? E_PROCEED : ST_OP(l, cur, e);
      const int target = eps ? ceps : ST_TARGET(l, cur, e);
      const int ver = f.ver, seq = run.seq;
      if (op == E_PROCEED || op == E_SKIP_PROCEED) {                 // :222-237
        if (d + 1 >= MAXD) { l.overflow = 1; return false; }
        Frame g;
        g.ver = f.ver;
        g.fl = f.fl & ((1u << FB_CBR) | (1u << FB_CIG));
        if (ST_NAME(l, target) != ST_NAME(l, cur) && !f.flag(FB_CBR) && !f.flag(FB_CIG)) {   // isForwardingToNextStage :343-349
          const int nv = dw_add_stage<W>(l, ver);
          if (nv < 0) return false;
          g.ver = nv;                                                // setVersion (a fresh stage: flags clear)
          g.fl = 0;
        }
        g.st = op == E_SKIP_PROCEED ? fr_st(target, EPS_NONE, f.prev_sid(), f.prev_eps())
                                    : fr_st(target, EPS_NONE, cur, ceps);
        g.before = 0;
        f.before = l.tlen;
        fr[d++] = f;                                                  // suspend the parent
        f = g;
        if (!frame_enter<W>(l, f, run)) return false;
        continue;
      }
      const int prev = f.prev_sid();
      if (op == E_TAKE) {                                            // :238-255
        if (!push_t(l, mk_run(cur, cur, ver, l.r, seq, false, false))) return false;
        int pv = ver;
        if (!(!f.flag(FB_BRANCHING) || f.flag(FB_IGNORED))) { pv = dw_add_run<W>(l, ver, 1); if (pv < 0) return false; }
        KPH_BEGIN(l, 2);
        if (prev >= 0) buf_put5<W>(l, cur, l.r, prev, run.ev, pv);
        else buf_put3<W>(l, cur, l.r, pv);
        KPH_END(l, 2);
        if (l.err || l.overflow) return false;
        f.set(FB_CONSUMED);
      } else if (op == E_BEGIN) {                                    // :256-271
        KPH_BEGIN(l, 2);
        if (prev >= 0) buf_put5<W>(l, cur, l.r, prev, run.ev, ver);
        else buf_put3<W>(l, cur, l.r, ver);
        KPH_END(l, 2);
        if (l.err || l.overflow) return false;
        if (!push_t(l, mk_run(cur, target, ver, l.r, seq, false, false))) return false;
        f.set(FB_CONSUMED);
      } else if (op == E_IGNORE) {                                   // :272-285
        if (!f.flag(FB_BRANCHING) && !push_t(l, mk_run(r_sid(run), r_eps(run), f.ver, run.ev, run.seq, false, true)))
          return false;
      }
      continue;
    }
    // ---- after the edge loop ----
    const int ver = f.ver, seq = run.seq, pev = run.ev;
    const int cur = f.cur_sid(), prev = f.prev_sid();
    const bool consumed = f.flag(FB_CONSUMED);
    if (f.flag(FB_BRANCHING)) {                                      // :289-317
      if (consumed) {
        const int nseq = next_seq<W>(l);
        const int last = f.flag(FB_IGNORED) ? pev : l.r;
        if (prev < 0) { l.err = CEP_E_NPE; return false; }           // Stage.newEpsilonState(null, ...)
        const bool pb = is_begin(l, prev);
        const int nv = dw_add_run<W>(l, ver, pb ? 2 : 1);
        if (nv < 0) return false;
        if (!push_t(l, mk_run(prev, cur, nv, last, nseq, true, false))) return false;
        for (int k = 0; k < KCEP_PROG(l).ndefined; k++) {                    // AggregatesStoreImpl.branch
          const int st = KCEP_PROG(l).defined[k];
          int32_t t;
          int64_t v;
          if (!agg_read<W>(l, st, seq, t, v)) return false;
          if (t && !agg_write<W>(l, st, nseq, t, v)) return false;           // (a new sequence's row is null)
        }
        if (!pb) {
          KPH_BEGIN(l, 2);
          buf_branch<W>(l, prev, pev, ver);
          KPH_END(l, 2);
          if (l.err) return false;
        }
      } else if (!f.flag(FB_PROCEED)) {
        if (!push_t(l, fr_cs(f, run))) return false;
      }
    }
    if (consumed && f.cur_eps() == EPS_NONE && ST_NFOLDS(l, cur) > 0) {   // evaluateAggregates :319-321, :362-369
      const DevStage& s = stg(l, cur);
      for (int k = 0; k < s.nfolds; k++) {
        int32_t ct;
        int64_t cv;
        if (!agg_read<W>(l, s.fold_state[k], seq, ct, cv)) return false;
        Ctx c{seq, -1, -1, ver, true, ct, cv};
        int64_t v;
        if (!run_code<W>(l, s.fold_code[k], c, v)) return false;
        if (!agg_write<W>(l, s.fold_state[k], seq, s.fold_type[k], v)) return false;
        l.ov_own = 1;
      }
    }
    const int csid = r_sid(run), ceps = r_eps(run);
    if (is_begin(l, csid) && !is_forwarding(l, csid, ceps)) {         // begin re-add :323-338
      if (consumed) {
        const int nseq = next_seq<W>(l);
        int nv = ver;
        if (l.tlen != f.nbase()) { nv = dw_add_run<W>(l, ver, 1); if (nv < 0) return false; }
        if (!push_t(l, mk_run(csid, ceps, nv, -1, nseq, false, false))) return false;
      } else {
        if (!push_t(l, fr_cs(f, run))) return false;
      }
    }
    if (d == 0) return true;
    f = fr[--d];                                                      // resume the parent
    if (l.tlen > f.before) f.set(FB_PROCEED);                         // its child produced runs
  }
}

// room for the longest buffer walk: it visits strictly earlier events, so at
// most one node per event of the key
__device__ __forceinline__ bool reserve_walk(Lane& l) {
  if (l.out_top + 4 > l.outcap && !regrow(l, l.out, l.outcap, l.out_top, int64_t(l.out_top) + 4, AK_OUT))
    return false;
  const int need_ent = 3 * (l.etop + l.nev);
  if (need_ent > l.ecap && !regrow(l, l.oent, l.ecap, int64_t(3) * l.etop, need_ent, AK_OUT)) return false;
  const int need_heap = 2 * l.nev + 2;
  if (l.heap_top + need_heap > l.heapcap &&
      !regrow(l, l.heap, l.heapcap, l.heap_top, int64_t(l.heap_top) + need_heap, AK_HEAP))
    return false;
  return true;
}

// matchConstruction of one final run: remove + Sequence entries (:151-158);
// the walk's (slot, event) pairs go to scratch at the heap top first
__device__ __forceinline__ bool emit_match(Lane& l, const Run& y) {
  if (!reserve_walk(l)) return false;
  int32_t* tmp = l.heap + l.heap_top;
  const int cnt = buf_peek(l, r_sid(y), y.ev, y.ver, true, tmp, l.nev + 1);
  if (cnt < 0) return false;
  int32_t* o = l.out + l.out_top;
  const int64_t pos = a_pos(*l.A, l.g);
  o[0] = int32_t(uint32_t(uint64_t(pos)));
  o[1] = int32_t(uint32_t(uint64_t(pos) >> 32));
  o[2] = cnt;
  o[3] = l.etop;
  int32_t* en = l.oent + int64_t(3) * l.etop;
  for (int i = 0; i < cnt; i++) {
    const int64_t q = ev_pos(l, tmp[2 * i + 1]);
    en[3 * i] = SLOT_NAME(l, tmp[2 * i]);
    en[3 * i + 1] = int32_t(uint32_t(uint64_t(q)));
    en[3 * i + 2] = int32_t(uint32_t(uint64_t(q) >> 32));
  }
  l.out_top += 4;
  l.etop += cnt;
  l.nmatch++;
  return true;
}

// NFA.matchPattern(Event) (NFA.java:134-149) for local event r
__device__ __forceinline__ bool step(Lane& l, Frame* fr) {
  const int n = l.qlen;
  int qn = 0;
  l.flen = 0;
  for (int i = 0; i < n; i++) {
    const int4 x = reinterpret_cast<int4*>(l.qa)[i];
    Run run{x.x, x.y, x.z, x.w};
    l.tlen = 0;
    // window check (:179-188): every non-begin run sits on an epsilon stage
    // whose window is -1, so it never prunes; nothing to evaluate.
    KPH_BEGIN(l, 0);
    const bool good = evaluate(l, run, fr);
    KPH_END(l, 0);
    if (!good) return false;
    if (l.tlen == 0) {                                               // removePattern :160-163
      KPH_BEGIN(l, 3);
      const int rm = buf_peek(l, r_sid(run), run.ev, run.ver, true, nullptr, 0);
      KPH_END(l, 3);
      if (rm < 0) return false;
    }
    for (int t = 0; t < l.tlen; t++) {
      const int4 y = reinterpret_cast<int4*>(l.tq)[t];
      const Run u{y.x, y.y, y.z, y.w};
      if (is_fwd_final(l, r_sid(u), r_eps(u))) {
        if (!push_run(l, l.fq, l.fq_cap, l.flen, u)) return false;
      } else {
        if (!push_run(l, l.qb, l.qb_cap, qn, u)) return false;
      }
    }
  }
  int32_t* tmp = l.qa;                                              // swap queues
  l.qa = l.qb;
  l.qb = tmp;
  const int32_t tc = l.qa_cap;
  l.qa_cap = l.qb_cap;
  l.qb_cap = tc;
  l.qlen = qn;
  for (int k = 0; k < l.flen; k++) {                                // matchConstruction :151-158
    const int4 y = reinterpret_cast<int4*>(l.fq)[k];
    KPH_BEGIN(l, 4);
    const bool good = emit_match(l, Run{y.x, y.y, y.z, y.w});
    KPH_END(l, 4);
    if (!good) return false;
  }
  return true;
}

// ---- carried state: import / export (CEP_SESSION_CARRY) ----
__device__ __forceinline__ int hwm_find(const Lane& l, int32_t tp) {
  int h = 0;
  while (h < l.nhwm && l.hwm[3 * h] != tp) h++;
  return h;
}

__device__ __forceinline__ bool import_state(Lane& l, const int32_t* b) {
  const auto& P = KCEP_PROG(l);
  l.nhwm = b[CB_NHWM];
  const int qlen = b[CB_QLEN], nnode = b[CB_NNODE], npred = b[CB_NPRED], nver = b[CB_NVER], nseq = b[CB_NSEQ];
  const int ncols = b[CB_NCOLS], nst = b[CB_NSTATES];
  const int32_t* p = b + CB_HDR;
  for (int i = 0; i < 3 * l.nhwm; i++) l.hwm[i] = p[i];
  p += 3 * l.nhwm;
  const int32_t* q = p;
  p += 4 * qlen;
  p += int64_t(carry_evw(ncols)) * l.C;                             // events: read in place (l.cev)
  const int32_t* nd = p;
  p += 4 * nnode;
  const int32_t* pr = p;
  p += 4 * npred;
  const int32_t* vs = p;
  p += nver;
  const int32_t* ag = p;
  // heap: versions at [0, nver), predecessors after them
  const int PB = nver;
  if (PB + PW * npred > l.heapcap && !regrow(l, l.heap, l.heapcap, 0, int64_t(PB) + PW * npred + 64, AK_HEAP)) return false;
  for (int i = 0; i < nver; i++) l.heap[i] = vs[i];
  for (int i = 0; i < npred; i++) {
    int32_t* h = l.heap + PB + PW * i;
    const int v = pr[4 * i];
    h[0] = v; h[1] = pr[4 * i + 1]; h[2] = pr[4 * i + 2];
    h[3] = pr[4 * i + 3] >= 0 ? PB + PW * pr[4 * i + 3] : -1;
    h[4] = l.heap[v]; h[5] = l.heap[v + 1];
  }
  l.heap_top = PB + PW * npred;
  for (int e = 0; e < l.C; e++)
    for (int s = 0; s < P.nslots; s++) { int32_t* x = node(l, s, e); x[0] = 0; x[1] = -1; x[2] = -1; x[3] = 0; }
  for (int i = 0; i < nnode; i++) {
    int32_t* x = node(l, nd[4 * i], nd[4 * i + 1]);
    x[0] = nd[4 * i + 2];
    x[1] = nd[4 * i + 3] >= 0 ? PB + PW * nd[4 * i + 3] : -1;
    int t = x[1];
    while (t >= 0 && l.heap[t + 3] >= 0) t = l.heap[t + 3];
    x[2] = t;
    x[3] = NF_EXISTS;
  }
  if (qlen > l.qa_cap) {
    int32_t capw = l.qa_cap * 4;
    if (!regrow(l, l.qa, capw, 0, int64_t(qlen) * 4, AK_QUEUE)) return false;
    l.qa_cap = capw / 4;
  }
  for (int i = 0; i < 4 * qlen; i++) l.qa[i] = q[i];
  l.qlen = qlen;
  if (nst != P.nstates) { l.err = CEP_E_ARG; return false; }
  if (nseq > 0 && nst > 0) {
    if (!agg(l, 0, nseq - 1)) return false;
    for (int64_t i = 0; i < int64_t(3) * nst * nseq; i++) l.aggs[i] = ag[i];
  }
  l.runs = nseq > 0 ? nseq - 1 : 0;
  l.runs_delta = cw64(b + CB_RUNS_LO) - l.runs;
  return true;
}

__device__ __forceinline__ void copy_version(const Lane& l, int v, int32_t* dst) {
  const int len = l.heap[v];
  for (int i = 0; i <= len; i++) dst[i] = l.heap[v + i];
}

// Compacts the key's state into a blob in the carry pool; returns its offset or -1.
__device__ __forceinline__ int64_t export_state(Lane& l) {
  const auto& P = KCEP_PROG(l);
  const int ns = P.nslots;
  // (1) nodes the queue can reach: roots are the runs' (stage, last event) nodes;
  // predecessor pointers always point to earlier events, so one descending pass closes the set
  for (int i = 0; i < l.qlen; i++) {
    const int ev = l.qa[4 * i + 2];
    if (ev >= 0) {
      int32_t* x = node(l, slot_of(l, l.qa[4 * i] & 0xFF), ev);
      x[3] |= NF_NEED | (exists(x) ? NF_MARK : 0);
    }
  }
  int nnode = 0, npred = 0, nver = 0;
  for (int e = l.nev - 1; e >= 0; e--)
    for (int s = 0; s < ns; s++) {
      int32_t* x = node(l, s, e);
      if (!(x[3] & NF_MARK)) continue;
      nnode++;
      for (int p = x[1]; p >= 0; p = l.heap[p + 3]) {
        npred++;
        nver += l.heap[l.heap[p]] + 1;
        if (l.heap[p + 1] >= 0) {
          int32_t* t = node(l, l.heap[p + 1], l.heap[p + 2]);
          t[3] |= NF_NEED | (exists(t) ? NF_MARK : 0);
        }
      }
    }
  // (2) carried events: every event a run or a carried pointer names
  int32_t* evmap = nullptr;
  {
    int32_t capw = l.tq_cap * 4;
    if (capw < l.nev) {
      if (!regrow(l, l.tq, capw, 0, l.nev, AK_OTHER)) return -1;
      l.tq_cap = capw / 4;
    }
    evmap = l.tq;
  }
  int nev = 0;
  for (int e = 0; e < l.nev; e++) {
    bool need = false;
    for (int s = 0; s < ns && !need; s++) need = node(l, s, e)[3] & NF_NEED;
    evmap[e] = need ? nev++ : -1;
  }
  // (3) live run sequences (runs may share one: they share its aggregates)
  const int nst = P.nstates;
  int nseq = 0;
  int32_t* seqmap = l.fq;                                           // qlen entries: new id of run i's seq
  if (l.fq_cap < l.qlen) {
    int32_t capw = l.fq_cap * 4;
    if (!regrow(l, l.fq, capw, 0, int64_t(l.qlen) * 4, AK_OTHER)) return -1;
    l.fq_cap = capw / 4;
    seqmap = l.fq;
  }
  for (int i = 0; i < l.qlen; i++) {
    const int sq = l.qa[4 * i + 3];
    int id = -1;
    for (int j = 0; j < i && id < 0; j++)
      if (l.qa[4 * j + 3] == sq) id = seqmap[j];
    seqmap[i] = id >= 0 ? id : nseq++;
    nver += l.heap[l.qa[4 * i + 1]] + 1;
  }
  const int evw = carry_evw(P.ncols);
  const int64_t words = CB_HDR + 3 * l.nhwm + 4 * l.qlen + int64_t(evw) * nev + 4 * nnode + 4 * npred + nver +
                        int64_t(3) * nst * nseq;
  const unsigned long long at = atomicAdd(l.A->cpool_top, (unsigned long long)words);
  if (at + (unsigned long long)words > (unsigned long long)l.A->cpool_cap) {
    atomicAdd(&l.A->flags[1], 1);
    return -1;
  }
  int32_t* b = l.A->cpool + at;
  const int64_t real_runs = int64_t(l.runs) + l.runs_delta;
  b[CB_WORDS] = int32_t(words);
  b[CB_RUNS_LO] = int32_t(uint32_t(uint64_t(real_runs)));
  b[CB_RUNS_HI] = int32_t(uint32_t(uint64_t(real_runs) >> 32));
  b[CB_NHWM] = l.nhwm; b[CB_QLEN] = l.qlen; b[CB_NEV] = nev; b[CB_NNODE] = nnode; b[CB_NPRED] = npred;
  b[CB_NVER] = nver; b[CB_NSEQ] = nseq; b[CB_NCOLS] = P.ncols; b[CB_NSTATES] = nst;
  int32_t* p = b + CB_HDR;
  for (int i = 0; i < 3 * l.nhwm; i++) p[i] = l.hwm[i];
  p += 3 * l.nhwm;
  int32_t* qo = p;
  p += 4 * l.qlen;
  int32_t* evo = p;
  p += int64_t(evw) * nev;
  int32_t* ndo = p;
  p += 4 * nnode;
  int32_t* pro = p;
  p += 4 * npred;
  int32_t* vo = p;
  p += nver;
  int32_t* ago = p;
  int vtop = 0;
  for (int i = 0; i < l.qlen; i++) {
    qo[4 * i] = l.qa[4 * i];
    copy_version(l, l.qa[4 * i + 1], vo + vtop);
    qo[4 * i + 1] = vtop;
    vtop += vo[vtop] + 1;
    const int ev = l.qa[4 * i + 2];
    qo[4 * i + 2] = ev >= 0 ? evmap[ev] : -1;
    qo[4 * i + 3] = seqmap[i];
  }
  for (int e = 0; e < l.nev; e++) {
    if (evmap[e] < 0) continue;
    int32_t* o = evo + int64_t(evw) * evmap[e];
    const int64_t pos = ev_pos(l, e), off = ev_off(l, e), ts = ev_ts(l, e);
    o[0] = int32_t(uint32_t(uint64_t(pos))); o[1] = int32_t(uint32_t(uint64_t(pos) >> 32));
    o[2] = ev_topic(l, e); o[3] = ev_part(l, e);
    o[4] = int32_t(uint32_t(uint64_t(off))); o[5] = int32_t(uint32_t(uint64_t(off) >> 32));
    o[6] = int32_t(uint32_t(uint64_t(ts))); o[7] = int32_t(uint32_t(uint64_t(ts) >> 32));
    for (int c = 0; c < P.ncols; c++) {
      const int64_t v = ev_field(l, c, P.coltype[c], e);
      o[8 + 2 * c] = int32_t(uint32_t(uint64_t(v)));
      o[9 + 2 * c] = int32_t(uint32_t(uint64_t(v) >> 32));
    }
  }
  int ni = 0, pi = 0;
  for (int e = 0; e < l.nev; e++)
    for (int s = 0; s < ns; s++) {
      int32_t* x = node(l, s, e);
      if (!(x[3] & NF_MARK)) continue;
      ndo[4 * ni] = s; ndo[4 * ni + 1] = evmap[e]; ndo[4 * ni + 2] = x[0];
      ndo[4 * ni + 3] = x[1] >= 0 ? pi : -1;
      ni++;
      for (int q = x[1]; q >= 0; q = l.heap[q + 3]) {
        copy_version(l, l.heap[q], vo + vtop);
        pro[4 * pi] = vtop;
        vtop += vo[vtop] + 1;
        pro[4 * pi + 1] = l.heap[q + 1];
        pro[4 * pi + 2] = l.heap[q + 1] >= 0 ? evmap[l.heap[q + 2]] : 0;
        pro[4 * pi + 3] = l.heap[q + 3] >= 0 ? pi + 1 : -1;
        pi++;
      }
    }
  for (int i = 0; i < l.qlen; i++) {                                // one aggregate row per live sequence
    const int id = seqmap[i];
    bool first = true;
    for (int j = 0; j < i && first; j++) first = seqmap[j] != id;
    if (!first || nst == 0) continue;
    const int sq = l.qa[4 * i + 3];
    for (int s = 0; s < nst; s++) {
      const int32_t* a = sq < l.seqcap ? l.aggs + (int64_t(sq) * nst + s) * 3 : nullptr;
      int32_t* o = ago + (int64_t(id) * nst + s) * 3;
      o[0] = a ? a[0] : 0; o[1] = a ? a[1] : 0; o[2] = a ? a[2] : 0;
    }
  }
  return int64_t(at);
}

// Per-key setup shared by the lane kernel and the wave kernel (nfa_wave.h): workspace from the
// pool, carried state (NFAStoreImpl.find, CEPProcessor.loadNFA :111-124) or NFA.build.  Returns
// false if the key has nothing to run (its result words are then final).
// arena (wave kernel): LDS words for the key's hot workspace (hwm, nodes, queues, aggregates, heap);
// used when they fit, the match output stays in the pool (the compaction reads it after the kernel).
// Arrays that outgrow it are re-allocated like any other (generic pointers throughout): from the
// wave's scratch region (ka, wave kernel) or the pool.
__device__ __forceinline__ bool key_begin(Lane& l, const NfaArgs& A, int seg, int32_t* arena = nullptr,
                                         int64_t arena_words = 0, KeyAlloc* ka = nullptr) {
  l.A = &A;
  l.P = A.P;
  l.pool_words = 0;
  const auto& P = KCEP_PROG(l);
  l.seg0 = A.seg_start[seg];
  l.L = int32_t(A.seg_start[seg + 1] - l.seg0);
  l.g = l.seg0;
  l.wtop = nullptr; l.log = nullptr; l.log_cap = 0; l.log_n = 0; l.nph = 0; l.wgrow = 0;
  l.wpool = ka;
  l.cap_hit = 0;
  l.rec_etop = 0;
  l.rec_nmatch = 0;
  l.err = 0; l.overflow = 0; l.nmatch = 0; l.flen = 0; l.tlen = 0; l.qlen = 0;
  l.nhwm = 0; l.runs = 1; l.runs_delta = 0; l.slm = 0; l.sle = 0;
  l.C = 0; l.cev = nullptr;
  l.evw = carry_evw(P.ncols);
  A.res_matches[seg] = 0;
  A.res_words[seg] = 0;
  A.res_out[seg] = 0;
  A.res_ent[seg] = 0;
  A.res_err[seg] = 0;
  A.res_err_rec[seg] = -1;
  if (A.carry) A.res_carry[seg] = -1;
  const int32_t* blob = nullptr;
  if (A.carry) {
    const int32_t k = A.key[l.seg0];
    if (k < 0 || k >= A.max_keys) { atomicAdd(&A.flags[2], 1); return false; }
    const int64_t bo = A.ctab[k];
    if (bo >= 0) {
      blob = A.cpool + bo;
      l.C = blob[CB_NEV];
      l.cev = blob + CB_HDR + 3 * blob[CB_NHWM] + 4 * blob[CB_QLEN];
    }
  }
  l.nev = l.C + l.L;
  // workspace: hwm | nodes | 4 queues | aggregates | heap | output
  const int ns = P.nslots, nst = P.nstates;
  l.qa_cap = l.qb_cap = l.tq_cap = l.fq_cap = A.cap.q0;
  l.seqcap = A.cap.seq_base + l.L + (blob ? blob[CB_NSEQ] : 0);
  l.heapcap = A.cap.heap_base + A.cap.heap_mult * l.nev;
  l.outcap = 4 * (4 + l.L);                                             // match headers (grown on demand)
  l.ecap = A.cap.out_base + A.cap.out_mult * l.L;                        // their entries
  const int64_t fixed = 3 * HWM_MAX + int64_t(NW) * ns * l.nev + 16 * int64_t(A.cap.q0) +
                        int64_t(3) * nst * l.seqcap + l.heapcap;
  const bool in_lds = arena && fixed <= arena_words;
  l.arena_used = in_lds ? int32_t(fixed) : -1;
  int32_t* p = in_lds ? arena : pool_alloc(l, fixed, AK_WS);
  int32_t* out_at = p ? pool_alloc(l, l.outcap + l.ecap, AK_OUT, true) : nullptr;   // headers, then entries
  if (!p || !out_at) {
    if (A.last_attempt || l.cap_hit) {                                 // handed back per key
      A.res_err[seg] = CEP_E_RUN_CAPACITY;
      A.res_err_rec[seg] = a_pos(A, l.seg0);
      atomicOr(A.err_any, 1ull);                                       // the host reads res_err only then
    } else {
      atomicAdd(&A.flags[0], 1);
    }
    return false;
  }
  l.hwm = p; p += 3 * HWM_MAX;
  l.nodes = p; p += int64_t(NW) * ns * l.nev;
  l.qa = p; p += 4 * A.cap.q0;
  l.qb = p; p += 4 * A.cap.q0;
  l.tq = p; p += 4 * A.cap.q0;
  l.fq = p; p += 4 * A.cap.q0;
  l.aggs = p; p += int64_t(3) * nst * l.seqcap;
  l.heap = p;
  l.out = out_at;
  l.oent = out_at + l.outcap;
  l.heap_top = 0; l.out_top = 0; l.etop = 0;
  for (int64_t i = 0; i < int64_t(3) * nst * l.seqcap; i++) l.aggs[i] = 0;   // all states null
  if (blob) {
    if (!import_state(l, blob)) {
      if (l.overflow && (A.last_attempt || l.cap_hit)) {
        A.res_err[seg] = CEP_E_RUN_CAPACITY;
        A.res_err_rec[seg] = a_pos(A, l.seg0);
        atomicOr(A.err_any, 1ull);
        return false;
      }
      if (l.overflow) atomicAdd(&A.flags[0], 1);
      A.res_err[seg] = l.err;
      if (l.err) {
        A.res_err_rec[seg] = a_pos(A, l.seg0);
        atomicOr(A.err_any, 1ull);
      }
      return false;
    }
  } else {
    // NFA.build (NFA.java:73-79), Stages.initialComputationStage (Stages.java:53-60)
    const int v0 = heap_alloc(l, 2);
    l.heap[v0] = 1;
    l.heap[v0 + 1] = 1;
    reinterpret_cast<int4*>(l.qa)[0] = make_int4(P.begin | (EPS_NONE << 8), v0, -1, 1);
    l.qlen = 1;
    l.runs = 1;
  }
  return true;
}

// CEPProcessor's record filters before the step (:136-138 null key/value, :152-160 high-water
// mark); false: the record is dropped
__device__ __forceinline__ bool record_admitted(const Lane& l, int64_t g) {
  if (l.A->valid && !l.A->valid[g]) return false;
  const int h = hwm_find(l, b_topic(l, g));
  return !(h < l.nhwm && b_off(l, g) < cw64(l.hwm + 3 * h + 1));
}
// the high-water mark after a processed record; false: too many topics for one key
__device__ __forceinline__ bool record_hwm(Lane& l, int64_t g) {
  const int h = hwm_find(l, b_topic(l, g));
  if (h == l.nhwm) {
    if (l.nhwm == HWM_MAX) return false;
    l.nhwm++;
    l.hwm[3 * h] = b_topic(l, g);
  }
  const int64_t hw = b_off(l, g) + 1;
  l.hwm[3 * h + 1] = int32_t(uint32_t(uint64_t(hw)));
  l.hwm[3 * h + 2] = int32_t(uint32_t(uint64_t(hw) >> 32));
  return true;
}

// Per-key results: carried state (NFAStoreImpl.put :144-147), profile, the capacity hand-off,
// match counts.
// prof (profiling wave kernels): the key's allocator with its phase clocks and allocation counts
__device__ __forceinline__ void key_end(Lane& l, const NfaArgs& A, int seg, int64_t err_rec, int32_t live_max,
                                        int64_t evals, uint64_t t0, const KeyAlloc* prof = nullptr) {
  if (A.carry && !l.err && !l.overflow) {
    const int64_t at = export_state(l);
    if (at >= 0) A.res_carry[seg] = at;
  }
  atomicMax(&A.flags[3], live_max);
  if (A.profile) {
    int64_t* pr = A.profile + NFA_PROFILE_W * int64_t(seg);
    pr[0] = live_max;
    pr[1] = evals;
    pr[2] = int64_t(wall_clock64() - t0);
#if defined(KCEP_PHASES_LANE)
    for (int i = 0; i < 11; i++) pr[3 + i] = int64_t(l.ph[i]);
#elif defined(KCEP_PHASES)
    for (int i = 0; i < 11; i++) pr[3 + i] = prof ? int64_t(prof->ph[i]) : -1;
#else
    for (int i = 0; i < 11; i++) pr[3 + i] = -1;
#endif
    pr[14] = int64_t(t0);                                                // start (wall clock, 100 MHz)
    pr[15] = l.pool_words;
#ifdef KCEP_PHASES
    for (int i = 0; i <= AK_N; i++) pr[16 + i] = prof ? int64_t(prof->kw[i]) : -1;   // words per kind, the pool's share
#else
    for (int i = 0; i <= AK_N; i++) pr[16 + i] = -1;
#endif
  }
  if (l.overflow && (A.last_attempt || l.cap_hit)) {
    // over capacity: the key stops at this record and is handed back (CEP_E_RUN_CAPACITY); the
    // matches of its earlier records stand, like the records before a reference exception
    A.res_err[seg] = CEP_E_RUN_CAPACITY;
    A.res_err_rec[seg] = a_pos(A, l.g);
    l.overflow = 0;
    if (l.nmatch > l.rec_nmatch) {                                     // none of the failing record's
      l.nmatch = l.rec_nmatch;                                         // matches is emitted
      l.out_top = int32_t(4 * l.nmatch);
      l.etop = l.rec_etop;
    }
  } else {
    A.res_err[seg] = l.overflow ? 0 : l.err;
    A.res_err_rec[seg] = l.overflow ? -1 : err_rec;
  }
  if (l.overflow) atomicAdd(&A.flags[0], 1);
  if (A.res_err[seg]) atomicOr(A.err_any, 1ull);
  A.res_matches[seg] = l.nmatch;
  A.res_words[seg] = l.etop;                                           // entries
  A.res_out[seg] = int64_t(reinterpret_cast<uintptr_t>(l.out));
  A.res_ent[seg] = int64_t(reinterpret_cast<uintptr_t>(l.oent));
}

// One lane runs one key segment (A.spread segments per wave).
__device__ __forceinline__ void nfa_kernel_body(const NfaArgs& A) {
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  const int seg = (gid >> 6) * A.spread + (gid & 63);
  if ((gid & 63) >= A.spread || seg >= A.nseg) return;
  Lane l;
  if (!key_begin(l, A, seg)) return;
  const auto& P = KCEP_PROG(l);
  const int ns = P.nslots;
  Frame fr[MAXD];
  int64_t err_rec = -1;
  const bool proc = A.mode == CEP_MODE_PROCESSOR;
#ifdef KCEP_PHASES_LANE
  for (int i = 0; i < 11; i++) l.ph[i] = 0;
#endif
  int32_t live_max = l.qlen;                                         // live-run high-water mark of the key
  int64_t evals = 0;
  const uint64_t t0 = A.profile ? wall_clock64() : 0;
  for (int i = 0; i < l.L && !l.err && !l.overflow; i++) {
    const int r = l.C + i;
    const int64_t g = l.seg0 + i;
    l.r = r;
    l.g = g;
    for (int s = 0; s < ns; s++) { int32_t* nd = node(l, s, r); nd[0] = 0; nd[1] = -1; nd[2] = -1; nd[3] = 0; }
    if (proc) {
      if (!record_admitted(l, g)) continue;
      for (int k = 0; k < l.qlen; k++) l.qa[4 * k] &= ~(1 << 17);      // isIgnored not serialised (Q3)
    }
    eval_event_only(l);
    evals += l.qlen;
    l.rec_etop = l.etop;
    l.rec_nmatch = l.nmatch;
    if (!step(l, fr)) {
      if (l.err) err_rec = a_pos(A, g);
      break;
    }
    live_max = l.qlen > live_max ? l.qlen : live_max;
    if (proc && !record_hwm(l, g)) { l.overflow = 1; break; }
  }
  key_end(l, A, seg, err_rec, live_max, evals, t0);
}

}  // namespace kcep

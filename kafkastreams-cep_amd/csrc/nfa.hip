// nfa.hip — general NFA path: the full reference semantics on the GPU.
//
// One lane runs the NFA of one record key over that key's records in arrival
// order (per-key NFAs share nothing: buffer nodes are keyed by
// (stage, topic, partition, offset), aggregates by (key, state, run), the run
// counter is per key — SURVEY §8(e)).  Everything the reference keeps in its
// three state stores lives in a per-key arena in HBM:
//
//   run queues   ComputationStage (nfa/ComputationStage.java:30-185), 4 words:
//                stage id | epsilon target | isBranching | isIgnored, Dewey
//                version handle, last event, run sequence
//   heap         immutable DeweyVersions [len, digits...] (nfa/DeweyVersion.java)
//                and predecessor pointers {version, slot, event, next}
//                (state/internal/MatchedEvent.java:124-168)
//   nodes        dense [slot][event] -> {refs, first predecessor, exists}:
//                the shared versioned buffer (SharedVersionedBufferStoreImpl.java)
//                with slot = (stage name, stage type) as in Matched.java:31-35
//   aggregates   dense [state][run sequence] -> {boxed type, value}
//                (AggregatesStoreImpl.java:55-75)
//   output       per match: emitting record, traversal length, then
//                (stage name, event) pairs, final stage first
//
// The step follows NFA.matchPattern / evaluate (nfa/NFA.java:134-341) with the
// recursion on PROCEED/SKIP_PROCEED edges unrolled onto an explicit frame
// stack; the buffer operations follow put/branch/peek of
// SharedVersionedBufferStoreImpl.java:101-201 including the copy-on-read
// refcount semantics (decrements persist only at zero, deleted nodes can be
// resurrected).  Predicates and folds run the bytecode of compile.cpp.
//
// A key that outgrows its arena sets an overflow flag and stops; the host
// re-runs exactly those keys with a larger arena (still on the GPU).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/kcep.h"
#include "kcep_internal.h"

namespace kcep {



__host__ __device__ inline void nfa_layout(const NfaCaps& c, int nslots, int nstates, int64_t L, int64_t& qcap,
                                           int64_t& seqcap, int64_t& heapcap, int64_t& outcap, int64_t& words) {
  qcap = c.q_base + c.q_mult * L;
  seqcap = c.seq_base + c.seq_mult * L;
  heapcap = c.heap_base + c.heap_mult * L;
  outcap = c.out_base + c.out_mult * L;
  words = 64 + 16 * qcap + 3 * int64_t(nslots) * L + 3 * int64_t(nstates) * seqcap + heapcap + outcap;
}

namespace {

constexpr int32_t EPS_NONE = 0xFF;
constexpr int MAXD = NFA_MAX_STAGES + 2;
constexpr int STK = 32;

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

struct Lane {
  const NfaArgs* A;
  const DevProgram* P;
  int32_t* base;
  int64_t seg0;
  int32_t L;
  int32_t qcap, seqcap, heapcap, outcap;
  int32_t *hwm, *qa, *qb, *tq, *fq, *nodes, *aggs, *heap, *out;
  int32_t qlen, tlen, flen, heap_top, out_top;
  int32_t runs;
  int32_t err;
  int32_t overflow;
  int32_t r;                 // current record (local)
  int64_t nmatch;
};

// ---- stage references (real stage or Stage.newEpsilonState(src, target), Stage.java:247-251) ----
__device__ __forceinline__ const DevStage& stg(const Lane& l, int sid) { return l.P->st[sid]; }
__device__ __forceinline__ bool is_begin(const Lane& l, int sid) { return stg(l, sid).type == ST_BEGIN_; }
__device__ __forceinline__ bool is_forwarding(const Lane& l, int sid, int eps) {   // ComputationStage.java:134-137
  if (eps != EPS_NONE) return true;
  const DevStage& s = stg(l, sid);
  return s.nedges == 1 && s.op[0] == E_PROCEED;
}
__device__ __forceinline__ bool is_fwd_final(const Lane& l, int sid, int eps) {    // :143-147
  if (!is_forwarding(l, sid, eps)) return false;
  const int tgt = eps != EPS_NONE ? eps : stg(l, sid).target[0];
  return stg(l, tgt).type == ST_FINAL_;
}

// ---- heap: versions and predecessor pointers ----
__device__ __forceinline__ int heap_alloc(Lane& l, int words) {
  if (l.heap_top + words > l.heapcap) { l.overflow = 1; return -1; }
  const int at = l.heap_top;
  l.heap_top += words;
  return at;
}
__device__ int dw_add_stage(Lane& l, int v) {             // DeweyVersion.addStage :95-97
  const int len = l.heap[v];
  const int n = heap_alloc(l, len + 2);
  if (n < 0) return -1;
  l.heap[n] = len + 1;
  for (int i = 0; i < len; i++) l.heap[n + 1 + i] = l.heap[v + 1 + i];
  l.heap[n + 1 + len] = 0;
  return n;
}
__device__ int dw_add_run(Lane& l, int v, int off) {      // DeweyVersion.addRun :62-67
  const int len = l.heap[v];
  const int idx = len - off;
  if (idx < 0 || idx >= len) { l.err = CEP_E_INDEX; return -1; }
  const int n = heap_alloc(l, len + 1);
  if (n < 0) return -1;
  l.heap[n] = len;
  for (int i = 0; i < len; i++) l.heap[n + 1 + i] = l.heap[v + 1 + i];
  l.heap[n + 1 + idx] = int32_t(uint32_t(l.heap[n + 1 + idx]) + 1u);
  return n;
}
__device__ bool dw_compatible(const Lane& l, int a, int b) {   // a.isCompatible(b) :73-93
  const int la = l.heap[a], lb = l.heap[b];
  if (la > lb) {
    for (int i = 0; i < lb; i++)
      if (l.heap[a + 1 + i] != l.heap[b + 1 + i]) return false;
    return true;
  }
  if (la == lb) {
    for (int i = 0; i < la - 1; i++)
      if (l.heap[a + 1 + i] != l.heap[b + 1 + i]) return false;
    return l.heap[a + la] >= l.heap[b + lb];
  }
  return false;
}

// ---- shared versioned buffer ----
__device__ __forceinline__ int32_t* node(Lane& l, int slot, int ev) { return l.nodes + (int64_t(slot) * l.L + ev) * 3; }
__device__ __forceinline__ int slot_of(const Lane& l, int sid) { return stg(l, sid).slot; }

__device__ bool add_pred(Lane& l, int32_t* nd, int ver, int pslot, int pev) {   // MatchedEvent.addPredecessor
  const int p = heap_alloc(l, 4);
  if (p < 0) return false;
  l.heap[p] = ver; l.heap[p + 1] = pslot; l.heap[p + 2] = pev; l.heap[p + 3] = -1;
  if (nd[1] < 0) { nd[1] = p; return true; }
  int q = nd[1];
  while (l.heap[q + 3] >= 0) q = l.heap[q + 3];
  l.heap[q + 3] = p;
  return true;
}
// put 5-arg (SharedVersionedBufferStoreImpl.java:101-126)
__device__ void buf_put5(Lane& l, int cur_sid, int ev, int prev_sid, int pev, int ver) {
  if (pev < 0) { l.err = CEP_E_NPE; return; }
  const int ps = slot_of(l, prev_sid);
  if (!node(l, ps, pev)[2]) { l.err = CEP_E_ILLEGAL_STATE; return; }
  int32_t* c = node(l, slot_of(l, cur_sid), ev);
  if (!c[2]) { c[0] = 1; c[1] = -1; c[2] = 1; }
  add_pred(l, c, ver, ps, pev);
}
// put 3-arg (:149-157): a fresh node overwrites
__device__ void buf_put3(Lane& l, int cur_sid, int ev, int ver) {
  int32_t* c = node(l, slot_of(l, cur_sid), ev);
  c[0] = 1; c[1] = -1; c[2] = 1;
  add_pred(l, c, ver, -1, 0);
}
__device__ int first_compatible(const Lane& l, const int32_t* nd, int ver, int* prevp) {   // getPointerByVersion
  int pp = -1;
  for (int p = nd[1]; p >= 0; p = l.heap[p + 3]) {
    if (dw_compatible(l, ver, l.heap[p])) { if (prevp) *prevp = pp; return p; }
    pp = p;
  }
  return -1;
}
// branch (:132-142)
__device__ void buf_branch(Lane& l, int sid, int ev, int ver) {
  if (ev < 0) { l.err = CEP_E_NPE; return; }
  int slot = slot_of(l, sid), e = ev, pv = ver;
  for (;;) {
    int32_t* nd = node(l, slot, e);
    if (!nd[2]) { l.err = CEP_E_NPE; return; }
    nd[0]++;
    const int p = first_compatible(l, nd, pv, nullptr);
    if (p < 0 || l.heap[p + 1] < 0) return;
    pv = l.heap[p]; slot = l.heap[p + 1]; e = l.heap[p + 2];
  }
}
// peek (:176-201).  emit: traversal entries appended at out[out_top..]; returns the count or -1.
__device__ int buf_peek(Lane& l, int sid, int ev, int ver, bool remove, int32_t* dst, int dst_cap) {
  if (ev < 0) { l.err = CEP_E_NPE; return -1; }
  int slot = slot_of(l, sid), e = ev, pv = ver, cnt = 0;
  for (;;) {
    int32_t* nd = node(l, slot, e);
    if (!nd[2]) { l.err = CEP_E_NPE; return -1; }
    const int refs_left = nd[0] == 0 ? 0 : nd[0] - 1;     // decremented on a copy
    const bool single = nd[1] < 0 || l.heap[nd[1] + 3] < 0;
    if (dst) {
      if (cnt + 1 > dst_cap) { l.overflow = 1; return -1; }
      dst[2 * cnt] = l.P->slot_name[slot];
      dst[2 * cnt + 1] = e;
    }
    cnt++;
    int pp = -1;
    const int p = first_compatible(l, nd, pv, &pp);
    if (remove && p >= 0 && refs_left == 0) {
      nd[0] = 0;                                            // removePredecessor + put(copy)
      if (pp < 0) nd[1] = l.heap[p + 3]; else l.heap[pp + 3] = l.heap[p + 3];
      nd[2] = 1;
    } else if (remove && refs_left == 0 && single) {
      nd[2] = 0;                                            // delete
    }
    if (p < 0 || l.heap[p + 1] < 0) return cnt;
    pv = l.heap[p]; slot = l.heap[p + 1]; e = l.heap[p + 2];
  }
}

// ---- aggregates ----
__device__ __forceinline__ int32_t* agg(Lane& l, int state, int seq) {
  if (seq < 0 || seq >= l.seqcap) { l.overflow = 1; return nullptr; }
  return l.aggs + (int64_t(state) * l.seqcap + seq) * 3;
}

// ---- event fields ----
__device__ __forceinline__ int64_t rec(const Lane& l, int r) { return l.seg0 + r; }
__device__ __forceinline__ int32_t ev_topic(const Lane& l, int64_t g) { return l.A->topic ? l.A->topic[g] : 0; }
__device__ __forceinline__ int32_t ev_part(const Lane& l, int64_t g) { return l.A->partition ? l.A->partition[g] : 0; }
__device__ __forceinline__ int64_t ev_off(const Lane& l, int64_t g) { return l.A->offset ? l.A->offset[g] : g; }
__device__ __forceinline__ int64_t ev_ts(const Lane& l, int64_t g) { return l.A->ts ? l.A->ts[g] : g; }
__device__ __forceinline__ int64_t field(const Lane& l, int col, int t, int64_t g) {
  const void* c = l.A->cols[col];
  if (t == T_I32) return static_cast<const int32_t*>(c)[g];
  return static_cast<const int64_t*>(c)[g];            // i64, or f64 bits
}

__device__ __forceinline__ double as_f(int64_t b) { return __builtin_bit_cast(double, b); }
__device__ __forceinline__ int64_t as_b(double d) { return __builtin_bit_cast(int64_t, d); }
__device__ __forceinline__ int64_t sx32(int64_t x) { return int64_t(int32_t(uint32_t(uint64_t(x)))); }

// Event.compareTo (Event.java:118-122) == 0, for TreeSet de-duplication
__device__ bool ev_same(const Lane& l, int a, int b) {
  const int64_t ga = rec(l, a), gb = rec(l, b);
  if (ev_topic(l, ga) != ev_topic(l, gb) || ev_part(l, ga) != ev_part(l, gb)) return ev_ts(l, ga) == ev_ts(l, gb);
  return ev_off(l, ga) == ev_off(l, gb);
}

struct Ctx {
  int r, seq, prev_sid, pev, ver;   // prev_sid < 0: null previous stage
  bool in_fold;
  int32_t curr_tag;
  int64_t curr;
};

// SequenceMatcher: average of a column over buffer.get(Matched(prev, prevEvent), version)
// (SequenceMatcher.java:21-26), with Sequence's per-stage TreeSet de-duplication.
__device__ bool seq_avg(Lane& l, const Ctx& c, int col, int64_t& out) {
  if (c.prev_sid < 0 || c.pev < 0) { l.err = CEP_E_NPE; return false; }
  const int mark = l.heap_top;
  const int room = l.heapcap - l.heap_top;
  int32_t* tmp = l.heap + l.heap_top;
  const int cnt = buf_peek(l, c.prev_sid, c.pev, c.ver, false, tmp, room / 2);
  if (cnt < 0) return false;
  const int t = l.P->coltype[col];
  int64_t isum = 0;
  double fsum = 0;
  int64_t n = 0;
  for (int i = 0; i < cnt; i++) {
    bool dup = false;
    for (int j = 0; j < i && !dup; j++)
      dup = tmp[2 * j] == tmp[2 * i] && ev_same(l, tmp[2 * j + 1], tmp[2 * i + 1]);
    if (dup) continue;
    const int64_t v = field(l, col, t, rec(l, tmp[2 * i + 1]));
    if (t == T_F64) fsum += as_f(v); else isum += v;
    n++;
  }
  l.heap_top = mark;
  const double avg = n ? (t == T_F64 ? fsum : double(isum)) / double(n) : 0.0;
  out = as_b(avg);
  return true;
}

// bytecode interpreter; returns false on error (l.err / l.overflow set)
__device__ bool run_code(Lane& l, int pc, const Ctx& c, int64_t& result) {
  const int32_t* code = l.P->code;
  int64_t st[STK];
  int sp = 0;
  const int64_t g = rec(l, c.r);
  for (;;) {
    const int32_t w = code[pc++];
    const int op = w & 0xFF, a = (w >> 8) & 0xFF, b = (w >> 16) & 0xFF;
    if (sp >= STK - 1) { l.overflow = 1; return false; }
    switch (op) {
      case BC_END: result = st[sp - 1]; return true;
      case BC_PUSH: st[sp++] = int64_t(uint32_t(code[pc])) | (int64_t(code[pc + 1]) << 32); pc += 2; break;
      case BC_FIELD: st[sp++] = field(l, a, b, g); break;
      case BC_EV_KEY: st[sp++] = l.A->key[g]; break;
      case BC_EV_TS: st[sp++] = ev_ts(l, g); break;
      case BC_EV_OFFSET: st[sp++] = ev_off(l, g); break;
      case BC_EV_PARTITION: st[sp++] = ev_part(l, g); break;
      case BC_TOPIC_EQ: st[sp++] = ev_topic(l, g) == code[pc] ? 1 : 0; pc++; break;
      case BC_STATE_GET: case BC_STATE_GET_OR_ELSE: {          // States.get / getOrElse (States.java:56-78)
        const int32_t* e = agg(l, a, c.seq);
        if (!e) return false;
        if (e[0] == 0) {
          if (op == BC_STATE_GET) { l.err = CEP_E_UNKNOWN_AGGREGATE; return false; }
          pc++;                                                  // evaluate the default
          break;
        }
        if (e[0] != b) { l.err = CEP_E_CLASS_CAST; return false; }
        st[sp++] = int64_t(uint32_t(e[1])) | (int64_t(e[2]) << 32);
        if (op == BC_STATE_GET_OR_ELSE) pc += 1 + code[pc];
        break;
      }
      case BC_FOLD_CURR:
        if (!c.in_fold || c.curr_tag == 0) { l.err = CEP_E_NPE; return false; }
        if (c.curr_tag != b) { l.err = CEP_E_CLASS_CAST; return false; }
        st[sp++] = c.curr;
        break;
      case BC_SEQ_AVG: {
        int64_t v;
        if (!seq_avg(l, c, a, v)) return false;
        st[sp++] = v;
        break;
      }
      case BC_NOT: st[sp - 1] = st[sp - 1] ? 0 : 1; break;
      case BC_JZ_KEEP: if (st[sp - 1] == 0) pc += 1 + code[pc]; else { sp--; pc++; } break;
      case BC_JNZ_KEEP: if (st[sp - 1] != 0) pc += 1 + code[pc]; else { sp--; pc++; } break;
      case BC_POP: sp--; break;
      case BC_NEG_I32: st[sp - 1] = sx32(0 - st[sp - 1]); break;
      case BC_NEG_I64: st[sp - 1] = int64_t(0ull - uint64_t(st[sp - 1])); break;
      case BC_NEG_F64: st[sp - 1] = as_b(-as_f(st[sp - 1])); break;
      case BC_I64_TO_I32: st[sp - 1] = sx32(st[sp - 1]); break;
      case BC_I_TO_F64: st[sp - 1] = as_b(double(st[sp - 1])); break;
      case BC_F64_TO_I32: {
        const double d = as_f(st[sp - 1]);
        st[sp - 1] = d != d ? 0 : d >= 2147483647.0 ? INT32_MAX : d <= -2147483648.0 ? INT32_MIN : int64_t(int32_t(d));
        break;
      }
      case BC_F64_TO_I64: {
        const double d = as_f(st[sp - 1]);
        st[sp - 1] = d != d ? 0 : d >= 9223372036854775807.0 ? INT64_MAX : d <= -9223372036854775808.0 ? INT64_MIN : int64_t(d);
        break;
      }
      default: {
        const int64_t y = st[--sp], x = st[sp - 1];
        int64_t z = 0;
        switch (op) {
          case BC_ADD_I32: z = sx32(x + y); break;
          case BC_SUB_I32: z = sx32(x - y); break;
          case BC_MUL_I32: z = sx32(int64_t(uint64_t(x) * uint64_t(y))); break;
          case BC_DIV_I32:
            if (y == 0) { l.err = CEP_E_ARITHMETIC; return false; }
            z = (x == INT32_MIN && y == -1) ? INT32_MIN : x / y;
            break;
          case BC_REM_I32:
            if (y == 0) { l.err = CEP_E_ARITHMETIC; return false; }
            z = y == -1 ? 0 : x % y;
            break;
          case BC_ADD_I64: z = int64_t(uint64_t(x) + uint64_t(y)); break;
          case BC_SUB_I64: z = int64_t(uint64_t(x) - uint64_t(y)); break;
          case BC_MUL_I64: z = int64_t(uint64_t(x) * uint64_t(y)); break;
          case BC_DIV_I64:
            if (y == 0) { l.err = CEP_E_ARITHMETIC; return false; }
            z = (x == INT64_MIN && y == -1) ? INT64_MIN : x / y;
            break;
          case BC_REM_I64:
            if (y == 0) { l.err = CEP_E_ARITHMETIC; return false; }
            z = y == -1 ? 0 : x % y;
            break;
          case BC_ADD_F64: z = as_b(as_f(x) + as_f(y)); break;
          case BC_SUB_F64: z = as_b(as_f(x) - as_f(y)); break;
          case BC_MUL_F64: z = as_b(as_f(x) * as_f(y)); break;
          case BC_DIV_F64: z = as_b(as_f(x) / as_f(y)); break;
          case BC_REM_F64: z = as_b(fmod(as_f(x), as_f(y))); break;
          case BC_EQ_I: z = x == y; break;
          case BC_NE_I: z = x != y; break;
          case BC_LT_I: z = x < y; break;
          case BC_LE_I: z = x <= y; break;
          case BC_GT_I: z = x > y; break;
          case BC_GE_I: z = x >= y; break;
          case BC_EQ_F: z = as_f(x) == as_f(y); break;
          case BC_NE_F: z = as_f(x) != as_f(y); break;
          case BC_LT_F: z = as_f(x) < as_f(y); break;
          case BC_LE_F: z = as_f(x) <= as_f(y); break;
          case BC_GT_F: z = as_f(x) > as_f(y); break;
          case BC_GE_F: z = as_f(x) >= as_f(y); break;
          case BC_EQ_B: z = (x != 0) == (y != 0); break;
          case BC_NE_B: z = (x != 0) != (y != 0); break;
          default: l.err = CEP_E_BAD_IR; return false;
        }
        st[sp - 1] = z;
      }
    }
  }
}

__device__ __forceinline__ bool push_t(Lane& l, const Run& x) {
  if (l.tlen >= l.qcap) { l.overflow = 1; return false; }
  reinterpret_cast<int4*>(l.tq)[l.tlen++] = make_int4(x.w0, x.ver, x.ev, x.seq);
  return true;
}

struct Frame {
  Run cs;                          // ComputationContext.computationStage
  int16_t cur_sid, cur_eps, prev_sid, prev_eps;
  int8_t medge[NFA_MAX_EDGES];
  int8_t nm, i, pending;
  uint8_t branching, ignored, consumed, proceed;
  int32_t nbase, before;
};

// frame entry: matchEdgesAndGet (NFA.java:371-384) + isBranching (:392-397)
__device__ bool frame_enter(Lane& l, Frame& f) {
  f.nm = 0; f.i = 0; f.pending = 0; f.consumed = 0; f.proceed = 0;
  f.nbase = l.tlen;
  int has[5] = {0, 0, 0, 0, 0};
  const bool eps = f.cur_eps != EPS_NONE;
  const DevStage& s = stg(l, f.cur_sid);
  const int ne = eps ? 1 : s.nedges;
  for (int e = 0; e < ne; e++) {
    const int op = eps ? E_PROCEED : s.op[e];
    const int pc = eps ? -1 : s.pred[e];
    bool ok = true;
    if (pc >= 0) {
      Ctx c{l.r, f.cs.seq, f.prev_sid >= 0 ? int(f.prev_sid) : -1, f.cs.ev, f.cs.ver, false, 0, 0};
      int64_t v;
      if (!run_code(l, pc, c, v)) return false;
      ok = v != 0;
    }
    if (ok) { f.medge[f.nm++] = int8_t(e); has[op] = 1; }
  }
  f.branching = (has[E_PROCEED] && has[E_TAKE]) || (has[E_IGNORE] && has[E_TAKE]) || (has[E_IGNORE] && has[E_BEGIN]) ||
                (has[E_IGNORE] && has[E_PROCEED]);
  f.ignored = has[E_IGNORE];
  return true;
}

// NFA.evaluate (NFA.java:190-341) for one run; results appended to tq
__device__ bool evaluate(Lane& l, const Run& run, Frame* fr) {
  int d = 0;
  fr[0].cs = run;
  fr[0].cur_sid = int16_t(r_sid(run));
  fr[0].cur_eps = int16_t(r_eps(run));
  fr[0].prev_sid = -1;
  fr[0].prev_eps = EPS_NONE;
  if (!frame_enter(l, fr[0])) return false;
  for (;;) {
    Frame& f = fr[d];
    if (f.i < f.nm) {
      const int e = f.medge[f.i++];
      const bool eps = f.cur_eps != EPS_NONE;
      const DevStage& s = stg(l, f.cur_sid);
      const int op = eps ? E_PROCEED : s.op[e];
      const int target = eps ? f.cur_eps : s.target[e];
      const int ver = f.cs.ver, seq = f.cs.seq;
      if (op == E_PROCEED || op == E_SKIP_PROCEED) {                 // :222-237
        if (d + 1 >= MAXD) { l.overflow = 1; return false; }
        Frame& g = fr[d + 1];
        g.cs = f.cs;
        if (stg(l, target).name != s.name && !r_br(f.cs) && !r_ig(f.cs)) {   // isForwardingToNextStage :343-349
          const int nv = dw_add_stage(l, ver);
          if (nv < 0) return false;
          g.cs = mk_run(r_sid(f.cs), r_eps(f.cs), nv, f.cs.ev, f.cs.seq, false, false);   // setVersion
        }
        if (op == E_SKIP_PROCEED) { g.prev_sid = f.prev_sid; g.prev_eps = f.prev_eps; }
        else { g.prev_sid = f.cur_sid; g.prev_eps = f.cur_eps; }
        g.cur_sid = int16_t(target);
        g.cur_eps = EPS_NONE;
        f.before = l.tlen;
        f.pending = 1;
        d++;
        if (!frame_enter(l, fr[d])) return false;
        continue;
      }
      if (op == E_TAKE) {                                            // :238-255
        if (!push_t(l, mk_run(f.cur_sid, f.cur_sid, ver, l.r, seq, false, false))) return false;
        int pv = ver;
        if (!(!f.branching || f.ignored)) { pv = dw_add_run(l, ver, 1); if (pv < 0) return false; }
        if (f.prev_sid >= 0) buf_put5(l, f.cur_sid, l.r, f.prev_sid, f.cs.ev, pv);
        else buf_put3(l, f.cur_sid, l.r, pv);
        if (l.err || l.overflow) return false;
        f.consumed = 1;
      } else if (op == E_BEGIN) {                                    // :256-271
        if (f.prev_sid >= 0) buf_put5(l, f.cur_sid, l.r, f.prev_sid, f.cs.ev, ver);
        else buf_put3(l, f.cur_sid, l.r, ver);
        if (l.err || l.overflow) return false;
        if (!push_t(l, mk_run(f.cur_sid, target, ver, l.r, seq, false, false))) return false;
        f.consumed = 1;
      } else if (op == E_IGNORE) {                                   // :272-285
        if (!f.branching && !push_t(l, mk_run(r_sid(f.cs), r_eps(f.cs), f.cs.ver, f.cs.ev, f.cs.seq, false, true)))
          return false;
      }
      continue;
    }
    // ---- after the edge loop ----
    const int ver = f.cs.ver, seq = f.cs.seq, pev = f.cs.ev;
    const int32_t key = l.A->key[rec(l, l.r)];
    (void)key;
    if (f.branching) {                                               // :289-317
      if (f.consumed) {
        const int nseq = ++l.runs;
        const int last = f.ignored ? pev : l.r;
        if (f.prev_sid < 0) { l.err = CEP_E_NPE; return false; }    // Stage.newEpsilonState(null, ...)
        const bool pb = is_begin(l, f.prev_sid);
        const int nv = dw_add_run(l, ver, pb ? 2 : 1);
        if (nv < 0) return false;
        if (!push_t(l, mk_run(f.prev_sid, f.cur_sid, nv, last, nseq, true, false))) return false;
        for (int k = 0; k < l.P->ndefined; k++) {                    // AggregatesStoreImpl.branch
          const int32_t* src = agg(l, l.P->defined[k], seq);
          int32_t* dst = agg(l, l.P->defined[k], nseq);
          if (!src || !dst) return false;
          if (src[0]) { dst[0] = src[0]; dst[1] = src[1]; dst[2] = src[2]; }
        }
        if (!pb) { buf_branch(l, f.prev_sid, pev, ver); if (l.err) return false; }
      } else if (!f.proceed) {
        if (!push_t(l, f.cs)) return false;
      }
    }
    if (f.consumed && f.cur_eps == EPS_NONE) {                       // evaluateAggregates :319-321, :362-369
      const DevStage& s = stg(l, f.cur_sid);
      for (int k = 0; k < s.nfolds; k++) {
        int32_t* e = agg(l, s.fold_state[k], seq);
        if (!e) return false;
        Ctx c{l.r, seq, -1, -1, ver, true, e[0], int64_t(uint32_t(e[1])) | (int64_t(e[2]) << 32)};
        int64_t v;
        if (!run_code(l, s.fold_code[k], c, v)) return false;
        e = agg(l, s.fold_state[k], seq);
        e[0] = s.fold_type[k];
        e[1] = int32_t(uint32_t(uint64_t(v)));
        e[2] = int32_t(uint32_t(uint64_t(v) >> 32));
      }
    }
    const int csid = r_sid(f.cs), ceps = r_eps(f.cs);
    if (is_begin(l, csid) && !is_forwarding(l, csid, ceps)) {         // begin re-add :323-338
      if (f.consumed) {
        const int nseq = ++l.runs;
        int nv = ver;
        if (l.tlen != f.nbase) { nv = dw_add_run(l, ver, 1); if (nv < 0) return false; }
        if (!push_t(l, mk_run(csid, ceps, nv, -1, nseq, false, false))) return false;
      } else {
        if (!push_t(l, f.cs)) return false;
      }
    }
    if (d == 0) return true;
    d--;
    Frame& p = fr[d];
    if (p.pending) {
      if (l.tlen > p.before) p.proceed = 1;
      p.pending = 0;
    }
  }
}

// NFA.matchPattern(Event) (NFA.java:134-149) for local record r
__device__ bool step(Lane& l, Frame* fr) {
  const int n = l.qlen;
  int qn = 0;
  l.flen = 0;
  for (int i = 0; i < n; i++) {
    const int4 x = reinterpret_cast<int4*>(l.qa)[i];
    Run run{x.x, x.y, x.z, x.w};
    l.tlen = 0;
    // window check (:179-188): every non-begin run sits on an epsilon stage
    // whose window is -1, so it never prunes; nothing to evaluate.
    if (!evaluate(l, run, fr)) return false;
    if (l.tlen == 0) {                                               // removePattern :160-163
      if (buf_peek(l, r_sid(run), run.ev, run.ver, true, nullptr, 0) < 0) return false;
    }
    for (int t = 0; t < l.tlen; t++) {
      const int4 y = reinterpret_cast<int4*>(l.tq)[t];
      const Run u{y.x, y.y, y.z, y.w};
      if (is_fwd_final(l, r_sid(u), r_eps(u))) {
        if (l.flen >= l.qcap) { l.overflow = 1; return false; }
        reinterpret_cast<int4*>(l.fq)[l.flen++] = y;
      } else {
        if (qn >= l.qcap) { l.overflow = 1; return false; }
        reinterpret_cast<int4*>(l.qb)[qn++] = y;
      }
    }
  }
  int32_t* tmp = l.qa;                                              // swap queues
  l.qa = l.qb;
  l.qb = tmp;
  l.qlen = qn;
  for (int k = 0; k < l.flen; k++) {                                // matchConstruction :151-158
    const int4 y = reinterpret_cast<int4*>(l.fq)[k];
    if (l.out_top + 2 > l.outcap) { l.overflow = 1; return false; }
    int32_t* hdr = l.out + l.out_top;
    const int cnt = buf_peek(l, y.x & 0xFF, y.z, y.y, true, hdr + 2, (l.outcap - l.out_top - 2) / 2);
    if (cnt < 0) return false;
    hdr[0] = l.r;
    hdr[1] = cnt;
    l.out_top += 2 + 2 * cnt;
    l.nmatch++;
  }
  return true;
}

}  // namespace

__global__ __launch_bounds__(64) void nfa_kernel(NfaArgs A) {
  const int li = blockIdx.x * blockDim.x + threadIdx.x;
  if (li >= A.nlist) return;
  const int seg = A.seg_list ? A.seg_list[li] : li;
  const DevProgram* P = A.P;
  Lane l;
  l.A = &A;
  l.P = P;
  l.seg0 = A.seg_start[seg];
  l.L = int32_t(A.seg_start[seg + 1] - l.seg0);
  int64_t qcap, seqcap, heapcap, outcap, words;
  nfa_layout(A.cap, P->nslots, P->nstates, l.L, qcap, seqcap, heapcap, outcap, words);
  l.qcap = int32_t(qcap); l.seqcap = int32_t(seqcap); l.heapcap = int32_t(heapcap); l.outcap = int32_t(outcap);
  l.base = A.arena + A.arena_off[li];
  int32_t* p = l.base;
  l.hwm = p; p += 64;
  l.qa = p; p += 4 * qcap;
  l.qb = p; p += 4 * qcap;
  l.tq = p; p += 4 * qcap;
  l.fq = p; p += 4 * qcap;
  l.nodes = p; p += 3 * int64_t(P->nslots) * l.L;
  l.aggs = p; p += 3 * int64_t(P->nstates) * seqcap;
  l.heap = p; p += heapcap;
  l.out = p;
  l.err = 0; l.overflow = 0; l.nmatch = 0; l.heap_top = 0; l.out_top = 0; l.flen = 0; l.tlen = 0;
  for (int64_t i = 0; i < 3 * int64_t(P->nstates) * seqcap; i += 3) l.aggs[i] = 0;   // all states null
  int nhwm = 0;
  // NFA.build (NFA.java:73-79), Stages.initialComputationStage (Stages.java:53-60)
  const int v0 = heap_alloc(l, 2);
  l.heap[v0] = 1;
  l.heap[v0 + 1] = 1;
  reinterpret_cast<int4*>(l.qa)[0] = make_int4(P->begin | (EPS_NONE << 8), v0, -1, 1);
  l.qlen = 1;
  l.runs = 1;
  Frame fr[MAXD];
  int64_t err_rec = -1;
  const bool proc = A.mode == CEP_MODE_PROCESSOR;
  for (int r = 0; r < l.L && !l.err && !l.overflow; r++) {
    const int64_t g = l.seg0 + r;
    l.r = r;
    for (int s = 0; s < P->nslots; s++) { int32_t* nd = node(l, s, r); nd[0] = 0; nd[1] = -1; nd[2] = 0; }
    if (proc) {
      if (A.valid && !A.valid[g]) continue;                           // CEPProcessor.java:136-138
      for (int i = 0; i < l.qlen; i++) l.qa[4 * i] &= ~(1 << 17);      // isIgnored not serialised (Q3)
      const int32_t tp = ev_topic(l, g);
      int h = 0;
      while (h < nhwm && l.hwm[3 * h] != tp) h++;
      if (h < nhwm) {                                                  // checkHighWaterMark :152-160
        const int64_t hw = int64_t(uint32_t(l.hwm[3 * h + 1])) | (int64_t(l.hwm[3 * h + 2]) << 32);
        if (ev_off(l, g) < hw) continue;
      }
    }
    if (!step(l, fr)) {
      if (l.err) err_rec = g;
      break;
    }
    if (proc) {
      const int32_t tp = ev_topic(l, g);
      int h = 0;
      while (h < nhwm && l.hwm[3 * h] != tp) h++;
      if (h == nhwm) {
        if (nhwm == 16) { l.overflow = 1; break; }
        nhwm++;
        l.hwm[3 * h] = tp;
      }
      const int64_t hw = ev_off(l, g) + 1;
      l.hwm[3 * h + 1] = int32_t(uint32_t(uint64_t(hw)));
      l.hwm[3 * h + 2] = int32_t(uint32_t(uint64_t(hw) >> 32));
    }
  }
  A.res_matches[seg] = l.nmatch;
  A.res_words[seg] = l.out_top;
  A.res_out[seg] = int64_t(reinterpret_cast<uintptr_t>(l.out));
  A.res_err[seg] = l.overflow ? 0 : l.err;
  A.res_err_rec[seg] = l.overflow ? -1 : err_rec;
  A.res_overflow[seg] = l.overflow;
  if (l.overflow) atomicAdd(A.overflow_count, 1);
}

// ---- segments, scans, output compaction ----
__global__ void seg_mark(const int32_t* __restrict__ key, int64_t n, int64_t* __restrict__ flag) {
  const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n) flag[i] = (i == 0 || key[i] != key[i - 1]) ? 1 : 0;
}
__global__ void seg_scatter(const int64_t* __restrict__ flag, const int64_t* __restrict__ idx, int64_t n,
                            int64_t* __restrict__ seg_start) {
  const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n && flag[i]) seg_start[idx[i]] = i;
  if (i == 0) seg_start[idx[n - 1] + flag[n - 1]] = n;
}
__global__ void arena_sizes(const int64_t* __restrict__ seg_start, int64_t nseg, NfaCaps cap, int nslots,
                            int nstates, int64_t* __restrict__ words) {
  const int64_t s = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (s >= nseg) return;
  int64_t a, b, c, d, w;
  nfa_layout(cap, nslots, nstates, seg_start[s + 1] - seg_start[s], a, b, c, d, w);
  words[s] = (w + 3) & ~int64_t(3);
}

// exclusive scan, 1024 elements per block: (1) block sums, (2) scan of block sums
// in one block, (3) per-block scan + offset
__global__ void scan_blocks(const int64_t* __restrict__ in, int64_t n, int64_t* __restrict__ bsum) {
  __shared__ int64_t s[256];
  const int64_t b0 = int64_t(blockIdx.x) * 1024;
  int64_t acc = 0;
  for (int k = 0; k < 4; k++) {
    const int64_t i = b0 + threadIdx.x * 4 + k;
    if (i < n) acc += in[i];
  }
  s[threadIdx.x] = acc;
  __syncthreads();
  for (int d = 128; d > 0; d >>= 1) {
    if (threadIdx.x < d) s[threadIdx.x] += s[threadIdx.x + d];
    __syncthreads();
  }
  if (threadIdx.x == 0) bsum[blockIdx.x] = s[0];
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
      const int64_t y = threadIdx.x >= d ? s[threadIdx.x - d] : 0;
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
__global__ void scan_final(const int64_t* __restrict__ in, int64_t n, const int64_t* __restrict__ bsum,
                           int64_t* __restrict__ out) {
  __shared__ int64_t s[256];
  const int64_t b0 = int64_t(blockIdx.x) * 1024;
  int64_t v[4], acc = 0;
  for (int k = 0; k < 4; k++) {
    const int64_t i = b0 + threadIdx.x * 4 + k;
    v[k] = i < n ? in[i] : 0;
    acc += v[k];
  }
  s[threadIdx.x] = acc;
  __syncthreads();
  for (int d = 1; d < 256; d <<= 1) {
    const int64_t y = threadIdx.x >= d ? s[threadIdx.x - d] : 0;
    __syncthreads();
    s[threadIdx.x] += y;
    __syncthreads();
  }
  int64_t run = bsum[blockIdx.x] + s[threadIdx.x] - acc;
  for (int k = 0; k < 4; k++) {
    const int64_t i = b0 + threadIdx.x * 4 + k;
    if (i < n) out[i] = run;
    run += v[k];
  }
}

hipError_t nfa_launch(const NfaArgs& A, hipStream_t st) {
  if (A.nlist <= 0) return hipSuccess;
  hipLaunchKernelGGL(nfa_kernel, dim3(unsigned((A.nlist + 63) / 64)), dim3(64), 0, st, A);
  return hipGetLastError();
}
hipError_t nfa_segments(const int32_t* key, int64_t n, int64_t* flag, int64_t* idx, int64_t* seg_start, int64_t* nseg,
                        int64_t* tmp, hipStream_t st);
hipError_t nfa_arena_sizes(const int64_t* seg_start, int64_t nseg, const NfaCaps& cap, int nslots, int nstates,
                           int64_t* words, hipStream_t st) {
  if (nseg <= 0) return hipSuccess;
  hipLaunchKernelGGL(arena_sizes, dim3(unsigned((nseg + 255) / 256)), dim3(256), 0, st, seg_start, nseg, cap, nslots,
                     nstates, words);
  return hipGetLastError();
}

hipError_t exclusive_scan(const int64_t* in, int64_t n, int64_t* out, int64_t* total, int64_t* tmp,
                          hipStream_t st) {
  if (n <= 0) return hipMemsetAsync(total, 0, sizeof(int64_t), st);
  const int64_t nb = (n + 1023) / 1024;
  hipLaunchKernelGGL(scan_blocks, dim3(unsigned(nb)), dim3(256), 0, st, in, n, tmp);
  hipLaunchKernelGGL(scan_sums, dim3(1), dim3(256), 0, st, tmp, nb, total);
  hipLaunchKernelGGL(scan_final, dim3(unsigned(nb)), dim3(256), 0, st, in, n, tmp, out);
  return hipGetLastError();
}

__global__ void nfa_compact(const int64_t* __restrict__ seg_start, int64_t nseg,
                            const int32_t* __restrict__ key, const int64_t* __restrict__ res_out,
                            const int64_t* __restrict__ res_matches, const int64_t* __restrict__ moff,
                            const int64_t* __restrict__ eoff, int64_t* __restrict__ match_record,
                            int32_t* __restrict__ match_key, int64_t* __restrict__ ent_off,
                            int32_t* __restrict__ ent_name, int64_t* __restrict__ ent_record) {
  const int64_t s = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (s >= nseg) return;
  const int64_t s0 = seg_start[s];
  const int32_t* o = reinterpret_cast<const int32_t*>(uintptr_t(res_out[s]));
  int64_t m = moff[s], e = eoff[s];
  for (int64_t k = 0; k < res_matches[s]; k++) {
    const int r = o[0], cnt = o[1];
    match_record[m] = s0 + r;
    match_key[m] = key[s0];
    ent_off[m] = e;
    for (int i = 0; i < cnt; i++) {
      ent_name[e + i] = o[2 + 2 * i];
      ent_record[e + i] = s0 + o[3 + 2 * i];
    }
    e += cnt;
    m++;
    o += 2 + 2 * cnt;
  }
}
// entries per segment = words - 2 * matches, halved
__global__ void nfa_entry_counts(const int64_t* __restrict__ words, const int64_t* __restrict__ matches, int64_t nseg,
                                 int64_t* __restrict__ ents) {
  const int64_t s = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (s < nseg) ents[s] = (words[s] - 2 * matches[s]) / 2;
}

hipError_t nfa_segments(const int32_t* key, int64_t n, int64_t* flag, int64_t* idx, int64_t* seg_start, int64_t* nseg,
                        int64_t* tmp, hipStream_t st) {
  if (n <= 0) return hipMemsetAsync(nseg, 0, sizeof(int64_t), st);
  const unsigned b = unsigned((n + 255) / 256);
  hipLaunchKernelGGL(seg_mark, dim3(b), dim3(256), 0, st, key, n, flag);
  hipError_t e = exclusive_scan(flag, n, idx, nseg, tmp, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(seg_scatter, dim3(b), dim3(256), 0, st, flag, idx, n, seg_start);
  return hipGetLastError();
}

hipError_t nfa_entry_counts_launch(const int64_t* words, const int64_t* matches, int64_t nseg, int64_t* ents,
                                   hipStream_t st) {
  if (nseg <= 0) return hipSuccess;
  hipLaunchKernelGGL(nfa_entry_counts, dim3(unsigned((nseg + 255) / 256)), dim3(256), 0, st, words, matches, nseg, ents);
  return hipGetLastError();
}

hipError_t nfa_compact_launch(const int64_t* seg_start, int64_t nseg, const int32_t* key, const int64_t* res_out,
                              const int64_t* res_matches, const int64_t* moff, const int64_t* eoff,
                              int64_t* match_record, int32_t* match_key, int64_t* ent_off, int32_t* ent_name,
                              int64_t* ent_record, hipStream_t st) {
  if (nseg <= 0) return hipSuccess;
  hipLaunchKernelGGL(nfa_compact, dim3(unsigned((nseg + 255) / 256)), dim3(256), 0, st, seg_start, nseg, key, res_out,
                     res_matches, moff, eoff, match_record, match_key, ent_off, ent_name, ent_record);
  return hipGetLastError();
}

}  // namespace kcep

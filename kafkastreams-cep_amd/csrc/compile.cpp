// compile.cpp — pattern IR -> stage graph (+ device programs).
//
// The stage graph follows the reference compiler StagesFactory.make /
// buildStages (core/.../cep/pattern/StagesFactory.java:49-180): stage ids are
// assigned $final = 0, then the stages of the LAST pattern first; a pattern
// gets a main stage (BEGIN or TAKE edge, IGNORE per strategy, PROCEED for
// TAKE), internal stages for oneOrMore / times(n), and a SKIP_PROCEED edge on
// its entry stage when optional.  Invalid shapes raise the reference's
// InvalidPatternException as CEP_E_INVALID_PATTERN.
//
// The stencil lowering implements SURVEY Q9: a pattern whose stages are all
// strict-contiguity, cardinality ONE, not optional, without folds, with
// pairwise-distinct names and side-effect-free predicates emits, per key, a
// match at record j iff the k consecutive records j-k+1..j satisfy P1..Pk.
#include <math.h>
#include <string.h>

#include <algorithm>
#include <limits>

#include "kcep_internal.h"
#include "../../include/kcep.h"

namespace kcep {
namespace {

struct Reader {
  const uint8_t* p;
  size_t n, i = 0;
  bool bad = false;
  bool need(size_t k) {
    if (i + k > n) bad = true;
    return !bad;
  }
  template <class T>
  T get() {
    T v{};
    if (need(sizeof(T))) { memcpy(&v, p + i, sizeof(T)); i += sizeof(T); }
    return v;
  }
  bool str(std::string& s, bool& is_null) {
    uint16_t len = get<uint16_t>();
    is_null = len == 0xFFFF;
    if (is_null || bad) return !bad;
    if (!need(len)) return false;
    s.assign(reinterpret_cast<const char*>(p + i), len);
    i += len;
    return true;
  }
};

int intern(std::vector<std::string>& v, const std::string& s) {
  auto it = std::find(v.begin(), v.end(), s);
  if (it != v.end()) return int(it - v.begin());
  v.push_back(s);
  return int(v.size() - 1);
}

ExprP parse_expr(Reader& r, Program& P, int depth) {
  if (depth > 256 || r.bad) { r.bad = true; return nullptr; }
  auto e = std::make_shared<Expr>();
  e->op = r.get<uint8_t>();
  auto num = [](const ExprP& x) { return x && x->t != T_BOOL; };
  auto boo = [](const ExprP& x) { return x && x->t == T_BOOL; };
  switch (e->op) {
    case OP_TRUE: case OP_FALSE: e->t = T_BOOL; break;
    case OP_CONST_I32: e->t = T_I32; e->i32 = r.get<int32_t>(); break;
    case OP_CONST_I64: e->t = T_I64; e->i64 = r.get<int64_t>(); break;
    case OP_CONST_F64: e->t = T_F64; e->f64 = r.get<double>(); break;
    case OP_FIELD:
      e->col = r.get<uint16_t>();
      if (e->col >= int(P.coltypes.size())) { r.bad = true; return nullptr; }
      e->t = P.coltypes[e->col];
      break;
    case OP_EV_KEY: case OP_EV_PARTITION: e->t = T_I32; break;
    case OP_EV_TS: case OP_EV_OFFSET: e->t = T_I64; break;
    case OP_EV_TOPIC_EQ: e->t = T_BOOL; e->i32 = r.get<int32_t>(); break;
    case OP_STATE_GET: case OP_STATE_GET_OR_ELSE: {
      e->ct = e->t = r.get<uint8_t>();
      std::string s; bool isnull;
      if (!r.str(s, isnull) || isnull) { r.bad = true; return nullptr; }
      e->name = intern(P.states, s);
      if (e->op == OP_STATE_GET_OR_ELSE) {
        e->a = parse_expr(r, P, depth + 1);
        if (!num(e->a) || e->a->t != e->ct) { r.bad = true; return nullptr; }
      }
      if (e->ct < T_I32 || e->ct > T_F64) { r.bad = true; return nullptr; }
      break;
    }
    case OP_FOLD_CURR:
      e->ct = e->t = r.get<uint8_t>();
      if (e->ct < T_I32 || e->ct > T_F64) { r.bad = true; return nullptr; }
      break;
    case OP_SEQ_AVG:
      e->col = r.get<uint16_t>();
      e->t = T_F64;
      if (e->col >= int(P.coltypes.size())) { r.bad = true; return nullptr; }
      break;
    case OP_SEQ_AGG: {                        // u8 kind, u16 column, stage name (null: every stage)
      e->ct = r.get<uint8_t>();
      e->col = r.get<uint16_t>();
      bool isnull;
      if (!r.str(e->sname, isnull)) { r.bad = true; return nullptr; }
      e->name = isnull ? -1 : 0;              // resolved against the stage names at bytecode time
      if (e->col >= int(P.coltypes.size()) || e->ct < SEQ_SUM || e->ct > SEQ_LAST) { r.bad = true; return nullptr; }
      const uint8_t ctype = P.coltypes[e->col];
      if ((e->ct == SEQ_FIRST || e->ct == SEQ_LAST) && isnull) { r.bad = true; return nullptr; }
      // sum over a double column: DoubleStream.sum, compensated (nfa_dev.h jsum_*), a double
      e->t = e->ct == SEQ_COUNT ? T_I64 : e->ct == SEQ_SUM ? (ctype == T_F64 ? T_F64 : T_I64) : ctype;
      break;
    }
    case OP_NOT:
      e->a = parse_expr(r, P, depth + 1);
      if (!boo(e->a)) { r.bad = true; return nullptr; }
      e->t = T_BOOL;
      break;
    case OP_AND: case OP_OR:
      e->a = parse_expr(r, P, depth + 1);
      e->b = parse_expr(r, P, depth + 1);
      if (!boo(e->a) || !boo(e->b)) { r.bad = true; return nullptr; }
      e->t = T_BOOL;
      break;
    case OP_ADD: case OP_SUB: case OP_MUL: case OP_DIV: case OP_REM:
      e->a = parse_expr(r, P, depth + 1);
      e->b = parse_expr(r, P, depth + 1);
      if (!num(e->a) || !num(e->b)) { r.bad = true; return nullptr; }
      e->t = std::max(e->a->t, e->b->t);
      break;
    case OP_NEG:
      e->a = parse_expr(r, P, depth + 1);
      if (!num(e->a)) { r.bad = true; return nullptr; }
      e->t = e->a->t;
      break;
    case OP_EQ: case OP_NE: case OP_LT: case OP_LE: case OP_GT: case OP_GE:
      e->a = parse_expr(r, P, depth + 1);
      e->b = parse_expr(r, P, depth + 1);
      if (!e->a || !e->b || (e->a->t == T_BOOL) != (e->b->t == T_BOOL)) { r.bad = true; return nullptr; }
      if (e->a->t == T_BOOL && e->op != OP_EQ && e->op != OP_NE) { r.bad = true; return nullptr; }
      e->t = T_BOOL;
      break;
    case OP_CAST:
      e->ct = r.get<uint8_t>();
      e->a = parse_expr(r, P, depth + 1);
      if (!num(e->a) || e->ct < T_I32 || e->ct > T_F64) { r.bad = true; return nullptr; }
      e->t = e->ct;
      break;
    default: r.bad = true; return nullptr;
  }
  return r.bad ? nullptr : e;
}

ExprP mk(uint8_t op, ExprP a = nullptr, ExprP b = nullptr) {
  auto e = std::make_shared<Expr>();
  e->op = op; e->t = T_BOOL; e->a = a; e->b = b;
  return e;
}
ExprP mk_topic(int32_t topic) { auto e = mk(OP_EV_TOPIC_EQ); e->i32 = topic; return e; }

struct BuildErr { int code; std::string msg; };

// StagesFactory.buildStages (StagesFactory.java:77-172)
std::vector<StageDef> build_stages(Program& P, uint8_t type, int pi, int succ_stage, int succ_pat,
                                   const std::vector<StageDef>& built, int& next_id) {
  const PatternDef& pat = P.pats[pi];
  const bool many = pat.one_or_more;
  StageDef main{next_id++, pat.name_id, uint8_t(many ? ST_NORMAL : type), -1, pi, {}};
  int64_t w = pat.window_ms;
  if (w == -1 && succ_pat >= 0) w = P.pats[succ_pat].window_ms;
  main.window_ms = w;
  if (!pat.pred) throw BuildErr{CEP_E_NPE, "pattern '" + pat.name + "' has no predicate"};
  ExprP pred = pat.topic >= 0 ? mk(OP_AND, mk_topic(pat.topic), pat.pred) : pat.pred;
  const uint8_t first_op = many ? E_TAKE : E_BEGIN;
  main.edges.push_back({first_op, pred, succ_stage});
  if (pat.strategy == S_NULL) throw BuildErr{CEP_E_NPE, "selected strategy is null for '" + pat.name + "'"};
  ExprP ignore;
  if (pat.strategy == S_ANY) {
    ignore = mk(OP_TRUE);
    main.edges.push_back({E_IGNORE, ignore, -1});
  } else if (pat.strategy == S_NEXT) {
    ignore = mk(OP_NOT, pred);
    main.edges.push_back({E_IGNORE, ignore, -1});
  }
  const bool succ_final = built[succ_stage].type == ST_FINAL;
  if (first_op == E_TAKE) {
    if (succ_pat < 0 && succ_final)
      throw BuildErr{CEP_E_INVALID_PATTERN, "Cannot define a pattern with a final stage expecting multiple matching events"};
    const PatternDef& sp = P.pats[succ_pat];
    ExprP succ = sp.topic >= 0 ? mk(OP_AND, mk_topic(sp.topic), sp.pred) : sp.pred;
    ExprP proceed = pat.strategy == S_STRICT
                        ? mk(OP_OR, succ, mk(OP_NOT, pred))
                        : mk(OP_OR, succ, mk(OP_AND, mk(OP_NOT, pred), mk(OP_NOT, ignore)));
    main.edges.push_back({E_PROCEED, proceed, succ_stage});
  }
  std::vector<StageDef> out{main};
  int times = pat.times;
  if (many || times > 1) {
    do {
      StageDef in{next_id++, pat.name_id, type, w, pi, {}};
      in.edges.push_back({E_BEGIN, pred, out.back().id});
      if (ignore) in.edges.push_back({E_IGNORE, ignore, -1});
      out.push_back(in);
    } while (--times > 1);
  }
  if (pat.optional) {
    if (succ_pat < 0 && succ_final)
      throw BuildErr{CEP_E_INVALID_PATTERN, "Cannot define a pattern with an optional final stage"};
    // the successor predicate without its topic filter (StagesFactory.java:165)
    out.back().edges.push_back({E_SKIP_PROCEED, mk(OP_AND, P.pats[succ_pat].pred, mk(OP_NOT, pred)), succ_stage});
  }
  return out;
}

// ---------------------------------------------------------------- stencil DNF
struct Range { int64_t lo, hi; double dlo, dhi; };
struct Term { bool has_v = false, has_t = false; Range v{}, t{}; };
using DNF = std::vector<Term>;

constexpr int64_t IMIN = std::numeric_limits<int64_t>::min();
constexpr int64_t IMAX = std::numeric_limits<int64_t>::max();

struct Lowering {
  int col = -1;
  uint8_t coltype = 0;
  bool ok = true;
  std::string why;

  void fail(const std::string& w) { if (ok) { ok = false; why = w; } }

  static bool empty(const Range& r, bool isf) { return isf ? !(r.dlo <= r.dhi) : r.lo > r.hi; }

  bool intersect(Term& a, const Term& b) {
    bool isf = coltype == T_F64;
    if (b.has_v) {
      if (!a.has_v) { a.has_v = true; a.v = b.v; }
      else {
        a.v.lo = std::max(a.v.lo, b.v.lo); a.v.hi = std::min(a.v.hi, b.v.hi);
        a.v.dlo = std::max(a.v.dlo, b.v.dlo); a.v.dhi = std::min(a.v.dhi, b.v.dhi);
      }
      if (empty(a.v, isf)) return false;
    }
    if (b.has_t) {
      if (!a.has_t) { a.has_t = true; a.t = b.t; }
      else { a.t.lo = std::max(a.t.lo, b.t.lo); a.t.hi = std::min(a.t.hi, b.t.hi); }
      if (a.t.lo > a.t.hi) return false;
    }
    return true;
  }

  DNF conj(const DNF& x, const DNF& y) {
    DNF out;
    for (auto& a : x)
      for (auto& b : y) {
        Term t = a;
        if (intersect(t, b)) out.push_back(t);
      }
    if (out.size() > STENCIL_MAX_TERMS) fail("predicate needs too many terms");
    return out;
  }

  static DNF int_cmp(uint8_t op, int64_t k, bool topic) {
    auto mkT = [&](int64_t lo, int64_t hi) {
      Term t;
      if (topic) { t.has_t = true; t.t.lo = lo; t.t.hi = hi; }
      else { t.has_v = true; t.v.lo = lo; t.v.hi = hi; }
      return t;
    };
    DNF d;
    switch (op) {
      case OP_EQ: d.push_back(mkT(k, k)); break;
      case OP_NE:
        if (k != IMIN) d.push_back(mkT(IMIN, k - 1));
        if (k != IMAX) d.push_back(mkT(k + 1, IMAX));
        break;
      case OP_LT: if (k != IMIN) d.push_back(mkT(IMIN, k - 1)); break;
      case OP_LE: d.push_back(mkT(IMIN, k)); break;
      case OP_GT: if (k != IMAX) d.push_back(mkT(k + 1, IMAX)); break;
      case OP_GE: d.push_back(mkT(k, IMAX)); break;
    }
    return d;
  }

  static uint8_t flip(uint8_t op) {
    switch (op) { case OP_LT: return OP_GT; case OP_LE: return OP_GE; case OP_GT: return OP_LT; case OP_GE: return OP_LE; }
    return op;
  }
  static uint8_t negate(uint8_t op) {
    switch (op) {
      case OP_EQ: return OP_NE; case OP_NE: return OP_EQ; case OP_LT: return OP_GE;
      case OP_GE: return OP_LT; case OP_LE: return OP_GT; case OP_GT: return OP_LE;
    }
    return op;
  }

  DNF lower(const ExprP& e, bool neg) {
    if (!ok) return {};
    switch (e->op) {
      case OP_TRUE: case OP_FALSE: {
        bool v = (e->op == OP_TRUE) != neg;
        return v ? DNF{Term{}} : DNF{};
      }
      case OP_NOT: return lower(e->a, !neg);
      case OP_AND: case OP_OR: {
        bool is_and = (e->op == OP_AND) != neg;
        DNF x = lower(e->a, neg), y = lower(e->b, neg);
        if (is_and) return conj(x, y);
        x.insert(x.end(), y.begin(), y.end());
        if (x.size() > STENCIL_MAX_TERMS) fail("predicate needs too many terms");
        return x;
      }
      case OP_EV_TOPIC_EQ: return int_cmp(neg ? OP_NE : OP_EQ, e->i32, true);
      case OP_EQ: case OP_NE: case OP_LT: case OP_LE: case OP_GT: case OP_GE: {
        ExprP f = e->a, c = e->b;
        uint8_t op = e->op;
        if (f->op != OP_FIELD) { std::swap(f, c); op = flip(op); }
        if (f->op != OP_FIELD || !(c->op == OP_CONST_I32 || c->op == OP_CONST_I64 || c->op == OP_CONST_F64)) {
          fail("predicate is not a column/constant comparison");
          return {};
        }
        if (col >= 0 && f->col != col) { fail("predicates read more than one column"); return {}; }
        col = f->col;
        coltype = f->t;
        if (neg) op = negate(op);
        if (f->t == T_F64) {
          if (op == OP_NE || neg) { fail("negated comparison on a double column (NaN)"); return {}; }
          double k = c->op == OP_CONST_F64 ? c->f64 : c->op == OP_CONST_I32 ? double(c->i32) : double(c->i64);
          Term t; t.has_v = true;
          t.v.dlo = -INFINITY; t.v.dhi = INFINITY;
          switch (op) {
            case OP_EQ: t.v.dlo = t.v.dhi = k; break;
            case OP_LT: t.v.dhi = nextafter(k, -INFINITY); break;
            case OP_LE: t.v.dhi = k; break;
            case OP_GT: t.v.dlo = nextafter(k, INFINITY); break;
            case OP_GE: t.v.dlo = k; break;
          }
          if (isnan(k)) return {};
          return DNF{t};
        }
        if (c->op == OP_CONST_F64) { fail("integer column compared with a double constant"); return {}; }
        int64_t k = c->op == OP_CONST_I32 ? int64_t(c->i32) : c->i64;
        return int_cmp(op, k, false);
      }
      default:
        fail("predicate uses state, sequence, arithmetic or event metadata");
        return {};
    }
  }
};

// exact membership of (value, topic) in stage s of the lowered program
bool stage_accepts(const StencilProgram& S, int s, bool isf, int64_t vi, double vf, int64_t topic) {
  for (int t = 0; t < S.nterms[s]; t++) {
    bool ok = true;
    if (S.hasv[s][t]) ok = isf ? (S.vf[s][t].lo <= vf && vf <= S.vf[s][t].hi) : (S.vi[s][t].lo <= vi && vi <= S.vi[s][t].hi);
    ok = ok && S.tp[s][t].lo <= topic && topic <= S.tp[s][t].hi;
    if (ok) return true;
  }
  return false;
}

bool build_table(StencilProgram& S) {
  const bool isf = S.coltype == T_F64;
  std::vector<int64_t> bi;
  std::vector<double> bf;
  std::vector<int64_t> tb;
  for (int s = 0; s < STENCIL_MAX_K; s++)
    for (int t = 0; t < S.nterms[s]; t++) {
      if (S.hasv[s][t]) {
        if (isf) {
          if (S.vf[s][t].lo > -INFINITY) bf.push_back(S.vf[s][t].lo);
          if (S.vf[s][t].hi < INFINITY) bf.push_back(nextafter(S.vf[s][t].hi, INFINITY));
        } else {
          if (S.vi[s][t].lo > IMIN) bi.push_back(S.vi[s][t].lo);
          if (S.vi[s][t].hi < IMAX) bi.push_back(S.vi[s][t].hi + 1);
        }
      }
      if (S.tp[s][t].lo > IMIN) tb.push_back(S.tp[s][t].lo);
      if (S.tp[s][t].hi < IMAX) tb.push_back(S.tp[s][t].hi + 1);
    }
  auto uniq = [](auto& v) { std::sort(v.begin(), v.end()); v.erase(std::unique(v.begin(), v.end()), v.end()); };
  if (S.coltype == T_I32) {                       // the column is int32: clamp the cut points
    for (auto& b : bi) b = std::max<int64_t>(b, INT32_MIN);
    bi.erase(std::remove_if(bi.begin(), bi.end(), [](int64_t b) { return b > INT32_MAX; }), bi.end());
  }
  for (auto& b : tb) b = std::max<int64_t>(b, INT32_MIN);   // topic ids are int32
  tb.erase(std::remove_if(tb.begin(), tb.end(), [](int64_t b) { return b > INT32_MAX; }), tb.end());
  uniq(bi); uniq(bf); uniq(tb);
  const int nb = int(isf ? bf.size() : bi.size());
  if (nb > 15 || tb.size() > 3) return false;
  S.nbp = nb;
  S.ntbp = int(tb.size());
  for (int i = 0; i < nb; i++) { if (isf) S.bpf[i] = bf[i]; else S.bpi[i] = bi[i]; }
  for (size_t i = 0; i < tb.size(); i++) S.tbp[i] = int32_t(tb[i]);
  memset(S.table, 0, sizeof S.table);
  memset(S.nan_mask, 0, sizeof S.nan_mask);
  for (int it = 0; it <= S.ntbp; it++) {
    const int64_t trep = it == 0 ? (S.ntbp ? int64_t(S.tbp[0]) - 1 : 0) : int64_t(S.tbp[it - 1]);
    for (int iv = 0; iv <= nb; iv++) {
      int64_t vi = 0;
      double vf = 0;
      if (isf) vf = iv == 0 ? -INFINITY : bf[iv - 1];
      else vi = iv == 0 ? (nb ? bi[0] - (bi[0] > IMIN ? 1 : 0) : 0) : bi[iv - 1];
      uint8_t m = 0;
      for (int s = 0; s < STENCIL_MAX_K; s++) m |= uint8_t(stage_accepts(S, s, isf, vi, vf, trep)) << s;
      S.table[it * 16 + iv] = m;
    }
    uint8_t m = 0;
    for (int s = 0; s < STENCIL_MAX_K; s++) m |= uint8_t(stage_accepts(S, s, isf, 0, NAN, trep)) << s;
    S.nan_mask[it] = m;
  }
  S.lut_n = 0;
  S.lut_lo = 0;
  memset(S.lut, 0, sizeof S.lut);
  // (worth it from ~6 breakpoints: C5's 8 -> kernel -2 %, C2's 4 -> +0.5 %, profiles/r02_ab_c2_c5_lut.log)
  if (!isf && S.ntbp == 0 && nb >= 6 && bi.back() - bi.front() < int64_t(sizeof S.lut)) {
    S.lut_lo = bi.front();
    S.lut_n = int32_t(bi.back() - bi.front() + 1);
    for (int r = 0, iv = 0; r < S.lut_n; r++) {   // iv = #{breakpoints <= lut_lo + r}
      while (iv < nb && bi[iv] <= S.lut_lo + r) iv++;
      S.lut[r] = S.table[iv];
    }
  }
  return true;
}

// Chain extension of Q9: with optional() stages (not the first; a final
// optional is already rejected by StagesFactory) and nothing else that adds
// TAKE or IGNORE edges, no edge combination is branching (NFA.java:392-397), so
// every run is deterministic: on each record it either consumes it (BEGIN of
// its stage) or skips optional stages on it (SKIP_PROCEED, :222-237) until a
// BEGIN consumes it, or dies.  A run started at record j therefore emits at
// most one match, made of consecutive records; runs are queued oldest first,
// so matches of one record come out in ascending start order.  Every run
// carries its own first Dewey digit and nodes are shared only at a stage both
// runs consume, so the first-compatible traversal (MatchedEvent.java:90-99)
// always returns the run's own predecessors.
void analyse_stencil(Program& P) {
  auto no = [&](const std::string& w) { P.stencil_ok = false; P.stencil_why = w; };
  const int k = int(P.pats.size());
  if (k > STENCIL_MAX_K) return no("more than 8 stages");
  uint32_t opt = 0;
  for (int i = 0; i < k; i++) {
    const auto& p = P.pats[i];
    if (p.strategy != S_STRICT) return no("non-strict selection strategy");
    if (p.one_or_more || p.times > 1) return no("quantifier");
    if (p.optional) {
      if (i == 0) return no("optional first stage");
      opt |= 1u << i;
    }
    if (!p.folds.empty()) return no("fold");
    for (int j = 0; j < i; j++)
      if (P.pats[j].name_id == p.name_id) return no("duplicate stage names");
  }
  if (opt && k > CHAIN_MAX_K) return no("optional stages in a pattern of more than 4 stages");
  Lowering L;
  StencilProgram& S = P.stencil;
  memset(&S, 0, sizeof S);
  S.k = k;
  S.chain = opt ? 1 : 0;
  S.optmask = int32_t(opt);
  auto lower_slot = [&](int slot, const ExprP& pred) {
    DNF d = L.lower(pred, false);
    if (!L.ok) return;
    if (d.size() > STENCIL_MAX_TERMS) { L.fail("too many terms"); return; }
    S.nterms[slot] = int(d.size());
    S.pslots |= 1 << slot;
    for (size_t t = 0; t < d.size(); t++) {
      const Term& tm = d[t];
      S.vi[slot][t] = tm.has_v ? StencilAtomI{tm.v.lo, tm.v.hi} : StencilAtomI{IMIN, IMAX};
      S.vf[slot][t] = tm.has_v ? StencilAtomF{tm.v.dlo, tm.v.dhi} : StencilAtomF{-INFINITY, INFINITY};
      S.tp[slot][t] = tm.has_t ? StencilAtomI{tm.t.lo, tm.t.hi} : StencilAtomI{IMIN, IMAX};
      S.hasv[slot][t] = tm.has_v ? 1 : 0;
      if (tm.has_t) S.use_topic = 1;
    }
  };
  for (int i = 0; i < k && L.ok; i++) {
    const auto& p = P.pats[i];
    S.name[i] = p.name_id;
    lower_slot(i, p.topic >= 0 ? mk(OP_AND, mk_topic(p.topic), p.pred) : p.pred);
    // SKIP_PROCEED of an optional stage: successor predicate without its topic (StagesFactory.java:165)
    if (L.ok && (opt >> i & 1)) lower_slot(CHAIN_MAX_K + i, P.pats[i + 1].pred);
  }
  if (!L.ok) return no(L.why);
  if (L.col < 0) { L.col = 0; L.coltype = P.coltypes.empty() ? T_I32 : P.coltypes[0]; }
  S.col = L.col;
  S.coltype = L.coltype;
  if (!build_table(S)) return no("predicates cut the value axis into more than 16 intervals");
  P.stencil_ok = true;
  P.stencil_why.clear();
}

// ---------------------------------------------------------------- deterministic runs
bool same_expr(const ExprP& a, const ExprP& b) {
  if (!a || !b) return a == b;
  if (a->op != b->op || a->t != b->t || a->ct != b->ct) return false;
  switch (a->op) {
    case OP_CONST_I32: case OP_EV_TOPIC_EQ: if (a->i32 != b->i32) return false; break;
    case OP_CONST_I64: if (a->i64 != b->i64) return false; break;
    case OP_CONST_F64: if (memcmp(&a->f64, &b->f64, sizeof(double)) != 0) return false; break;
    case OP_FIELD: case OP_SEQ_AVG: if (a->col != b->col) return false; break;
    case OP_SEQ_AGG: if (a->col != b->col || a->sname != b->sname || a->name != b->name) return false; break;
    case OP_STATE_GET: case OP_STATE_GET_OR_ELSE: if (a->name != b->name) return false; break;
    default: break;
  }
  return same_expr(a->a, b->a) && same_expr(a->b, b->b);
}
bool is_cmp(uint8_t op) { return op >= OP_EQ && op <= OP_GE; }
bool complementary(uint8_t x, uint8_t y) {
  auto c = [](uint8_t o) -> uint8_t {
    switch (o) { case OP_EQ: return OP_NE; case OP_NE: return OP_EQ; case OP_LT: return OP_GE;
                 case OP_GE: return OP_LT; case OP_GT: return OP_LE; case OP_LE: return OP_GT; }
    return 0;
  };
  return c(x) == y;
}
uint8_t flip_cmp(uint8_t o) {
  switch (o) { case OP_LT: return OP_GT; case OP_LE: return OP_GE; case OP_GT: return OP_LT; case OP_GE: return OP_LE; }
  return o;
}
// p AND q can never both be true (whatever the run's states): structural
// complements, different topics, or disjoint value intervals of one column
bool disjoint(const ExprP& p, const ExprP& q) {
  if (!p || !q) return false;                                   // TRUE
  if (p->op == OP_FALSE || q->op == OP_FALSE) return true;
  if (p->op == OP_AND) return disjoint(p->a, q) || disjoint(p->b, q);
  if (q->op == OP_AND) return disjoint(p, q->a) || disjoint(p, q->b);
  if (p->op == OP_OR) return disjoint(p->a, q) && disjoint(p->b, q);
  if (q->op == OP_OR) return disjoint(p, q->a) && disjoint(p, q->b);
  if (p->op == OP_NOT && same_expr(p->a, q)) return true;
  if (q->op == OP_NOT && same_expr(q->a, p)) return true;
  if (p->op == OP_EV_TOPIC_EQ && q->op == OP_EV_TOPIC_EQ) return p->i32 != q->i32;
  if (is_cmp(p->op) && is_cmp(q->op)) {
    if (same_expr(p->a, q->a) && same_expr(p->b, q->b) && complementary(p->op, q->op)) return true;
    if (same_expr(p->a, q->b) && same_expr(p->b, q->a) && complementary(p->op, flip_cmp(q->op))) return true;
  }
  Lowering L;
  DNF a = L.lower(p, false), b = L.lower(q, false);
  if (!L.ok) return false;
  for (auto& ta : a)
    for (auto& tb : b) {
      Term t = ta;
      if (L.intersect(t, tb)) return false;
    }
  return true;
}
bool uses_seq(const ExprP& e) {
  return e && (e->op == OP_SEQ_AVG || e->op == OP_SEQ_AGG || uses_seq(e->a) || uses_seq(e->b));
}

// Strict patterns whose stages never take a branching edge combination
// (NFA.java:392-397): without IGNORE edges that needs TAKE and PROCEED of a
// oneOrMore stage to exclude each other, i.e. its predicate and its successor's
// to be disjoint (PROCEED = succ OR NOT pred, StagesFactory.java:131-137).  Then
// every run is one deterministic walk over consecutive records from the record
// its begin stage consumed: it owns a fresh run sequence (so its aggregates),
// its Dewey versions start with a digit no other run has, and its buffer
// traversal returns exactly the records it consumed.
void analyse_runs(Program& P) {
  auto no = [&](const std::string& w) { P.runs_ok = false; P.runs_why = w; };
  if (!P.general_ok) return no("not lowered to the device NFA");
  if (P.states.size() > size_t(RUNS_MAX_STATES)) return no("more than 8 aggregate states");
  const int k = int(P.pats.size());
  for (int i = 0; i < k; i++) {
    const auto& p = P.pats[i];
    if (p.strategy != S_STRICT) return no("non-strict selection strategy");
    if (i == 0 && (p.one_or_more || p.times > 1 || p.optional)) return no("quantifier on the first stage");
    if (p.one_or_more && (p.optional || p.times > 1)) return no("zeroOrMore");
    if (uses_seq(p.pred)) return no("sequence condition");
    for (auto& f : p.folds)
      if (uses_seq(f.expr)) return no("sequence condition");
    if (p.one_or_more) {
      const auto& q = P.pats[i + 1];
      ExprP pw = p.topic >= 0 ? mk(OP_AND, mk_topic(p.topic), p.pred) : p.pred;
      ExprP qw = q.topic >= 0 ? mk(OP_AND, mk_topic(q.topic), q.pred) : q.pred;
      if (!disjoint(pw, qw)) return no("oneOrMore predicate not provably exclusive of its successor's");
    }
  }
  P.runs_ok = true;
  P.runs_why.clear();
}

// ---------------------------------------------------------------- bytecode
struct CodeGen {
  const std::vector<std::string>* names = nullptr;   // stage names (OP_SEQ_AGG filters)
  std::vector<int32_t> code;
  bool ok = true;
  std::string why;
  int depth = 0, maxdepth = 0;      // operand-stack depth (the device keeps <= NFA_STACK slots in registers)

  static int effect(uint8_t o) {
    switch (o) {
      case BC_PUSH: case BC_FIELD: case BC_EV_KEY: case BC_EV_TS: case BC_EV_OFFSET: case BC_EV_PARTITION:
      case BC_TOPIC_EQ: case BC_STATE_GET: case BC_FOLD_CURR: case BC_SEQ_AVG: case BC_SEQ_AGG: return 1;
      case BC_END: case BC_STATE_GET_OR_ELSE: case BC_NOT: case BC_NEG_I32: case BC_NEG_I64: case BC_NEG_F64:
      case BC_I64_TO_I32: case BC_I_TO_F64: case BC_F64_TO_I32: case BC_F64_TO_I64: return 0;
      default: return -1;           // binary operators, POP, and the fall-through of JZ/JNZ_KEEP
    }
  }
  void op(uint8_t o, int a = 0, int b = 0) {
    code.push_back(int32_t(o) | (a << 8) | (b << 16));
    depth += effect(o);
    maxdepth = std::max(maxdepth, depth);
  }
  void push64(int64_t v) {
    op(BC_PUSH);
    code.push_back(int32_t(uint32_t(uint64_t(v))));
    code.push_back(int32_t(uint32_t(uint64_t(v) >> 32)));
  }
  int jump(uint8_t o) {
    op(o);
    code.push_back(0);
    return int(code.size()) - 1;
  }
  void patch(int at) { code[at] = int32_t(code.size()) - (at + 1); }
  void cvt(uint8_t from, uint8_t to) {
    if (from == to || (from == T_I32 && to == T_I64)) return;     // ints are kept sign-extended
    if (to == T_F64) op(BC_I_TO_F64);
    else if (from == T_F64) op(to == T_I32 ? BC_F64_TO_I32 : BC_F64_TO_I64);
    else op(BC_I64_TO_I32);
  }
  void arith(uint8_t eop, uint8_t t) {
    static const uint8_t base[3] = {BC_ADD_I32, BC_ADD_I64, BC_ADD_F64};
    const int k = t == T_I32 ? 0 : t == T_I64 ? 1 : 2;
    const int off = eop == OP_ADD ? 0 : eop == OP_SUB ? 1 : eop == OP_MUL ? 2 : eop == OP_DIV ? 3 : eop == OP_REM ? 4 : 5;
    op(uint8_t(base[k] + off));
  }
  // x itself when it is an int, or the int under a cast of an int to double; else null
  static ExprP int32_operand(const ExprP& x) {
    if (x->t == T_I32) return x;
    if (x->op == OP_CAST && x->ct == T_F64 && x->a && x->a->t == T_I32) return x->a;
    return nullptr;
  }
  void gen(const ExprP& e) {
    if (!ok) return;
    switch (e->op) {
      case OP_TRUE: push64(1); break;
      case OP_FALSE: push64(0); break;
      case OP_CONST_I32: push64(e->i32); break;
      case OP_CONST_I64: push64(e->i64); break;
      case OP_CONST_F64: { int64_t b; memcpy(&b, &e->f64, 8); push64(b); break; }
      case OP_FIELD: op(BC_FIELD, e->col, e->t); break;
      case OP_EV_KEY: op(BC_EV_KEY); break;
      case OP_EV_TS: op(BC_EV_TS); break;
      case OP_EV_OFFSET: op(BC_EV_OFFSET); break;
      case OP_EV_PARTITION: op(BC_EV_PARTITION); break;
      case OP_EV_TOPIC_EQ: op(BC_TOPIC_EQ); code.push_back(e->i32); break;
      case OP_STATE_GET: op(BC_STATE_GET, e->name, e->ct); break;
      case OP_STATE_GET_OR_ELSE: {
        op(BC_STATE_GET_OR_ELSE, e->name, e->ct);
        code.push_back(0);
        const int at = int(code.size()) - 1;
        gen(e->a);
        patch(at);
        break;
      }
      case OP_FOLD_CURR: op(BC_FOLD_CURR, 0, e->ct); break;
      case OP_SEQ_AVG: op(BC_SEQ_AVG, e->col); break;
      case OP_SEQ_AGG: {                      // a = column, b = kind; next word: stage name id
        int sid = SEQ_ANY_STAGE;
        if (e->name >= 0) {
          const auto it = std::find(names->begin(), names->end(), e->sname);
          sid = it == names->end() ? -2 : int(it - names->begin());   // unknown: never present
        }
        op(BC_SEQ_AGG, e->col, e->ct);
        code.push_back(sid);
        break;
      }
      case OP_NOT: gen(e->a); op(BC_NOT); break;
      case OP_AND: { gen(e->a); int j = jump(BC_JZ_KEEP); gen(e->b); patch(j); break; }
      case OP_OR: { gen(e->a); int j = jump(BC_JNZ_KEEP); gen(e->b); patch(j); break; }
      case OP_ADD: case OP_SUB: case OP_MUL: case OP_DIV: case OP_REM:
        gen(e->a); cvt(e->a->t, e->t); gen(e->b); cvt(e->b->t, e->t); arith(e->op, e->t); break;
      case OP_NEG: gen(e->a); arith(OP_NEG, e->t); break;
      case OP_EQ: case OP_NE: case OP_LT: case OP_LE: case OP_GT: case OP_GE: {
        if (e->a->t == T_BOOL) {
          gen(e->a); gen(e->b); op(e->op == OP_EQ ? BC_EQ_B : BC_NE_B);
          break;
        }
        const uint8_t t = std::max(e->a->t, e->b->t);
        const int off = e->op - OP_EQ;
        // two int values compared as doubles (e.g. `(sum / count).asDouble() >= value`): every int fits a
        // double exactly, so the int comparison gives the same answer without the two conversions
        const ExprP ia = int32_operand(e->a), ib = int32_operand(e->b);
        if (t == T_F64 && ia && ib) {
          gen(ia); gen(ib);
          op(uint8_t(BC_EQ_I + off));
          break;
        }
        gen(e->a); cvt(e->a->t, t); gen(e->b); cvt(e->b->t, t);
        op(uint8_t((t == T_F64 ? BC_EQ_F : BC_EQ_I) + off));
        break;
      }
      case OP_CAST: gen(e->a); cvt(e->a->t, e->ct); break;
      default: ok = false; why = "unsupported expression opcode"; break;
    }
  }
  int emit(const ExprP& e, uint8_t result_type = 0xFF) {
    const int at = int(code.size());
    depth = 0;
    gen(e);
    if (result_type != 0xFF) cvt(e->t, result_type);
    op(BC_END);
    return at;
  }
};

// an edge predicate that reads nothing but the current record's fields
// (no States, fold accumulator or partial sequence) has one value per record
// whatever run evaluates it
bool event_only(const ExprP& e) {
  if (!e) return true;
  switch (e->op) {
    case OP_STATE_GET: case OP_STATE_GET_OR_ELSE: case OP_FOLD_CURR: case OP_SEQ_AVG: case OP_SEQ_AGG: return false;
    default: return event_only(e->a) && event_only(e->b);
  }
}

}  // namespace

int lower_general(Program& P, std::string& why) {
  DevProgram& D = P.dev;
  memset(&D, 0, sizeof D);
  if (P.stages.size() > size_t(NFA_MAX_STAGES)) { why = "too many stages"; return CEP_E_UNSUPPORTED; }
  if (P.states.size() > size_t(NFA_MAX_STATES)) { why = "too many states"; return CEP_E_UNSUPPORTED; }
  if (P.coltypes.size() > 16) { why = "too many columns"; return CEP_E_UNSUPPORTED; }
  D.nstages = int32_t(P.stages.size());
  D.begin = P.begin;
  D.nstates = int32_t(P.states.size());
  D.ncols = int32_t(P.coltypes.size());
  // NFA.evaluate recurses along PROCEED / SKIP_PROCEED edges, which always lead
  // to a later pattern's stage: the longest such path bounds the frame stack
  {
    std::vector<int> depth(P.stages.size(), 1);
    for (int id = 0; id < int(P.stages.size()); id++)           // targets have smaller ids (built last-first)
      for (auto& e : P.stages[id].edges)
        if ((e.op == E_PROCEED || e.op == E_SKIP_PROCEED) && e.target >= 0)
          depth[id] = std::max(depth[id], depth[e.target] + 1);
    int m = 0;
    for (int d : depth) m = std::max(m, d);
    D.maxdepth = m + 1;                                          // + the epsilon frame a run starts on
    if (D.maxdepth > NFA_MAX_FRAMES) { why = "PROCEED chain deeper than the device frame stack"; return CEP_E_UNSUPPORTED; }
  }
  for (size_t c = 0; c < P.coltypes.size(); c++) D.coltype[c] = P.coltypes[c];
  D.ndefined = int32_t(P.defined_states.size());
  for (size_t i = 0; i < P.defined_states.size(); i++) D.defined[i] = P.defined_states[i];
  // buffer-node slots: one per (stage name, stage type) pair (Matched.java:31-35)
  std::vector<std::pair<int, int>> slots;
  CodeGen cg;
  cg.names = &P.names;
  for (auto& s : P.stages) {
    DevStage& d = D.st[s.id];
    d.name = s.name;
    d.type = s.type;
    auto key = std::make_pair(s.name, int(s.type));
    auto it = std::find(slots.begin(), slots.end(), key);
    if (it == slots.end()) { slots.push_back(key); it = slots.end() - 1; }
    d.slot = int32_t(it - slots.begin());
    if (s.edges.size() > size_t(NFA_MAX_EDGES)) { why = "too many edges"; return CEP_E_UNSUPPORTED; }
    d.nedges = int32_t(s.edges.size());
    for (size_t e = 0; e < s.edges.size(); e++) {
      d.op[e] = s.edges[e].op;
      d.target[e] = s.edges[e].target;
      d.pred[e] = s.edges[e].pred ? cg.emit(s.edges[e].pred) : -1;
      d.sl[e] = -1;
      if (d.pred[e] >= 0 && event_only(s.edges[e].pred) && D.nsl < NFA_MAX_SL) {
        d.sl[e] = D.nsl;
        D.sl_pc[D.nsl++] = d.pred[e];
      }
    }
    if (s.pattern >= 0) {
      const auto& folds = P.pats[s.pattern].folds;
      if (folds.size() > size_t(NFA_MAX_FOLDS)) { why = "too many folds"; return CEP_E_UNSUPPORTED; }
      d.nfolds = int32_t(folds.size());
      for (size_t f = 0; f < folds.size(); f++) {
        d.fold_state[f] = folds[f].state;
        d.fold_type[f] = folds[f].type;
        d.fold_code[f] = cg.emit(folds[f].expr, folds[f].type);
      }
    }
  }
  if (!cg.ok) { why = cg.why; return CEP_E_UNSUPPORTED; }
  if (cg.maxdepth > NFA_STACK) { why = "expression nests deeper than the device operand stack"; return CEP_E_UNSUPPORTED; }
  if (slots.size() > size_t(NFA_MAX_SLOTS)) { why = "too many buffer slots"; return CEP_E_UNSUPPORTED; }
  if (cg.code.size() > size_t(NFA_MAX_CODE)) { why = "predicate code too large"; return CEP_E_UNSUPPORTED; }
  D.nslots = int32_t(slots.size());
  for (size_t i = 0; i < slots.size(); i++) D.slot_name[i] = slots[i].first;
  memcpy(D.code, cg.code.data(), cg.code.size() * sizeof(int32_t));
  return CEP_OK;
}

int compile_ir(const uint8_t* ir, size_t len, Program& P, std::string& err) {
  Reader r{ir, len};
  if (len < 8 || memcmp(ir, "KCEP", 4) != 0) { err = "bad magic"; return CEP_E_BAD_IR; }
  r.i = 4;
  if (r.get<uint32_t>() != 1) { err = "unsupported IR version"; return CEP_E_BAD_IR; }
  uint16_t ncols = r.get<uint16_t>();
  for (int i = 0; i < ncols; i++) {
    uint8_t t = r.get<uint8_t>();
    if (t < T_I32 || t > T_F64) r.bad = true;
    P.coltypes.push_back(t);
  }
  P.names.push_back("$final");
  uint16_t npat = r.get<uint16_t>();
  if (npat == 0) r.bad = true;
  for (int i = 0; i < npat && !r.bad; i++) {
    PatternDef pd;
    bool isnull = false;
    r.str(pd.name, isnull);
    pd.level = r.get<int32_t>();
    if (isnull) pd.name = std::to_string(pd.level);            // Pattern.getName (Pattern.java:181-183)
    pd.name_id = intern(P.names, pd.name);
    pd.strategy = r.get<uint8_t>();
    pd.topic = r.get<int32_t>();
    pd.one_or_more = r.get<uint8_t>();
    pd.optional = r.get<uint8_t>();
    pd.times = r.get<int32_t>();
    pd.window_ms = r.get<int64_t>();
    if (r.get<uint8_t>()) pd.pred = parse_expr(r, P, 0);
    uint16_t nf = r.get<uint16_t>();
    for (int f = 0; f < nf && !r.bad; f++) {
      std::string s;
      if (!r.str(s, isnull) || isnull) { r.bad = true; break; }
      Fold fd;
      fd.state = intern(P.states, s);
      fd.type = r.get<uint8_t>();
      fd.expr = parse_expr(r, P, 0);
      if (!fd.expr || fd.expr->t == T_BOOL || fd.type < T_I32 || fd.type > T_F64) r.bad = true;
      pd.folds.push_back(fd);
    }
    P.pats.push_back(std::move(pd));
  }
  if (r.bad || r.i != len) { err = "malformed pattern IR"; return CEP_E_BAD_IR; }

  // StagesFactory.make (StagesFactory.java:49-70)
  try {
    int next_id = 0;
    P.stages.push_back(StageDef{next_id++, 0, ST_FINAL, -1, -1, {}});
    int succ_stage = 0, succ_pat = -1;
    for (int cur = int(P.pats.size()) - 1; cur >= 0; cur--) {
      auto st = build_stages(P, cur > 0 ? ST_NORMAL : ST_BEGIN, cur, succ_stage, succ_pat, P.stages, next_id);
      for (auto& s : st) P.stages.push_back(std::move(s));
      succ_stage = int(P.stages.size()) - 1;
      succ_pat = cur;
    }
  } catch (const BuildErr& e) {
    err = e.msg;
    return e.code;
  }
  for (auto& s : P.stages)                                       // Stages.getBeginingStage (Stages.java:49-51)
    if (s.type == ST_BEGIN) { P.begin = s.id; break; }
  for (auto& s : P.stages) {                                     // Stages.getDefinedStates (Stages.java:62-67)
    if (s.pattern < 0) continue;
    for (auto& f : P.pats[s.pattern].folds)
      if (std::find(P.defined_states.begin(), P.defined_states.end(), f.state) == P.defined_states.end())
        P.defined_states.push_back(f.state);
  }
  analyse_stencil(P);
  P.general_ok = lower_general(P, P.general_why) == CEP_OK;
  analyse_runs(P);
  P.has_seq = false;
  for (const auto& pd : P.pats) {
    P.has_seq = P.has_seq || uses_seq(pd.pred);
    for (const auto& f : pd.folds) P.has_seq = P.has_seq || uses_seq(f.expr);
  }
  return CEP_OK;
}

// a pattern whose evaluations read or write more than the current record: aggregates (folds, defined
// states, state reads) or partial sequences -- the wave kernel's stateful round machinery (nfa_wave.h)
bool wave_stateful(const DevProgram& D) {
  if (D.nstates || D.ndefined) return true;
  for (int s = 0; s < D.nstages; s++) {
    const DevStage& t = D.st[s];
    if (t.nfolds) return true;
    for (int e = 0; e < t.nedges; e++)
      if (t.pred[e] >= 0 && t.sl[e] < 0) return true;
  }
  return false;
}

}  // namespace kcep

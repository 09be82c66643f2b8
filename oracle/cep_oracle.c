/*
 * cep_oracle.c — TEST INFRASTRUCTURE ONLY (see cep_oracle.h).
 *
 * Plain-C restatement of the reference's per-record NFA evaluation path.  Every
 * function cites the reference file:line it follows.  Paths are relative to
 * /root/reference/core/src/main/java/com/github/fhuss/kafka/streams/cep/.
 *
 * Storage emulation: the reference keeps the shared buffer and the aggregates in
 * Kafka KeyValueStores of serialised bytes, so every get() returns a fresh copy
 * and only explicit put()s persist (Q4 in SURVEY.md).  Here the stores are hash
 * maps and the copy-on-read is modelled by computing the would-be copy and
 * writing it back exactly where the reference calls put()/delete().
 */
#include "cep_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------- */
/* small utilities                                                           */
/* ------------------------------------------------------------------------- */
#define T_BOOL ORC_T_BOOL
#define T_I32 ORC_T_I32
#define T_I64 ORC_T_I64
#define T_F64 ORC_T_F64

static void* xmalloc(size_t n) {
  void* p = malloc(n ? n : 1);
  if (!p) { fprintf(stderr, "oracle: out of memory\n"); abort(); }
  return p;
}
static void* xrealloc(void* p, size_t n) {
  p = realloc(p, n ? n : 1);
  if (!p) { fprintf(stderr, "oracle: out of memory\n"); abort(); }
  return p;
}
static void* xcalloc(size_t a, size_t b) {
  void* p = calloc(a ? a : 1, b ? b : 1);
  if (!p) { fprintf(stderr, "oracle: out of memory\n"); abort(); }
  return p;
}

#define VEC(T) struct { T* a; int64_t n, cap; }
#define VPUSH(v, x) do { if ((v).n == (v).cap) { (v).cap = (v).cap ? (v).cap * 2 : 16; \
      (v).a = xrealloc((v).a, (size_t)(v).cap * sizeof(*(v).a)); } (v).a[(v).n++] = (x); } while (0)
#define VFREE(v) do { free((v).a); (v).a = NULL; (v).n = (v).cap = 0; } while (0)

/* bump arena for immutable DeweyVersions */
typedef struct Chunk { struct Chunk* next; size_t used, cap; char data[]; } Chunk;
typedef struct { Chunk* head; } Arena;
static void* arena_alloc(Arena* a, size_t n) {
  n = (n + 7) & ~(size_t)7;
  if (!a->head || a->head->used + n > a->head->cap) {
    size_t cap = n > (1u << 20) ? n : (1u << 20);
    Chunk* c = xmalloc(sizeof(Chunk) + cap);
    c->next = a->head; c->used = 0; c->cap = cap; a->head = c;
  }
  void* p = a->head->data + a->head->used;
  a->head->used += n;
  return p;
}
static void arena_free(Arena* a) {
  Chunk* c = a->head;
  while (c) { Chunk* n = c->next; free(c); c = n; }
  a->head = NULL;
}

/* open-addressing map: 4 x int64 key -> int64 value */
typedef struct { int64_t k[4]; } Key4;
typedef struct { Key4* keys; int64_t* vals; uint8_t* st; int64_t cap, n, used; } Map;
static uint64_t mix64(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
  return x;
}
static uint64_t key_hash(const Key4* k) {
  uint64_t h = 0x9e3779b97f4a7c15ULL;
  for (int i = 0; i < 4; i++) h = mix64(h ^ (uint64_t)k->k[i]) + 0x9e3779b97f4a7c15ULL * (uint64_t)(i + 1);
  return h;
}
static void map_init(Map* m) { memset(m, 0, sizeof(*m)); }
static void map_free(Map* m) { free(m->keys); free(m->vals); free(m->st); memset(m, 0, sizeof(*m)); }
static void map_rehash(Map* m, int64_t ncap);
static int64_t* map_find(const Map* m, const Key4* k) {
  if (!m->cap) return NULL;
  uint64_t mask = (uint64_t)m->cap - 1, i = key_hash(k) & mask;
  for (;;) {
    if (m->st[i] == 0) return NULL;
    if (m->st[i] == 1 && !memcmp(&m->keys[i], k, sizeof(Key4))) return &m->vals[i];
    i = (i + 1) & mask;
  }
}
static void map_put(Map* m, const Key4* k, int64_t v) {
  int64_t* p = map_find(m, k);
  if (p) { *p = v; return; }
  if ((m->used + 1) * 4 >= m->cap * 3) map_rehash(m, m->cap ? (m->n * 2 >= m->cap / 2 ? m->cap * 2 : m->cap) : 64);
  uint64_t mask = (uint64_t)m->cap - 1, i = key_hash(k) & mask;
  while (m->st[i] == 1) i = (i + 1) & mask;
  if (m->st[i] == 0) m->used++;
  m->st[i] = 1; m->keys[i] = *k; m->vals[i] = v; m->n++;
}
static int map_del(Map* m, const Key4* k) {
  if (!m->cap) return 0;
  uint64_t mask = (uint64_t)m->cap - 1, i = key_hash(k) & mask;
  for (;;) {
    if (m->st[i] == 0) return 0;
    if (m->st[i] == 1 && !memcmp(&m->keys[i], k, sizeof(Key4))) { m->st[i] = 2; m->n--; return 1; }
    i = (i + 1) & mask;
  }
}
static void map_rehash(Map* m, int64_t ncap) {
  Map o = *m;
  m->cap = ncap; m->n = 0; m->used = 0;
  m->keys = xmalloc((size_t)ncap * sizeof(Key4));
  m->vals = xmalloc((size_t)ncap * sizeof(int64_t));
  m->st = xcalloc((size_t)ncap, 1);
  for (int64_t i = 0; i < o.cap; i++)
    if (o.st[i] == 1) map_put(m, &o.keys[i], o.vals[i]);
  free(o.keys); free(o.vals); free(o.st);
}

/* ------------------------------------------------------------------------- */
/* expression IR (kcep/expr.py)                                              */
/* ------------------------------------------------------------------------- */
enum {
  OP_TRUE = 0x01, OP_FALSE = 0x02, OP_CONST_I32 = 0x03, OP_CONST_I64 = 0x04, OP_CONST_F64 = 0x05,
  OP_FIELD = 0x10, OP_EV_KEY = 0x11, OP_EV_TS = 0x12, OP_EV_TOPIC_EQ = 0x13, OP_EV_OFFSET = 0x14,
  OP_EV_PARTITION = 0x15, OP_STATE_GET = 0x20, OP_STATE_GET_OR_ELSE = 0x21, OP_FOLD_CURR = 0x22,
  OP_SEQ_AVG = 0x23, OP_SEQ_AGG = 0x24, OP_NOT = 0x30, OP_AND = 0x31, OP_OR = 0x32, OP_ADD = 0x40, OP_SUB = 0x41,
  OP_MUL = 0x42, OP_DIV = 0x43, OP_REM = 0x44, OP_NEG = 0x45, OP_EQ = 0x50, OP_NE = 0x51,
  OP_LT = 0x52, OP_LE = 0x53, OP_GT = 0x54, OP_GE = 0x55, OP_CAST = 0x60
};

typedef struct Expr {
  uint8_t op, t, ct;
  int32_t i32;
  int64_t i64;
  double f64;
  int col, name;
  struct Expr *a, *b;
} Expr;

typedef struct { uint8_t t; union { int32_t i; int64_t l; double d; int b; } u; } Val;
/* SequenceMatcher reductions (OP_SEQ_AGG kind) */
enum { SEQ_SUM = 1, SEQ_COUNT = 2, SEQ_MIN = 3, SEQ_MAX = 4, SEQ_FIRST = 5, SEQ_LAST = 6 };

/* ------------------------------------------------------------------------- */
/* compiled pattern (StagesFactory.java:49-180, Stage.java:40-252)           */
/* ------------------------------------------------------------------------- */
enum { ST_BEGIN = 0, ST_NORMAL = 1, ST_FINAL = 2 };                  /* Stage.StateType */
enum { E_BEGIN = 0, E_TAKE = 1, E_PROCEED = 2, E_SKIP_PROCEED = 3, E_IGNORE = 4 }; /* EdgeOperation */
enum { S_STRICT = 0, S_NEXT = 1, S_ANY = 2, S_NULL = 0xFF };          /* Strategy */

typedef struct { int op; Expr* pred; int target; } Edge;
typedef struct {
  char* name_str; int name; int level; int strategy; int topic; int card; int optional; int times;
  int64_t window; Expr* pred; int nfolds; int* fold_state; int* fold_type; Expr** fold_expr;
} Pat;
typedef struct {
  int id, name, type; int64_t window; int nedges; Edge e[4]; int pat; /* -1: no aggregates */
} Stage;
typedef VEC(Stage) StageVec;
typedef VEC(char*) StrVec;
typedef VEC(int64_t) I64Vec;

struct orc_pattern {
  int ncols; uint8_t* coltype;
  int npat; Pat* pats;
  int nstages; Stage* st;
  StrVec names;             /* stage names; 0 = "$final" */
  StrVec states;            /* aggregate state names */
  VEC(Expr*) pool;          /* all allocated Expr nodes */
  int begin;                /* Stages.getBeginingStage() */
  int* defined;             /* Stages.getDefinedStates() */
  int ndefined;
};

static Expr* new_expr(orc_pattern* p, uint8_t op) {
  Expr* e = xcalloc(1, sizeof(Expr));
  e->op = op;
  VPUSH(p->pool, e);
  return e;
}
static int intern(StrVec* v, const char* s) {
  for (int64_t i = 0; i < v->n; i++) if (!strcmp(v->a[i], s)) return (int)i;
  char* c = xmalloc(strlen(s) + 1);
  strcpy(c, s);
  VPUSH(*v, c);
  return (int)(v->n - 1);
}

typedef struct { const uint8_t* p; size_t n, i; int bad; } Rd;
static int rd_ok(Rd* r, size_t k) { if (r->i + k > r->n) { r->bad = 1; return 0; } return 1; }
static uint8_t rd_u8(Rd* r) { if (!rd_ok(r, 1)) return 0; return r->p[r->i++]; }
static uint16_t rd_u16(Rd* r) { uint16_t v = 0; if (!rd_ok(r, 2)) return 0; memcpy(&v, r->p + r->i, 2); r->i += 2; return v; }
static uint32_t rd_u32(Rd* r) { uint32_t v = 0; if (!rd_ok(r, 4)) return 0; memcpy(&v, r->p + r->i, 4); r->i += 4; return v; }
static int64_t rd_i64(Rd* r) { int64_t v = 0; if (!rd_ok(r, 8)) return 0; memcpy(&v, r->p + r->i, 8); r->i += 8; return v; }
static double rd_f64(Rd* r) { double v = 0; if (!rd_ok(r, 8)) return 0; memcpy(&v, r->p + r->i, 8); r->i += 8; return v; }
static char* rd_str(Rd* r) {
  uint16_t n = rd_u16(r);
  if (n == 0xFFFF) return NULL;
  if (!rd_ok(r, n)) return NULL;
  char* s = xmalloc((size_t)n + 1);
  memcpy(s, r->p + r->i, n); s[n] = 0; r->i += n;
  return s;
}

static int promote(int a, int b) { return a > b ? a : b; }

/* parse + static typing (Java binary numeric promotion) */
static Expr* rd_expr(orc_pattern* p, Rd* r, int depth) {
  if (depth > 256 || r->bad) { r->bad = 1; return NULL; }
  uint8_t op = rd_u8(r);
  Expr* e = new_expr(p, op);
  switch (op) {
    case OP_TRUE: case OP_FALSE: e->t = T_BOOL; break;
    case OP_CONST_I32: e->t = T_I32; e->i32 = (int32_t)rd_u32(r); break;
    case OP_CONST_I64: e->t = T_I64; e->i64 = rd_i64(r); break;
    case OP_CONST_F64: e->t = T_F64; e->f64 = rd_f64(r); break;
    case OP_FIELD:
      e->col = rd_u16(r);
      if (e->col >= p->ncols) { r->bad = 1; return NULL; }
      e->t = p->coltype[e->col];
      break;
    case OP_EV_KEY: e->t = T_I32; break;
    case OP_EV_TS: e->t = T_I64; break;
    case OP_EV_OFFSET: e->t = T_I64; break;
    case OP_EV_PARTITION: e->t = T_I32; break;
    case OP_EV_TOPIC_EQ: e->t = T_BOOL; e->i32 = (int32_t)rd_u32(r); break;
    case OP_STATE_GET: case OP_STATE_GET_OR_ELSE: {
      e->ct = rd_u8(r); e->t = e->ct;
      char* s = rd_str(r);
      if (!s) { r->bad = 1; return NULL; }
      e->name = intern(&p->states, s); free(s);
      if (op == OP_STATE_GET_OR_ELSE) {
        e->a = rd_expr(p, r, depth + 1);
        if (!e->a || e->a->t != e->ct) { r->bad = 1; return NULL; }
      }
      break;
    }
    case OP_FOLD_CURR: e->ct = rd_u8(r); e->t = e->ct; break;
    case OP_SEQ_AVG:
      e->col = rd_u16(r); e->t = T_F64;
      if (e->col >= p->ncols) { r->bad = 1; return NULL; }
      break;
    case OP_SEQ_AGG: {                /* kind, column, stage name (null: every stage) */
      e->ct = rd_u8(r); e->col = rd_u16(r);
      if (!rd_ok(r, 2)) { r->bad = 1; return NULL; }
      const int isnull = r->p[r->i] == 0xFF && r->p[r->i + 1] == 0xFF;
      char* s = rd_str(r);
      if (r->bad || (!s && !isnull)) { r->bad = 1; return NULL; }
      e->name = -1;                   /* every stage */
      if (s) {                        /* a stage no one declared never appears: -2 */
        e->name = -2;
        for (int64_t i = 0; i < p->names.n; i++) if (!strcmp(p->names.a[i], s)) e->name = (int)i;
        free(s);
      }
      if (e->col >= p->ncols || e->ct < SEQ_SUM || e->ct > SEQ_LAST) { r->bad = 1; return NULL; }
      if ((e->ct == SEQ_FIRST || e->ct == SEQ_LAST) && isnull) { r->bad = 1; return NULL; }
      /* sum over a double column: DoubleStream.sum (compensated, below) stays a double */
      e->t = e->ct == SEQ_COUNT ? T_I64 : e->ct == SEQ_SUM ? (p->coltype[e->col] == T_F64 ? T_F64 : T_I64)
                                                          : p->coltype[e->col];
      break;
    }
    case OP_NOT:
      e->a = rd_expr(p, r, depth + 1);
      if (!e->a || e->a->t != T_BOOL) { r->bad = 1; return NULL; }
      e->t = T_BOOL; break;
    case OP_AND: case OP_OR:
      e->a = rd_expr(p, r, depth + 1); e->b = rd_expr(p, r, depth + 1);
      if (!e->a || !e->b || e->a->t != T_BOOL || e->b->t != T_BOOL) { r->bad = 1; return NULL; }
      e->t = T_BOOL; break;
    case OP_ADD: case OP_SUB: case OP_MUL: case OP_DIV: case OP_REM:
      e->a = rd_expr(p, r, depth + 1); e->b = rd_expr(p, r, depth + 1);
      if (!e->a || !e->b || e->a->t == T_BOOL || e->b->t == T_BOOL) { r->bad = 1; return NULL; }
      e->t = (uint8_t)promote(e->a->t, e->b->t); break;
    case OP_NEG:
      e->a = rd_expr(p, r, depth + 1);
      if (!e->a || e->a->t == T_BOOL) { r->bad = 1; return NULL; }
      e->t = e->a->t; break;
    case OP_EQ: case OP_NE: case OP_LT: case OP_LE: case OP_GT: case OP_GE:
      e->a = rd_expr(p, r, depth + 1); e->b = rd_expr(p, r, depth + 1);
      if (!e->a || !e->b) { r->bad = 1; return NULL; }
      if ((e->a->t == T_BOOL) != (e->b->t == T_BOOL)) { r->bad = 1; return NULL; }
      e->t = T_BOOL; break;
    case OP_CAST:
      e->ct = rd_u8(r);
      e->a = rd_expr(p, r, depth + 1);
      if (!e->a || e->a->t == T_BOOL || e->ct == T_BOOL || e->ct > T_F64) { r->bad = 1; return NULL; }
      e->t = e->ct; break;
    default: r->bad = 1; return NULL;
  }
  if (r->bad) return NULL;
  return e;
}

static Expr* mk_true(orc_pattern* p) { Expr* e = new_expr(p, OP_TRUE); e->t = T_BOOL; return e; }
static Expr* mk_not(orc_pattern* p, Expr* a) { Expr* e = new_expr(p, OP_NOT); e->t = T_BOOL; e->a = a; return e; }
static Expr* mk_bin(orc_pattern* p, uint8_t op, Expr* a, Expr* b) {
  Expr* e = new_expr(p, op); e->t = T_BOOL; e->a = a; e->b = b; return e;
}
static Expr* mk_topic(orc_pattern* p, int topic) {
  Expr* e = new_expr(p, OP_EV_TOPIC_EQ); e->t = T_BOOL; e->i32 = topic; return e;
}

static int fail(char* err, size_t errlen, int code, const char* fmt, ...) {
  if (err && errlen) { va_list ap; va_start(ap, fmt); vsnprintf(err, errlen, fmt, ap); va_end(ap); }
  return code;
}

/* StagesFactory.buildStages (StagesFactory.java:77-172) */
static int build_stages(orc_pattern* p, int type, int pi, int succ_stage, int succ_pat, StageVec* out,
                        char* err, size_t errlen, int* next_id) {
  Pat* P = &p->pats[pi];
  int card = P->card, cur_type = type;
  int mandatory = (card == 1);                       /* :86-88 */
  if (mandatory) cur_type = ST_NORMAL;
  Stage s; memset(&s, 0, sizeof s);
  s.id = (*next_id)++; s.name = P->name; s.type = cur_type; s.pat = pi;  /* :90 */
  int64_t window = -1;                               /* getWindowLengthMs :174-180 */
  if (P->window != -1) window = P->window;
  else if (succ_pat >= 0 && p->pats[succ_pat].window != -1) window = p->pats[succ_pat].window;
  s.window = window;
  if (!P->pred) return fail(err, errlen, ORC_E_NPE, "pattern '%s' has no predicate", P->name_str);
  Expr* pred = P->topic >= 0 ? mk_bin(p, OP_AND, mk_topic(p, P->topic), P->pred) : P->pred; /* :97-99 */
  int op = card == 0 ? E_BEGIN : E_TAKE;             /* :101 */
  s.e[s.nedges++] = (Edge){op, pred, succ_stage};
  Expr* ignore = NULL;
  if (P->strategy == S_NULL)                         /* strategy null -> NPE at :106 */
    return fail(err, errlen, ORC_E_NPE, "selected strategy is null for '%s'", P->name_str);
  if (P->strategy == S_ANY) { ignore = mk_true(p); s.e[s.nedges++] = (Edge){E_IGNORE, ignore, -1}; }   /* :106-109 */
  if (P->strategy == S_NEXT) { ignore = mk_not(p, pred); s.e[s.nedges++] = (Edge){E_IGNORE, ignore, -1}; } /* :112-115 */
  if (op == E_TAKE) {                                /* :117-139 */
    if (succ_pat < 0 && out->a[succ_stage].type == ST_FINAL)
      return fail(err, errlen, ORC_E_INVALID_PATTERN,
                  "Cannot define a pattern with a final stage expecting multiple matching events");
    Pat* S = &p->pats[succ_pat];
    Expr* sp = S->pred;
    if (!sp) return fail(err, errlen, ORC_E_NPE, "successor without predicate");
    if (S->topic >= 0) sp = mk_bin(p, OP_AND, mk_topic(p, S->topic), sp);
    Expr* proceed;
    if (P->strategy == S_STRICT) proceed = mk_bin(p, OP_OR, sp, mk_not(p, pred));
    else proceed = mk_bin(p, OP_OR, sp, mk_bin(p, OP_AND, mk_not(p, pred), mk_not(p, ignore)));
    s.e[s.nedges++] = (Edge){E_PROCEED, proceed, succ_stage};
  }
  VPUSH(*out, s);
  int last = (int)out->n - 1;
  int times = P->times;
  if (mandatory || times > 1) {                      /* :144-157 */
    do {
      Stage in; memset(&in, 0, sizeof in);
      in.id = (*next_id)++; in.name = P->name; in.type = type; in.pat = pi; in.window = window;
      in.e[in.nedges++] = (Edge){E_BEGIN, pred, out->a[last].id};
      if (ignore) in.e[in.nedges++] = (Edge){E_IGNORE, ignore, -1};
      VPUSH(*out, in);
      last = (int)out->n - 1;
    } while (--times > 1);
  }
  if (P->optional) {                                 /* :159-169 */
    if (succ_pat < 0 && out->a[succ_stage].type == ST_FINAL)
      return fail(err, errlen, ORC_E_INVALID_PATTERN, "Cannot define a pattern with an optional final stage");
    Pat* S = &p->pats[succ_pat];
    Expr* skip = mk_bin(p, OP_AND, S->pred, mk_not(p, pred));   /* note: no topic filter (:165) */
    Stage* L = &out->a[last];
    L->e[L->nedges++] = (Edge){E_SKIP_PROCEED, skip, succ_stage};
  }
  return ORC_OK;
}

void orc_pattern_free(orc_pattern* p) {
  if (!p) return;
  for (int i = 0; i < p->npat; i++) {
    free(p->pats[i].name_str); free(p->pats[i].fold_state); free(p->pats[i].fold_type); free(p->pats[i].fold_expr);
  }
  free(p->pats); free(p->st); free(p->coltype); free(p->defined);
  for (int64_t i = 0; i < p->names.n; i++) free(p->names.a[i]);
  for (int64_t i = 0; i < p->states.n; i++) free(p->states.a[i]);
  for (int64_t i = 0; i < p->pool.n; i++) free(p->pool.a[i]);
  VFREE(p->names); VFREE(p->states); VFREE(p->pool);
  free(p);
}

int orc_compile(const uint8_t* ir, size_t len, orc_pattern** out, char* err, size_t errlen) {
  *out = NULL;
  Rd r = {ir, len, 0, 0};
  if (len < 8 || memcmp(ir, "KCEP", 4)) return fail(err, errlen, ORC_E_BAD_IR, "bad magic");
  r.i = 4;
  if (rd_u32(&r) != 1) return fail(err, errlen, ORC_E_BAD_IR, "bad IR version");
  orc_pattern* p = xcalloc(1, sizeof(orc_pattern));
  p->ncols = rd_u16(&r);
  p->coltype = xcalloc((size_t)p->ncols + 1, 1);
  for (int i = 0; i < p->ncols; i++) {
    p->coltype[i] = rd_u8(&r);
    if (p->coltype[i] < T_I32 || p->coltype[i] > T_F64) r.bad = 1;
  }
  intern(&p->names, "$final");
  p->npat = rd_u16(&r);
  if (p->npat == 0) r.bad = 1;
  p->pats = xcalloc((size_t)p->npat + 1, sizeof(Pat));
  for (int i = 0; i < p->npat && !r.bad; i++) {
    Pat* P = &p->pats[i];
    P->name_str = rd_str(&r);
    P->level = (int32_t)rd_u32(&r);
    if (!P->name_str) {                              /* Pattern.getName(): level when unnamed */
      char buf[32]; snprintf(buf, sizeof buf, "%d", P->level);
      P->name_str = xmalloc(strlen(buf) + 1); strcpy(P->name_str, buf);
    }
    P->name = intern(&p->names, P->name_str);
    P->strategy = rd_u8(&r);
    P->topic = (int32_t)rd_u32(&r);
    P->card = rd_u8(&r);
    P->optional = rd_u8(&r);
    P->times = (int32_t)rd_u32(&r);
    P->window = rd_i64(&r);
    P->pred = rd_u8(&r) ? rd_expr(p, &r, 0) : NULL;
    P->nfolds = rd_u16(&r);
    P->fold_state = xcalloc((size_t)P->nfolds + 1, sizeof(int));
    P->fold_type = xcalloc((size_t)P->nfolds + 1, sizeof(int));
    P->fold_expr = xcalloc((size_t)P->nfolds + 1, sizeof(Expr*));
    for (int f = 0; f < P->nfolds && !r.bad; f++) {
      char* s = rd_str(&r);
      if (!s) { r.bad = 1; break; }
      P->fold_state[f] = intern(&p->states, s); free(s);
      P->fold_type[f] = rd_u8(&r);
      P->fold_expr[f] = rd_expr(p, &r, 0);
      if (!P->fold_expr[f] || P->fold_expr[f]->t == T_BOOL) r.bad = 1;
    }
  }
  if (r.bad || r.i != len) { orc_pattern_free(p); return fail(err, errlen, ORC_E_BAD_IR, "malformed IR"); }

  /* StagesFactory.make (StagesFactory.java:49-70): last pattern first */
  StageVec sv = {0};
  int next_id = 0;
  Stage fin; memset(&fin, 0, sizeof fin);
  fin.id = next_id++; fin.name = 0; fin.type = ST_FINAL; fin.window = -1; fin.pat = -1;
  VPUSH(sv, fin);
  int succ_stage = 0, succ_pat = -1, cur = p->npat - 1, rc = ORC_OK;
  while (cur > 0 && rc == ORC_OK) {
    rc = build_stages(p, ST_NORMAL, cur, succ_stage, succ_pat, &sv, err, errlen, &next_id);
    if (rc) break;
    succ_stage = (int)sv.n - 1; succ_pat = cur; cur--;
  }
  if (rc == ORC_OK) rc = build_stages(p, ST_BEGIN, 0, succ_stage, succ_pat, &sv, err, errlen, &next_id);
  if (rc) { VFREE(sv); orc_pattern_free(p); return rc; }
  p->st = sv.a; p->nstages = (int)sv.n;
  p->begin = -1;
  for (int i = 0; i < p->nstages; i++) if (p->st[i].type == ST_BEGIN) { p->begin = i; break; } /* Stages.java:49-51 */
  /* Stages.getDefinedStates (Stages.java:62-67) */
  p->defined = xcalloc((size_t)p->states.n + 1, sizeof(int));
  for (int i = 0; i < p->nstages; i++) {
    if (p->st[i].pat < 0) continue;
    Pat* P = &p->pats[p->st[i].pat];
    for (int f = 0; f < P->nfolds; f++) {
      int s = P->fold_state[f], seen = 0;
      for (int k = 0; k < p->ndefined; k++) if (p->defined[k] == s) seen = 1;
      if (!seen) p->defined[p->ndefined++] = s;
    }
  }
  *out = p;
  return ORC_OK;
}

int orc_n_stages(const orc_pattern* p) { return p->nstages; }
int orc_n_names(const orc_pattern* p) { return (int)p->names.n; }
const char* orc_name(const orc_pattern* p, int id) { return (id >= 0 && id < p->names.n) ? p->names.a[id] : NULL; }
int orc_stage_info(const orc_pattern* p, int sid, int* name_id, int* type, int64_t* window, int* ops, int* targets) {
  const Stage* s = &p->st[sid];
  *name_id = s->name; *type = s->type; *window = s->window;
  for (int i = 0; i < s->nedges; i++) { ops[i] = s->e[i].op; targets[i] = s->e[i].target; }
  return s->nedges;
}

/* ------------------------------------------------------------------------- */
/* DeweyVersion (nfa/DeweyVersion.java:25-105)                               */
/* ------------------------------------------------------------------------- */
typedef struct { int len; int32_t d[]; } Dewey;

static Dewey* dw_new(Arena* a, int len) {
  Dewey* v = arena_alloc(a, sizeof(Dewey) + sizeof(int32_t) * (size_t)(len > 0 ? len : 1));
  v->len = len;
  return v;
}
/* addRun(offset) :62-67 ; returns NULL on ArrayIndexOutOfBoundsException */
static Dewey* dw_add_run(Arena* a, const Dewey* v, int off) {
  int idx = v->len - off;
  if (idx < 0 || idx >= v->len) return NULL;
  Dewey* n = dw_new(a, v->len);
  memcpy(n->d, v->d, sizeof(int32_t) * (size_t)v->len);
  n->d[idx] = (int32_t)((uint32_t)n->d[idx] + 1u);
  return n;
}
/* addStage :95-97 */
static Dewey* dw_add_stage(Arena* a, const Dewey* v) {
  Dewey* n = dw_new(a, v->len + 1);
  memcpy(n->d, v->d, sizeof(int32_t) * (size_t)v->len);
  n->d[v->len] = 0;
  return n;
}
/* isCompatible :73-93 */
static int dw_compatible(const Dewey* t, const Dewey* o) {
  if (t->len > o->len) {
    for (int i = 0; i < o->len; i++) if (t->d[i] != o->d[i]) return 0;
    return 1;
  } else if (t->len == o->len) {
    int last = t->len - 1;
    for (int i = 0; i < last; i++) if (t->d[i] != o->d[i]) return 0;
    return t->d[last] >= o->d[last];
  }
  return 0;
}
static void dw_str(const Dewey* v, char* out, size_t cap) {
  size_t k = 0;
  if (cap) out[0] = 0;
  for (int i = 0; i < v->len && k + 1 < cap; i++) {
    int w = snprintf(out + k, cap - k, i ? ".%d" : "%d", v->d[i]);
    if (w < 0) break;
    k += (size_t)w;
  }
}
static Dewey* dw_parse(Arena* a, const char* s) {
  int len = 1;
  for (const char* c = s; *c; c++) if (*c == '.') len++;
  Dewey* v = dw_new(a, len);
  const char* c = s;
  for (int i = 0; i < len; i++) { v->d[i] = (int32_t)strtol(c, (char**)&c, 10); if (*c == '.') c++; }
  return v;
}
int orc_dewey_compatible(const char* a, const char* b) {
  Arena ar = {0};
  int r = dw_compatible(dw_parse(&ar, a), dw_parse(&ar, b));
  arena_free(&ar);
  return r;
}
int orc_dewey_add_run(const char* v, int off, char* out, size_t cap) {
  Arena ar = {0};
  Dewey* n = dw_add_run(&ar, dw_parse(&ar, v), off);
  if (n) dw_str(n, out, cap);
  arena_free(&ar);
  return n ? 0 : ORC_E_INDEX;
}
int orc_dewey_add_stage(const char* v, char* out, size_t cap) {
  Arena ar = {0};
  dw_str(dw_add_stage(&ar, dw_parse(&ar, v)), out, cap);
  arena_free(&ar);
  return 0;
}

/* ------------------------------------------------------------------------- */
/* runs, buffer nodes, aggregates                                            */
/* ------------------------------------------------------------------------- */
/* A stage reference: a real compiled stage, or Stage.newEpsilonState(src,target)
 * (Stage.java:247-251) which copies (id, name, type) of src and carries one
 * PROCEED(true) edge to target, window -1, no aggregates. */
typedef struct { int sid; int eps; } SRef;

/* ComputationStage (nfa/ComputationStage.java:30-185) */
typedef struct {
  SRef st; Dewey* ver; int64_t ev; int64_t ts; int64_t seq; uint8_t br, ig;
} Run;

typedef VEC(Run) RunVec;

/* Matched key (state/internal/Matched.java:31-66): (stageName, stageType, topic, partition, offset) */
typedef struct { Dewey* ver; int has; Key4 key; } Pointer;   /* MatchedEvent.Pointer :124-168 */
typedef struct { int64_t refs; int64_t ev; int n, cap; Pointer* preds; } Node; /* MatchedEvent :27-34 */

typedef struct {
  int32_t key; VEC(Run) q; int64_t runs;
  int nh; int32_t h_topic[16]; int64_t h_off[16];    /* NFAStates.latestOffsets */
} Inst;

typedef struct { int64_t record; int32_t key; int64_t eb, ee; int64_t gb, ge; } Match;

struct orc_run {
  const orc_pattern* p;
  int mode;
  Arena arena;
  Map nodes; VEC(Node) pool;                   /* shared versioned buffer store */
  Map aggs; VEC(Val) aggv;                     /* aggregates store */
  Map inst_idx; VEC(Inst) inst;
  VEC(Match) m;
  VEC(int32_t) ent_name; VEC(int64_t) ent_ev;  /* traversal entries */
  VEC(int32_t) grp_name; VEC(int64_t) grp_cnt; VEC(int64_t) grp_ev; VEC(int64_t) grp_evoff;
  const orc_batch* b;
  int64_t err_record; char err_msg[256];
};

static int32_t ev_topic(const orc_batch* b, int64_t r) { return b->topic ? b->topic[r] : 0; }
static int32_t ev_part(const orc_batch* b, int64_t r) { return b->partition ? b->partition[r] : 0; }
static int64_t ev_off(const orc_batch* b, int64_t r) { return b->offset ? b->offset[r] : r; }
static int64_t ev_ts(const orc_batch* b, int64_t r) { return b->ts ? b->ts[r] : r; }

static int sr_name(const orc_pattern* p, SRef s) { return p->st[s.sid].name; }
static int sr_type(const orc_pattern* p, SRef s) { return p->st[s.sid].type; }
static int sr_is_begin(const orc_pattern* p, SRef s) { return sr_type(p, s) == ST_BEGIN; }
static int sr_nedges(const orc_pattern* p, SRef s) { return s.eps >= 0 ? 1 : p->st[s.sid].nedges; }
static Edge sr_edge(const orc_pattern* p, SRef s, int i) {
  if (s.eps >= 0) { Edge e = {E_PROCEED, NULL /* TruePredicate */, s.eps}; return e; }
  return p->st[s.sid].e[i];
}
/* ComputationStage.isForwarding :134-137 */
static int sr_forwarding(const orc_pattern* p, SRef s) { return sr_nedges(p, s) == 1 && sr_edge(p, s, 0).op == E_PROCEED; }
/* ComputationStage.isForwardingToFinalState :143-147 */
static int sr_fwd_final(const orc_pattern* p, SRef s) {
  return sr_forwarding(p, s) && p->st[sr_edge(p, s, 0).target].type == ST_FINAL;
}
static int64_t sr_window(const orc_pattern* p, SRef s) { return s.eps >= 0 ? -1 : p->st[s.sid].window; }
static SRef eps_of(SRef src, int target) { SRef r = {src.sid, target}; return r; }

static Key4 matched_key(const orc_run* R, SRef s, int64_t ev) {
  Key4 k;
  k.k[0] = ((int64_t)sr_name(R->p, s) << 8) | sr_type(R->p, s);
  k.k[1] = ev_topic(R->b, ev);
  k.k[2] = ev_part(R->b, ev);
  k.k[3] = ev_off(R->b, ev);
  return k;
}
static int key_name(const Key4* k) { return (int)(k->k[0] >> 8); }

static Node* node_get(orc_run* R, const Key4* k) {
  int64_t* i = map_find(&R->nodes, k);
  return i ? &R->pool.a[*i] : NULL;
}
static Node* node_new(orc_run* R, const Key4* k, int64_t ev, int64_t refs) {
  Node n; memset(&n, 0, sizeof n);
  n.refs = refs; n.ev = ev;
  VPUSH(R->pool, n);
  map_put(&R->nodes, k, R->pool.n - 1);
  return &R->pool.a[R->pool.n - 1];
}
static void node_add_pred(Node* n, Dewey* v, const Key4* k) {   /* MatchedEvent.addPredecessor :101-105 */
  if (n->n == n->cap) { n->cap = n->cap ? n->cap * 2 : 2; n->preds = xrealloc(n->preds, (size_t)n->cap * sizeof(Pointer)); }
  Pointer* pt = &n->preds[n->n++];
  pt->ver = v; pt->has = k != NULL;
  if (k) pt->key = *k; else memset(&pt->key, 0, sizeof(Key4));
}
/* MatchedEvent.getPointerByVersion :90-99 */
static int node_ptr(const Node* n, const Dewey* v) {
  for (int i = 0; i < n->n; i++) if (dw_compatible(v, n->preds[i].ver)) return i;
  return -1;
}

static int err_at(orc_run* R, int code, const char* fmt, ...) {
  va_list ap; va_start(ap, fmt); vsnprintf(R->err_msg, sizeof R->err_msg, fmt, ap); va_end(ap);
  return code;
}

/* SharedVersionedBufferStoreImpl.put 5-arg (:101-126) */
static int buf_put5(orc_run* R, SRef cur, int64_t ev, SRef prev, int64_t pev, Dewey* ver) {
  if (pev < 0) return err_at(R, ORC_E_NPE, "Matched.from(prevStage, null event)");
  Key4 pk = matched_key(R, prev, pev), ck = matched_key(R, cur, ev);
  if (!node_get(R, &pk)) return err_at(R, ORC_E_ILLEGAL_STATE, "Cannot find predecessor event");
  Node* c = node_get(R, &ck);
  if (!c) c = node_new(R, &ck, ev, 1);
  node_add_pred(c, ver, &pk);
  return ORC_OK;
}
/* put 3-arg (:149-157): overwrite with a fresh node */
static int buf_put3(orc_run* R, SRef cur, int64_t ev, Dewey* ver) {
  Key4 ck = matched_key(R, cur, ev);
  Node* c = node_get(R, &ck);
  if (c) { free(c->preds); memset(c, 0, sizeof *c); c->refs = 1; c->ev = ev; }
  else c = node_new(R, &ck, ev, 1);
  node_add_pred(c, ver, NULL);
  return ORC_OK;
}
/* branch (:132-142) */
static int buf_branch(orc_run* R, SRef st, int64_t ev, Dewey* ver) {
  if (ev < 0) return err_at(R, ORC_E_NPE, "Matched.from(stage, null event)");
  Key4 k = matched_key(R, st, ev);
  Dewey* pv = ver;
  for (;;) {
    Node* n = node_get(R, &k);
    if (!n) return err_at(R, ORC_E_NPE, "branch through deleted node");
    n->refs++;
    int i = node_ptr(n, pv);
    if (i < 0 || !n->preds[i].has) break;
    pv = n->preds[i].ver;
    k = n->preds[i].key;
  }
  return ORC_OK;
}
/* peek (:176-201): traversal emitted into R->ent_* ; returns error code */
static int buf_peek(orc_run* R, SRef st, int64_t ev, Dewey* ver, int remove, int64_t* eb, int64_t* ee) {
  if (ev < 0) return err_at(R, ORC_E_NPE, "Matched.from(stage, null event)");
  Key4 k = matched_key(R, st, ev);
  Dewey* pv = ver;
  *eb = R->ent_name.n;
  for (;;) {
    int64_t* ix = map_find(&R->nodes, &k);
    if (!ix) return err_at(R, ORC_E_NPE, "traversal reached a deleted buffer node");
    Node* n = &R->pool.a[*ix];
    int64_t refs_left = n->refs == 0 ? 0 : n->refs - 1;     /* decrementRefAndGet on a copy */
    int del = remove && refs_left == 0 && n->n <= 1;
    VPUSH(R->ent_name, key_name(&k));
    VPUSH(R->ent_ev, n->ev);
    int pi = node_ptr(n, pv);
    int has = pi >= 0;
    Pointer ptr; memset(&ptr, 0, sizeof ptr);
    if (has) ptr = n->preds[pi];
    if (remove && has && refs_left == 0) {
      /* removePredecessor + put(copy): a deleted node comes back (Q5) */
      n->refs = 0;
      memmove(&n->preds[pi], &n->preds[pi + 1], sizeof(Pointer) * (size_t)(n->n - pi - 1));
      n->n--;
    } else if (del) {
      free(n->preds); n->preds = NULL; n->n = n->cap = 0;
      map_del(&R->nodes, &k);
    }
    if (!has || !ptr.has) break;
    pv = ptr.ver; k = ptr.key;
  }
  *ee = R->ent_name.n;
  return ORC_OK;
}

/* AggregatesStoreImpl (:55-75), key (record key, state name, run seq) */
static Key4 agg_key(int32_t key, int state, int64_t seq) { Key4 k = {{key, state, seq, 0}}; return k; }
static Val* agg_find(orc_run* R, int32_t key, int state, int64_t seq) {
  Key4 k = agg_key(key, state, seq);
  int64_t* i = map_find(&R->aggs, &k);
  return i ? &R->aggv.a[*i] : NULL;
}
static void agg_put(orc_run* R, int32_t key, int state, int64_t seq, Val v) {
  Key4 k = agg_key(key, state, seq);
  int64_t* i = map_find(&R->aggs, &k);
  if (i) { R->aggv.a[*i] = v; return; }
  VPUSH(R->aggv, v);
  map_put(&R->aggs, &k, R->aggv.n - 1);
}

/* ------------------------------------------------------------------------- */
/* Sequence materialisation: Sequence.Builder + java.util.TreeMap insertion   */
/* (cep/Sequence.java:490-517, Event.compareTo Event.java:118-122)           */
/* ------------------------------------------------------------------------- */
typedef struct TNode { int64_t ev; struct TNode *l, *r, *p; int red; } TNode;
typedef struct { TNode* root; TNode* pool; int n; } TSet;

static int ev_cmp(const orc_batch* b, int64_t x, int64_t y) {
  if (ev_topic(b, x) != ev_topic(b, y) || ev_part(b, x) != ev_part(b, y)) {
    int64_t a = ev_ts(b, x), c = ev_ts(b, y);
    return a < c ? -1 : (a > c ? 1 : 0);
  }
  int64_t a = ev_off(b, x), c = ev_off(b, y);
  return a < c ? -1 : (a > c ? 1 : 0);
}
static void rot_left(TSet* t, TNode* p) {
  if (!p) return;
  TNode* r = p->r; p->r = r->l; if (r->l) r->l->p = p; r->p = p->p;
  if (!p->p) t->root = r; else if (p->p->l == p) p->p->l = r; else p->p->r = r;
  r->l = p; p->p = r;
}
static void rot_right(TSet* t, TNode* p) {
  if (!p) return;
  TNode* l = p->l; p->l = l->r; if (l->r) l->r->p = p; l->p = p->p;
  if (!p->p) t->root = l; else if (p->p->r == p) p->p->r = l; else p->p->l = l;
  l->r = p; p->p = l;
}
#define PAR(x) ((x) ? (x)->p : NULL)
#define LEFT(x) ((x) ? (x)->l : NULL)
#define RIGHT(x) ((x) ? (x)->r : NULL)
#define RED(x) ((x) ? (x)->red : 0)
#define SETC(x, c) do { if (x) (x)->red = (c); } while (0)
static void ts_insert(TSet* t, const orc_batch* b, int64_t ev) {   /* TreeMap.put + fixAfterInsertion */
  if (!t->root) { TNode* e = &t->pool[t->n++]; memset(e, 0, sizeof *e); e->ev = ev; t->root = e; return; }
  TNode *x = t->root, *parent = NULL; int c = 0;
  do { parent = x; c = ev_cmp(b, ev, x->ev); if (c < 0) x = x->l; else if (c > 0) x = x->r; else return; } while (x);
  TNode* e = &t->pool[t->n++]; memset(e, 0, sizeof *e); e->ev = ev; e->p = parent;
  if (c < 0) parent->l = e; else parent->r = e;
  x = e; x->red = 1;
  while (x && x != t->root && x->p->red) {
    if (PAR(x) == LEFT(PAR(PAR(x)))) {
      TNode* y = RIGHT(PAR(PAR(x)));
      if (RED(y)) { SETC(PAR(x), 0); SETC(y, 0); SETC(PAR(PAR(x)), 1); x = PAR(PAR(x)); }
      else {
        if (x == RIGHT(PAR(x))) { x = PAR(x); rot_left(t, x); }
        SETC(PAR(x), 0); SETC(PAR(PAR(x)), 1); rot_right(t, PAR(PAR(x)));
      }
    } else {
      TNode* y = LEFT(PAR(PAR(x)));
      if (RED(y)) { SETC(PAR(x), 0); SETC(y, 0); SETC(PAR(PAR(x)), 1); x = PAR(PAR(x)); }
      else {
        if (x == LEFT(PAR(x))) { x = PAR(x); rot_right(t, x); }
        SETC(PAR(x), 0); SETC(PAR(PAR(x)), 1); rot_left(t, PAR(PAR(x)));
      }
    }
  }
  t->root->red = 0;
}
static void ts_walk(const TNode* n, I64Vec* out) {
  if (!n) return;
  ts_walk(n->l, out); VPUSH(*out, n->ev); ts_walk(n->r, out);
}

/* Builds the groups of one traversal [eb,ee) into R->grp_* ; returns first group index */
static void materialise(orc_run* R, int64_t eb, int64_t ee, int64_t* gb, int64_t* ge) {
  int64_t n = ee - eb;
  int ng = 0;
  int32_t* gname = xmalloc(sizeof(int32_t) * (size_t)(n + 1));
  TSet* sets = xcalloc((size_t)n + 1, sizeof(TSet));
  for (int64_t i = 0; i < n; i++) sets[i].pool = NULL;
  for (int64_t i = eb; i < ee; i++) {                /* Builder.add: first-seen stage order */
    int32_t nm = R->ent_name.a[i]; int g = -1;
    for (int k = 0; k < ng; k++) if (gname[k] == nm) { g = k; break; }
    if (g < 0) { g = ng++; gname[g] = nm; sets[g].pool = xmalloc(sizeof(TNode) * (size_t)n); }
    ts_insert(&sets[g], R->b, R->ent_ev.a[i]);
  }
  *gb = R->grp_name.n;
  for (int g = ng - 1; g >= 0; g--) {               /* build(true): reversed */
    I64Vec evs = {0};
    ts_walk(sets[g].root, &evs);
    VPUSH(R->grp_name, gname[g]);
    VPUSH(R->grp_cnt, evs.n);
    VPUSH(R->grp_evoff, R->grp_ev.n);
    for (int64_t i = 0; i < evs.n; i++) VPUSH(R->grp_ev, evs.a[i]);
    VFREE(evs);
  }
  *ge = R->grp_name.n;
  for (int g = 0; g < ng; g++) free(sets[g].pool);
  free(sets); free(gname);
}

/* ------------------------------------------------------------------------- */
/* expression evaluation with Java semantics                                 */
/* ------------------------------------------------------------------------- */
typedef struct {
  orc_run* R; int64_t rec; int32_t key; int64_t seq;
  int has_prev; SRef prev; int64_t pev; Dewey* ver;   /* MatcherContext */
  int in_fold; const Val* curr;                        /* Aggregator.aggregate(k, v, curr) */
} EC;

static Val conv(Val v, int t) {
  Val o; o.t = (uint8_t)t;
  if (v.t == t) return v;
  switch (t) {
    case T_I32:
      if (v.t == T_I64) o.u.i = (int32_t)(uint32_t)(uint64_t)v.u.l;
      else { double d = v.u.d; o.u.i = isnan(d) ? 0 : d >= 2147483647.0 ? INT32_MAX : d <= -2147483648.0 ? INT32_MIN : (int32_t)d; }
      break;
    case T_I64:
      if (v.t == T_I32) o.u.l = v.u.i;
      else { double d = v.u.d; o.u.l = isnan(d) ? 0 : d >= 9223372036854775807.0 ? INT64_MAX : d <= -9223372036854775808.0 ? INT64_MIN : (int64_t)d; }
      break;
    case T_F64:
      o.u.d = v.t == T_I32 ? (double)v.u.i : (double)v.u.l;
      break;
  }
  return o;
}

static int eval(const Expr* e, EC* c, Val* out);

static int read_col(const orc_batch* b, const orc_pattern* p, int col, int64_t r, Val* out) {
  out->t = p->coltype[col];
  if (col >= b->ncols || !b->cols[col]) return ORC_E_NPE;
  if (out->t == T_I32) out->u.i = ((const int32_t*)b->cols[col])[r];
  else if (out->t == T_I64) out->u.l = ((const int64_t*)b->cols[col])[r];
  else out->u.d = ((const double*)b->cols[col])[r];
  return ORC_OK;
}

/* Java 8's compensated double summation (Collectors.sumWithCompensation / computeFinalSum, which
   DoubleStream.sum and DoubleStream.average / DoubleSummaryStatistics use): a Kahan sum plus the
   simple sum, finished as sum + compensation (JDK 8 adds the compensation term), the simple sum
   when that is NaN and the simple sum is infinite.  Values in Sequence order. */
typedef struct { double s, c, simple; } JSum;
static void jsum_add(JSum* j, double d) {
  const double tmp = d - j->c;
  const double velvel = j->s + tmp;
  j->c = (velvel - j->s) - tmp;
  j->s = velvel;
  j->simple += d;
}
static double jsum_final(const JSum* j) {
  const double tmp = j->s + j->c;
  return isnan(tmp) && isinf(j->simple) ? j->simple : tmp;
}

static int seq_avg(EC* c, int col, Val* out) {
  /* SequenceMatcher.accept (SequenceMatcher.java:21-26): buffer.get(Matched.from(prev, prevEvent), version) */
  orc_run* R = c->R;
  if (!c->has_prev || c->pev < 0) return err_at(R, ORC_E_NPE, "SequenceMatcher without previous stage/event");
  int64_t eb, ee;
  int rc = buf_peek(R, c->prev, c->pev, c->ver, 0, &eb, &ee);
  if (rc) return rc;
  int64_t gb, ge;
  materialise(R, eb, ee, &gb, &ge);
  JSum js = {0, 0, 0}; int64_t cnt = 0; int64_t isum = 0;
  for (int64_t g = gb; g < ge; g++)
    for (int64_t i = 0; i < R->grp_cnt.a[g]; i++) {
      Val v; rc = read_col(R->b, R->p, col, R->grp_ev.a[R->grp_evoff.a[g] + i], &v);
      if (rc) return rc;
      if (v.t == T_F64) jsum_add(&js, v.u.d); else isum += (v.t == T_I32 ? v.u.i : v.u.l);
      cnt++;
    }
  /* drop the temporary traversal + groups */
  R->ent_name.n = eb; R->ent_ev.n = eb;
  R->grp_ev.n = ge > gb ? R->grp_evoff.a[gb] : R->grp_ev.n;
  R->grp_name.n = gb; R->grp_cnt.n = gb; R->grp_evoff.n = gb;
  out->t = T_F64;
  out->u.d = cnt ? (R->p->coltype[col] == T_F64 ? jsum_final(&js) : (double)isum) / (double)cnt : 0.0;
  return ORC_OK;
}

/* Reductions a SequenceMatcher computes over the same partial Sequence (Sequence.java:57-60,
   116-167): every event, or getByName(stage).getEvents() -- a TreeSet in Event.compareTo order
   (Event.java:118-122), null for a stage the sequence lacks (NPE).  sum/count as Java longs
   (mapToLong(..).sum(), count()), min/max as LongStream / DoubleStream (Math.min / max), first /
   last the TreeSet's ends. */
static int seq_agg(EC* c, int kind, int col, int stage, uint8_t t, Val* out) {
  orc_run* R = c->R;
  if (!c->has_prev || c->pev < 0) return err_at(R, ORC_E_NPE, "SequenceMatcher without previous stage/event");
  int64_t eb, ee;
  int rc = buf_peek(R, c->prev, c->pev, c->ver, 0, &eb, &ee);
  if (rc) return rc;
  int64_t gb, ge;
  materialise(R, eb, ee, &gb, &ge);
  int64_t n = 0; uint64_t isum = 0; Val acc = {0}; int64_t first = -1, last = -1;
  JSum js = {0, 0, 0};
  const uint8_t ctype = R->p->coltype[col];
  for (int64_t g = gb; g < ge && !rc; g++) {
    if (stage != -1 && R->grp_name.a[g] != stage) continue;
    for (int64_t i = 0; i < R->grp_cnt.a[g] && !rc; i++) {
      const int64_t ev = R->grp_ev.a[R->grp_evoff.a[g] + i];
      if (first < 0) first = ev;
      last = ev;
      Val v;
      rc = read_col(R->b, R->p, col, ev, &v);
      if (rc) break;
      if (kind == SEQ_SUM && v.t == T_F64) jsum_add(&js, v.u.d);
      else if (kind == SEQ_SUM) isum += (uint64_t)(v.t == T_I32 ? (int64_t)v.u.i : v.u.l);
      else if (kind == SEQ_MIN || kind == SEQ_MAX) {
        if (n == 0) acc = v;
        else if (ctype == T_F64) {
          const double a = acc.u.d, b = v.u.d;
          int take;
          if (a != a) take = 0;
          else if (b != b) take = 1;
          else if (kind == SEQ_MIN) take = b < a || (b == 0 && a == 0 && signbit(b) && !signbit(a));
          else take = b > a || (b == 0 && a == 0 && !signbit(b) && signbit(a));
          if (take) acc = v;
        } else {
          const int64_t a = acc.t == T_I32 ? acc.u.i : acc.u.l, b = v.t == T_I32 ? v.u.i : v.u.l;
          if (kind == SEQ_MIN ? b < a : b > a) acc = v;
        }
      }
      n++;
    }
  }
  R->ent_name.n = eb; R->ent_ev.n = eb;                /* drop the temporary traversal + groups */
  R->grp_ev.n = ge > gb ? R->grp_evoff.a[gb] : R->grp_ev.n;
  R->grp_name.n = gb; R->grp_cnt.n = gb; R->grp_evoff.n = gb;
  if (rc) return rc;
  if (n == 0 && (stage != -1 || kind == SEQ_MIN || kind == SEQ_MAX))
    return err_at(R, ORC_E_NPE, "Sequence.getByName: no such stage in the partial sequence");
  out->t = t;
  if (kind == SEQ_COUNT) out->u.l = n;
  else if (kind == SEQ_SUM && t == T_F64) out->u.d = jsum_final(&js);
  else if (kind == SEQ_SUM) out->u.l = (int64_t)isum;
  else if (kind == SEQ_MIN || kind == SEQ_MAX) *out = acc;
  else return read_col(R->b, R->p, col, kind == SEQ_FIRST ? first : last, out);
  return ORC_OK;
}

static int eval(const Expr* e, EC* c, Val* out) {
  orc_run* R = c->R;
  Val a, b;
  int rc;
  switch (e->op) {
    case OP_TRUE: out->t = T_BOOL; out->u.b = 1; return 0;
    case OP_FALSE: out->t = T_BOOL; out->u.b = 0; return 0;
    case OP_CONST_I32: out->t = T_I32; out->u.i = e->i32; return 0;
    case OP_CONST_I64: out->t = T_I64; out->u.l = e->i64; return 0;
    case OP_CONST_F64: out->t = T_F64; out->u.d = e->f64; return 0;
    case OP_FIELD: return read_col(R->b, R->p, e->col, c->rec, out);
    case OP_EV_KEY: out->t = T_I32; out->u.i = R->b->key[c->rec]; return 0;
    case OP_EV_TS: out->t = T_I64; out->u.l = ev_ts(R->b, c->rec); return 0;
    case OP_EV_OFFSET: out->t = T_I64; out->u.l = ev_off(R->b, c->rec); return 0;
    case OP_EV_PARTITION: out->t = T_I32; out->u.i = ev_part(R->b, c->rec); return 0;
    case OP_EV_TOPIC_EQ: out->t = T_BOOL; out->u.b = ev_topic(R->b, c->rec) == e->i32; return 0;
    case OP_STATE_GET: case OP_STATE_GET_OR_ELSE: {      /* States.get/getOrElse (States.java:56-78) */
      Val* v = agg_find(R, c->key, e->name, c->seq);
      if (!v) {
        if (e->op == OP_STATE_GET)
          return err_at(R, ORC_E_UNKNOWN_AGGREGATE, "No state found for name '%s'", R->p->states.a[e->name]);
        return eval(e->a, c, out);
      }
      if (v->t != e->ct) return err_at(R, ORC_E_CLASS_CAST, "state '%s' has another boxed type", R->p->states.a[e->name]);
      *out = *v; return 0;
    }
    case OP_FOLD_CURR:
      if (!c->in_fold || !c->curr) return err_at(R, ORC_E_NPE, "null aggregate value unboxed");
      if (c->curr->t != e->ct) return err_at(R, ORC_E_CLASS_CAST, "aggregate has another boxed type");
      *out = *c->curr; return 0;
    case OP_SEQ_AVG: return seq_avg(c, e->col, out);
    case OP_SEQ_AGG: return seq_agg(c, e->ct, e->col, e->name, e->t, out);
    case OP_NOT:
      if ((rc = eval(e->a, c, &a))) return rc;
      out->t = T_BOOL; out->u.b = !a.u.b; return 0;
    case OP_AND:                                          /* Matcher.and: && short-circuit */
      if ((rc = eval(e->a, c, &a))) return rc;
      if (!a.u.b) { *out = a; return 0; }
      return eval(e->b, c, out);
    case OP_OR:
      if ((rc = eval(e->a, c, &a))) return rc;
      if (a.u.b) { *out = a; return 0; }
      return eval(e->b, c, out);
    case OP_NEG:
      if ((rc = eval(e->a, c, &a))) return rc;
      out->t = a.t;
      if (a.t == T_I32) out->u.i = (int32_t)(0u - (uint32_t)a.u.i);
      else if (a.t == T_I64) out->u.l = (int64_t)(0ull - (uint64_t)a.u.l);
      else out->u.d = -a.u.d;
      return 0;
    case OP_CAST:
      if ((rc = eval(e->a, c, &a))) return rc;
      *out = conv(a, e->ct); return 0;
    case OP_ADD: case OP_SUB: case OP_MUL: case OP_DIV: case OP_REM: {
      if ((rc = eval(e->a, c, &a))) return rc;
      if ((rc = eval(e->b, c, &b))) return rc;
      int t = e->t; a = conv(a, t); b = conv(b, t); out->t = (uint8_t)t;
      if (t == T_I32) {
        uint32_t x = (uint32_t)a.u.i, y = (uint32_t)b.u.i;
        switch (e->op) {
          case OP_ADD: out->u.i = (int32_t)(x + y); break;
          case OP_SUB: out->u.i = (int32_t)(x - y); break;
          case OP_MUL: out->u.i = (int32_t)(x * y); break;
          case OP_DIV:
            if (!b.u.i) return err_at(R, ORC_E_ARITHMETIC, "/ by zero");
            out->u.i = (a.u.i == INT32_MIN && b.u.i == -1) ? INT32_MIN : a.u.i / b.u.i; break;
          default:
            if (!b.u.i) return err_at(R, ORC_E_ARITHMETIC, "/ by zero");
            out->u.i = b.u.i == -1 ? 0 : a.u.i % b.u.i; break;
        }
      } else if (t == T_I64) {
        uint64_t x = (uint64_t)a.u.l, y = (uint64_t)b.u.l;
        switch (e->op) {
          case OP_ADD: out->u.l = (int64_t)(x + y); break;
          case OP_SUB: out->u.l = (int64_t)(x - y); break;
          case OP_MUL: out->u.l = (int64_t)(x * y); break;
          case OP_DIV:
            if (!b.u.l) return err_at(R, ORC_E_ARITHMETIC, "/ by zero");
            out->u.l = (a.u.l == INT64_MIN && b.u.l == -1) ? INT64_MIN : a.u.l / b.u.l; break;
          default:
            if (!b.u.l) return err_at(R, ORC_E_ARITHMETIC, "/ by zero");
            out->u.l = b.u.l == -1 ? 0 : a.u.l % b.u.l; break;
        }
      } else {
        switch (e->op) {
          case OP_ADD: out->u.d = a.u.d + b.u.d; break;
          case OP_SUB: out->u.d = a.u.d - b.u.d; break;
          case OP_MUL: out->u.d = a.u.d * b.u.d; break;
          case OP_DIV: out->u.d = a.u.d / b.u.d; break;
          default: out->u.d = fmod(a.u.d, b.u.d); break;
        }
      }
      return 0;
    }
    case OP_EQ: case OP_NE: case OP_LT: case OP_LE: case OP_GT: case OP_GE: {
      if ((rc = eval(e->a, c, &a))) return rc;
      if ((rc = eval(e->b, c, &b))) return rc;
      int r;
      if (a.t == T_BOOL) r = e->op == OP_EQ ? a.u.b == b.u.b : a.u.b != b.u.b;
      else {
        int t = promote(a.t, b.t); a = conv(a, t); b = conv(b, t);
        if (t == T_F64) {
          double x = a.u.d, y = b.u.d;
          switch (e->op) { case OP_EQ: r = x == y; break; case OP_NE: r = x != y; break; case OP_LT: r = x < y; break;
            case OP_LE: r = x <= y; break; case OP_GT: r = x > y; break; default: r = x >= y; }
        } else {
          int64_t x = t == T_I32 ? a.u.i : a.u.l, y = t == T_I32 ? b.u.i : b.u.l;
          switch (e->op) { case OP_EQ: r = x == y; break; case OP_NE: r = x != y; break; case OP_LT: r = x < y; break;
            case OP_LE: r = x <= y; break; case OP_GT: r = x > y; break; default: r = x >= y; }
        }
      }
      out->t = T_BOOL; out->u.b = r; return 0;
    }
  }
  return err_at(R, ORC_E_BAD_IR, "bad opcode");
}

/* ------------------------------------------------------------------------- */
/* NFA.evaluate (nfa/NFA.java:190-341)                                       */
/* ------------------------------------------------------------------------- */
typedef struct { orc_run* R; Inst* I; int64_t rec; } Step;

static Run mk_run(SRef s, Dewey* v, int64_t ev, int64_t ts, int64_t seq, int br, int ig) {
  Run r; r.st = s; r.ver = v; r.ev = ev; r.ts = ts; r.seq = seq; r.br = (uint8_t)br; r.ig = (uint8_t)ig;
  return r;
}

static int evaluate(Step* S, const Run* cs, SRef cur, const SRef* prev, RunVec* next) {
  orc_run* R = S->R;
  const orc_pattern* p = R->p;
  int64_t rec = S->rec;
  int32_t key = R->b->key[rec];
  const int64_t seq = cs->seq, pev = cs->ev;
  Dewey* ver = cs->ver;

  /* matchEdgesAndGet (:371-384): every edge predicate, in edge order */
  int ne = sr_nedges(p, cur), nm = 0;
  Edge matched[4];
  int has_op[5] = {0};
  for (int i = 0; i < ne; i++) {
    Edge e = sr_edge(p, cur, i);
    int ok = 1;
    if (e.pred) {
      EC c; memset(&c, 0, sizeof c);
      c.R = R; c.rec = rec; c.key = key; c.seq = seq; c.has_prev = prev != NULL;
      if (prev) c.prev = *prev;
      c.pev = pev; c.ver = ver;
      Val v; int rc = eval(e.pred, &c, &v);
      if (rc) return rc;
      ok = v.u.b;
    }
    if (ok) { matched[nm++] = e; has_op[e.op] = 1; }
  }
  /* isBranching (:392-397) */
  const int branching = (has_op[E_PROCEED] && has_op[E_TAKE]) || (has_op[E_IGNORE] && has_op[E_TAKE]) ||
                        (has_op[E_IGNORE] && has_op[E_BEGIN]) || (has_op[E_IGNORE] && has_op[E_PROCEED]);
  const int64_t start = sr_is_begin(p, cs->st) ? ev_ts(R->b, rec) : cs->ts;   /* getFirstPatternTimestamp :423-425 */
  int consumed = 0, proceed = 0;
  const int ignored = has_op[E_IGNORE];
  int64_t nbase = next->n;

  for (int i = 0; i < nm; i++) {
    Edge e = matched[i];
    int rc;
    switch (e.op) {
      case E_PROCEED: case E_SKIP_PROCEED: {        /* :222-237 */
        Run nctx = *cs;
        const Run* use = cs;
        if (p->st[e.target].name != sr_name(p, cur) && !cs->br && !cs->ig) {   /* isForwardingToNextStage :343-349 */
          nctx = mk_run(cs->st, dw_add_stage(&R->arena, ver), cs->ev, cs->ts, cs->seq, 0, 0); /* setVersion */
          use = &nctx;
        }
        const SRef* pv = e.op == E_SKIP_PROCEED ? prev : &cur;
        SRef tgt = {e.target, -1};
        int64_t before = next->n;
        if ((rc = evaluate(S, use, tgt, pv, next))) return rc;
        if (next->n > before) proceed = 1;
        break;
      }
      case E_TAKE: {                                  /* :238-255 */
        VPUSH(*next, mk_run(eps_of(cur, cur.sid), ver, rec, start, seq, 0, 0));
        Dewey* pv = ver;
        if (!(!branching || ignored)) { pv = dw_add_run(&R->arena, ver, 1); if (!pv) return err_at(R, ORC_E_INDEX, "addRun"); }
        rc = prev ? buf_put5(R, cur, rec, *prev, pev, pv) : buf_put3(R, cur, rec, pv);
        if (rc) return rc;
        consumed = 1;
        break;
      }
      case E_BEGIN: {                                 /* :256-271 */
        rc = prev ? buf_put5(R, cur, rec, *prev, pev, ver) : buf_put3(R, cur, rec, ver);
        if (rc) return rc;
        VPUSH(*next, mk_run(eps_of(cur, e.target), ver, rec, start, seq, 0, 0));
        consumed = 1;
        break;
      }
      case E_IGNORE:                                  /* :272-285 */
        if (!branching) VPUSH(*next, mk_run(cs->st, cs->ver, cs->ev, cs->ts, cs->seq, 0, 1));
        break;
    }
  }

  if (branching) {                                    /* :289-317 */
    if (consumed) {
      int64_t nseq = ++S->I->runs;
      int64_t last = ignored ? pev : rec;
      if (!prev) return err_at(R, ORC_E_NPE, "Stage.newEpsilonState(null previousStage)");
      SRef st = eps_of(*prev, cur.sid);
      Dewey* nv = dw_add_run(&R->arena, ver, sr_is_begin(p, *prev) ? 2 : 1);
      if (!nv) return err_at(R, ORC_E_INDEX, "DeweyVersion.addRun");
      VPUSH(*next, mk_run(st, nv, last, start, nseq, 1, 0));
      for (int k = 0; k < p->ndefined; k++) {         /* AggregatesStoreImpl.branch :55-60 */
        Val* v = agg_find(R, key, p->defined[k], seq);
        if (v) { Val cp = *v; agg_put(R, key, p->defined[k], nseq, cp); }
      }
      if (!sr_is_begin(p, *prev)) {
        int rc = buf_branch(R, *prev, pev, ver);
        if (rc) return rc;
      }
    } else if (!proceed) {
      VPUSH(*next, *cs);
    }
  }

  if (consumed && cur.eps < 0 && p->st[cur.sid].pat >= 0) {   /* evaluateAggregates :319-321, :362-369 */
    const Pat* P = &p->pats[p->st[cur.sid].pat];
    for (int f = 0; f < P->nfolds; f++) {
      Val* cv = agg_find(R, key, P->fold_state[f], seq);
      Val curv; if (cv) curv = *cv;
      EC c; memset(&c, 0, sizeof c);
      c.R = R; c.rec = rec; c.key = key; c.seq = seq; c.in_fold = 1; c.curr = cv ? &curv : NULL;
      Val nv; int rc = eval(P->fold_expr[f], &c, &nv);
      if (rc) return rc;
      if (nv.t != P->fold_type[f]) nv = conv(nv, P->fold_type[f]);
      agg_put(R, key, P->fold_state[f], seq, nv);
    }
  }

  if (sr_is_begin(p, cs->st) && !sr_forwarding(p, cs->st)) {   /* begin re-add :323-338 */
    if (consumed) {
      int64_t nseq = ++S->I->runs;
      Dewey* nv = ver;
      if (next->n != nbase) { nv = dw_add_run(&R->arena, ver, 1); if (!nv) return err_at(R, ORC_E_INDEX, "addRun"); }
      VPUSH(*next, mk_run(cs->st, nv, -1, -1, nseq, 0, 0));
    } else {
      VPUSH(*next, *cs);
    }
  }
  return ORC_OK;
}

/* NFA.matchPattern(Event) (:134-149) */
static int match_pattern(Step* S) {
  orc_run* R = S->R;
  Inst* I = S->I;
  const orc_pattern* p = R->p;
  int64_t n = I->q.n;
  RunVec finals = {0}, states = {0}, q2 = {0};
  int rc = ORC_OK;
  for (int64_t i = 0; i < n; i++) {
    Run cs = I->q.a[i];
    states.n = 0;
    /* window check (:179-188); inert in practice (Q1) but restated */
    int64_t w = sr_window(p, cs.st);
    int out_of_window = !sr_is_begin(p, cs.st) && w != -1 && (ev_ts(R->b, S->rec) - cs.ts) > w;
    if (!out_of_window) {
      rc = evaluate(S, &cs, cs.st, NULL, &states);
      if (rc) break;
    }
    if (states.n == 0) {                              /* removePattern :160-163 */
      int64_t eb, ee;
      rc = buf_peek(R, cs.st, cs.ev, cs.ver, 1, &eb, &ee);
      if (rc) break;
      R->ent_name.n = eb; R->ent_ev.n = eb;          /* result discarded */
    } else {
      for (int64_t k = 0; k < states.n; k++)
        if (sr_fwd_final(p, states.a[k].st)) VPUSH(finals, states.a[k]);
    }
    for (int64_t k = 0; k < states.n; k++)
      if (!sr_fwd_final(p, states.a[k].st)) VPUSH(q2, states.a[k]);
  }
  if (rc == ORC_OK) {
    /* the queue is polled n times and appended to: the result is q2 (the
     * reference queue had exactly n entries at entry) */
    VFREE(I->q);
    I->q.a = q2.a; I->q.n = q2.n; I->q.cap = q2.cap; q2.a = NULL;
    for (int64_t k = 0; k < finals.n && rc == ORC_OK; k++) {   /* matchConstruction :151-158 */
      Match m; memset(&m, 0, sizeof m);
      m.record = S->rec; m.key = R->b->key[S->rec];
      rc = buf_peek(R, finals.a[k].st, finals.a[k].ev, finals.a[k].ver, 1, &m.eb, &m.ee);
      if (rc) break;
      materialise(R, m.eb, m.ee, &m.gb, &m.ge);
      VPUSH(R->m, m);
    }
  }
  VFREE(finals); VFREE(states); VFREE(q2);
  return rc;
}

/* ------------------------------------------------------------------------- */
/* driver: NFATest-style single NFA, or CEPProcessor.process (:134-160)      */
/* ------------------------------------------------------------------------- */
orc_run* orc_run_new(const orc_pattern* p, int mode) {
  orc_run* R = xcalloc(1, sizeof(orc_run));
  R->p = p; R->mode = mode; R->err_record = -1;
  map_init(&R->nodes); map_init(&R->aggs); map_init(&R->inst_idx);
  return R;
}
void orc_run_free(orc_run* R) {
  if (!R) return;
  for (int64_t i = 0; i < R->pool.n; i++) free(R->pool.a[i].preds);
  for (int64_t i = 0; i < R->inst.n; i++) VFREE(R->inst.a[i].q);
  VFREE(R->pool); VFREE(R->aggv); VFREE(R->inst); VFREE(R->m);
  VFREE(R->ent_name); VFREE(R->ent_ev); VFREE(R->grp_name); VFREE(R->grp_cnt); VFREE(R->grp_ev); VFREE(R->grp_evoff);
  map_free(&R->nodes); map_free(&R->aggs); map_free(&R->inst_idx);
  arena_free(&R->arena);
  free(R);
}

static Inst* get_inst(orc_run* R, int32_t key, int create) {
  Key4 k = {{R->mode == ORC_MODE_NFA_SINGLE ? 0 : key, 0, 0, 0}};
  int64_t* ix = map_find(&R->inst_idx, &k);
  if (ix) return &R->inst.a[*ix];
  if (!create) return NULL;
  Inst I; memset(&I, 0, sizeof I);                    /* NFA.build (NFA.java:73-79), Stages.java:53-60 */
  I.key = key; I.runs = 1;
  Dewey* v = dw_new(&R->arena, 1); v->d[0] = 1;
  SRef b = {R->p->begin, -1};
  VPUSH(I.q, mk_run(b, v, -1, -1, 1, 0, 0));
  VPUSH(R->inst, I);
  map_put(&R->inst_idx, &k, R->inst.n - 1);
  return &R->inst.a[R->inst.n - 1];
}

static int run_from(orc_run* R, const orc_batch* b, int64_t r0);

int orc_run_batch(orc_run* R, const orc_batch* b) { return run_from(R, b, 0); }

/* CEPProcessor.process for records r0..n-1 of the bound batch (:134-160) */
static int run_from(orc_run* R, const orc_batch* b, int64_t r0) {
  R->b = b;
  if (R->p->begin < 0) return ORC_E_NPE;
  for (int64_t r = r0; r < b->n; r++) {
    int proc = R->mode == ORC_MODE_PROCESSOR;
    if (proc && b->valid && !b->valid[r]) continue;   /* CEPProcessor.java:136-138 */
    Inst* I = get_inst(R, b->key[r], 1);
    if (proc) {
      /* the run queue was serialised after the previous record: isIgnored is
       * not part of the wire format (ComputationStageSerde.java:118-136) */
      for (int64_t i = 0; i < I->q.n; i++) I->q.a[i].ig = 0;
      /* checkHighWaterMark (:152-160) */
      int32_t tp = ev_topic(b, r);
      int64_t latest = -1;
      for (int h = 0; h < I->nh; h++) if (I->h_topic[h] == tp) latest = I->h_off[h];
      if (ev_off(b, r) < latest) continue;
    }
    Step S = {R, I, r};
    int rc = match_pattern(&S);
    if (rc) { R->err_record = r; return rc; }
    I = get_inst(R, b->key[r], 0);
    if (proc) {
      int32_t tp = ev_topic(b, r); int h;
      for (h = 0; h < I->nh; h++) if (I->h_topic[h] == tp) break;
      if (h == I->nh) { if (I->nh == 16) return ORC_E_CAPACITY; I->h_topic[I->nh++] = tp; }
      I->h_off[h] = ev_off(b, r) + 1;
    }
  }
  return ORC_OK;
}

/* ------------------------------------------------------------------------- */
/* continuing a key from its state in the reference's terms ("KCRF", libkcep  */
/* cep_state_to_reference): NFAStates (runs, run queue, latestOffsets), the   */
/* buffer's MatchedEvent nodes and the aggregates, rebuilt as the reference   */
/* stores would hold them (NFAStates.java:33-109, MatchedEvent.java:27-169,   */
/* AggregatesStoreImpl.java:30-76); then CEPProcessor.process per record.     */
/* ------------------------------------------------------------------------- */
static int32_t rd_i32(Rd* r) { return (int32_t)rd_u32(r); }
static char* rd_lstr(Rd* r) {                      /* i32 length + bytes */
  int32_t n = rd_i32(r);
  if (n < 0 || !rd_ok(r, (size_t)n)) { r->bad = 1; return NULL; }
  char* c = xmalloc((size_t)n + 1);
  memcpy(c, r->p + r->i, (size_t)n); c[n] = 0; r->i += (size_t)n;
  return c;
}
static Dewey* rd_dewey(orc_run* R, Rd* r) {
  int32_t nd = rd_i32(r);
  if (nd < 0 || nd > 1 << 20) { r->bad = 1; return NULL; }
  Dewey* v = dw_new(&R->arena, nd);
  for (int i = 0; i < nd; i++) v->d[i] = rd_i32(r);
  return v;
}
static int name_id(const orc_pattern* p, const char* s) {
  for (int64_t i = 0; i < p->names.n; i++) if (!strcmp(p->names.a[i], s)) return (int)i;
  return -1;
}
static int state_id(const orc_pattern* p, const char* s) {
  for (int64_t i = 0; i < p->states.n; i++) if (!strcmp(p->states.a[i], s)) return (int)i;
  return -1;
}

int orc_run_resume(orc_run* R, const orc_batch* b, const uint8_t* st, size_t len) {
  Rd r = {st, len, 0, 0};
  R->b = b;
  if (rd_u32(&r) != 0x4652434Bu || rd_u32(&r) != 1) return ORC_E_BAD_IR;
  const int32_t key = rd_i32(&r), ncols = rd_i32(&r);
  const int64_t runs = rd_i64(&r);
  if (ncols != R->p->ncols) return ORC_E_BAD_IR;
  Inst* I = get_inst(R, key, 1);
  VFREE(I->q); memset(&I->q, 0, sizeof I->q);
  I->runs = runs;
  I->nh = rd_i32(&r);
  if (I->nh < 0 || I->nh > 16) return ORC_E_BAD_IR;
  for (int h = 0; h < I->nh; h++) { I->h_topic[h] = rd_i32(&r); I->h_off[h] = rd_i64(&r); }
  const int32_t nev = rd_i32(&r);
  if (nev < 0 || nev > b->n) return ORC_E_BAD_IR;
  for (int32_t e = 0; e < nev && !r.bad; e++) {    /* the batch starts with exactly these events */
    rd_i64(&r);
    const int32_t tp = rd_i32(&r), part = rd_i32(&r);
    const int64_t off = rd_i64(&r), ts = rd_i64(&r);
    for (int c = 0; c < ncols; c++) rd_i64(&r);
    if (b->key[e] != key || ev_topic(b, e) != tp || ev_part(b, e) != part || ev_off(b, e) != off || ev_ts(b, e) != ts)
      return ORC_E_BAD_IR;
  }
  const int32_t qlen = rd_i32(&r);
  for (int32_t i = 0; i < qlen && !r.bad; i++) {
    SRef sr;
    sr.sid = rd_i32(&r); sr.eps = rd_i32(&r);
    const int32_t flags = rd_i32(&r);
    const int64_t seq = rd_i64(&r);
    const int32_t ev = rd_i32(&r);
    const int64_t ts = rd_i64(&r);
    Dewey* v = rd_dewey(R, &r);
    if (r.bad || sr.sid < 0 || sr.sid >= R->p->nstages || sr.eps >= R->p->nstages || ev >= nev) return ORC_E_BAD_IR;
    VPUSH(I->q, mk_run(sr, v, ev, ts, seq, flags & 1, (flags >> 1) & 1));
  }
  const int32_t nnode = rd_i32(&r);
  for (int32_t i = 0; i < nnode && !r.bad; i++) {
    char* nm = rd_lstr(&r);
    const int32_t type = rd_i32(&r), ev = rd_i32(&r);
    const int64_t refs = rd_i64(&r);
    const int32_t np = rd_i32(&r);
    const int id = nm ? name_id(R->p, nm) : -1;
    free(nm);
    if (id < 0 || ev < 0 || ev >= nev || np < 0) return ORC_E_BAD_IR;
    Key4 k = {{((int64_t)id << 8) | type, ev_topic(b, ev), ev_part(b, ev), ev_off(b, ev)}};
    Node* n = node_new(R, &k, ev, refs);
    for (int32_t j = 0; j < np && !r.bad; j++) {
      Dewey* v = rd_dewey(R, &r);
      const int32_t has = rd_i32(&r);
      char* pn = rd_lstr(&r);
      const int32_t ptype = rd_i32(&r), pev = rd_i32(&r);
      const int pid = has && pn ? name_id(R->p, pn) : -1;
      free(pn);
      if (has && (pid < 0 || pev < 0 || pev >= nev)) return ORC_E_BAD_IR;
      Key4 pk = {{((int64_t)pid << 8) | ptype, has ? ev_topic(b, pev) : 0, has ? ev_part(b, pev) : 0,
                  has ? ev_off(b, pev) : 0}};
      n = node_get(R, &k);                            /* (node_new may move the pool) */
      node_add_pred(n, v, has ? &pk : NULL);
    }
  }
  const int32_t nagg = rd_i32(&r);
  for (int32_t i = 0; i < nagg && !r.bad; i++) {
    char* sn = rd_lstr(&r);
    const int64_t seq = rd_i64(&r);
    const int32_t t = rd_i32(&r);
    const int64_t bits = rd_i64(&r);
    const int sid = sn ? state_id(R->p, sn) : -1;
    free(sn);
    if (sid < 0 || t < ORC_T_I32 || t > ORC_T_F64) return ORC_E_BAD_IR;
    Val v; memset(&v, 0, sizeof v);
    v.t = (uint8_t)t;
    if (t == ORC_T_I32) v.u.i = (int32_t)bits;
    else if (t == ORC_T_I64) v.u.l = bits;
    else memcpy(&v.u.d, &bits, 8);
    agg_put(R, key, sid, seq, v);
  }
  if (r.bad || r.i != len) return ORC_E_BAD_IR;
  return run_from(R, b, nev);
}

int64_t orc_err_record(const orc_run* R) { return R->err_record; }
const char* orc_err_msg(const orc_run* R) { return R->err_msg; }
int64_t orc_n_matches(const orc_run* R) { return R->m.n; }
void orc_match(const orc_run* R, int64_t m, int64_t* record, int32_t* key, int64_t* eb, int64_t* ee) {
  const Match* x = &R->m.a[m];
  *record = x->record; *key = x->key; *eb = x->eb; *ee = x->ee;
}
void orc_entry(const orc_run* R, int64_t e, int32_t* name, int64_t* ev) { *name = R->ent_name.a[e]; *ev = R->ent_ev.a[e]; }
int64_t orc_seq_groups(const orc_run* R, int64_t m, int32_t* names, int64_t* cnts, int64_t cap) {
  const Match* x = &R->m.a[m];
  int64_t n = x->ge - x->gb;
  for (int64_t i = 0; i < n && i < cap; i++) { names[i] = R->grp_name.a[x->gb + i]; cnts[i] = R->grp_cnt.a[x->gb + i]; }
  return n;
}
int64_t orc_seq_events(const orc_run* R, int64_t m, int64_t* evs, int64_t cap) {
  const Match* x = &R->m.a[m];
  int64_t k = 0;
  for (int64_t g = x->gb; g < x->ge; g++)
    for (int64_t i = 0; i < R->grp_cnt.a[g]; i++) {
      if (k < cap) evs[k] = R->grp_ev.a[R->grp_evoff.a[g] + i];
      k++;
    }
  return k;
}
int orc_inst_state(const orc_run* R, int32_t key, int64_t* runs, int64_t* qs) {
  Inst* I = get_inst((orc_run*)R, key, 0);
  if (!I) return -1;
  *runs = I->runs; *qs = I->q.n;
  return 0;
}
int orc_queue_entry(const orc_run* R, int32_t key, int64_t idx, int32_t* sid, int32_t* eps, int64_t* seq,
                    int64_t* ev, char* ver, size_t vcap) {
  Inst* I = get_inst((orc_run*)R, key, 0);
  if (!I || idx < 0 || idx >= I->q.n) return -1;
  Run* r = &I->q.a[idx];
  *sid = r->st.sid; *eps = r->st.eps; *seq = r->seq; *ev = r->ev;
  dw_str(r->ver, ver, vcap);
  return 0;
}

/* ------------------------------------------------------------------------- */
/* direct buffer access for SharedVersionedBufferTest.java:50-87: puts and a  */
/* get (peek without remove, :164-175) on the events of a bound batch         */
/* ------------------------------------------------------------------------- */
void orc_svb_bind(orc_run* R, const orc_batch* b) { R->b = b; }
/* psid < 0: the 3-arg put (:149-157), else the 5-arg put (:101-126) */
int orc_svb_put(orc_run* R, int sid, int64_t ev, int psid, int64_t pev, const char* version) {
  SRef cur = {sid, -1};
  Dewey* v = dw_parse(&R->arena, version);
  if (psid < 0) return buf_put3(R, cur, ev, v);
  SRef prev = {psid, -1};
  return buf_put5(R, cur, ev, prev, pev, v);
}
/* buffer.get(Matched.from(stage, ev), version): appended to the run's matches */
int orc_svb_get(orc_run* R, int sid, int64_t ev, const char* version, int remove) {
  SRef cur = {sid, -1};
  Match m; memset(&m, 0, sizeof m);
  m.record = ev; m.key = R->b->key[ev];
  int rc = buf_peek(R, cur, ev, dw_parse(&R->arena, version), remove, &m.eb, &m.ee);
  if (rc) return rc;
  materialise(R, m.eb, m.ee, &m.gb, &m.ge);
  VPUSH(R->m, m);
  return ORC_OK;
}

/* ------------------------------------------------------------------------- */
/* CPU baseline: key-sharded threads over a key-grouped batch                */
/* ------------------------------------------------------------------------- */
typedef struct {
  const orc_pattern* p; const orc_batch* b; int mode; int64_t lo, hi;
  int64_t matches; uint64_t sum; int err;
  int csr;                                            /* also keep every match, in emission order */
  VEC(int64_t) mrec; VEC(int32_t) mkey; VEC(int64_t) elen; VEC(int32_t) ename; VEC(int64_t) erec;
} Shard;

static void* shard_main(void* arg) {
  Shard* s = arg;
  const int64_t CH = 1 << 16;                         /* whole-key chunks bound the memory */
  int64_t r = s->lo;
  while (r < s->hi) {
    int64_t e = r + CH < s->hi ? r + CH : s->hi;
    while (e < s->hi && s->b->key[e] == s->b->key[e - 1]) e++;
    orc_batch sub = *s->b;
    sub.n = e - r;
    sub.key = s->b->key + r;
    if (s->b->valid) sub.valid = s->b->valid + r;
    if (s->b->topic) sub.topic = s->b->topic + r;
    if (s->b->partition) sub.partition = s->b->partition + r;
    int64_t* off = NULL; int64_t* ts = NULL;
    if (s->b->offset) sub.offset = s->b->offset + r;
    else { off = xmalloc(sizeof(int64_t) * (size_t)sub.n); for (int64_t i = 0; i < sub.n; i++) off[i] = r + i; sub.offset = off; }
    if (s->b->ts) sub.ts = s->b->ts + r;
    else { ts = xmalloc(sizeof(int64_t) * (size_t)sub.n); for (int64_t i = 0; i < sub.n; i++) ts[i] = r + i; sub.ts = ts; }
    const void* cols[16];
    for (int c = 0; c < s->b->ncols && c < 16; c++) {
      int t = s->p->coltype[c];
      size_t w = t == T_I32 ? 4 : 8;
      cols[c] = (const char*)s->b->cols[c] + (size_t)r * w;
    }
    sub.cols = cols;
    orc_run* R = orc_run_new(s->p, s->mode);
    int rc = orc_run_batch(R, &sub);
    if (rc) s->err = rc;
    for (int64_t m = 0; m < R->m.n; m++) {
      const Match* x = &R->m.a[m];
      uint64_t h = mix64((uint64_t)(x->record + r) * 0x9e3779b97f4a7c15ULL);
      for (int64_t i = x->eb; i < x->ee; i++)
        h = mix64(h ^ ((uint64_t)(R->ent_ev.a[i] + r) << 8) ^ (uint64_t)R->ent_name.a[i]);
      s->sum += h;
      if (s->csr) {
        VPUSH(s->mrec, x->record + r);
        VPUSH(s->mkey, x->key);
        VPUSH(s->elen, x->ee - x->eb);
        for (int64_t i = x->eb; i < x->ee; i++) { VPUSH(s->ename, R->ent_name.a[i]); VPUSH(s->erec, R->ent_ev.a[i] + r); }
      }
    }
    s->matches += R->m.n;
    orc_run_free(R);
    free(off); free(ts);
    r = e;
  }
  return NULL;
}

static Shard* run_shards(const orc_pattern* p, const orc_batch* b, int mode, int nthreads, int csr) {
  Shard* sh = xcalloc((size_t)nthreads, sizeof(Shard));
  pthread_t* th = xcalloc((size_t)nthreads, sizeof(pthread_t));
  int64_t prev = 0;
  for (int t = 0; t < nthreads; t++) {
    int64_t hi = t == nthreads - 1 ? b->n : (b->n * (t + 1)) / nthreads;
    if (hi < prev) hi = prev;
    while (hi > 0 && hi < b->n && b->key[hi] == b->key[hi - 1]) hi++;
    sh[t].p = p; sh[t].b = b; sh[t].mode = mode; sh[t].lo = prev; sh[t].hi = hi; sh[t].csr = csr;
    prev = hi;
  }
  for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, shard_main, &sh[t]);
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  free(th);
  return sh;
}

int64_t orc_baseline(const orc_pattern* p, const orc_batch* b, int mode, int nthreads, uint64_t* checksum, int* err) {
  if (nthreads < 1) nthreads = 1;
  Shard* sh = run_shards(p, b, mode, nthreads, 0);
  int64_t total = 0; uint64_t sum = 0; int e = 0;
  for (int t = 0; t < nthreads; t++) { total += sh[t].matches; sum += sh[t].sum; if (sh[t].err) e = sh[t].err; }
  free(sh);
  if (checksum) *checksum = sum;
  if (err) *err = e;
  return total;
}

/* The same run keeping every match: the batch's CSR in key order (shards are contiguous whole-key
   ranges), per key in emission order -- the order cep_collect returns for a key-grouped batch. */
struct orc_csr { Shard* sh; int n; int64_t nm, ne; int err; };
orc_csr* orc_baseline_csr(const orc_pattern* p, const orc_batch* b, int mode, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  orc_csr* c = xcalloc(1, sizeof(orc_csr));
  c->sh = run_shards(p, b, mode, nthreads, 1);
  c->n = nthreads;
  for (int t = 0; t < nthreads; t++) { c->nm += c->sh[t].mrec.n; c->ne += c->sh[t].ename.n; if (c->sh[t].err) c->err = c->sh[t].err; }
  return c;
}
void orc_csr_sizes(const orc_csr* c, int64_t* n_matches, int64_t* n_entries, int* err) {
  *n_matches = c->nm; *n_entries = c->ne; *err = c->err;
}
void orc_csr_copy(const orc_csr* c, int64_t* match_record, int32_t* match_key, int64_t* ent_off, int32_t* ent_name,
                  int64_t* ent_record) {
  int64_t m = 0, e = 0;
  for (int t = 0; t < c->n; t++) {
    const Shard* s = &c->sh[t];
    for (int64_t i = 0; i < s->mrec.n; i++, m++) {
      match_record[m] = s->mrec.a[i]; match_key[m] = s->mkey.a[i]; ent_off[m] = e; e += s->elen.a[i];
    }
    memcpy(ent_name + (e - s->ename.n), s->ename.a, sizeof(int32_t) * (size_t)s->ename.n);
    memcpy(ent_record + (e - s->erec.n), s->erec.a, sizeof(int64_t) * (size_t)s->erec.n);
  }
  ent_off[m] = e;
}
void orc_csr_free(orc_csr* c) {
  if (!c) return;
  for (int t = 0; t < c->n; t++) {
    Shard* s = &c->sh[t];
    VFREE(s->mrec); VFREE(s->mkey); VFREE(s->elen); VFREE(s->ename); VFREE(s->erec);
  }
  free(c->sh);
  free(c);
}

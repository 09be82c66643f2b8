// kcep_internal.h — compiled-pattern representation shared by the host
// compiler (compile.cpp) and the HIP kernels (stencil.hip, nfa.hip).
#pragma once
#include <stdint.h>

#include <memory>
#include <string>
#include <vector>

namespace kcep {

// ---- static types / opcodes of the expression IR (kcep/expr.py) ----
enum : uint8_t { T_BOOL = 0, T_I32 = 1, T_I64 = 2, T_F64 = 3 };
enum : uint8_t {
  OP_TRUE = 0x01, OP_FALSE = 0x02, OP_CONST_I32 = 0x03, OP_CONST_I64 = 0x04, OP_CONST_F64 = 0x05,
  OP_FIELD = 0x10, OP_EV_KEY = 0x11, OP_EV_TS = 0x12, OP_EV_TOPIC_EQ = 0x13, OP_EV_OFFSET = 0x14,
  OP_EV_PARTITION = 0x15, OP_STATE_GET = 0x20, OP_STATE_GET_OR_ELSE = 0x21, OP_FOLD_CURR = 0x22,
  OP_SEQ_AVG = 0x23, OP_NOT = 0x30, OP_AND = 0x31, OP_OR = 0x32, OP_ADD = 0x40, OP_SUB = 0x41,
  OP_MUL = 0x42, OP_DIV = 0x43, OP_REM = 0x44, OP_NEG = 0x45, OP_EQ = 0x50, OP_NE = 0x51,
  OP_LT = 0x52, OP_LE = 0x53, OP_GT = 0x54, OP_GE = 0x55, OP_CAST = 0x60
};

// Stage.StateType (nfa/Stage.java:243-245) and EdgeOperation (nfa/EdgeOperation.java:20-46)
enum : uint8_t { ST_BEGIN = 0, ST_NORMAL = 1, ST_FINAL = 2 };
enum : uint8_t { E_BEGIN = 0, E_TAKE = 1, E_PROCEED = 2, E_SKIP_PROCEED = 3, E_IGNORE = 4 };
enum : uint8_t { S_STRICT = 0, S_NEXT = 1, S_ANY = 2, S_NULL = 0xFF };

struct Expr {
  uint8_t op = 0, t = 0, ct = 0;
  int32_t i32 = 0;
  int64_t i64 = 0;
  double f64 = 0;
  int col = 0, name = 0;
  std::shared_ptr<Expr> a, b;
};
using ExprP = std::shared_ptr<Expr>;

struct Fold {
  int state;
  uint8_t type;
  ExprP expr;
};

struct PatternDef {                 // one select() of the DSL (pattern/Pattern.java)
  std::string name;
  int name_id = 0, level = 0;
  uint8_t strategy = S_STRICT;
  int32_t topic = -1;
  uint8_t one_or_more = 0, optional = 0;
  int32_t times = 1;
  int64_t window_ms = -1;
  ExprP pred;
  std::vector<Fold> folds;
};

struct EdgeDef {
  uint8_t op;
  ExprP pred;                       // nullptr = Matcher.TruePredicate
  int target;                       // stage id, -1 for IGNORE
};

struct StageDef {                   // nfa/Stage.java
  int id, name;
  uint8_t type;
  int64_t window_ms;
  int pattern;                      // index into patterns (aggregates), -1 for $final
  std::vector<EdgeDef> edges;
};

// ---- stencil (strict single-cardinality fast path) ----
constexpr int STENCIL_MAX_K = 8;
constexpr int STENCIL_MAX_TERMS = 6;
constexpr int STENCIL_MAX_ATOMS = 2;   // per term: one value-column range + one topic range

struct StencilAtomI { int64_t lo, hi; };
struct StencilAtomF { double lo, hi; };

// Predicate slot p (0..7): OR over terms of (value in [lo,hi] AND topic in [tlo,thi]).
// Slots 0..k-1 are the stage predicates (BEGIN edges, topic filter included).
// Chain patterns (strict with optional() stages, k <= 4) also use slot 4+i for
// the SKIP_PROCEED edge of optional stage i: the successor's predicate without
// its topic filter (StagesFactory.java:159-169); the edge is that AND NOT slot i.
constexpr int CHAIN_MAX_K = 4;
struct StencilProgram {
  int32_t k;
  int32_t col;                       // value column read by every predicate
  int32_t coltype;                   // T_I32 / T_I64 / T_F64
  int32_t use_topic;                 // 1 if any atom constrains the topic
  int32_t chain;                     // 1: some stage is optional (variable-length matches)
  int32_t optmask;                   // bit i: stage i is optional
  int32_t pslots;                    // bit p: predicate slot p is in use
  int32_t nterms[STENCIL_MAX_K];
  int32_t hasv[STENCIL_MAX_K][STENCIL_MAX_TERMS];   // 0: term does not constrain the value
  StencilAtomI vi[STENCIL_MAX_K][STENCIL_MAX_TERMS];
  StencilAtomF vf[STENCIL_MAX_K][STENCIL_MAX_TERMS];
  StencilAtomI tp[STENCIL_MAX_K][STENCIL_MAX_TERMS];
  int32_t name[STENCIL_MAX_K];       // stage name id of pattern s
  // Interval table: the breakpoints of every value/topic atom cut the value
  // (topic) axis into intervals on which each stage predicate is constant, so
  // a record's k-bit stage mask is table[it * 16 + iv] with iv = #{value
  // breakpoints <= v} and it = #{topic breakpoints <= topic}.
  int32_t nbp;                       // value breakpoints (<= 15), sorted ascending
  int32_t ntbp;                      // topic breakpoints (<= 3)
  int64_t bpi[15];                   // integer columns (clamped to int32 for i32 columns)
  double bpf[15];                    // double columns
  int32_t tbp[3];
  uint8_t table[64];
  uint8_t nan_mask[4];               // double columns: mask of a NaN value per topic interval
};

// ---- general NFA path: flat device program ----
// Predicates and folds become postfix bytecode over 64-bit slots (ints kept
// sign-extended, doubles as bits); the compiler inserts Java's binary numeric
// promotions.  AND/OR short-circuit with conditional jumps so that exceptions
// (unknown state, / by zero, ...) are raised exactly when Java would.
enum : uint8_t {
  BC_END = 0, BC_PUSH, BC_FIELD, BC_EV_KEY, BC_EV_TS, BC_EV_OFFSET, BC_EV_PARTITION, BC_TOPIC_EQ,
  BC_STATE_GET, BC_STATE_GET_OR_ELSE, BC_FOLD_CURR, BC_SEQ_AVG, BC_NOT, BC_JZ_KEEP, BC_JNZ_KEEP, BC_POP,
  BC_ADD_I32, BC_SUB_I32, BC_MUL_I32, BC_DIV_I32, BC_REM_I32, BC_NEG_I32,
  BC_ADD_I64, BC_SUB_I64, BC_MUL_I64, BC_DIV_I64, BC_REM_I64, BC_NEG_I64,
  BC_ADD_F64, BC_SUB_F64, BC_MUL_F64, BC_DIV_F64, BC_REM_F64, BC_NEG_F64,
  BC_EQ_I, BC_NE_I, BC_LT_I, BC_LE_I, BC_GT_I, BC_GE_I,
  BC_EQ_F, BC_NE_F, BC_LT_F, BC_LE_F, BC_GT_F, BC_GE_F,
  BC_EQ_B, BC_NE_B,
  BC_I64_TO_I32, BC_I_TO_F64, BC_F64_TO_I32, BC_F64_TO_I64,
};
// instruction word: op | a << 8 | b << 16 (a, b: small operands); BC_PUSH is
// followed by two words (lo, hi); jumps carry a signed word offset in the next word.

constexpr int NFA_MAX_STAGES = 64;
constexpr int NFA_MAX_EDGES = 4;
constexpr int NFA_MAX_FOLDS = 8;
constexpr int NFA_MAX_STATES = 16;
constexpr int NFA_MAX_SLOTS = 64;
constexpr int NFA_MAX_CODE = 4096;
constexpr int NFA_MAX_SL = 64;     // event-only edge predicates evaluated once per record
constexpr int NFA_STACK = 8;       // operand stack of the device interpreter (registers)
constexpr int NFA_MAX_FRAMES = 16; // NFA.evaluate recursion depth of the device kernel
constexpr int RUNS_MAX_STATES = 8; // aggregate registers of one deterministic run

struct DevStage {
  int32_t name, type, slot, nedges, nfolds;
  int32_t op[NFA_MAX_EDGES], target[NFA_MAX_EDGES], pred[NFA_MAX_EDGES];   // pred: code offset, -1 = TRUE
  int32_t sl[NFA_MAX_EDGES];       // index of the edge's event-only predicate, -1 = evaluate per run
  int32_t fold_state[NFA_MAX_FOLDS], fold_type[NFA_MAX_FOLDS], fold_code[NFA_MAX_FOLDS];
};

struct DevProgram {
  int32_t nstages, begin, nslots, nstates, ndefined, ncols, mode, maxdepth;
  int32_t nsl;                      // event-only edge predicates (read only the current record's fields)
  int32_t sl_pc[NFA_MAX_SL];        // their code offsets
  int32_t slot_name[NFA_MAX_SLOTS];
  int32_t defined[NFA_MAX_STATES];
  int32_t coltype[16];
  DevStage st[NFA_MAX_STAGES];
  int32_t code[NFA_MAX_CODE];
};

struct Program {
  std::vector<uint8_t> coltypes;
  std::vector<PatternDef> pats;
  std::vector<StageDef> stages;
  std::vector<std::string> names;    // stage names, 0 = "$final"
  std::vector<std::string> states;   // aggregate state names
  std::vector<int> defined_states;   // Stages.getDefinedStates()
  int begin = -1;
  bool general_ok = false;
  std::string general_why;
  DevProgram dev{};
  bool stencil_ok = false;
  std::string stencil_why;           // reason the stencil path does not apply
  bool runs_ok = false;              // deterministic strict runs (compile.cpp analyse_runs)
  std::string runs_why;
  StencilProgram stencil{};
};

// ---- launch interfaces shared by abi.cpp and the .hip files ----
struct StencilLaunch {
  const int32_t* key;
  const void* val;
  const int32_t* topic;
  int64_t n;
  const StencilProgram* prog_dev;
  int k, coltype, use_topic, chain;
  int32_t* slots;                 // per-tile match slots, ST_TILE * k ints each
  int64_t* tile_count;            // matches per tile
  int64_t* tile_pre;              // their exclusive prefix
  int64_t* scan_tmp;
  int32_t* out;                   // contiguous output, k ints per match
  int64_t out_cap;                // matches
  int64_t* total;                 // device: number of matches
};

// Per-key workspace of the general NFA kernel.  Every key segment draws its
// workspace from a batch-wide pool (one atomic per lane, aggregated per wave);
// arrays that outgrow their first allocation are re-allocated from the pool at
// twice the size (all internal references are offsets, so a copy relocates).
struct NfaCaps {
  int32_t q0;                     // initial run-queue capacity (runs)
  int32_t heap_base, heap_mult;   // initial heap: base + mult * events (words)
  int32_t out_base, out_mult;     // initial match output: base + mult * records (words)
  int32_t seq_base;               // initial aggregate rows: seq_base + records
};

// Carried per-key state (CEP_SESSION_CARRY): the NFAStates of the key
// (state/internal/NFAStates.java:33-109: run queue, runs counter, per-topic
// high-water marks) plus the shared-buffer nodes and aggregates the queue can
// still reach, as one relocatable blob of int32 words in the session's carry
// pool.  Events referenced by the carried buffer travel with it
// (MatchedEvent.java:29-34 keeps key/value/timestamp in the buffer too).
enum : int32_t {
  CB_WORDS = 0, CB_RUNS_LO, CB_RUNS_HI, CB_NHWM, CB_QLEN, CB_NEV, CB_NNODE, CB_NPRED, CB_NVER, CB_NSEQ,
  CB_NCOLS, CB_NSTATES, CB_HDR
};
// sections after the header: hwm[3*nhwm] (topic, hwm lo, hi); queue[4*qlen]
// (w0, version offset, event, seq); events[(8+2*ncols)*nev] (stream position,
// topic, partition, offset, ts, columns as 64-bit); nodes[4*nnode] (slot, event,
// refs, first pred); preds[4*npred] (version offset, prev slot, prev event, next
// pred); versions[nver] ([len, digits...]); aggs[3*nstates*nseq] (tag, lo, hi).
__host__ __device__ inline int32_t carry_evw(int32_t ncols) { return 8 + 2 * ncols; }

struct NfaArgs {
  const DevProgram* P;
  const int32_t* key;
  const uint8_t* valid;
  const int32_t* topic;
  const int32_t* partition;
  const int64_t* offset;
  const int64_t* ts;
  const void* cols[16];
  int64_t n;
  int64_t base;                   // stream position of batch record 0 (carry sessions; else 0)
  int32_t mode;
  int32_t nseg;
  const int64_t* seg_start;       // nseg + 1
  int32_t* pool;                  // per-batch workspace pool
  int64_t pool_cap;
  unsigned long long* pool_top;
  NfaCaps cap;
  int32_t carry;                  // 1: import/export carried state
  int32_t max_keys;               // carry: key ids are dense in [0, max_keys)
  const int64_t* ctab;            // carry: per key id, word offset of its blob in cpool (-1 none)
  int32_t* cpool;
  int64_t cpool_cap;
  unsigned long long* cpool_top;
  int64_t* res_carry;             // carry: per segment, offset of the new blob (-1 none)
  int64_t* res_matches;           // per segment
  int64_t* res_words;
  int64_t* res_out;               // device address of the key's output region
  int32_t* res_err;
  int64_t* res_err_rec;
  int32_t* flags;                 // [0] pool overflow lanes, [1] carry-pool overflow lanes, [2] bad key ids
};

// deterministic-runs path (runs.hip)
struct RunsArgs {
  const DevProgram* P;
  const int32_t* key;
  const int32_t* topic;
  const int32_t* partition;
  const int64_t* offset;
  const int64_t* ts;
  const void* cols[16];
  int64_t n;
  int64_t base;
  unsigned long long* nmatch;     // match counter (append position)
  unsigned long long* match_key;  // appended (end << 31 | start), sorted afterwards
  int64_t match_cap;
  unsigned long long* err_min;    // min over failing runs of (record << 31 | start)
  int32_t* err_code;              // per start record (valid where it failed)
};

// compile.cpp
int lower_general(Program& P, std::string& why);
int compile_ir(const uint8_t* ir, size_t len, Program& out, std::string& err);

}  // namespace kcep

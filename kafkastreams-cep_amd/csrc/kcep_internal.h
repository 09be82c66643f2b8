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

// per stage s (pattern order, first..last): OR over terms of (value in [lo,hi] AND topic in [tlo,thi])
struct StencilProgram {
  int32_t k;
  int32_t col;                       // value column read by every predicate
  int32_t coltype;                   // T_I32 / T_I64 / T_F64
  int32_t use_topic;                 // 1 if any atom constrains the topic
  int32_t nterms[STENCIL_MAX_K];
  int32_t hasv[STENCIL_MAX_K][STENCIL_MAX_TERMS];   // 0: term does not constrain the value
  StencilAtomI vi[STENCIL_MAX_K][STENCIL_MAX_TERMS];
  StencilAtomF vf[STENCIL_MAX_K][STENCIL_MAX_TERMS];
  StencilAtomI tp[STENCIL_MAX_K][STENCIL_MAX_TERMS];
  int32_t name[STENCIL_MAX_K];       // stage name id of pattern s
};

struct Program {
  std::vector<uint8_t> coltypes;
  std::vector<PatternDef> pats;
  std::vector<StageDef> stages;
  std::vector<std::string> names;    // stage names, 0 = "$final"
  std::vector<std::string> states;   // aggregate state names
  std::vector<int> defined_states;   // Stages.getDefinedStates()
  int begin = -1;
  bool stencil_ok = false;
  std::string stencil_why;           // reason the stencil path does not apply
  StencilProgram stencil{};
};

// compile.cpp
int compile_ir(const uint8_t* ir, size_t len, Program& out, std::string& err);

}  // namespace kcep

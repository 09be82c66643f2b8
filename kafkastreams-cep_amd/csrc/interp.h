// interp.h — device interpreter of the predicate / fold bytecode (compile.cpp CodeGen).
//
// Java semantics of Matcher.accept / Aggregator.aggregate bodies: 32/64-bit
// wrap-around, integer "/ by zero" -> ArithmeticException, boxed-type checks on
// state reads (ClassCastException), States.get on an unset state ->
// UnknownAggregateException (States.java:56-60), short-circuit && and ||.
// The operand stack is a shift register of NFA_STACK slots (s[0] is the top):
// the compiler bounds every program's depth, so it stays in registers.
//
// Env supplies the record and run context:
//   int64_t field(int col, int type); int64_t key(); int64_t ts(); int64_t off();
//   int64_t part(); int32_t topic();
//   bool state(int idx, int32_t& tag, int64_t& bits);   // false: failure already recorded
//   bool seq_avg(int col, int64_t& bits);
//   bool seq_agg(int kind, int col, int stage, int64_t& bits);
//   void fail(int code);
//   bool in_fold; int32_t curr_tag; int64_t curr;        // Aggregator's current value
#pragma once
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#endif
#include <stdint.h>

#include "../../include/kcep.h"
#include "kcep_dev.h"

namespace kcep {

// read-only program memory addressed wave-uniformly: constant address space,
// so the compiler emits scalar loads (scalar cache) instead of vector loads
typedef const int32_t __attribute__((address_space(4))) cint32_t;
typedef const DevStage __attribute__((address_space(4))) cDevStage;
typedef const DevProgram __attribute__((address_space(4))) cDevProgram;

__device__ __forceinline__ double bc_f(int64_t b) { return __builtin_bit_cast(double, b); }
__device__ __forceinline__ int64_t bc_b(double d) { return __builtin_bit_cast(int64_t, d); }
__device__ __forceinline__ int64_t bc_sx32(int64_t x) { return int64_t(int32_t(uint32_t(uint64_t(x)))); }

// 32-bit integer division without a branch: the float-reciprocal estimate of 2^32 / d refined once,
// then the quotient corrected twice (the same exact sequence the compiler expands `/` into, but as
// straight-line selects: a predicate's divide is then one basic block, so two predicates of a stage
// that divide the same operands share it, and no exec-mask juggling surrounds it).  d != 0.
__device__ __forceinline__ uint32_t bc_udiv32(uint32_t n, uint32_t d) {
  uint32_t inv = uint32_t(__builtin_amdgcn_rcpf(float(d)) * 4294966784.0f);   // 0x4f7ffffe
  inv += __umulhi(inv, (0u - d) * inv);
  uint32_t q = __umulhi(n, inv);
  uint32_t r = n - q * d;
  const bool c1 = r >= d;
  q = c1 ? q + 1 : q;
  r = c1 ? r - d : r;
  return r >= d ? q + 1 : q;
}
// Java int division / remainder (wrapping: MIN_VALUE / -1 == MIN_VALUE, MIN_VALUE % -1 == 0); y != 0
__device__ __forceinline__ int32_t bc_sdiv32(int32_t x, int32_t y) {
  const uint32_t ax = x < 0 ? 0u - uint32_t(x) : uint32_t(x), ay = y < 0 ? 0u - uint32_t(y) : uint32_t(y);
  const uint32_t q = bc_udiv32(ax, ay);
  return int32_t((x ^ y) < 0 ? 0u - q : q);
}
__device__ __forceinline__ int32_t bc_srem32(int32_t x, int32_t y) {
  return int32_t(uint32_t(x) - uint32_t(bc_sdiv32(x, y)) * uint32_t(y));
}

// One binary opcode with Java semantics: 0, or the exception it raises.  The
// interpreters call it with a loaded opcode, the per-pattern kernels (jit.cpp)
// with a constant one, so both evaluate every operator through this one body.
__device__ __forceinline__ int bc_bin(int op, int64_t x, int64_t y, int64_t& z) {
  z = 0;
  switch (op) {
    case BC_ADD_I32: z = bc_sx32(x + y); break;
    case BC_SUB_I32: z = bc_sx32(x - y); break;
    case BC_MUL_I32: z = bc_sx32(int64_t(uint64_t(x) * uint64_t(y))); break;
    // int operands are sign-extended 32-bit values: a 32-bit divide (the 64-bit one is a long
    // software sequence); y == -1 is a negation (Integer.MIN_VALUE / -1 wraps, JLS 15.17.2).  The
    // divisor is made safe instead of branching around the divide, so a predicate's failure checks
    // stay branch-free (jit.cpp)
    case BC_DIV_I32: {
      const int32_t yy = y == 0 ? 1 : int32_t(y);
      z = y == 0 ? 0 : int64_t(bc_sdiv32(int32_t(x), yy));
      return y == 0 ? CEP_E_ARITHMETIC : 0;
    }
    case BC_REM_I32: {
      const int32_t yy = y == 0 ? 1 : int32_t(y);
      z = y == 0 ? 0 : int64_t(bc_srem32(int32_t(x), yy));
      return y == 0 ? CEP_E_ARITHMETIC : 0;
    }
    case BC_ADD_I64: z = int64_t(uint64_t(x) + uint64_t(y)); break;
    case BC_SUB_I64: z = int64_t(uint64_t(x) - uint64_t(y)); break;
    case BC_MUL_I64: z = int64_t(uint64_t(x) * uint64_t(y)); break;
    // long operands that fit 32 bits (the common case) take the 32-bit divide too
    case BC_DIV_I64: {
      const int64_t yy = (y == 0 || y == -1) ? 1 : y;
      z = y == 0 ? 0 : y == -1 ? int64_t(0ull - uint64_t(x))
          : (bc_sx32(x) == x && bc_sx32(yy) == yy) ? int64_t(bc_sdiv32(int32_t(x), int32_t(yy))) : x / yy;
      return y == 0 ? CEP_E_ARITHMETIC : 0;
    }
    case BC_REM_I64: {
      const int64_t yy = (y == 0 || y == -1) ? 1 : y;
      z = (y == 0 || y == -1) ? 0 : (bc_sx32(x) == x && bc_sx32(yy) == yy) ? int64_t(bc_srem32(int32_t(x), int32_t(yy))) : x % yy;
      return y == 0 ? CEP_E_ARITHMETIC : 0;
    }
    case BC_ADD_F64: z = bc_b(bc_f(x) + bc_f(y)); break;
    case BC_SUB_F64: z = bc_b(bc_f(x) - bc_f(y)); break;
    case BC_MUL_F64: z = bc_b(bc_f(x) * bc_f(y)); break;
    case BC_DIV_F64: z = bc_b(bc_f(x) / bc_f(y)); break;
    case BC_REM_F64: z = bc_b(fmod(bc_f(x), bc_f(y))); break;
    case BC_EQ_I: z = x == y; break;
    case BC_NE_I: z = x != y; break;
    case BC_LT_I: z = x < y; break;
    case BC_LE_I: z = x <= y; break;
    case BC_GT_I: z = x > y; break;
    case BC_GE_I: z = x >= y; break;
    case BC_EQ_F: z = bc_f(x) == bc_f(y); break;
    case BC_NE_F: z = bc_f(x) != bc_f(y); break;
    case BC_LT_F: z = bc_f(x) < bc_f(y); break;
    case BC_LE_F: z = bc_f(x) <= bc_f(y); break;
    case BC_GT_F: z = bc_f(x) > bc_f(y); break;
    case BC_GE_F: z = bc_f(x) >= bc_f(y); break;
    case BC_EQ_B: z = (x != 0) == (y != 0); break;
    case BC_NE_B: z = (x != 0) != (y != 0); break;
    default: return CEP_E_BAD_IR;
  }
  return 0;
}

// unary opcodes (none raises)
__device__ __forceinline__ int64_t bc_un(int op, int64_t x) {
  switch (op) {
    case BC_NOT: return x ? 0 : 1;
    case BC_NEG_I32: return bc_sx32(0 - x);
    case BC_NEG_I64: return int64_t(0ull - uint64_t(x));
    case BC_NEG_F64: return bc_b(-bc_f(x));
    case BC_I64_TO_I32: return bc_sx32(x);
    case BC_I_TO_F64: return bc_b(double(x));
    case BC_F64_TO_I32: {
      const double d = bc_f(x);
      return d != d ? 0 : d >= 2147483647.0 ? INT32_MAX : d <= -2147483648.0 ? INT32_MIN : int64_t(int32_t(d));
    }
    case BC_F64_TO_I64: {
      const double d = bc_f(x);
      return d != d ? 0 : d >= 9223372036854775807.0 ? INT64_MAX : d <= -9223372036854775808.0 ? INT64_MIN : int64_t(d);
    }
  }
  return 0;
}

struct BcStack {
  int64_t s[NFA_STACK];
  __device__ __forceinline__ void push(int64_t v) {
#pragma unroll
    for (int i = NFA_STACK - 1; i > 0; i--) s[i] = s[i - 1];
    s[0] = v;
  }
  __device__ __forceinline__ void pop() {
#pragma unroll
    for (int i = 0; i < NFA_STACK - 1; i++) s[i] = s[i + 1];
  }
};

template <class Env>
__device__ __forceinline__ bool interp(const int32_t* __restrict__ code, int pc, Env& env, int64_t& result) {
  BcStack st;
#pragma unroll
  for (int i = 0; i < NFA_STACK; i++) st.s[i] = 0;
  for (;;) {
    const int32_t w = code[pc++];
    const int op = w & 0xFF, a = (w >> 8) & 0xFF, b = (w >> 16) & 0xFF;
    switch (op) {
      case BC_END: result = st.s[0]; return true;
      case BC_PUSH: st.push(int64_t(uint32_t(code[pc])) | (int64_t(code[pc + 1]) << 32)); pc += 2; break;
      case BC_FIELD: st.push(env.field(a, b)); break;
      case BC_EV_KEY: st.push(env.key()); break;
      case BC_EV_TS: st.push(env.ts()); break;
      case BC_EV_OFFSET: st.push(env.off()); break;
      case BC_EV_PARTITION: st.push(env.part()); break;
      case BC_TOPIC_EQ: st.push(env.topic() == code[pc] ? 1 : 0); pc++; break;
      case BC_STATE_GET: case BC_STATE_GET_OR_ELSE: {          // States.get / getOrElse (States.java:56-78)
        int32_t tag;
        int64_t v;
        if (!env.state(a, tag, v)) return false;
        if (tag == 0) {
          if (op == BC_STATE_GET) { env.fail(CEP_E_UNKNOWN_AGGREGATE); return false; }
          pc++;                                                  // evaluate the default
          break;
        }
        if (tag != b) { env.fail(CEP_E_CLASS_CAST); return false; }
        st.push(v);
        if (op == BC_STATE_GET_OR_ELSE) pc += 1 + code[pc];
        break;
      }
      case BC_FOLD_CURR:
        if (!env.in_fold || env.curr_tag == 0) { env.fail(CEP_E_NPE); return false; }
        if (env.curr_tag != b) { env.fail(CEP_E_CLASS_CAST); return false; }
        st.push(env.curr);
        break;
      case BC_SEQ_AVG: {
        int64_t v;
        if (!env.seq_avg(a, v)) return false;
        st.push(v);
        break;
      }
      case BC_SEQ_AGG: {
        int64_t v;
        if (!env.seq_agg(b, a, code[pc], v)) return false;
        pc++;
        st.push(v);
        break;
      }
      case BC_JZ_KEEP: if (st.s[0] == 0) pc += 1 + code[pc]; else { st.pop(); pc++; } break;
      case BC_JNZ_KEEP: if (st.s[0] != 0) pc += 1 + code[pc]; else { st.pop(); pc++; } break;
      case BC_POP: st.pop(); break;
      case BC_NOT: case BC_NEG_I32: case BC_NEG_I64: case BC_NEG_F64: case BC_I64_TO_I32: case BC_I_TO_F64:
      case BC_F64_TO_I32: case BC_F64_TO_I64:
        st.s[0] = bc_un(op, st.s[0]);
        break;
      default: {
        int64_t z;
        const int e = bc_bin(op, st.s[1], st.s[0], z);
        if (e) { env.fail(e); return false; }
        st.pop();
        st.s[0] = z;
      }
    }
  }
}

// Lock-step variant: every lane of the wave walks the same program with a
// wave-uniform pc (the opcode switch is a scalar branch, no divergence); lanes
// not taking part (active = false) or jumped over a region (short-circuit &&,
// ||, getOrElse) follow along inactive until their resume point.  Jumps are
// forward and nested, so a lane resumes exactly at its target instruction.
// Returns false for a lane that raised (env.fail) -- only active lanes raise.
template <class Env>
__device__ __forceinline__ bool interp_ls(const int32_t* __restrict__ code_flat, int pc0, Env& env, bool active,
                                          int64_t& result) {
  const cint32_t* code = (const cint32_t*)code_flat;   // pc is wave-uniform: scalar fetches
  BcStack st;
#pragma unroll
  for (int i = 0; i < NFA_STACK; i++) st.s[i] = 0;
  int pc = __builtin_amdgcn_readfirstlane(pc0);
  int resume = active ? -1 : 0x7FFFFFFF;
  bool ok = true;
  result = 0;
  for (;;) {
    if (resume == pc) resume = -1;
    const bool on = resume < 0 && ok;
    const int32_t w = code[pc];
    const int op = w & 0xFF, a = (w >> 8) & 0xFF, b = (w >> 16) & 0xFF;
    pc++;
    switch (op) {
      case BC_END: if (on) result = st.s[0]; return ok;
      case BC_PUSH: if (on) st.push(int64_t(uint32_t(code[pc])) | (int64_t(code[pc + 1]) << 32)); pc += 2; break;
      case BC_FIELD: if (on) st.push(env.field(a, b)); break;
      case BC_EV_KEY: if (on) st.push(env.key()); break;
      case BC_EV_TS: if (on) st.push(env.ts()); break;
      case BC_EV_OFFSET: if (on) st.push(env.off()); break;
      case BC_EV_PARTITION: if (on) st.push(env.part()); break;
      case BC_TOPIC_EQ: if (on) st.push(env.topic() == code[pc] ? 1 : 0); pc++; break;
      case BC_STATE_GET: {
        if (on) {
          int32_t tag;
          int64_t v;
          if (!env.state(a, tag, v)) ok = false;
          else if (tag == 0) { env.fail(CEP_E_UNKNOWN_AGGREGATE); ok = false; }
          else if (tag != b) { env.fail(CEP_E_CLASS_CAST); ok = false; }
          else st.push(v);
        }
        break;
      }
      case BC_STATE_GET_OR_ELSE: {                              // the default's code follows; skip it if set
        const int target = pc + 1 + code[pc];
        if (on) {
          int32_t tag;
          int64_t v;
          if (!env.state(a, tag, v)) ok = false;
          else if (tag != 0) {
            if (tag != b) { env.fail(CEP_E_CLASS_CAST); ok = false; }
            else { st.push(v); resume = target; }
          }
        }
        pc++;
        break;
      }
      case BC_FOLD_CURR:
        if (on) {
          if (!env.in_fold || env.curr_tag == 0) { env.fail(CEP_E_NPE); ok = false; }
          else if (env.curr_tag != b) { env.fail(CEP_E_CLASS_CAST); ok = false; }
          else st.push(env.curr);
        }
        break;
      case BC_SEQ_AVG: {
        if (on) {
          int64_t v;
          if (!env.seq_avg(a, v)) ok = false;
          else st.push(v);
        }
        break;
      }
      case BC_SEQ_AGG: {
        if (on) {
          int64_t v;
          if (!env.seq_agg(b, a, code[pc], v)) ok = false;
          else st.push(v);
        }
        pc++;
        break;
      }
      case BC_JZ_KEEP: case BC_JNZ_KEEP: {
        const int target = pc + 1 + code[pc];
        if (on) {
          const bool jump = op == BC_JZ_KEEP ? st.s[0] == 0 : st.s[0] != 0;
          if (jump) resume = target;
          else st.pop();
        }
        pc++;
        break;
      }
      case BC_POP: if (on) st.pop(); break;
      case BC_NOT: case BC_NEG_I32: case BC_NEG_I64: case BC_NEG_F64: case BC_I64_TO_I32: case BC_I_TO_F64:
      case BC_F64_TO_I32: case BC_F64_TO_I64:
        if (on) st.s[0] = bc_un(op, st.s[0]);
        break;
      default: {
        int64_t z;
        const int e = bc_bin(op, st.s[1], st.s[0], z);
        if (on && e) { env.fail(e); ok = false; }
        else if (on) { st.pop(); st.s[0] = z; }
      }
    }
  }
}

// The program table of the built-in kernels: the pattern's DevProgram in
// device memory (wave-uniform reads through the scalar cache), predicates and
// folds interpreted in lock-step.  jit.cpp's JitTab has the same interface.
struct InterpTab {
  const DevProgram* raw;
  __device__ __forceinline__ const cDevProgram& prog() const { return *(const cDevProgram*)raw; }
  template <class Env>
  __device__ __forceinline__ bool eval(int pc, Env& env, bool active, int64_t& v) const {
    return interp_ls(raw->code, pc, env, active, v);
  }
};

}  // namespace kcep

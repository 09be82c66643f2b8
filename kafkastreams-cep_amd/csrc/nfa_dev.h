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

// The engine body (nfa_dev_body.h) is compiled in two address-space modes: here, in namespace kcep,
// with the key workspace addressed through generic pointers (kp_t: the workspace may sit in the pool
// or in the wave kernel's LDS arena), and by nfa_wave.h in namespace kcep::ldsm with LDS pointers, for
// keys whose whole workspace fits the arena (ds instructions instead of flat ones).
// queue entries (4 words) through either address space: a clang vector type, not HIP's int4 class, whose
// members take generic references
typedef int i4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ i4v mk4(int a, int b, int c, int d) { return i4v{a, b, c, d}; }
typedef int32_t* kp_t;
typedef const int32_t* kcp_t;
typedef i4v* kp4_t;
typedef const i4v* kcp4_t;
#define KCEP_LDSM 0
#define KCEP_NS kcep
#include "nfa_dev_body.h"
#undef KCEP_NS
#undef KCEP_LDSM

}  // namespace kcep

// jit.h — per-pattern kernels (jit.cpp).
#pragma once
#include <hip/hip_runtime.h>

#include <memory>
#include <string>

#include "kcep_internal.h"

namespace kcep {

// One pattern's specialised kernels, loaded from a code object hiprtc built.
// Shared by every session of the same program text (process-wide cache).
struct JitModule {
  hipModule_t mod = nullptr;
  hipFunction_t runs_sim = nullptr;     // runs_dev.h runs_sim_body<JitTab>
  hipFunction_t runs_write = nullptr;   // runs_dev.h runs_write_body<JitTab>
  hipFunction_t nfa = nullptr;          // nfa_dev.h nfa_kernel_body (general path)
  hipFunction_t nfa_wave = nullptr;     // nfa_wave.h nfa_wave_body, one key per wave (general path)
  hipFunction_t nfa_order = nullptr;    // nfa_dev.h nfa_order_bits_body, the wave kernel's schedule estimate
  ~JitModule();
};

// The HIP source of the pattern's runs kernels: the DevProgram as a constexpr
// table plus every predicate / fold as straight-line code (empty + why if some
// bytecode cannot be translated).
std::string jit_source_runs(const Program& P, std::string& why);

// Compile (or fetch from the cache) and load the runs kernels; nullptr + why on failure.
std::shared_ptr<const JitModule> jit_runs(const Program& P, std::string& why);

// Generate and compile only (no device needed): false + why if either fails.
bool jit_check_runs(const Program& P, std::string& why);

// the same for the general NFA path's kernel (nfa_dev.h)
std::string jit_source_general(const Program& P, std::string& why, bool phases = false);
// phases: the profiling build (KCEP_PHASES clocks, CEP_SESSION_PROFILE sessions)
std::shared_ptr<const JitModule> jit_general(const Program& P, std::string& why, bool phases = false);
bool jit_check_general(const Program& P, std::string& why);

}  // namespace kcep

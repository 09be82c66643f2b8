// jit.cpp — per-pattern kernels built with hiprtc.
//
// The built-in runs / general kernels interpret each predicate and fold
// (interp.h): per bytecode op a scalar dispatch plus predicated shifts of the
// register operand stack, ~200 instructions per op (SQ_INSTS_* of runs_sim).
// A pattern is fixed for the life of a session, so the session can instead run
// kernels compiled for it:
//   * the DevProgram becomes a constexpr table, so the engine's loops over
//     stages, edges and folds unroll and every table read folds to a constant;
//   * every predicate / fold becomes a straight-line function: the bytecode's
//     stack depth is static at every pc (compile.cpp CodeGen), so slot i is the
//     local s<i>, short-circuit jumps are forward gotos, and each operator is
//     the same bc_bin / bc_un body the interpreter uses (Java semantics shared
//     by construction, with -ffp-contract=off so no multiply-add is fused).
// The engine text (runs_dev.h, interp.h, kcep_dev.h, kcep.h) is embedded in the
// library at build time (build/jit_src.inc) and compiled with the generated
// part in-process; code objects are cached per (device, source) for the
// process, and hiprtc's own cache keeps repeat compiles across processes cheap.
#include "jit.h"

#include <hip/hiprtc.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <functional>
#include <map>
#include <mutex>
#include <set>
#include <vector>

#include "../../include/kcep.h"

namespace kcep {

namespace {
#include "jit_src.inc"   // kJitNames[], kJitTexts[], kJitCount (Makefile: embedded headers)

void put_arr(std::string& o, const int32_t* v, int n) {
  while (n > 0 && v[n - 1] == 0) n--;
  o += '{';
  for (int i = 0; i < n; i++) {
    if (i) o += ',';
    o += std::to_string(v[i]);
  }
  o += '}';
}

// DevProgram as a positional aggregate initializer (kcep_dev.h member order)
std::string program_table(const DevProgram& d) {
  std::string o = "{";
  for (int32_t v : {d.nstages, d.begin, d.nslots, d.nstates, d.ndefined, d.ncols, d.mode, d.maxdepth, d.nsl})
    o += std::to_string(v) + ",";
  put_arr(o, d.sl_pc, NFA_MAX_SL);
  o += ',';
  put_arr(o, d.slot_name, NFA_MAX_SLOTS);
  o += ',';
  put_arr(o, d.defined, NFA_MAX_STATES);
  o += ',';
  put_arr(o, d.coltype, 16);
  o += ",{";
  for (int s = 0; s < d.nstages; s++) {
    const DevStage& t = d.st[s];
    if (s) o += ',';
    o += '{';
    for (int32_t v : {t.name, t.type, t.slot, t.nedges, t.nfolds}) o += std::to_string(v) + ",";
    put_arr(o, t.op, NFA_MAX_EDGES);
    o += ',';
    put_arr(o, t.target, NFA_MAX_EDGES);
    o += ',';
    put_arr(o, t.pred, NFA_MAX_EDGES);
    o += ',';
    put_arr(o, t.sl, NFA_MAX_EDGES);
    o += ',';
    put_arr(o, t.fold_state, NFA_MAX_FOLDS);
    o += ',';
    put_arr(o, t.fold_type, NFA_MAX_FOLDS);
    o += ',';
    put_arr(o, t.fold_code, NFA_MAX_FOLDS);
    o += '}';
  }
  o += "}}";                                    // code[] stays zero: predicates are compiled
  return o;
}

std::string sv(int i) { return "s" + std::to_string(i); }

// one predicate / fold body starting at pc0, as template <class Env> bool jf_<pc0>(Env&, int64_t&)
// branchfree (the runs kernels, whose Env.state never fails): a body without sequence reads keeps its
// first failure in a register and tests it once at the end, instead of a divergent branch per check
// (state tag, Curr, division by zero) -- the ops after a failure compute discarded values and have no
// side effects, so the result and the reported failure are the same; && / || jumps stay branches, so
// what they skip never runs (Java's short circuit)
bool gen_entry(const DevProgram& d, int pc0, std::string& o, std::string& why, bool branchfree) {
  auto word = [&](int pc) { return pc >= 0 && pc < NFA_MAX_CODE ? d.code[pc] : 0; };
  std::set<int> labels;
  bool has_seq = false;
  for (int pc = pc0;;) {                        // pass 1: jump targets
    if (pc < 0 || pc >= NFA_MAX_CODE) { why = "code out of range"; return false; }
    const int op = word(pc) & 0xFF;
    pc++;
    if (op == BC_SEQ_AVG || op == BC_SEQ_AGG) has_seq = true;
    if (op == BC_END) break;
    if (op == BC_PUSH) pc += 2;
    else if (op == BC_TOPIC_EQ || op == BC_SEQ_AGG) pc++;
    else if (op == BC_STATE_GET_OR_ELSE || op == BC_JZ_KEEP || op == BC_JNZ_KEEP) {
      labels.insert(pc + 1 + word(pc));
      pc++;
    }
  }
  const bool bf = branchfree && !has_seq;      // (a jump stays a branch: the ops it skips never run)
  std::string b;
  char buf[256];
  int depth = 0, maxd = 0;
  auto need = [&](int k) {
    if (depth < k) { why = "stack underflow"; return false; }
    return true;
  };
  for (int pc = pc0;;) {
    if (labels.count(pc)) b += "L" + std::to_string(pc) + ":;\n";
    const int32_t w = word(pc);
    const int op = w & 0xFF, a = (w >> 8) & 0xFF, c = (w >> 16) & 0xFF;
    pc++;
    const std::string top = depth > 0 ? sv(depth - 1) : "";
    switch (op) {
      case BC_END:
        if (!need(1)) return false;
        if (bf) b += "if (e) { env.fail(e); return false; }\n";
        b += "r = " + top + "; return true;\n";
        goto done;
      case BC_PUSH: {
        const uint64_t v = uint64_t(uint32_t(word(pc))) | (uint64_t(uint32_t(word(pc + 1))) << 32);
        snprintf(buf, sizeof buf, "%s = int64_t(0x%016llxull);\n", sv(depth).c_str(), (unsigned long long)v);
        b += buf;
        depth++;
        pc += 2;
        break;
      }
      case BC_FIELD: b += sv(depth++) + " = env.field(" + std::to_string(a) + ", " + std::to_string(c) + ");\n"; break;
      case BC_EV_KEY: b += sv(depth++) + " = env.key();\n"; break;
      case BC_EV_TS: b += sv(depth++) + " = env.ts();\n"; break;
      case BC_EV_OFFSET: b += sv(depth++) + " = env.off();\n"; break;
      case BC_EV_PARTITION: b += sv(depth++) + " = env.part();\n"; break;
      case BC_TOPIC_EQ:
        b += sv(depth++) + " = env.topic() == " + std::to_string(word(pc)) + " ? 1 : 0;\n";
        pc++;
        break;
      case BC_STATE_GET:
        if (bf) {
          snprintf(buf, sizeof buf,
                   "{ int32_t tg; int64_t v; env.state(%d, tg, v); "
                   "e = e ? e : tg == 0 ? CEP_E_UNKNOWN_AGGREGATE : tg != %d ? CEP_E_CLASS_CAST : 0; %s = v; }\n",
                   a, c, sv(depth).c_str());
          b += buf;
          depth++;
          break;
        }
        snprintf(buf, sizeof buf,
                 "{ int32_t tg; int64_t v; if (!env.state(%d, tg, v)) return false; "
                 "if (tg == 0) { env.fail(CEP_E_UNKNOWN_AGGREGATE); return false; } "
                 "if (tg != %d) { env.fail(CEP_E_CLASS_CAST); return false; } %s = v; }\n",
                 a, c, sv(depth).c_str());
        b += buf;
        depth++;
        break;
      case BC_STATE_GET_OR_ELSE: {               // set: push and skip the default's code
        const int target = pc + 1 + word(pc);
        if (bf) {
          snprintf(buf, sizeof buf,
                   "{ int32_t tg; int64_t v; env.state(%d, tg, v); if (tg != 0) { "
                   "e = e ? e : tg != %d ? CEP_E_CLASS_CAST : 0; %s = v; goto L%d; } }\n",
                   a, c, sv(depth).c_str(), target);
          b += buf;
          pc++;
          break;
        }
        snprintf(buf, sizeof buf,
                 "{ int32_t tg; int64_t v; if (!env.state(%d, tg, v)) return false; if (tg != 0) { "
                 "if (tg != %d) { env.fail(CEP_E_CLASS_CAST); return false; } %s = v; goto L%d; } }\n",
                 a, c, sv(depth).c_str(), target);
        b += buf;
        pc++;
        break;
      }
      case BC_FOLD_CURR:
        if (bf) {
          snprintf(buf, sizeof buf,
                   "e = e ? e : (!env.in_fold || env.curr_tag == 0) ? CEP_E_NPE : env.curr_tag != %d ? CEP_E_CLASS_CAST : 0; "
                   "%s = env.curr;\n",
                   c, sv(depth).c_str());
          b += buf;
          depth++;
          break;
        }
        snprintf(buf, sizeof buf,
                 "if (!env.in_fold || env.curr_tag == 0) { env.fail(CEP_E_NPE); return false; } "
                 "if (env.curr_tag != %d) { env.fail(CEP_E_CLASS_CAST); return false; } %s = env.curr;\n",
                 c, sv(depth).c_str());
        b += buf;
        depth++;
        break;
      case BC_SEQ_AVG:
        snprintf(buf, sizeof buf, "{ int64_t v; if (!env.seq_avg(%d, v)) return false; %s = v; }\n", a,
                 sv(depth).c_str());
        b += buf;
        depth++;
        break;
      case BC_SEQ_AGG:
        snprintf(buf, sizeof buf, "{ int64_t v; if (!env.seq_agg(%d, %d, %d, v)) return false; %s = v; }\n", c, a,
                 word(pc), sv(depth).c_str());
        b += buf;
        depth++;
        pc++;
        break;
      case BC_JZ_KEEP: case BC_JNZ_KEEP: {         // jump keeps the operand; fall-through pops it
        if (!need(1)) return false;
        const int target = pc + 1 + word(pc);
        b += "if (" + top + (op == BC_JZ_KEEP ? " == 0" : " != 0") + ") goto L" + std::to_string(target) + ";\n";
        depth--;
        pc++;
        break;
      }
      case BC_POP:
        if (!need(1)) return false;
        depth--;
        break;
      case BC_NOT: case BC_NEG_I32: case BC_NEG_I64: case BC_NEG_F64: case BC_I64_TO_I32: case BC_I_TO_F64:
      case BC_F64_TO_I32: case BC_F64_TO_I64:
        if (!need(1)) return false;
        b += top + " = bc_un(" + std::to_string(op) + ", " + top + ");\n";
        break;
      default: {
        if (op < BC_ADD_I32 || op > BC_NE_B) { why = "unknown opcode " + std::to_string(op); return false; }
        if (!need(2)) return false;
        if (bf)
          snprintf(buf, sizeof buf, "{ int64_t z; const int ee = bc_bin(%d, %s, %s, z); e = e ? e : ee; %s = z; }\n",
                   op, sv(depth - 2).c_str(), sv(depth - 1).c_str(), sv(depth - 2).c_str());
        else
          snprintf(buf, sizeof buf, "{ int64_t z; const int e = bc_bin(%d, %s, %s, z); if (e) { env.fail(e); return false; } %s = z; }\n",
                   op, sv(depth - 2).c_str(), sv(depth - 1).c_str(), sv(depth - 2).c_str());
        b += buf;
        depth--;
      }
    }
    maxd = std::max(maxd, depth);
  }
done:
  o += "template <class Env>\n__device__ __forceinline__ bool jf_" + std::to_string(pc0) + "(Env& env, int64_t& r) {\n";
  if (bf) o += "  int e = 0;\n";
  if (maxd > 0) {
    o += "  int64_t ";
    for (int i = 0; i < maxd; i++) o += (i ? ", " : "") + sv(i) + " = 0";
    o += ";\n";
  }
  o += b + "}\n";
  return true;
}

// int f(int i) returning v[i] computed from 64-bit immediates (bit fields of a fixed width, the word
// picked by comparisons): the stage table's small fields without a memory access -- a lookup in the
// constexpr DevProgram with a lane-divergent stage id is a vector load from the code object's constant
// data, which sat on every evaluation's dependency chain (nfa_dev.h ST_* accessors)
void gen_packed(std::string& o, const char* name, const std::vector<int>& v) {
  int lo = 0, hi = 0;
  for (int x : v) { lo = std::min(lo, x); hi = std::max(hi, x); }
  int bits = 1;
  while ((int64_t(1) << bits) <= int64_t(hi) - lo) bits++;
  const int per = 64 / bits;
  const int nw = std::max<int>(1, int((v.size() + per - 1) / per));
  std::vector<uint64_t> w(size_t(nw), 0);
  for (size_t i = 0; i < v.size(); i++)
    w[i / per] |= uint64_t(int64_t(v[i]) - lo) << (bits * (i % per));
  char buf[96];
  o += "__device__ __forceinline__ int " + std::string(name) + "(int i) {\n  uint64_t w = ";
  for (int k = nw - 1; k > 0; k--) {
    snprintf(buf, sizeof buf, "i >= %d ? 0x%016llxull : ", k * per, (unsigned long long)w[size_t(k)]);
    o += buf;
  }
  snprintf(buf, sizeof buf, "0x%016llxull;\n", (unsigned long long)w[0]);
  o += buf;
  o += "  int s = i;\n";
  for (int k = nw - 1; k > 0; k--) o += "  if (i >= " + std::to_string(k * per) + ") s = i - " + std::to_string(k * per) + ";\n" +
                                     (k > 1 ? "  else\n" : "");
  snprintf(buf, sizeof buf, "  return int((w >> (s * %d)) & 0x%llxull) + (%d);\n}\n", bits,
           (unsigned long long)((uint64_t(1) << bits) - 1), lo);
  o += buf;
}

// the generated part shared by every kernel family: program table, predicates, JitTab
bool gen_program(const Program& P, std::string& o, std::string& why, bool branchfree = false) {
  const DevProgram& d = P.dev;
  std::set<int> entries;
  for (int s = 0; s < d.nstages; s++) {
    const DevStage& t = d.st[s];
    for (int e = 0; e < t.nedges; e++)
      if (t.pred[e] >= 0) entries.insert(t.pred[e]);
    for (int f = 0; f < t.nfolds; f++) entries.insert(t.fold_code[f]);
  }
  for (int i = 0; i < d.nsl; i++) entries.insert(d.sl_pc[i]);
  o += "namespace kcep {\n";
  o += "constexpr DevProgram kcep_prog = " + program_table(d) + ";\n";
  {                                               // the stage table's hot fields as immediates
    std::vector<int> ty, nm, sl, ne, nf, op, tg, pr, es, sn;
    for (int s = 0; s < d.nstages; s++) {
      const DevStage& t = d.st[s];
      ty.push_back(t.type); nm.push_back(t.name); sl.push_back(t.slot); ne.push_back(t.nedges); nf.push_back(t.nfolds);
      for (int e = 0; e < NFA_MAX_EDGES; e++) {
        op.push_back(t.op[e]); tg.push_back(t.target[e]); pr.push_back(t.pred[e]); es.push_back(t.sl[e]);
      }
    }
    for (int s = 0; s < std::max(1, d.nslots); s++) sn.push_back(d.slot_name[s]);
    gen_packed(o, "jst_type", ty); gen_packed(o, "jst_name", nm); gen_packed(o, "jst_slot", sl);
    gen_packed(o, "jst_nedges", ne); gen_packed(o, "jst_nfolds", nf); gen_packed(o, "jst_op", op);
    gen_packed(o, "jst_target", tg); gen_packed(o, "jst_pred", pr); gen_packed(o, "jst_sl", es);
    gen_packed(o, "jst_slot_name", sn);
  }
  for (int pc : entries)
    if (!gen_entry(d, pc, o, why, branchfree)) return false;
  o += "template <class Env>\n__device__ __forceinline__ bool jit_eval(int pc, Env& env, int64_t& r) {\n  switch (pc) {\n";
  for (int pc : entries) o += "    case " + std::to_string(pc) + ": return jf_" + std::to_string(pc) + "(env, r);\n";
  o += "  }\n  env.fail(CEP_E_BAD_IR);\n  return false;\n}\n";
  o += R"(struct JitTab {
  __device__ __forceinline__ const DevProgram& prog() const { return kcep_prog; }
  // every lane evaluates (a pure function of its env, which the caller keeps loadable for idle lanes;
  // their results are dropped): with no branch around a predicate, the first computation of a
  // subexpression dominates its repeats in the stage's later predicates and folds, and the compiler
  // folds them (C3: the running average's divide, three per record on the oneOrMore stage -> one)
  template <class Env>
  __device__ __forceinline__ bool eval(int pc, Env& env, bool active, int64_t& v) const {
    int64_t r = 0;
    const bool ok = jit_eval(pc, env, r);
    v = active ? r : 0;
    return ok || !active;
  }
};
}  // namespace kcep
)";
  return true;
}

struct Cache {
  std::mutex mu;
  std::map<std::pair<int, std::string>, std::shared_ptr<const JitModule>> mods;
};
Cache& cache() {
  static Cache* c = new Cache();              // never destroyed: modules live for the process
  return *c;
}

bool compile(const std::string& src, std::vector<char>& code, std::string& why) {
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, src.c_str(), "kcep_jit.hip", kJitCount, kJitTexts, kJitNames) != HIPRTC_SUCCESS) {
    why = "hiprtcCreateProgram failed";
    return false;
  }
  const char* opts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-DKCEP_JIT=1"};
  const hiprtcResult rc = hiprtcCompileProgram(prog, 5, opts);
  if (rc != HIPRTC_SUCCESS) {
    size_t n = 0;
    hiprtcGetProgramLogSize(prog, &n);
    std::string log(n + 1, '\0');
    hiprtcGetProgramLog(prog, &log[0]);
    why = "hiprtc: " + std::string(hiprtcGetErrorString(rc)) + ": " + log.substr(0, 2000);
    hiprtcDestroyProgram(&prog);
    return false;
  }
  size_t n = 0;
  hiprtcGetCodeSize(prog, &n);
  code.resize(n);
  hiprtcGetCode(prog, code.data());
  hiprtcDestroyProgram(&prog);
  if (const char* dir = getenv("KCEP_JIT_DUMP")) {          // inspection: source + code object per build
    const std::string stem = std::string(dir) + "/kcep_jit_" + std::to_string(std::hash<std::string>()(src) & 0xFFFFFF);
    if (FILE* f = fopen((stem + ".hip").c_str(), "w")) { fwrite(src.data(), 1, src.size(), f); fclose(f); }
    if (FILE* f = fopen((stem + ".co").c_str(), "wb")) { fwrite(code.data(), 1, code.size(), f); fclose(f); }
  }
  return true;
}

std::shared_ptr<const JitModule> build(const std::string& src, const char* const* kernels,
                                       hipFunction_t JitModule::* const* slots, int nk, std::string& why) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) { why = "no HIP device"; return nullptr; }
  Cache& c = cache();
  std::lock_guard<std::mutex> lk(c.mu);
  auto it = c.mods.find({dev, src});
  if (it != c.mods.end()) return it->second;
  std::vector<char> code;
  if (!compile(src, code, why)) return nullptr;
  auto m = std::make_shared<JitModule>();
  if (hipModuleLoadData(&m->mod, code.data()) != hipSuccess) {
    why = "hipModuleLoadData failed";
    return nullptr;
  }
  for (int i = 0; i < nk; i++)
    if (hipModuleGetFunction(&(m.get()->*slots[i]), m->mod, kernels[i]) != hipSuccess) {
      why = std::string("kernel not found: ") + kernels[i];
      return nullptr;
    }
  c.mods[{dev, src}] = m;
  return m;
}
}  // namespace

JitModule::~JitModule() {}

std::string jit_source_runs(const Program& P, std::string& why) {
  std::string o = "#include \"interp.h\"\n";
  if (!gen_program(P, o, why, true)) return "";
  o += R"(#include "runs_dev.h"
extern "C" __global__ __launch_bounds__(kcep::RT) void kcep_runs_sim(kcep::RunsArgs A, int64_t* __restrict__ flag,
                                                                     int32_t* __restrict__ end_of) {
  kcep::runs_sim_body(kcep::JitTab{}, kcep::runs_args_dev(A), flag, end_of);
}
extern "C" __global__ __launch_bounds__(kcep::RT) void kcep_runs_write(kcep::WriteArgs W) {
  kcep::runs_write_body(kcep::JitTab{}, W);
}
)";
  return o;
}

std::shared_ptr<const JitModule> jit_runs(const Program& P, std::string& why) {
  const std::string src = jit_source_runs(P, why);
  if (src.empty()) return nullptr;
  static const char* const names[] = {"kcep_runs_sim", "kcep_runs_write"};
  static hipFunction_t JitModule::* const slots[] = {&JitModule::runs_sim, &JitModule::runs_write};
  return build(src, names, slots, 2, why);
}

std::string jit_source_general(const Program& P, std::string& why, bool phases) {
  std::string o = phases ? "#define KCEP_PHASES 1\n#include \"interp.h\"\n" : "#include \"interp.h\"\n";
  if (!gen_program(P, o, why)) return "";
  // waves per SIMD the register budgets are cut for: the lane kernel 2; the wave kernel 3 (166 VGPRs, no
  // spills).  r05, C4 with 16-byte frames: 4 waves (128 VGPRs) ran the kernel in 4.67 vs 4.92 ms but
  // spilled ~50 VGPRs, whose scratch lines reach HBM: 5.5 GB per launch against 0.28 GB
  // (profiles/r05_c4_occupancy.txt); r02: 2: 13.3, 3: 10.8, 4: 11.8 ms.  The wave kernel's LDS arena
  // (nfa_wave.h WAVE_ARENA) is 1664 words: C4 kernel 512 5.82-5.85, 1024 4.97-4.98, 1280 4.95-4.97,
  // 1536 4.94-4.96, 1664 4.94, 1792 5.25-5.26, 2048 5.21-5.24 ms (past ~1700 words a CU holds fewer
  // waves); HBM bytes per launch 1024: 275 MB, 1536: 234, 1664: 232 (profiles/r05_c4_arena.txt)
  const int waves = 2, wave_occ = 3;
  const std::string agg = wave_stateful(P.dev) || P.has_seq ? "true" : "false";
  o += "#include \"nfa_dev.h\"\n#include \"nfa_wave.h\"\nextern \"C\" __global__ __launch_bounds__(64) "
       "__attribute__((amdgpu_waves_per_eu(" + std::to_string(waves) + R"())) void kcep_nfa_kernel(kcep::NfaArgs A) {
  kcep::nfa_kernel_body(A);
}
extern "C" __global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu()" + std::to_string(wave_occ) + R"())) void kcep_nfa_wave(kcep::NfaArgs A) {
  kcep::nfa_wave_body<)" + agg + R"(>(A);
}
extern "C" __global__ __launch_bounds__(256) void kcep_nfa_order(kcep::NfaArgs A, uint8_t* bits) {
  kcep::nfa_order_bits_body(A, bits);
}
)";
  return o;
}

std::shared_ptr<const JitModule> jit_general(const Program& P, std::string& why, bool phases) {
  const std::string src = jit_source_general(P, why, phases);
  if (src.empty()) return nullptr;
  static const char* const names[] = {"kcep_nfa_kernel", "kcep_nfa_wave", "kcep_nfa_order"};
  static hipFunction_t JitModule::* const slots[] = {&JitModule::nfa, &JitModule::nfa_wave, &JitModule::nfa_order};
  return build(src, names, slots, 3, why);
}

bool jit_check_general(const Program& P, std::string& why) {
  const std::string src = jit_source_general(P, why);
  std::vector<char> code;
  return !src.empty() && compile(src, code, why);
}

bool jit_check_runs(const Program& P, std::string& why) {
  const std::string src = jit_source_runs(P, why);
  std::vector<char> code;
  return !src.empty() && compile(src, code, why);
}

}  // namespace kcep

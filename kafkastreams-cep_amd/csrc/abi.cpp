// abi.cpp — the C-ABI of include/kcep.h.
//
// A session plays the role of one CEPProcessor (processor/CEPProcessor.java:45-171)
// bound to one GPU: it owns the device workspace, receives whole batches of
// records (struct-of-arrays, grouped by key) instead of one process(K,V) call
// per record, launches the HIP kernels on the caller's stream and hands back
// the emitted sequences as a CSR.  There is no CPU evaluation path: if a
// pattern or batch cannot be lowered to a device path, the call fails with a
// status code.
//
// Two device paths:
//   stencil  (stencil.hip)  strict single-cardinality patterns, SURVEY Q9
//   general  (nfa.hip)      every pattern the IR expresses: one lane per key
//                           running the reference NFA over an HBM arena
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <memory>
#include <string>
#include <vector>

#include "../../include/kcep.h"
#include "kcep_internal.h"

namespace kcep {
hipError_t stencil_launch(const StencilLaunch& L, hipStream_t st);
int64_t stencil_tiles(int64_t n);
hipError_t stencil_post(const int32_t* key, const int32_t* out, int k, int64_t nm, int32_t* mkey,
                        const StencilProgram* P, unsigned long long* sum, hipStream_t st);

hipError_t nfa_launch(const NfaArgs& A, hipStream_t st);
hipError_t nfa_segments(const int32_t* key, int64_t n, int64_t* flag, int64_t* idx, int64_t* seg_start, int64_t* nseg,
                        int64_t* tmp, hipStream_t st);
hipError_t nfa_arena_sizes(const int64_t* seg_start, int64_t nseg, const NfaCaps& cap, int nslots, int nstates,
                           int64_t* words, hipStream_t st);
hipError_t nfa_entry_counts_launch(const int64_t* words, const int64_t* matches, int64_t nseg, int64_t* ents,
                                   hipStream_t st);
hipError_t exclusive_scan(const int64_t* in, int64_t n, int64_t* out, int64_t* total, int64_t* tmp, hipStream_t st);
hipError_t nfa_compact_launch(const int64_t* seg_start, int64_t nseg, const int32_t* key, const int64_t* res_out,
                              const int64_t* res_matches, const int64_t* moff, const int64_t* eoff,
                              int64_t* match_record, int32_t* match_key, int64_t* ent_off, int32_t* ent_name,
                              int64_t* ent_record, hipStream_t st);
}  // namespace kcep

using namespace kcep;

namespace {
thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIPCHECK(x)                                                                                \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess) return fail(CEP_E_HIP, std::string(#x ": ") + hipGetErrorString(e_));    \
  } while (0)

size_t type_size(int t) { return t == T_I32 ? 4 : 8; }

// device buffer that only grows
struct DBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap && p) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    hipError_t e = hipMalloc(&p, bytes ? bytes : 16);
    if (e == hipSuccess) cap = bytes ? bytes : 16;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T* as() const { return static_cast<T*>(p); }
};

uint64_t mix64(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
  return x;
}

// default per-key capacities of the general path (words; scaled on overflow)
constexpr NfaCaps kCaps{16, 2, 8, 4, 256, 48, 64, 16};
constexpr int kMaxRegrow = 6;                      // x4 each: up to 4096x the default arena
}  // namespace

struct cep_pattern {
  Program prog;
};

struct cep_session {
  const cep_pattern* pat = nullptr;
  cep_opts opts{};
  int path = 0;                 // preferred path
  int last_path = 0;            // path of the last batch
  int device = 0;
  hipStream_t stream = nullptr;
  int64_t n = 0;
  bool pending = false;
  hipEvent_t ev0 = nullptr, ev1 = nullptr, eb0 = nullptr, eb1 = nullptr;
  // ---- stencil workspace ----
  DBuf prog, out, status, counter, total, sum, mkey;
  int64_t out_cap = 0;
  uint32_t epoch = 0;
  const int32_t* d_key = nullptr;
  // ---- staging of host-resident batches ----
  DBuf h_key, h_valid, h_topic, h_part, h_off, h_ts;
  DBuf h_cols[16];
  // ---- general workspace ----
  DBuf dprog, flag, idx, seg, scan_tmp, scal, words, aoff, arena, r_matches, r_words, r_out, r_err, r_errrec, r_ovf,
      ents, moff, eoff, o_record, o_key, o_entoff, o_name, o_entrec, list, list_off;
  std::vector<std::unique_ptr<DBuf>> rerun_arenas;
  int64_t nseg = 0, g_matches = 0, g_entries = 0;
  int32_t g_err = CEP_OK;
  int64_t g_err_rec = -1;
  // ---- host CSR of the last collect ----
  std::vector<int64_t> match_record, ent_off, ent_record;
  std::vector<int32_t> match_key, ent_name, out_host;
};

namespace {

int push_stencil(cep_session* s, const cep_batch* b, hipStream_t st) {
  const StencilProgram& SP = s->pat->prog.stencil;
  const void* col = b->n_cols ? b->cols[SP.col] : nullptr;
  const int32_t* key = b->key_id;
  const int32_t* topic = SP.use_topic ? b->topic : nullptr;
  const size_t vs = type_size(SP.coltype);
  if (b->mem == CEP_MEM_HOST && b->n > 0) {
    if (s->h_key.ensure(size_t(b->n) * 4) || s->h_cols[0].ensure(size_t(b->n) * vs) ||
        (SP.use_topic && s->h_topic.ensure(size_t(b->n) * 4)))
      return fail(CEP_E_HIP, "staging allocation failed");
    HIPCHECK(hipMemcpyAsync(s->h_key.p, key, size_t(b->n) * 4, hipMemcpyHostToDevice, st));
    HIPCHECK(hipMemcpyAsync(s->h_cols[0].p, col, size_t(b->n) * vs, hipMemcpyHostToDevice, st));
    key = s->h_key.as<int32_t>();
    col = s->h_cols[0].p;
    if (SP.use_topic) {
      if (b->topic) HIPCHECK(hipMemcpyAsync(s->h_topic.p, b->topic, size_t(b->n) * 4, hipMemcpyHostToDevice, st));
      else HIPCHECK(hipMemsetAsync(s->h_topic.p, 0, size_t(b->n) * 4, st));
      topic = s->h_topic.as<int32_t>();
    }
  } else if (SP.use_topic && !b->topic && b->n > 0) {
    if (s->h_topic.ensure(size_t(b->n) * 4)) return fail(CEP_E_HIP, "staging allocation failed");
    HIPCHECK(hipMemsetAsync(s->h_topic.p, 0, size_t(b->n) * 4, st));
    topic = s->h_topic.as<int32_t>();
  }
  if ((reinterpret_cast<uintptr_t>(key) | reinterpret_cast<uintptr_t>(col) | reinterpret_cast<uintptr_t>(topic)) & 15)
    return fail(CEP_E_ARG, "device columns must be 16-byte aligned");
  s->d_key = key;
  // epoch tags the look-back granules of this launch; reset the status words when it wraps
  s->epoch = (s->epoch % 0xFFFFu) + 1;
  if (s->epoch == 1) HIPCHECK(hipMemsetAsync(s->status.p, 0, s->status.cap, st));
  StencilLaunch L{key, col, topic, b->n, s->prog.as<StencilProgram>(), SP.k, SP.coltype, SP.use_topic, SP.chain,
                  s->out.as<int32_t>(), s->out_cap, s->status.as<uint64_t>(), s->counter.as<uint32_t>(),
                  s->total.as<int64_t>(), s->epoch};
  HIPCHECK(hipEventRecord(s->ev0, st));
  HIPCHECK(stencil_launch(L, st));
  HIPCHECK(hipEventRecord(s->ev1, st));
  HIPCHECK(hipEventRecord(s->eb1, st));
  return CEP_OK;
}

template <class T>
int stage(cep_session* s, DBuf& buf, const T* src, int64_t n, hipStream_t st, const T** dst) {
  *dst = src;
  if (!src || n <= 0) return CEP_OK;
  if (buf.ensure(size_t(n) * sizeof(T))) return fail(CEP_E_HIP, "staging allocation failed");
  HIPCHECK(hipMemcpyAsync(buf.p, src, size_t(n) * sizeof(T), hipMemcpyHostToDevice, st));
  *dst = buf.as<T>();
  return CEP_OK;
}

int64_t read_i64(const void* dev, hipStream_t st, int* rc) {
  int64_t v = 0;
  if (hipMemcpyAsync(&v, dev, sizeof v, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    *rc = CEP_E_HIP;
  return v;
}

int push_general(cep_session* s, const cep_batch* b, hipStream_t st) {
  const Program& P = s->pat->prog;
  const int64_t n = b->n;
  NfaArgs A{};
  A.P = s->dprog.as<DevProgram>();
  A.n = n;
  A.mode = s->opts.mode;
  int rc = CEP_OK;
  if (b->mem == CEP_MEM_HOST) {
    if ((rc = stage(s, s->h_key, b->key_id, n, st, &A.key)) || (rc = stage(s, s->h_valid, b->valid, n, st, &A.valid)) ||
        (rc = stage(s, s->h_topic, b->topic, n, st, &A.topic)) ||
        (rc = stage(s, s->h_part, b->partition, n, st, &A.partition)) ||
        (rc = stage(s, s->h_off, b->offset, n, st, &A.offset)) || (rc = stage(s, s->h_ts, b->ts, n, st, &A.ts)))
      return rc;
    for (int c = 0; c < b->n_cols; c++) {
      const size_t w = type_size(P.coltypes[c]);
      if (n > 0) {
        if (s->h_cols[c].ensure(size_t(n) * w)) return fail(CEP_E_HIP, "staging allocation failed");
        HIPCHECK(hipMemcpyAsync(s->h_cols[c].p, b->cols[c], size_t(n) * w, hipMemcpyHostToDevice, st));
      }
      A.cols[c] = s->h_cols[c].p;
    }
  } else {
    A.key = b->key_id; A.valid = b->valid; A.topic = b->topic; A.partition = b->partition;
    A.offset = b->offset; A.ts = b->ts;
    for (int c = 0; c < b->n_cols; c++) A.cols[c] = b->cols[c];
  }
  s->d_key = A.key;
  s->g_err = CEP_OK;
  s->g_err_rec = -1;
  s->g_matches = s->g_entries = 0;
  s->nseg = 0;
  s->rerun_arenas.clear();
  if (n == 0) {
    HIPCHECK(hipEventRecord(s->ev0, st));
    HIPCHECK(hipEventRecord(s->ev1, st));
    HIPCHECK(hipEventRecord(s->eb1, st));
    return CEP_OK;
  }
  // segments: one per key run of the grouped batch
  const size_t nb = size_t(n / 1024 + 2) * 8;
  if (s->flag.ensure(size_t(n) * 8) || s->idx.ensure(size_t(n) * 8) || s->seg.ensure(size_t(n + 1) * 8) ||
      s->scan_tmp.ensure(nb) || s->scal.ensure(64))
    return fail(CEP_E_HIP, "allocation failed");
  int64_t* scal = s->scal.as<int64_t>();
  HIPCHECK(nfa_segments(A.key, n, s->flag.as<int64_t>(), s->idx.as<int64_t>(), s->seg.as<int64_t>(), scal,
                        s->scan_tmp.as<int64_t>(), st));
  const int64_t nseg = read_i64(scal, st, &rc);
  if (rc) return fail(rc, "segment count");
  if (nseg >= (int64_t(1) << 31)) return fail(CEP_E_ARG, "too many keys in one batch");
  s->nseg = nseg;
  A.seg_start = s->seg.as<int64_t>();
  const DevProgram& D = P.dev;
  NfaCaps cap = kCaps;
  const double scale = s->opts.arena_scale > 0 ? s->opts.arena_scale : 1.0;
  cap.heap_mult = int32_t(cap.heap_mult * scale);
  cap.out_mult = int32_t(cap.out_mult * scale);
  cap.q_mult = int32_t(cap.q_mult * scale + 0.5);
  cap.seq_mult = int32_t(cap.seq_mult * scale + 0.5);
  const size_t sb = size_t(nseg) * 8;
  if (s->words.ensure(sb) || s->aoff.ensure(sb) || s->r_matches.ensure(sb) || s->r_words.ensure(sb) ||
      s->r_out.ensure(sb) || s->r_err.ensure(sb) || s->r_errrec.ensure(sb) || s->r_ovf.ensure(sb) || s->ents.ensure(sb) ||
      s->moff.ensure(sb) || s->eoff.ensure(sb))
    return fail(CEP_E_HIP, "allocation failed");
  HIPCHECK(nfa_arena_sizes(A.seg_start, nseg, cap, D.nslots, D.nstates, s->words.as<int64_t>(), st));
  HIPCHECK(exclusive_scan(s->words.as<int64_t>(), nseg, s->aoff.as<int64_t>(), scal + 1, s->scan_tmp.as<int64_t>(), st));
  const int64_t total_words = read_i64(scal + 1, st, &rc);
  if (rc) return fail(rc, "arena size");
  if (s->arena.ensure(size_t(total_words) * 4)) return fail(CEP_E_RUN_CAPACITY, "cannot allocate the NFA arena");
  HIPCHECK(hipMemsetAsync(scal + 2, 0, 8, st));
  A.nlist = int32_t(nseg);
  A.seg_list = nullptr;
  A.arena = s->arena.as<int32_t>();
  A.arena_off = s->aoff.as<int64_t>();
  A.cap = cap;
  A.res_matches = s->r_matches.as<int64_t>();
  A.res_words = s->r_words.as<int64_t>();
  A.res_out = s->r_out.as<int64_t>();
  A.res_err = s->r_err.as<int32_t>();
  A.res_err_rec = s->r_errrec.as<int64_t>();
  A.res_overflow = s->r_ovf.as<int32_t>();
  A.overflow_count = reinterpret_cast<int32_t*>(scal + 2);
  HIPCHECK(hipEventRecord(s->ev0, st));
  HIPCHECK(nfa_launch(A, st));
  HIPCHECK(hipEventRecord(s->ev1, st));
  // keys that outgrew their arena: re-run exactly those with a 4x larger one
  std::vector<int64_t> seg_host;
  for (int round = 0;; round++) {
    int32_t novf = 0;
    HIPCHECK(hipMemcpyAsync(&novf, scal + 2, 4, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipStreamSynchronize(st));
    if (novf == 0) break;
    if (round >= kMaxRegrow) return fail(CEP_E_RUN_CAPACITY, "a key exceeded the largest NFA arena");
    std::vector<int32_t> ovf(static_cast<size_t>(nseg));
    HIPCHECK(hipMemcpy(ovf.data(), s->r_ovf.p, sb / 2, hipMemcpyDeviceToHost));
    if (seg_host.empty()) {
      seg_host.resize(size_t(nseg) + 1);
      HIPCHECK(hipMemcpy(seg_host.data(), s->seg.p, (size_t(nseg) + 1) * 8, hipMemcpyDeviceToHost));
    }
    cap.q_mult *= 4; cap.q_base *= 4; cap.seq_mult *= 4; cap.seq_base *= 4;
    cap.heap_mult *= 4; cap.heap_base *= 4; cap.out_mult *= 4; cap.out_base *= 4;
    std::vector<int32_t> lst;
    std::vector<int64_t> off;
    int64_t tot = 0;
    for (int64_t i = 0; i < nseg; i++)
      if (ovf[size_t(i)]) {
        int64_t a, b2, c, d, w;
        const int64_t L = seg_host[size_t(i) + 1] - seg_host[size_t(i)];
        a = cap.q_base + cap.q_mult * L; b2 = cap.seq_base + cap.seq_mult * L;
        c = cap.heap_base + cap.heap_mult * L; d = cap.out_base + cap.out_mult * L;
        w = 64 + 16 * a + 3 * int64_t(D.nslots) * L + 3 * int64_t(D.nstates) * b2 + c + d;
        lst.push_back(int32_t(i));
        off.push_back(tot);
        tot += (w + 3) & ~int64_t(3);
      }
    auto ar = std::make_unique<DBuf>();
    if (ar->ensure(size_t(tot) * 4) || s->list.ensure(lst.size() * 4) || s->list_off.ensure(off.size() * 8))
      return fail(CEP_E_RUN_CAPACITY, "cannot allocate the regrown NFA arena");
    HIPCHECK(hipMemcpy(s->list.p, lst.data(), lst.size() * 4, hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(s->list_off.p, off.data(), off.size() * 8, hipMemcpyHostToDevice));
    HIPCHECK(hipMemsetAsync(scal + 2, 0, 8, st));
    A.nlist = int32_t(lst.size());
    A.seg_list = s->list.as<int32_t>();
    A.arena = ar->as<int32_t>();
    A.arena_off = s->list_off.as<int64_t>();
    A.cap = cap;
    HIPCHECK(nfa_launch(A, st));
    s->rerun_arenas.push_back(std::move(ar));
  }
  // compaction into the CSR
  HIPCHECK(nfa_entry_counts_launch(s->r_words.as<int64_t>(), s->r_matches.as<int64_t>(), nseg, s->ents.as<int64_t>(), st));
  HIPCHECK(exclusive_scan(s->r_matches.as<int64_t>(), nseg, s->moff.as<int64_t>(), scal + 3, s->scan_tmp.as<int64_t>(), st));
  HIPCHECK(exclusive_scan(s->ents.as<int64_t>(), nseg, s->eoff.as<int64_t>(), scal + 4, s->scan_tmp.as<int64_t>(), st));
  int64_t tots[2] = {0, 0};
  HIPCHECK(hipMemcpyAsync(tots, scal + 3, 16, hipMemcpyDeviceToHost, st));
  HIPCHECK(hipStreamSynchronize(st));
  s->g_matches = tots[0];
  s->g_entries = tots[1];
  const size_t nm = size_t(std::max<int64_t>(tots[0], 1)), ne = size_t(std::max<int64_t>(tots[1], 1));
  if (s->o_record.ensure(nm * 8) || s->o_key.ensure(nm * 4) || s->o_entoff.ensure(nm * 8) ||
      s->o_name.ensure(ne * 4) || s->o_entrec.ensure(ne * 8))
    return fail(CEP_E_HIP, "allocation failed");
  HIPCHECK(nfa_compact_launch(A.seg_start, nseg, A.key, s->r_out.as<int64_t>(), s->r_matches.as<int64_t>(),
                              s->moff.as<int64_t>(), s->eoff.as<int64_t>(), s->o_record.as<int64_t>(),
                              s->o_key.as<int32_t>(), s->o_entoff.as<int64_t>(), s->o_name.as<int32_t>(),
                              s->o_entrec.as<int64_t>(), st));
  HIPCHECK(hipEventRecord(s->eb1, st));
  // the reference fails the task at its first exception: report the earliest failing record
  std::vector<int32_t> err(static_cast<size_t>(nseg));
  std::vector<int64_t> erec(static_cast<size_t>(nseg));
  HIPCHECK(hipMemcpyAsync(err.data(), s->r_err.p, size_t(nseg) * 4, hipMemcpyDeviceToHost, st));
  HIPCHECK(hipMemcpyAsync(erec.data(), s->r_errrec.p, size_t(nseg) * 8, hipMemcpyDeviceToHost, st));
  HIPCHECK(hipStreamSynchronize(st));
  for (int64_t i = 0; i < nseg; i++)
    if (err[size_t(i)] && (s->g_err_rec < 0 || erec[size_t(i)] < s->g_err_rec)) {
      s->g_err = err[size_t(i)];
      s->g_err_rec = erec[size_t(i)];
    }
  return CEP_OK;
}

}  // namespace

extern "C" {

const char* cep_last_error(void) { return g_err.c_str(); }
const char* cep_version(void) { return "kcep 0.1 (gfx950)"; }

int cep_compile(const uint8_t* ir, size_t len, cep_pattern** out) {
  if (!ir || !out) return fail(CEP_E_ARG, "null argument");
  *out = nullptr;
  auto* p = new cep_pattern();
  std::string err;
  int rc = compile_ir(ir, len, p->prog, err);
  if (rc) {
    delete p;
    return fail(rc, err);
  }
  *out = p;
  return CEP_OK;
}

void cep_pattern_free(cep_pattern* p) { delete p; }

int cep_pattern_get_info(const cep_pattern* p, cep_pattern_info* o) {
  if (!p || !o) return fail(CEP_E_ARG, "null argument");
  const Program& P = p->prog;
  o->n_stages = int32_t(P.stages.size());
  o->n_names = int32_t(P.names.size());
  o->n_patterns = int32_t(P.pats.size());
  o->n_cols = int32_t(P.coltypes.size());
  o->stencil_ok = P.stencil_ok && !P.stencil.chain ? 1 : 0;
  o->stencil_k = P.stencil_ok ? P.stencil.k : 0;
  o->chain_ok = P.stencil_ok && P.stencil.chain ? 1 : 0;
  return CEP_OK;
}

const char* cep_pattern_name(const cep_pattern* p, int32_t id) {
  if (!p || id < 0 || id >= int32_t(p->prog.names.size())) return nullptr;
  return p->prog.names[id].c_str();
}

int32_t cep_pattern_stage(const cep_pattern* p, int32_t sid, int32_t* name_id, int32_t* type, int64_t* window_ms,
                          int32_t* ops, int32_t* targets, int32_t cap) {
  if (!p || sid < 0 || sid >= int32_t(p->prog.stages.size())) return -1;
  const StageDef& st = p->prog.stages[sid];
  if (name_id) *name_id = st.name;
  if (type) *type = st.type;
  if (window_ms) *window_ms = st.window_ms;
  const int32_t ne = int32_t(st.edges.size());
  for (int32_t i = 0; i < ne && i < cap; i++) {
    if (ops) ops[i] = st.edges[i].op;
    if (targets) targets[i] = st.edges[i].target;
  }
  return ne;
}

int cep_session_open(const cep_pattern* p, const cep_opts* opts, cep_session** out) {
  if (!p || !opts || !out) return fail(CEP_E_ARG, "null argument");
  *out = nullptr;
  if (opts->mode != CEP_MODE_NFA && opts->mode != CEP_MODE_PROCESSOR) return fail(CEP_E_ARG, "bad mode");
  const Program& P = p->prog;
  int path = opts->force_path;
  const int fast = P.stencil.chain ? CEP_PATH_CHAIN : CEP_PATH_STENCIL;   // the streaming kernel's flavour
  if (path == 0) path = P.stencil_ok ? fast : CEP_PATH_GENERAL;
  if ((path == CEP_PATH_STENCIL || path == CEP_PATH_CHAIN) && !P.stencil_ok)
    return fail(CEP_E_UNSUPPORTED, "stencil path does not apply: " + P.stencil_why);
  if (path == CEP_PATH_STENCIL || path == CEP_PATH_CHAIN) path = fast;
  if (path == CEP_PATH_GENERAL && !P.general_ok)
    return fail(CEP_E_UNSUPPORTED, "pattern cannot be lowered to the device NFA: " + P.general_why);
  if (path != CEP_PATH_STENCIL && path != CEP_PATH_CHAIN && path != CEP_PATH_GENERAL) return fail(CEP_E_ARG, "bad path");
  HIPCHECK(hipSetDevice(opts->device));
  auto* s = new cep_session();
  s->pat = p;
  s->opts = *opts;
  s->path = path;
  s->device = opts->device;
  auto cleanup = [&](int rc) {
    cep_session_close(s);
    return rc;
  };
  const int64_t cap = std::max<int64_t>(opts->max_events, 1);
  if (cap >= (int64_t(1) << 31)) return cleanup(fail(CEP_E_ARG, "max_events must be < 2^31 per batch"));
  if (s->scal.ensure(64) || hipMemset(s->scal.p, 0, 64)) return cleanup(fail(CEP_E_HIP, "device allocation failed"));
  if (P.stencil_ok && path != CEP_PATH_GENERAL) {
    const int k = P.stencil.k;
    if (s->prog.ensure(sizeof(StencilProgram)) || s->status.ensure(sizeof(uint64_t) * (stencil_tiles(cap) + 1)) ||
        s->counter.ensure(64) || s->total.ensure(64) || s->sum.ensure(64) ||
        s->out.ensure(sizeof(int32_t) * size_t(k) * size_t(cap)))
      return cleanup(fail(CEP_E_HIP, "device allocation failed"));
    s->out_cap = cap;
    if (hipMemcpy(s->prog.p, &P.stencil, sizeof(StencilProgram), hipMemcpyHostToDevice) ||
        hipMemset(s->status.p, 0, s->status.cap) || hipMemset(s->counter.p, 0, s->counter.cap) ||
        hipMemset(s->total.p, 0, s->total.cap))
      return cleanup(fail(CEP_E_HIP, "device init failed"));
  }
  if (P.general_ok) {
    if (s->dprog.ensure(sizeof(DevProgram)) ||
        hipMemcpy(s->dprog.p, &P.dev, sizeof(DevProgram), hipMemcpyHostToDevice))
      return cleanup(fail(CEP_E_HIP, "device allocation failed"));
  }
  if (hipEventCreate(&s->ev0) || hipEventCreate(&s->ev1) || hipEventCreate(&s->eb0) || hipEventCreate(&s->eb1))
    return cleanup(fail(CEP_E_HIP, "event create failed"));
  *out = s;
  return CEP_OK;
}

void cep_session_close(cep_session* s) {
  if (!s) return;
  for (DBuf* b : {&s->prog, &s->out, &s->status, &s->counter, &s->total, &s->sum, &s->mkey, &s->h_key, &s->h_valid,
                  &s->h_topic, &s->h_part, &s->h_off, &s->h_ts, &s->dprog, &s->flag, &s->idx, &s->seg, &s->scan_tmp,
                  &s->scal, &s->words, &s->aoff, &s->arena, &s->r_matches, &s->r_words, &s->r_out, &s->r_err,
                  &s->r_errrec, &s->r_ovf, &s->ents, &s->moff, &s->eoff, &s->o_record, &s->o_key, &s->o_entoff,
                  &s->o_name, &s->o_entrec, &s->list, &s->list_off})
    b->release();
  for (auto& c : s->h_cols) c.release();
  s->rerun_arenas.clear();
  if (s->ev0) (void)hipEventDestroy(s->ev0);
  if (s->ev1) (void)hipEventDestroy(s->ev1);
  if (s->eb0) (void)hipEventDestroy(s->eb0);
  if (s->eb1) (void)hipEventDestroy(s->eb1);
  delete s;
}

int cep_session_path(const cep_session* s) { return s ? s->path : 0; }

int cep_push_batch(cep_session* s, const cep_batch* b, void* stream) {
  if (!s || !b) return fail(CEP_E_ARG, "null argument");
  const Program& P = s->pat->prog;
  if (b->n < 0 || b->n > s->opts.max_events) return fail(CEP_E_ARG, "batch larger than the session capacity");
  if (b->n > 0 && !b->key_id) return fail(CEP_E_ARG, "key_id is required");
  if (b->n_cols != int32_t(P.coltypes.size())) return fail(CEP_E_ARG, "column count does not match the pattern schema");
  for (int c = 0; c < b->n_cols; c++)
    if (b->n > 0 && !b->cols[c]) return fail(CEP_E_ARG, "null value column");
  hipStream_t st = static_cast<hipStream_t>(stream);
  HIPCHECK(hipSetDevice(s->device));
  s->stream = st;
  s->n = b->n;
  s->pending = true;
  HIPCHECK(hipEventRecord(s->eb0, st));
  // records the processor would drop (null key/value, re-delivered offsets)
  // break contiguity: the stencil only takes batches without them
  const bool stencil_batch = !b->valid && !(s->opts.mode == CEP_MODE_PROCESSOR && b->offset &&
                                            !(b->flags & CEP_BATCH_OFFSETS_MONOTONE));
  if (s->path != CEP_PATH_GENERAL && stencil_batch) {
    s->last_path = s->path;
    return push_stencil(s, b, st);
  }
  if (!P.general_ok)
    return fail(CEP_E_UNSUPPORTED, "batch needs the general NFA path, which this pattern cannot use: " + P.general_why);
  s->last_path = CEP_PATH_GENERAL;
  return push_general(s, b, st);
}

const int64_t* cep_device_match_count(const cep_session* s) { return s ? s->total.as<int64_t>() : nullptr; }

int cep_last_kernel_ms(cep_session* s, float* ms) {
  if (!s || !ms) return fail(CEP_E_ARG, "null argument");
  HIPCHECK(hipEventSynchronize(s->ev1));
  HIPCHECK(hipEventElapsedTime(ms, s->ev0, s->ev1));
  return CEP_OK;
}

int cep_last_batch_ms(cep_session* s, float* ms) {
  if (!s || !ms) return fail(CEP_E_ARG, "null argument");
  HIPCHECK(hipEventSynchronize(s->eb1));
  HIPCHECK(hipEventElapsedTime(ms, s->eb0, s->eb1));
  return CEP_OK;
}

int cep_collect(cep_session* s, cep_matches* o) {
  if (!s || !o) return fail(CEP_E_ARG, "null argument");
  memset(o, 0, sizeof *o);
  HIPCHECK(hipSetDevice(s->device));
  if (s->last_path == CEP_PATH_GENERAL) {
    HIPCHECK(hipStreamSynchronize(s->stream));
    const int64_t nm = s->g_matches, ne = s->g_entries;
    s->match_record.resize(size_t(nm));
    s->match_key.resize(size_t(nm));
    s->ent_off.resize(size_t(nm) + 1);
    s->ent_name.resize(size_t(ne));
    s->ent_record.resize(size_t(ne));
    if (nm > 0) {
      HIPCHECK(hipMemcpy(s->match_record.data(), s->o_record.p, size_t(nm) * 8, hipMemcpyDeviceToHost));
      HIPCHECK(hipMemcpy(s->match_key.data(), s->o_key.p, size_t(nm) * 4, hipMemcpyDeviceToHost));
      HIPCHECK(hipMemcpy(s->ent_off.data(), s->o_entoff.p, size_t(nm) * 8, hipMemcpyDeviceToHost));
    }
    if (ne > 0) {
      HIPCHECK(hipMemcpy(s->ent_name.data(), s->o_name.p, size_t(ne) * 4, hipMemcpyDeviceToHost));
      HIPCHECK(hipMemcpy(s->ent_record.data(), s->o_entrec.p, size_t(ne) * 8, hipMemcpyDeviceToHost));
    }
    s->ent_off[size_t(nm)] = ne;
    o->n_matches = nm;
    o->n_entries = ne;
    o->path = CEP_PATH_GENERAL;
    o->err = s->g_err;
    o->err_record = s->g_err_rec;
    if (s->g_err) g_err = "the reference NFA raises an exception on this batch";
  } else {
    const StencilProgram& SP = s->pat->prog.stencil;
    const int k = SP.k;
    int64_t nm = 0;
    if (s->pending && s->n > 0) HIPCHECK(hipMemcpyAsync(&nm, s->total.p, sizeof nm, hipMemcpyDeviceToHost, s->stream));
    HIPCHECK(hipStreamSynchronize(s->stream));
    if (nm > s->out_cap) return fail(CEP_E_RUN_CAPACITY, "match output exceeded the session capacity");
    s->out_host.resize(size_t(nm) * k);
    s->match_key.resize(size_t(nm));
    if (nm > 0) {
      if (s->mkey.ensure(size_t(nm) * 4)) return fail(CEP_E_HIP, "allocation failed");
      HIPCHECK(stencil_post(s->d_key, s->out.as<int32_t>(), k, nm, s->mkey.as<int32_t>(), s->prog.as<StencilProgram>(),
                            nullptr, s->stream));
      HIPCHECK(hipMemcpyAsync(s->out_host.data(), s->out.p, size_t(nm) * k * 4, hipMemcpyDeviceToHost, s->stream));
      HIPCHECK(hipMemcpyAsync(s->match_key.data(), s->mkey.p, size_t(nm) * 4, hipMemcpyDeviceToHost, s->stream));
      HIPCHECK(hipStreamSynchronize(s->stream));
    }
    // traversal order of SharedVersionedBufferStoreImpl.peek: final stage first;
    // chain matches carry -1 for the optional stages they skipped
    s->match_record.resize(size_t(nm));
    s->ent_off.resize(size_t(nm) + 1);
    s->ent_name.resize(size_t(nm) * k);
    s->ent_record.resize(size_t(nm) * k);
    int64_t ne = 0;
    for (int64_t m = 0; m < nm; m++) {
      s->match_record[m] = s->out_host[m * k + k - 1];
      s->ent_off[m] = ne;
      for (int i = 0; i < k; i++) {
        const int st = k - 1 - i;
        const int32_t r = s->out_host[m * k + st];
        if (r < 0) continue;
        s->ent_name[ne] = SP.name[st];
        s->ent_record[ne] = r;
        ne++;
      }
    }
    s->ent_off[nm] = ne;
    s->ent_name.resize(size_t(ne));
    s->ent_record.resize(size_t(ne));
    o->n_matches = nm;
    o->n_entries = ne;
    o->path = s->last_path;
    o->err = CEP_OK;
    o->err_record = -1;
  }
  o->match_record = s->match_record.data();
  o->match_key = s->match_key.data();
  o->ent_off = s->ent_off.data();
  o->ent_name = s->ent_name.data();
  o->ent_record = s->ent_record.data();
  s->pending = false;
  return CEP_OK;
}

int cep_checksum(cep_session* s, uint64_t* sum, int64_t* n_matches) {
  if (!s || !sum) return fail(CEP_E_ARG, "null argument");
  HIPCHECK(hipSetDevice(s->device));
  if (s->last_path == CEP_PATH_GENERAL) {
    cep_matches m;
    int rc = cep_collect(s, &m);
    if (rc) return rc;
    uint64_t h_all = 0;
    for (int64_t i = 0; i < m.n_matches; i++) {
      uint64_t h = mix64(uint64_t(m.match_record[i]) * 0x9e3779b97f4a7c15ULL);
      for (int64_t e = m.ent_off[i]; e < m.ent_off[i + 1]; e++)
        h = mix64(h ^ (uint64_t(m.ent_record[e]) << 8) ^ uint64_t(m.ent_name[e]));
      h_all += h;
    }
    *sum = h_all;
    if (n_matches) *n_matches = m.n_matches;
    return CEP_OK;
  }
  int64_t nm = 0;
  HIPCHECK(hipMemcpyAsync(&nm, s->total.p, sizeof nm, hipMemcpyDeviceToHost, s->stream));
  HIPCHECK(hipStreamSynchronize(s->stream));
  nm = std::min(nm, s->out_cap);
  HIPCHECK(hipMemsetAsync(s->sum.p, 0, 8, s->stream));
  const StencilProgram& SP = s->pat->prog.stencil;
  HIPCHECK(stencil_post(s->d_key, s->out.as<int32_t>(), SP.k, nm, nullptr, s->prog.as<StencilProgram>(),
                        s->sum.as<unsigned long long>(), s->stream));
  uint64_t h = 0;
  HIPCHECK(hipMemcpyAsync(&h, s->sum.p, 8, hipMemcpyDeviceToHost, s->stream));
  HIPCHECK(hipStreamSynchronize(s->stream));
  *sum = h;
  if (n_matches) *n_matches = nm;
  return CEP_OK;
}

}  // extern "C"

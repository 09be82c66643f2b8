// abi.cpp — the C-ABI of include/kcep.h.
//
// A session plays the role of one CEPProcessor (processor/CEPProcessor.java:45-171)
// bound to one GPU: it owns the device workspace, receives whole batches of
// records (struct-of-arrays, grouped by key) instead of one process(K,V) call
// per record, launches the HIP kernels on the caller's stream and hands back
// the emitted sequences as a CSR.  There is no CPU evaluation path: if a
// pattern or batch cannot be lowered to a device path, the call fails with a
// status code.
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/kcep.h"
#include "kcep_internal.h"

namespace kcep {
struct StencilLaunch {
  const int32_t* key;
  const void* val;
  const int32_t* topic;
  int64_t n;
  const StencilProgram* prog_dev;
  int k, coltype, use_topic;
  int32_t* out;
  int64_t out_cap;
  uint64_t* status;
  uint32_t* counter;
  int64_t* total;
  uint32_t epoch;
};
hipError_t stencil_launch(const StencilLaunch& L, hipStream_t st);
int64_t stencil_tiles(int64_t n);
hipError_t stencil_post(const int32_t* key, const int32_t* out, int k, int64_t nm, int32_t* mkey,
                        const StencilProgram* P, unsigned long long* sum, hipStream_t st);
}  // namespace kcep

using namespace kcep;

namespace {
thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIPCHECK(x)                                                                    \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) return fail(CEP_E_HIP, std::string(#x ": ") + hipGetErrorString(e_)); \
  } while (0)

size_t type_size(int t) { return t == T_I32 ? 4 : 8; }

// device buffer that only grows
struct DBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    hipError_t e = hipMalloc(&p, bytes ? bytes : 16);
    if (e == hipSuccess) cap = bytes;
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
}  // namespace

struct cep_pattern {
  Program prog;
};

struct cep_session {
  const cep_pattern* pat = nullptr;
  cep_opts opts{};
  int path = 0;
  int device = 0;
  // stencil workspace
  DBuf prog, out, status, counter, total, sum, mkey;
  int64_t out_cap = 0;
  uint32_t epoch = 0;
  // staging of host-resident batches
  DBuf h_key, h_col, h_topic;
  // last batch
  hipStream_t stream = nullptr;
  int64_t n = 0;
  const int32_t* d_key = nullptr;
  bool pending = false;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  // host CSR of the last collect
  std::vector<int64_t> match_record, ent_off, ent_record;
  std::vector<int32_t> match_key, ent_name, out_host;
};

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
  o->stencil_ok = P.stencil_ok ? 1 : 0;
  o->stencil_k = P.stencil_ok ? P.stencil.k : 0;
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
  int path = opts->force_path;
  if (path == 0) path = p->prog.stencil_ok ? CEP_PATH_STENCIL : CEP_PATH_GENERAL;
  if (path == CEP_PATH_STENCIL && !p->prog.stencil_ok)
    return fail(CEP_E_UNSUPPORTED, "stencil path does not apply: " + p->prog.stencil_why);
  if (path == CEP_PATH_GENERAL)
    return fail(CEP_E_UNSUPPORTED, "general NFA path not built into this library yet (" + p->prog.stencil_why + ")");
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
  const int k = p->prog.stencil.k;
  if (s->prog.ensure(sizeof(StencilProgram)) || s->status.ensure(sizeof(uint64_t) * (stencil_tiles(cap) + 1)) ||
      s->counter.ensure(64) || s->total.ensure(64) || s->sum.ensure(64) ||
      s->out.ensure(sizeof(int32_t) * size_t(k) * size_t(cap)))
    return cleanup(fail(CEP_E_HIP, "device allocation failed"));
  s->out_cap = cap;
  if (hipMemcpy(s->prog.p, &p->prog.stencil, sizeof(StencilProgram), hipMemcpyHostToDevice) ||
      hipMemset(s->status.p, 0, s->status.cap) || hipMemset(s->counter.p, 0, s->counter.cap) ||
      hipMemset(s->total.p, 0, s->total.cap))
    return cleanup(fail(CEP_E_HIP, "device init failed"));
  if (hipEventCreate(&s->ev0) || hipEventCreate(&s->ev1)) return cleanup(fail(CEP_E_HIP, "event create failed"));
  *out = s;
  return CEP_OK;
}

void cep_session_close(cep_session* s) {
  if (!s) return;
  for (DBuf* b : {&s->prog, &s->out, &s->status, &s->counter, &s->total, &s->sum, &s->mkey, &s->h_key, &s->h_col,
                  &s->h_topic})
    b->release();
  if (s->ev0) (void)hipEventDestroy(s->ev0);
  if (s->ev1) (void)hipEventDestroy(s->ev1);
  delete s;
}

int cep_session_path(const cep_session* s) { return s ? s->path : 0; }

int cep_push_batch(cep_session* s, const cep_batch* b, void* stream) {
  if (!s || !b) return fail(CEP_E_ARG, "null argument");
  const Program& P = s->pat->prog;
  if (b->n < 0 || b->n > s->opts.max_events) return fail(CEP_E_ARG, "batch larger than the session capacity");
  if (b->n > 0 && !b->key_id) return fail(CEP_E_ARG, "key_id is required");
  if (b->n_cols != int32_t(P.coltypes.size())) return fail(CEP_E_ARG, "column count does not match the pattern schema");
  hipStream_t st = static_cast<hipStream_t>(stream);
  HIPCHECK(hipSetDevice(s->device));
  s->stream = st;
  s->n = b->n;
  s->pending = true;

  const StencilProgram& SP = P.stencil;
  // records that the processor would drop (null key/value, re-delivered
  // offsets) break contiguity: the stencil only takes batches without them
  if (b->valid) return fail(CEP_E_UNSUPPORTED, "stencil path: batches with null records need the general path");
  if (s->opts.mode == CEP_MODE_PROCESSOR && b->offset && !(b->flags & CEP_BATCH_OFFSETS_MONOTONE))
    return fail(CEP_E_UNSUPPORTED, "stencil path: offsets must be flagged CEP_BATCH_OFFSETS_MONOTONE");
  const void* col = b->n_cols ? b->cols[SP.col] : nullptr;
  const int32_t* key = b->key_id;
  const int32_t* topic = SP.use_topic ? b->topic : nullptr;
  if (SP.use_topic && !b->topic && b->n) {
    // topic defaults to 0 for every record: the host copy below synthesises it
  }
  const size_t vs = type_size(SP.coltype);
  if (b->mem == CEP_MEM_HOST && b->n > 0) {
    if (s->h_key.ensure(size_t(b->n) * 4) || s->h_col.ensure(size_t(b->n) * vs) ||
        (SP.use_topic && s->h_topic.ensure(size_t(b->n) * 4)))
      return fail(CEP_E_HIP, "staging allocation failed");
    HIPCHECK(hipMemcpyAsync(s->h_key.p, key, size_t(b->n) * 4, hipMemcpyHostToDevice, st));
    HIPCHECK(hipMemcpyAsync(s->h_col.p, col, size_t(b->n) * vs, hipMemcpyHostToDevice, st));
    key = s->h_key.as<int32_t>();
    col = s->h_col.p;
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
  StencilLaunch L{key, col, topic, b->n, s->prog.as<StencilProgram>(), SP.k, SP.coltype, SP.use_topic,
                  s->out.as<int32_t>(), s->out_cap, s->status.as<uint64_t>(), s->counter.as<uint32_t>(),
                  s->total.as<int64_t>(), s->epoch};
  HIPCHECK(hipEventRecord(s->ev0, st));
  HIPCHECK(stencil_launch(L, st));
  HIPCHECK(hipEventRecord(s->ev1, st));
  return CEP_OK;
}

const int64_t* cep_device_match_count(const cep_session* s) { return s ? s->total.as<int64_t>() : nullptr; }

int cep_last_kernel_ms(cep_session* s, float* ms) {
  if (!s || !ms) return fail(CEP_E_ARG, "null argument");
  HIPCHECK(hipEventSynchronize(s->ev1));
  HIPCHECK(hipEventElapsedTime(ms, s->ev0, s->ev1));
  return CEP_OK;
}

int cep_checksum(cep_session* s, uint64_t* sum, int64_t* n_matches) {
  if (!s || !sum) return fail(CEP_E_ARG, "null argument");
  HIPCHECK(hipSetDevice(s->device));
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

int cep_collect(cep_session* s, cep_matches* o) {
  if (!s || !o) return fail(CEP_E_ARG, "null argument");
  memset(o, 0, sizeof *o);
  HIPCHECK(hipSetDevice(s->device));
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
  // traversal order of SharedVersionedBufferStoreImpl.peek: final stage first
  s->match_record.resize(size_t(nm));
  s->ent_off.resize(size_t(nm) + 1);
  s->ent_name.resize(size_t(nm) * k);
  s->ent_record.resize(size_t(nm) * k);
  for (int64_t m = 0; m < nm; m++) {
    s->match_record[m] = s->out_host[m * k + k - 1];
    s->ent_off[m] = m * k;
    for (int i = 0; i < k; i++) {
      const int st = k - 1 - i;
      s->ent_name[m * k + i] = SP.name[st];
      s->ent_record[m * k + i] = s->out_host[m * k + st];
    }
  }
  s->ent_off[nm] = nm * k;
  o->n_matches = nm;
  o->n_entries = nm * k;
  o->match_record = s->match_record.data();
  o->match_key = s->match_key.data();
  o->ent_off = s->ent_off.data();
  o->ent_name = s->ent_name.data();
  o->ent_record = s->ent_record.data();
  o->path = s->path;
  o->err = CEP_OK;
  o->err_record = -1;
  s->pending = false;
  return CEP_OK;
}

}  // extern "C"

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
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <memory>
#include <string>
#include <vector>

#include "../../include/kcep.h"
#include "build_id.h"   // KCEP_BUILD_ID (Makefile: hash of the library sources)
#include "kcep_internal.h"
#include "jit.h"

namespace kcep {
hipError_t stencil_launch(const StencilLaunch& L, hipEvent_t ev0, hipEvent_t ev1, hipStream_t st);
int64_t stencil_tiles(int64_t n);
hipError_t stencil_post(const int32_t* key, const int32_t* out, int k, int64_t nm, int32_t* mkey,
                        const StencilProgram* P, unsigned long long* sum, hipStream_t st);
hipError_t stencil_resolve_launch(const int32_t* key, const int32_t* out, int k, int64_t nm, const StencilCarry& C,
                                  int64_t* pos, const StencilProgram* P, unsigned long long* sum, hipStream_t st);
hipError_t stencil_deliver_launch(const int32_t* key, const int32_t* out, int k, const int64_t* total, int64_t out_cap,
                                  const StencilCarry& C, int64_t host_cap, int64_t* hdr, int32_t* hkey, int64_t* hpos,
                                  int32_t* dkey, int64_t* dpos, hipStream_t st);

hipError_t nfa_launch(const NfaArgs& A, hipStream_t st, hipFunction_t jf);
hipError_t nfa_wave_launch(const NfaArgs& A, int64_t grid, hipStream_t st, const JitModule* j);
int64_t nfa_wave_grid(int64_t nseg, bool agg, const JitModule* j);
hipError_t nfa_segments(const int32_t* key, int64_t n, int64_t* flag, int64_t* idx, int64_t* seg_start, int64_t* nseg,
                        int64_t* tmp, hipStream_t st);
hipError_t exclusive_scan(const int64_t* in, int64_t n, int64_t* out, int64_t* total, int64_t* tmp, hipStream_t st);
hipError_t set_words_launch(int64_t* w, int n, int at, int64_t v, hipStream_t st);
hipError_t nfa_order_launch(const NfaArgs& A, int64_t nseg, uint8_t* bits, unsigned* bcnt, int32_t* order,
                            hipStream_t st, const JitModule* j, int lo);
// The schedule's estimate buckets (log2 of the segment weight) below this one keep arrival order
// behind the heavier ones: only a key that could end the grid late needs to start early, and every
// key moved forward adds scratch lines in flight beside the other heavy keys (C4, lowest ordered
// bucket 0 / 4 / 6 / 8 / 10: kernel 4.240 / 4.255 / 4.282 / 4.273 / 4.573 ms, kcep_nfa_wave
// 201.2 / 201.3 / 200.9 / 197.6 / 183.0 MB per launch; profiles/r05_c4_order_lo.txt)
constexpr int NFA_ORDER_LO = 8;
hipError_t gather_words_launch(const int64_t* a, int na, const int64_t* b, int nb, int64_t* h, hipStream_t st);
hipError_t exclusive_scan_pair(const int64_t* in0, const int64_t* in1, int64_t n, const int64_t* n_dev, int64_t* out0,
                               int64_t* out1, int64_t* total0, int64_t* total1, int64_t* tmp, hipStream_t st);
hipError_t nfa_compact_launch(int64_t nseg, const int64_t* nseg_dev, int64_t nm, int64_t ne, const int64_t* tot_dev,
                              const int32_t* key, const int64_t* seg_start, const int64_t* res_out, const int64_t* res_ent,
                              const int64_t* moff, const int64_t* eoff, int64_t* match_record, int32_t* match_key,
                              int64_t* ent_off, int32_t* ent_name, int64_t* ent_record, hipStream_t st);
hipError_t carry_commit_launch(int64_t nseg, const int32_t* key, const int64_t* seg_start, const int64_t* res_carry,
                               const int32_t* res_err, int64_t* ctab, hipStream_t st);
hipError_t carry_keycheck_launch(int64_t max_seg, const int64_t* nseg, const int32_t* key, const int64_t* seg_start,
                                int32_t max_keys, int32_t* stamp, int32_t batch_no, unsigned long long* flags,
                                hipStream_t st);
hipError_t carry_sizes_launch(const int64_t* ctab, int64_t nkeys, const int32_t* cpool, int64_t* words,
                              hipStream_t st);
hipError_t runs_sim_launch(const RunsArgs& A, int64_t* flag, int32_t* end_of, hipStream_t st, hipFunction_t jf);
hipError_t runs_expand_launch(const RunsArgs& R, const unsigned long long* sorted, int64_t nm, const int64_t* ent_off,
                              int64_t ne, int64_t* match_record, int32_t* match_key, int64_t* ent_off_out, int32_t* ent_name,
                              int64_t* ent_record, hipStream_t st);
hipError_t runs_compact_launch(const int64_t* stat, const int32_t* end_of, int64_t n, int32_t chunk, int64_t* pre,
                               unsigned long long* out, int64_t* tot_cnt, int64_t* tot_len, int64_t* scan_tmp,
                               hipStream_t st, int64_t n_grid);
int64_t runs_sim_waves(int64_t n, int32_t chunk);
bool runs_emit_scan(const int64_t* stat, int64_t n, int32_t chunk, int64_t* pre, int64_t* tot_cnt, int64_t* tot_len,
                    hipStream_t st, const int64_t* n_dev);
hipError_t runs_emit_launch(const RunsArgs& R, const int32_t* end_of, const int64_t* pre, int span, int64_t* match_record,
                            int32_t* match_key, int64_t* ent_off, int32_t* ent_name, int64_t* ent_record, hipStream_t st,
                            int64_t n_grid);
hipError_t runs_results_launch(const unsigned long long* ctl, const int64_t* nm, const int64_t* top, int64_t* h,
                               hipStream_t st, const int64_t* x);
hipError_t runs_order_launch(const unsigned long long* in, int64_t nm, int w, unsigned long long* out, int64_t* len,
                             hipStream_t st);
hipError_t runs_sort(const unsigned long long* in, unsigned long long* out, int64_t nm, int bits, void* tmp,
                     size_t* tmp_bytes, hipStream_t st);
hipError_t runs_write_launch(const RunsArgs& R, const unsigned long long* sorted, int64_t nm, int64_t* len,
                             int64_t* ent_off, int64_t* total, int64_t* scan_tmp, int64_t* match_record,
                             int32_t* match_key, int64_t* ent_off_out, int32_t* ent_name, int64_t* ent_record,
                             hipStream_t st, bool lengths_only, hipFunction_t jf);
hipError_t carry_move_launch(int64_t* ctab, int64_t nkeys, const int32_t* src, const int64_t* off, int32_t* dst,
                             hipStream_t st);
}  // namespace kcep

using namespace kcep;

namespace {
thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
}  // namespace
namespace kcep {
int set_error(int code, const std::string& msg) { return fail(code, msg); }
}  // namespace kcep
namespace {

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

// The wave kernel (nfa_wave.h) evaluates a record's runs in parallel: it needs a pattern whose
// evaluations read nothing but the record -- every edge predicate event-only, no folds, no states.
// the wave kernel takes every pattern: rounds whose runs share a sequence that one of them folds into
// (or that read a partial sequence after a run of the round died) are evaluated again sequentially
// (nfa_wave.h).

// first allocation of a key's workspace on the general path (grown on demand from the pool)
constexpr NfaCaps kCaps{16, 64, 32, 32, 8, 16};
constexpr int kMaxRetry = 24;                      // pool regrowths (each toward free HBM) before CEP_E_RUN_CAPACITY
constexpr int kPoolQuiet = 4;                      // batches within the estimate before a grown pool is given back
constexpr int64_t kRunsErrCap = int64_t(1) << 20;  // runs path: failing runs listed per batch (cep_batch_errors)
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
  bool timing = true;                      // cep_session_set_timing: stencil/chain batches record events
  // ---- stencil workspace ----
  DBuf prog, out, status, counter, total, sum, mkey, slots;   // status: tile counts + prefixes; counter: scan scratch
  int64_t out_cap = 0;
  const int32_t* d_key = nullptr;
  // ---- staging of host-resident batches (stage_host): a pinned ring the caller's columns are copied
  // into in chunks, each chunk moved by one async copy into one packed device image; caller memory
  // that is itself pinned is copied from directly and the push waits for that copy ----
  DBuf dstage, h_topic;
  void* ring[2] = {nullptr, nullptr};
  size_t ring_cap[2] = {0, 0};
  hipEvent_t ring_ev[2] = {nullptr, nullptr};
  int ring_next = 0;
  hipEvent_t h2d_ev = nullptr;
  // ---- CEP_BATCH_DELIVER (carry stencil / chain sessions): the matches handed to pinned host memory by
  // the device during the push; cep_collect then only waits ----
  void* dl[2] = {nullptr, nullptr};   // dl_layout: header, host_cap keys, host_cap * k positions; by stamp parity
  int64_t dl_pid[2] = {-1, -1};       // the batch (push number) each holds: a host pushes batch i + 1 before it
                                      // collects batch i (cep_collect_batch)
  int64_t push_id = 0;                // cep_push_batch calls so far (cep_batch_id)
  int64_t dl_cap = 0;
  DBuf dl_ticket;                 // device: workgroups of the delivery kernel done
  int64_t dl_stamp = 0;           // the last delivery's number
  bool delivered = false;
  bool h2d_wait = false;          // the push copied from pinned caller memory: wait for h2d_ev
  int zc_slot = -1;               // the push's kernels read ring slot zc_slot in place (zero copy)
  // ---- general workspace ----
  DBuf dprog, flag, idx, seg, scan_tmp, scal, ctl, pool, r_matches, r_words, r_out, r_ent, r_err, r_errrec, r_carry,
      moff, eoff, o_record, o_key, o_entoff, o_name, o_entrec, ord, ord_bucket, ord_cnt;
  int64_t pool_words = 0;       // pool capacity this batch uses
  int64_t pool_est = 0;         // the batches' estimated pool (largest so far)
  int64_t pool_learned = 0;     // what the last overflowing batch grew the pool to (0: none): later batches start
                                // there, without re-running, until kPoolQuiet batches in a row fit the estimate
  int pool_quiet = 0;
  int last_attempts = 0;        // general path: kernel attempts of the last batch (1 + pool regrowths)
  int64_t nseg = 0, g_matches = 0, g_entries = 0;
  int64_t nseg_hint = 0;        // the last general batch's segment count (pool estimate of the next)
  // ---- carried per-key state (CEP_SESSION_CARRY): NFAStore equivalent ----
  bool carry = false;
  int64_t base = 0;             // stream position of the next batch's record 0
  DBuf ctab, cpool;             // per key id: blob offset (-1 none); blobs (int32 words)
  DBuf kstamp;                  // per key id: number of the last batch that had a segment of it
  int32_t batch_no = 0;
  // ---- carried halos of the stencil path (CEP_SESSION_CARRY, kcep_internal.h HaloHdr) ----
  DBuf halo, hpos, hflags, opos;
  int32_t halo_stamp = 0;
  int64_t halo_base = 0;        // stream position of the last stencil batch's record 0
  int64_t cpool_words = 0, cpool_used = 0;
  // ---- deterministic runs workspace ----
  DBuf rk, rk_sorted, rk_tmp, r_len, r_entoff, r_errcode, r_endof, r_segs, r_blk, r_errlist;
  // kernels compiled for the pattern (jit.cpp); null: the built-in interpreting kernels run
  bool jit_on = false;                     // allowed (not CEP_SESSION_INTERPRET / KCEP_JIT=0)
  std::shared_ptr<const JitModule> jit;    // runs path
  std::shared_ptr<const JitModule> jitg;   // general path (built at open, or at the first general batch)
  bool jitg_tried = false;
  int64_t live_hwm = 0;                    // general path: most live runs any key held in the last batch
  bool wave = false;                       // general path: one key per wave (nfa_wave.h) for this pattern
  DBuf wscratch;                           // the wave kernel's recycled per-workgroup workspace regions
  bool g_any_err = false;                  // general path: some key of the last batch raised
  DBuf r_prof;                             // CEP_SESSION_PROFILE: per key segment {live max, evaluations, cycles}
  std::string jit_why;
  int32_t g_err = CEP_OK;
  int64_t g_err_rec = -1;
  std::vector<int64_t> e_rec;              // every failing key's (record, code) of the last batch
  std::vector<int32_t> e_code;
  // ---- host CSR of the last collect ----
  std::vector<int64_t> match_record, ent_off, ent_record;
  std::vector<int32_t> match_key, ent_name, out_host;
  // ---- carried tails of the runs path (CEP_SESSION_CARRY, runs.hip) ----
  DBuf rtab, rpool, rpool2, rtop, e_key, e_topic, e_part, e_seg, e_off, e_ts, e_pos, rc_a, rc_b, rc_c, rc_d, gc_len, gc_off;
  DBuf e_cols[16];
  int64_t rpool_cap = 0, rpool_used = 0;   // tail records (5 + ncols int64 words each)
  int64_t* h_res = nullptr;                // runs / general paths: the batch's counts, written by the device into
                                           // pinned memory (16 words)
  // ---- CEP_BATCH_ARRIVAL_ORDER (group.hip): the batch grouped by key on the device ----
  DBuf g_key, g_arr, g_pos, g_valid, g_topic, g_part, g_off, g_ts, g_head, g_top, g_nodes, g_start, a_cnt,
      a_ecnt, a_head, a_moff, a_moffe, a_tmp, a_record, a_key, a_entoff, a_name, a_entrec;
  uint32_t group_stamp = 0;                // the groupings so far (epoch of the per-key list heads)
  DBuf g_cols[16];
  const int64_t* cur_pos = nullptr;        // the batch being pushed: stream position per grouped record (else null)
  const int64_t* last_gpos = nullptr;      // ... of the last stencil / chain batch (carry_args)
  bool collected = false;                  // the CSR above is the last batch's: a second collect re-uses it
  cep_matches last{};
  std::vector<uint8_t> evict_buf;          // cep_state_evict's blobs
};

namespace {

// roctx ranges around the C-ABI calls (SURVEY §5 tracing), for rocprofv3 --marker-trace: on with
// KCEP_ROCTX=1, the roctx library loaded at the first call (no link-time dependency, no cost when off)
struct Roctx {
  int (*push)(const char*) = nullptr;
  int (*pop)() = nullptr;
  Roctx() {
    const char* on = getenv("KCEP_ROCTX");
    if (!on || on[0] != '1') return;
    void* h = dlopen("librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("libroctx64.so.4", RTLD_NOW | RTLD_LOCAL);
    if (!h) return;
    push = reinterpret_cast<int (*)(const char*)>(dlsym(h, "roctxRangePushA"));
    pop = reinterpret_cast<int (*)()>(dlsym(h, "roctxRangePop"));
    if (!push || !pop) push = nullptr;
  }
};
const Roctx& roctx() {
  static const Roctx r;
  return r;
}
struct RoctxRange {
  bool on;
  explicit RoctxRange(const char* name) : on(roctx().push != nullptr) { if (on) roctx().push(name); }
  ~RoctxRange() { if (on) roctx().pop(); }
};

// an environment switch for A/B runs ("1" on)
bool getenv_flag(const char* name) {
  const char* v = getenv(name);
  return v && v[0] == '1';
}
// an on-by-default path switched off by NAME=0
bool getenv_flag_off(const char* name) {
  const char* v = getenv(name);
  return v && v[0] == '0' && v[1] == 0;
}

// the halo arguments of the last stencil batch (its stamp and stream position)
StencilCarry carry_args(const cep_session* s) {
  return StencilCarry{s->halo.as<HaloHdr>(), s->hpos.as<int64_t>(), s->pat->prog.stencil.k - 1, s->halo_stamp,
                      int32_t(std::min<int64_t>(s->opts.max_keys, INT32_MAX)), s->halo_base,
                      s->hflags.as<unsigned long long>() + (s->halo_stamp & 1), s->last_gpos};
}

// Host-resident batch columns -> one packed device image (s->dstage), 256-B aligned per column.  The
// caller's memory is borrowed only for the call (kcep.h cep_push_batch):
//  - pageable memory (a JVM heap array, a numpy buffer) is copied into the session's pinned ring in
//    chunks of 2 MB, each chunk moved by one async copy while the next one is filled; the
//    call returns once the last chunk is in the ring;
//  - memory that is itself pinned is copied from directly, and the call waits for that copy (the
//    kernels are already enqueued behind it).
struct HostArr {
  const void* src;
  size_t bytes;
  const void** dst;               // receives the device address (null src: left null)
};
// zero copy only pays for small batches: the kernel then reads the batch over the link itself, which
// for an 8 MB batch (1 M records) cost 706 us per flush against ~280 us by DMA (r04 bench)
constexpr size_t kZeroCopyMax = size_t(1) << 20;

bool host_pinned(const void* p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();      // pageable memory is unknown to the runtime: not an error
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

int stage_host(cep_session* s, HostArr* arrs, int na, hipStream_t st, bool zero_copy = false) {
  size_t total = 0;
  std::vector<size_t> at(size_t(na), 0);
  for (int i = 0; i < na; i++) {
    if (!arrs[i].src || !arrs[i].bytes) continue;
    at[size_t(i)] = total;
    total += (arrs[i].bytes + 255) & ~size_t(255);
  }
  if (!total) return CEP_OK;
  // zero copy (the stencil path's one streaming pass, batches up to kZeroCopyMax): the kernel reads the
  // pinned ring over the link itself, no copy into HBM first.
  // Pinned caller memory takes it too: one host memcpy beats waiting for a DMA before the call may
  // return (r04 flush probe, 64 k records: 55.8 us per flush through the ring, 67-69 us pinned by DMA)
  if (zero_copy && total <= kZeroCopyMax) {
    const int j = s->ring_next;
    s->ring_next ^= 1;
    if (s->ring_ev[j]) HIPCHECK(hipEventSynchronize(s->ring_ev[j]));
    else HIPCHECK(hipEventCreateWithFlags(&s->ring_ev[j], hipEventDisableTiming));
    if (s->ring_cap[j] < total) {
      if (s->ring[j]) HIPCHECK(hipHostFree(s->ring[j]));
      s->ring[j] = nullptr;
      s->ring_cap[j] = 0;
      HIPCHECK(hipHostMalloc(&s->ring[j], std::max(total, size_t(1) << 20), hipHostMallocMapped));
      s->ring_cap[j] = std::max(total, size_t(1) << 20);
    }
    uint8_t* h = static_cast<uint8_t*>(s->ring[j]);
    void* dptr = nullptr;
    HIPCHECK(hipHostGetDevicePointer(&dptr, h, 0));
    for (int i = 0; i < na; i++)
      if (arrs[i].src && arrs[i].bytes) {
        memcpy(h + at[size_t(i)], arrs[i].src, arrs[i].bytes);
        *arrs[i].dst = static_cast<uint8_t*>(dptr) + at[size_t(i)];
      }
    s->zc_slot = j;                                   // its event is recorded behind the kernels that read it
    return CEP_OK;
  }
  bool pinned = true;
  for (int i = 0; i < na && pinned; i++)
    if (arrs[i].src && arrs[i].bytes) pinned = host_pinned(arrs[i].src);
  if (s->dstage.ensure(total)) return fail(CEP_E_HIP, "staging allocation failed");
  uint8_t* dev = s->dstage.as<uint8_t>();
  for (int i = 0; i < na; i++)
    if (arrs[i].src && arrs[i].bytes) *arrs[i].dst = dev + at[size_t(i)];
  if (pinned) {                                       // DMA straight from the caller's pinned memory
    for (int i = 0; i < na; i++)
      if (arrs[i].src && arrs[i].bytes)
        HIPCHECK(hipMemcpyAsync(dev + at[size_t(i)], arrs[i].src, arrs[i].bytes, hipMemcpyHostToDevice, st));
    if (!s->h2d_ev) HIPCHECK(hipEventCreateWithFlags(&s->h2d_ev, hipEventDisableTiming));
    HIPCHECK(hipEventRecord(s->h2d_ev, st));
    s->h2d_wait = true;                               // cep_push_batch waits for it before returning
    return CEP_OK;
  }
  // pageable: through the pinned ring, in chunks so that the copy of one overlaps the filling of the next
  // (2 MB chunks: the copy of chunk i overlaps the filling of chunk i + 1; a smaller batch is one chunk)
  const size_t chunk = std::min(total, size_t(2) << 20);
  for (size_t c0 = 0; c0 < total; c0 += chunk) {
    const size_t c1 = std::min(total, c0 + chunk);
    const int j = s->ring_next;
    s->ring_next ^= 1;
    if (s->ring_ev[j]) HIPCHECK(hipEventSynchronize(s->ring_ev[j]));
    else HIPCHECK(hipEventCreateWithFlags(&s->ring_ev[j], hipEventDisableTiming));
    const size_t want = std::min(total, chunk);
    if (s->ring_cap[j] < want) {
      if (s->ring[j]) HIPCHECK(hipHostFree(s->ring[j]));
      s->ring[j] = nullptr;
      s->ring_cap[j] = 0;
      HIPCHECK(hipHostMalloc(&s->ring[j], want, hipHostMallocMapped));   // (the slot may serve a zero-copy batch later)
      s->ring_cap[j] = want;
    }
    uint8_t* h = static_cast<uint8_t*>(s->ring[j]);
    for (int i = 0; i < na; i++) {                    // the parts of the columns inside [c0, c1)
      if (!arrs[i].src || !arrs[i].bytes) continue;
      const size_t a = std::max(c0, at[size_t(i)]), b = std::min(c1, at[size_t(i)] + arrs[i].bytes);
      if (a < b) memcpy(h + (a - c0), static_cast<const uint8_t*>(arrs[i].src) + (a - at[size_t(i)]), b - a);
    }
    HIPCHECK(hipMemcpyAsync(dev + c0, h, c1 - c0, hipMemcpyHostToDevice, st));
    HIPCHECK(hipEventRecord(s->ring_ev[j], st));
  }
  return CEP_OK;
}

// CEP_BATCH_DELIVER host buffer: {match count, error flags, completion stamp, 0}, host_cap keys (int32,
// padded to 8 bytes), then host_cap x k stream positions
void dl_layout(const cep_session* s, int slot, int64_t*& hdr, int32_t*& hkey, int64_t*& hpos) {
  hdr = static_cast<int64_t*>(s->dl[slot]);
  hkey = reinterpret_cast<int32_t*>(hdr + 4);
  hpos = hdr + 4 + (s->dl_cap + 1) / 2 + 1;
}

int push_stencil(cep_session* s, const cep_batch* b, hipStream_t st) {
  const StencilProgram& SP = s->pat->prog.stencil;
  const void* col = b->n_cols ? b->cols[SP.col] : nullptr;
  const int32_t* key = b->key_id;
  const int32_t* topic = SP.use_topic ? b->topic : nullptr;
  const size_t vs = type_size(SP.coltype);
  if (b->mem == CEP_MEM_HOST && b->n > 0) {
    HostArr arrs[3] = {{key, size_t(b->n) * 4, reinterpret_cast<const void**>(&key)},
                       {col, size_t(b->n) * vs, &col},
                       {topic, size_t(b->n) * 4, reinterpret_cast<const void**>(&topic)}};
    int rc = stage_host(s, arrs, SP.use_topic ? 3 : 2, st, true);
    if (rc) return rc;
  }
  if (SP.use_topic && !topic && b->n > 0) {          // no topic column: every record on topic id 0
    if (s->h_topic.ensure(size_t(b->n) * 4)) return fail(CEP_E_HIP, "staging allocation failed");
    HIPCHECK(hipMemsetAsync(s->h_topic.p, 0, size_t(b->n) * 4, st));
    topic = s->h_topic.as<int32_t>();
  }
  if ((reinterpret_cast<uintptr_t>(key) | reinterpret_cast<uintptr_t>(col) | reinterpret_cast<uintptr_t>(topic)) & 15)
    return fail(CEP_E_ARG, "device columns must be 16-byte aligned");
  s->d_key = key;
  int64_t* tc = s->status.as<int64_t>();
  const int64_t ntiles = stencil_tiles(b->n);
  StencilLaunch L{key, col, topic, b->n, s->prog.as<StencilProgram>(), SP.k, SP.coltype, SP.use_topic, SP.chain,
                  s->slots.as<int32_t>(), tc, tc + ntiles + 1, s->counter.as<int64_t>(), s->out.as<int32_t>(),
                  s->out_cap, s->total.as<int64_t>(), StencilCarry{}, !getenv_flag("KCEP_STENCIL_KEYED"), nullptr};
  if (s->carry) {                                // the keys' halos: read the previous, write the next
    // the batch's error flags: one of two words by the stamp's parity; the other one, cleared by this
    // batch's scan kernel, serves the next batch (no memset launch per batch)
    L.clear_flag = s->hflags.as<unsigned long long>() + (s->halo_stamp & 1);
    L.carry = StencilCarry{s->halo.as<HaloHdr>(), s->hpos.as<int64_t>(), SP.k - 1, ++s->halo_stamp,
                           int32_t(std::min<int64_t>(s->opts.max_keys, INT32_MAX)), s->base,
                           s->hflags.as<unsigned long long>() + (s->halo_stamp & 1), s->cur_pos,
                           s->cur_pos ? 1 : 0};
    s->last_gpos = s->cur_pos;
    s->halo_base = s->base;
    s->base += b->n;
  }
  if (s->carry && (b->flags & CEP_BATCH_DELIVER)) {   // the matches to pinned host memory, by the device
    const int k = SP.k;
    const int64_t host_cap = std::min<int64_t>(s->out_cap, int64_t(1) << 20);
    if (!s->dl[0]) {
      const size_t bytes = 8 * (4 + size_t(host_cap + 1) / 2 + 1) + size_t(host_cap) * size_t(k) * 8;   // see dl_layout
      for (int j = 0; j < 2; j++) {
        HIPCHECK(hipHostMalloc(&s->dl[j], bytes, hipHostMallocMapped | hipHostMallocCoherent));
        memset(s->dl[j], 0, 32);
      }
      s->dl_cap = host_cap;
      if (s->dl_ticket.ensure(16)) return fail(CEP_E_HIP, "allocation failed");
      HIPCHECK(hipMemsetAsync(s->dl_ticket.p, 0, 16, st));
    }
    if (s->out_cap > host_cap &&
        (s->mkey.ensure(size_t(s->out_cap) * 4) || s->opos.ensure(size_t(s->out_cap) * size_t(k) * 8)))
      return fail(CEP_E_HIP, "allocation failed");
    const int slot = int((s->dl_stamp + 1) & 1);   // the next stamp's buffer (the other holds the batch before)
    dl_layout(s, slot, L.deliver.hdr, L.deliver.hkey, L.deliver.hpos);
    s->dl_pid[slot] = s->push_id;
    L.deliver.dkey = s->mkey.as<int32_t>();
    L.deliver.dpos = s->opos.as<int64_t>();
    L.deliver.host_cap = s->dl_cap;
    L.deliver.ticket = s->dl_ticket.as<unsigned>();
    L.deliver.stamp = ++s->dl_stamp;
    if (s->cur_pos && b->n > 0) {                  // arrival order: rows delivered by their completing record's arrival
      if (s->a_moff.ensure(size_t(b->n) * 8) || s->a_tmp.ensure(size_t(b->n / 1024 + 4) * 8) || s->scal.ensure(64))
        return fail(CEP_E_HIP, "allocation failed");
      L.deliver.a_cnt = s->a_cnt.as<int64_t>();
      L.deliver.a_head = s->a_head.as<int32_t>();
      L.deliver.a_moff = s->a_moff.as<int64_t>();
      L.deliver.a_tot = s->scal.as<int64_t>() + 6;
      L.deliver.a_tmp = s->a_tmp.as<int64_t>();
      L.deliver.a_n = b->n;
    }
    s->delivered = true;
  }
  HIPCHECK(stencil_launch(L, s->timing ? s->ev0 : nullptr, s->timing ? s->ev1 : nullptr, st));
  if (s->timing) HIPCHECK(hipEventRecord(s->eb1, st));
  return CEP_OK;
}

int64_t read_i64(const void* dev, hipStream_t st, int* rc) {
  int64_t v = 0;
  if (hipMemcpyAsync(&v, dev, sizeof v, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    *rc = CEP_E_HIP;
  return v;
}

// Carry pool: the live blobs move to a fresh buffer (dropping the blobs that
// later batches superseded); the table is rewritten in place.
int carry_gc(cep_session* s, int64_t min_words, hipStream_t st) {
  const int64_t nk = s->opts.max_keys;
  int rc = CEP_OK;
  if (s->flag.ensure(size_t(nk) * 8) || s->idx.ensure(size_t(nk) * 8) ||
      s->scan_tmp.ensure(size_t(nk / 1024 + 2) * 8) || s->scal.ensure(64))
    return fail(CEP_E_HIP, "allocation failed");
  int64_t* scal = s->scal.as<int64_t>();
  HIPCHECK(carry_sizes_launch(s->ctab.as<int64_t>(), nk, s->cpool.as<int32_t>(), s->flag.as<int64_t>(), st));
  HIPCHECK(exclusive_scan(s->flag.as<int64_t>(), nk, s->idx.as<int64_t>(), scal + 5, s->scan_tmp.as<int64_t>(), st));
  const int64_t live = read_i64(scal + 5, st, &rc);
  if (rc) return fail(rc, "carry size");
  const int64_t cap = std::max<int64_t>({2 * live, min_words, int64_t(1) << 20});
  DBuf fresh;
  if (fresh.ensure(size_t(cap) * 4)) return fail(CEP_E_RUN_CAPACITY, "cannot allocate the carried-state pool");
  HIPCHECK(carry_move_launch(s->ctab.as<int64_t>(), nk, s->cpool.as<int32_t>(), s->idx.as<int64_t>(),
                             fresh.as<int32_t>(), st));
  HIPCHECK(hipStreamSynchronize(st));
  s->cpool.release();
  s->cpool = fresh;
  fresh.p = nullptr;
  s->cpool_words = cap;
  s->cpool_used = live;
  return CEP_OK;
}

// batch columns on the device (host batches staged through the session's buffers)
int stage_inputs(cep_session* s, const cep_batch* b, hipStream_t st, NfaArgs& A) {
  const Program& P = s->pat->prog;
  const int64_t n = b->n;
  A.key = b->key_id; A.valid = b->valid; A.topic = b->topic; A.partition = b->partition;
  A.offset = b->offset; A.ts = b->ts;
  for (int c = 0; c < b->n_cols; c++) A.cols[c] = b->cols[c];
  if (b->mem == CEP_MEM_HOST && n > 0) {
    HostArr arrs[6 + 16] = {{A.key, size_t(n) * 4, reinterpret_cast<const void**>(&A.key)},
                            {A.valid, size_t(n), reinterpret_cast<const void**>(&A.valid)},
                            {A.topic, size_t(n) * 4, reinterpret_cast<const void**>(&A.topic)},
                            {A.partition, size_t(n) * 4, reinterpret_cast<const void**>(&A.partition)},
                            {A.offset, size_t(n) * 8, reinterpret_cast<const void**>(&A.offset)},
                            {A.ts, size_t(n) * 8, reinterpret_cast<const void**>(&A.ts)}};
    for (int c = 0; c < b->n_cols; c++)
      arrs[6 + c] = HostArr{A.cols[c], size_t(n) * type_size(P.coltypes[c]), &A.cols[c]};
    return stage_host(s, arrs, 6 + b->n_cols, st);
  }
  return CEP_OK;
}

// Deterministic strict runs (runs.hip): one lane per start record, completed runs
// ordered by (completing record, start), traversals written into the general CSR.
int tail_rw(const cep_session* s) { return 5 + int(s->pat->prog.coltypes.size()); }
bool tail_session(const cep_session* s) { return s->carry && s->path == CEP_PATH_RUNS; }

// the tail pool with room for `more` records beyond the used ones (compacted / grown when short)
int tail_reserve(cep_session* s, int64_t more, hipStream_t st) {
  if (s->rpool_used + more <= s->rpool_cap) return CEP_OK;
  const int RW = tail_rw(s);
  const int64_t nk = s->opts.max_keys;
  const int64_t cap = std::max<int64_t>(2 * (s->rpool_used + more), int64_t(1) << 16);
  if (s->rpool2.ensure(size_t(cap) * RW * 8) || s->gc_len.ensure(size_t(nk + 1) * 8) || s->gc_off.ensure(size_t(nk + 1) * 8) ||
      s->scan_tmp.ensure(size_t(nk / 1024 + 4) * 8))
    return fail(CEP_E_HIP, "tail pool allocation failed");
  if (s->rpool_used > 0)
    HIPCHECK(runs_carry_gc(s->rtab.as<int64_t>(), nk, RW, s->rpool.as<int64_t>(), s->rpool2.as<int64_t>(),
                           s->gc_len.as<int64_t>(), s->gc_off.as<int64_t>(), s->rtop.as<int64_t>(), s->scan_tmp.as<int64_t>(),
                           st));
  else
    HIPCHECK(hipMemsetAsync(s->rtop.p, 0, 8, st));
  int64_t live = 0;
  HIPCHECK(hipMemcpyAsync(&live, s->rtop.p, 8, hipMemcpyDeviceToHost, st));
  HIPCHECK(hipStreamSynchronize(st));
  std::swap(s->rpool, s->rpool2);
  s->rpool2.release();
  s->rpool_cap = cap;
  s->rpool_used = live;
  return CEP_OK;
}

// Deterministic strict runs (runs.hip): one lane per start record, completed runs
// ordered by (completing record, start), traversals written into the general CSR.
// Carry sessions prefix every key's records with its carried tail (runs.hip) and keep the tails of
// the runs still open at the batch end.
int push_runs(cep_session* s, const cep_batch* b, hipStream_t st) {
  const int64_t nb = b->n;                        // the batch's records
  int64_t n = nb;                                 // records simulated (carry: plus the keys' tails)
  NfaArgs in{};
  int rc = stage_inputs(s, b, st, in);
  if (rc) return rc;
  s->d_key = in.key;
  s->g_err = CEP_OK;
  s->g_err_rec = -1;
  s->e_rec.clear();
  s->e_code.clear();
  s->g_matches = s->g_entries = 0;
  HIPCHECK(hipEventRecord(s->ev0, st));
  if (n == 0) {                                   // cep_device_match_count reads scal[3]: zero it
    if (s->scal.ensure(64)) return fail(CEP_E_HIP, "allocation failed");
    HIPCHECK(hipMemsetAsync(s->scal.as<int64_t>() + 3, 0, 16, st));
    HIPCHECK(hipEventRecord(s->ev1, st));
    HIPCHECK(hipEventRecord(s->eb1, st));
    return CEP_OK;
  }
  const bool rcarry = tail_session(s);
  bool nosync = false;                            // carry: the extended batch's size read after the launches
  RcExt X{};
  const int32_t* bkey = in.key;                   // the batch's own key column (segments index it)
  if (rcarry) {
    const Program& PP = s->pat->prog;
    if (s->flag.ensure(size_t(nb) * 8) || s->idx.ensure(size_t(nb) * 8) || s->seg.ensure(size_t(nb + 1) * 8) ||
        s->scan_tmp.ensure(size_t(nb / 1024 + 4) * 8) || s->rc_a.ensure(size_t(nb + 2) * 8) ||
        s->rc_b.ensure(size_t(nb + 2) * 8) || s->ctl.ensure(64))
      return fail(CEP_E_HIP, "allocation failed");
    int64_t* scal = s->scal.as<int64_t>();
    HIPCHECK(nfa_segments(in.key, nb, s->flag.as<int64_t>(), s->idx.as<int64_t>(), s->seg.as<int64_t>(), scal,
                          s->scan_tmp.as<int64_t>(), st));
    HIPCHECK(hipMemsetAsync(scal + 1, 0, 8, st));
    HIPCHECK(carry_keycheck_launch(nb, scal, in.key, s->seg.as<int64_t>(), int32_t(std::min<int64_t>(s->opts.max_keys, INT32_MAX)),
                                   s->kstamp.as<int32_t>(), ++s->batch_no, reinterpret_cast<unsigned long long*>(scal + 1), st));
    RcIn B{};
    B.pos = s->cur_pos;
    B.key = in.key; B.topic = in.topic; B.partition = in.partition; B.offset = in.offset; B.ts = in.ts;
    for (int c = 0; c < 16; c++) B.cols[c] = in.cols[c];
    const int32_t mk = int32_t(std::min<int64_t>(s->opts.max_keys, INT32_MAX));
    HIPCHECK(runs_carry_build(B, nb, s->base, s->flag.as<int64_t>(), s->idx.as<int64_t>(), s->seg.as<int64_t>(), scal,
                              s->rtab.as<int64_t>(), s->rpool.as<int64_t>(), s->rc_a.as<int64_t>(), s->rc_b.as<int64_t>(),
                              scal + 5, s->scan_tmp.as<int64_t>(), X, st, true, mk));
    // The extended batch's size (the batch plus its keys' carried tails) stays on the device: the launches
    // are sized by a bound -- the batch plus every tail record the pool holds -- and read the count
    // (scal[7]); the key checks are read with the batch's results, and a failing batch leaves the tail
    // pool and table untouched (rc_tail_*).  Unless a forced ordering path or a batch too large for the
    // one-workgroup chunk scan needs the count first.
    const int64_t nmax = nb + s->rpool_used;
    nosync = !getenv_flag("KCEP_RUNS_RADIX") && !getenv_flag_off("KCEP_RUNS_EMIT") && nmax < (int64_t(1) << 31) &&
             (nmax + runs_chunk(nmax) - 1) / runs_chunk(nmax) <= (int64_t(1) << 16);
    if (nosync) {
      n = nmax;
      if ((rc = tail_reserve(s, n, st))) return rc;  // room for the new tails (at most every record)
      HIPCHECK(runs_carry_count(scal + 7, nb, scal + 5, nmax, st));
    } else {
      int64_t h[6];
      HIPCHECK(hipMemcpyAsync(h, scal, sizeof h, hipMemcpyDeviceToHost, st));
      HIPCHECK(hipStreamSynchronize(st));
      if (h[1] & 1) return fail(CEP_E_ARG, "carry sessions need key ids in [0, max_keys)");
      if (h[1] & 2) return fail(CEP_E_ARG, "carry batch is not grouped by key: a key has two segments");
      n = nb + h[5];
      if (n >= (int64_t(1) << 31)) return fail(CEP_E_RUN_CAPACITY, "carried tails make the batch exceed 2^31 records");
    }
    const size_t e4 = size_t(n) * 4, e8 = size_t(n) * 8;
    if (s->e_key.ensure(e4) || s->e_topic.ensure(e4) || s->e_part.ensure(e4) || s->e_seg.ensure(e4) ||
        s->e_off.ensure(e8) || s->e_ts.ensure(e8) || s->e_pos.ensure(e8))
      return fail(CEP_E_HIP, "allocation failed");
    X.key = s->e_key.as<int32_t>(); X.topic = s->e_topic.as<int32_t>(); X.partition = s->e_part.as<int32_t>();
    X.seg = s->e_seg.as<int32_t>(); X.offset = s->e_off.as<int64_t>(); X.ts = s->e_ts.as<int64_t>();
    X.pos = s->e_pos.as<int64_t>();
    X.cap = n;
    X.ncols = int32_t(PP.coltypes.size());
    for (int c = 0; c < X.ncols; c++) {
      X.coltype[c] = PP.coltypes[c];
      if (s->e_cols[c].ensure(size_t(n) * type_size(PP.coltypes[c]))) return fail(CEP_E_HIP, "allocation failed");
      X.cols[c] = s->e_cols[c].p;
    }
    HIPCHECK(runs_carry_build(B, nb, s->base, s->flag.as<int64_t>(), s->idx.as<int64_t>(), s->seg.as<int64_t>(), scal,
                              s->rtab.as<int64_t>(), s->rpool.as<int64_t>(), s->rc_a.as<int64_t>(), s->rc_b.as<int64_t>(),
                              scal + 5, s->scan_tmp.as<int64_t>(), X, st, false, mk));
    in.key = X.key; in.topic = X.topic; in.partition = X.partition; in.offset = X.offset; in.ts = X.ts;
    for (int c = 0; c < X.ncols; c++) in.cols[c] = X.cols[c];
    if (!nosync && (rc = tail_reserve(s, n, st))) return rc;   // room for the new tails (at most every record)
  }
  const int64_t n_grid = n;                       // what the runs_sim grid is sized by
  if (s->rk.ensure(size_t(n) * 8) || s->rk_sorted.ensure(size_t(n) * 8) || s->r_errcode.ensure(size_t(n) * 4) ||
      s->ctl.ensure(64) || s->scal.ensure(64) || s->scan_tmp.ensure(size_t(n / 1024 + 4) * 8) ||
      s->flag.ensure(size_t(6 * runs_sim_waves(n, runs_chunk(n)) + 8) * 8) ||
      s->idx.ensure(size_t(2 * runs_sim_waves(n, runs_chunk(n)) + 8) * 8) || s->r_endof.ensure(size_t(n) * 4) ||
      s->r_segs.ensure(size_t(n) * RUNS_MAX_SEGS * 2) ||
      s->r_errlist.ensure(size_t(std::min<int64_t>(n, kRunsErrCap)) * 24))
    return fail(CEP_E_HIP, "allocation failed");
  RunsArgs A{};
  A.P = s->dprog.as<DevProgram>();
  A.key = in.key; A.topic = in.topic; A.partition = in.partition; A.offset = in.offset; A.ts = in.ts;
  for (int c = 0; c < 16; c++) A.cols[c] = in.cols[c];
  A.n = n;
  A.n_dev = nosync ? s->scal.as<int64_t>() + 7 : nullptr;
  A.base = 0;
  A.pos = rcarry ? X.pos : nullptr;               // carry: stream positions; runs ending in a tail are old
  A.emit_from = s->base;
  A.chunk = runs_chunk(n);
  unsigned long long* ctl = s->ctl.as<unsigned long long>();
  A.nmatch = ctl;
  A.err_min = ctl + 1;
  A.match_key = s->rk.as<unsigned long long>();
  A.match_cap = n;
  A.err_code = s->r_errcode.as<int32_t>();
  A.segs = s->r_segs.as<uint16_t>();             // the runs' consumed stages, for runs_emit / runs_expand
  A.segn = s->pat->prog.dev.nstages - 1 <= 4 ? 4 : RUNS_MAX_SEGS;   // (a run consumes each stage at most once)
  A.seg_over = ctl + 3;
  A.err_list = s->r_errlist.as<unsigned long long>();
  A.err_n = ctl + 5;
  A.err_cap = std::min<int64_t>(n, kRunsErrCap);
  A.max_span = ctl + 4;
  // matches, first exception, entries, segment overflow, longest span, failing runs
  const unsigned long long init[6] = {0, ~0ull, 0, 0, 0, 0};
  HIPCHECK(hipMemcpyAsync(ctl, init, sizeof init, hipMemcpyHostToDevice, st));
  HIPCHECK(runs_sim_launch(A, s->flag.as<int64_t>(), s->r_endof.as<int32_t>(), st,
                           s->jit ? s->jit->runs_sim : nullptr));
  HIPCHECK(hipEventRecord(s->ev1, st));
  int64_t* scal0 = s->scal.as<int64_t>();
  // the completed runs counted by the chunk they end in and scanned (runs_emit's placement), or -- too
  // many chunks for that scan, or the sort forced -- compacted in start order for runs_order / the sort
  // (KCEP_RUNS_EMIT=0 / KCEP_RUNS_RADIX=1: the tests' hooks onto those paths for batches runs_emit takes)
  const bool emit_scan = !getenv_flag("KCEP_RUNS_RADIX") && !getenv_flag_off("KCEP_RUNS_EMIT") &&
                         runs_emit_scan(s->flag.as<int64_t>(), n, A.chunk, s->idx.as<int64_t>(), scal0 + 3,
                                        reinterpret_cast<int64_t*>(ctl + 2), st, A.n_dev);
  if (!emit_scan)                                  // (never with nosync: it was decided on the same bound)
    HIPCHECK(runs_compact_launch(s->flag.as<int64_t>(), s->r_endof.as<int32_t>(), n, A.chunk, s->idx.as<int64_t>(),
                                 s->rk.as<unsigned long long>(), scal0 + 3, reinterpret_cast<int64_t*>(ctl + 2),
                                 s->scan_tmp.as<int64_t>(), st, n_grid));
  if (rcarry) {                                    // the keys' new tails: from their oldest still-open start
    if (s->rc_c.ensure(size_t(nb + 2) * 8) || s->rc_d.ensure(size_t(nb + 2) * 8))
      return fail(CEP_E_HIP, "allocation failed");
    HIPCHECK(runs_carry_tails(X, n, nb, scal0, s->seg.as<int64_t>(), bkey, s->rc_b.as<int64_t>(), s->r_endof.as<int32_t>(),
                              reinterpret_cast<unsigned long long*>(s->rc_a.as<int64_t>()), s->rc_c.as<int64_t>(),
                              s->rc_d.as<int64_t>(), scal0 + 6, s->scan_tmp.as<int64_t>(), s->rtop.as<int64_t>(),
                              s->rpool.as<int64_t>(), s->rtab.as<int64_t>(), st, A.n_dev, scal0 + 1));
  }
  // the batch's one host synchronisation: completed runs, entries, first exception, segment overflow (one
  // small kernel writes them into pinned host memory: no copy commands, which cost ~25 us of gaps)
  if (!s->h_res) HIPCHECK(hipHostMalloc(reinterpret_cast<void**>(&s->h_res), 128, hipHostMallocMapped | hipHostMallocCoherent));
  int64_t* h_res_dev = nullptr;
  HIPCHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&h_res_dev), s->h_res, 0));
  HIPCHECK(runs_results_launch(ctl, scal0 + 3, rcarry ? s->rtop.as<int64_t>() : nullptr, h_res_dev, st,
                               rcarry ? scal0 : nullptr));
  HIPCHECK(hipStreamSynchronize(st));
  if (nosync) {                                    // the key checks and the extended batch's size, now
    if (s->h_res[7] & 1) return fail(CEP_E_ARG, "carry sessions need key ids in [0, max_keys)");
    if (s->h_res[7] & 2) return fail(CEP_E_ARG, "carry batch is not grouped by key: a key has two segments");
    n = nb + s->h_res[8];
    A.n = n;
    A.n_dev = nullptr;
  }
  unsigned long long res[6];
  for (int q = 0; q < 6; q++) res[q] = (unsigned long long)s->h_res[q];
  const int64_t top = s->h_res[6];
  if (rcarry) {
    s->rpool_used = top;
    s->base += nb;
  }
  const int64_t nm = int64_t(res[0]), ne = int64_t(res[2]);
  if (nm > n) return fail(CEP_E_RUN_CAPACITY, "more completed runs than records");
  if (res[1] != ~0ull) {                           // the reference's first exception
    int64_t at = int64_t(res[1] >> 31);
    const int64_t j = int64_t(res[1] & 0x7FFFFFFFull);
    int32_t code = 0;
    HIPCHECK(hipMemcpy(&code, s->r_errcode.as<int32_t>() + j, 4, hipMemcpyDeviceToHost));
    if (code == CEP_E_UNSUPPORTED) return fail(CEP_E_UNSUPPORTED, "sequence condition on the runs path");
    if (rcarry) HIPCHECK(hipMemcpy(&at, X.pos + at, 8, hipMemcpyDeviceToHost));   // its stream position
    s->g_err = code;
    s->g_err_rec = at;
    const int64_t nerr = int64_t(res[5]);
    if (nerr <= A.err_cap) {                       // every failing key's first exception (cep_batch_errors)
      std::vector<unsigned long long> el(size_t(nerr) * 3);
      HIPCHECK(hipMemcpy(el.data(), A.err_list, el.size() * 8, hipMemcpyDeviceToHost));
      std::vector<size_t> ord(static_cast<size_t>(nerr));
      for (size_t q = 0; q < ord.size(); q++) ord[q] = q;
      // per key the smallest (record << 31 | start): its first failure in the reference's order
      std::sort(ord.begin(), ord.end(), [&](size_t x, size_t y) {
        const uint32_t kx = uint32_t(el[3 * x + 2] >> 32), ky = uint32_t(el[3 * y + 2] >> 32);
        return kx != ky ? kx < ky : el[3 * x] < el[3 * y];
      });
      std::vector<std::pair<int64_t, int32_t>> first;
      for (size_t q = 0; q < ord.size(); q++) {
        const size_t x = ord[q];
        if (q > 0 && (el[3 * x + 2] >> 32) == (el[3 * ord[q - 1] + 2] >> 32)) continue;
        first.emplace_back(int64_t(el[3 * x + 1]), int32_t(uint32_t(el[3 * x + 2])));
      }
      std::sort(first.begin(), first.end());
      for (const auto& f : first) {
        s->e_rec.push_back(f.first);
        s->e_code.push_back(f.second);
      }
    } else {                                       // more failing runs than the list holds: the first only
      s->e_rec.push_back(at);
      s->e_code.push_back(code);
    }
  }
  int bits = 1;                                    // bits of the completing record
  while ((int64_t(1) << bits) <= n) bits++;
  size_t tmp_bytes = 0;
  HIPCHECK(runs_sort(nullptr, nullptr, nm, bits, nullptr, &tmp_bytes, st));
  const size_t nmb = size_t(std::max<int64_t>(nm, 1)), neb = size_t(std::max<int64_t>(ne, 1));
  if (s->rk_tmp.ensure(std::max<size_t>(tmp_bytes, 16)) || s->r_len.ensure(nmb * 8) || s->r_entoff.ensure(nmb * 8) ||
      s->scan_tmp.ensure(size_t(nm / 1024 + 4) * 8) || s->o_record.ensure(nmb * 8) || s->o_key.ensure(nmb * 4) ||
      s->o_entoff.ensure(nmb * 8) || s->o_name.ensure(neb * 4) || s->o_entrec.ensure(neb * 8))
    return fail(CEP_E_HIP, "allocation failed");
  int64_t* scal = s->scal.as<int64_t>();
  if (emit_scan && nm > 0 && !res[3] && res[4] < uint64_t(A.chunk)) {
    // every run shorter than a chunk: the CSR in one pass over the end chunks (runs_emit)
    HIPCHECK(runs_emit_launch(A, s->r_endof.as<int32_t>(), s->idx.as<int64_t>(), int(res[4]), s->o_record.as<int64_t>(),
                              s->o_key.as<int32_t>(), s->o_entoff.as<int64_t>(), s->o_name.as<int32_t>(),
                              s->o_entrec.as<int64_t>(), st, n_grid));
    HIPCHECK(hipEventRecord(s->eb1, st));
    s->g_matches = nm;
    s->g_entries = ne;
    return CEP_OK;
  }
  if (emit_scan)                                   // (the start-ordered list the paths below read)
    HIPCHECK(runs_compact_launch(s->flag.as<int64_t>(), s->r_endof.as<int32_t>(), n, A.chunk, s->idx.as<int64_t>(),
                                 s->rk.as<unsigned long long>(), scal0 + 3, reinterpret_cast<int64_t*>(ctl + 2),
                                 s->scan_tmp.as<int64_t>(), st, n_grid));
  // (completing record, start) order: a windowed rank when every run spans <= 1024 records
  // (runs_order), else rocPRIM's radix sort over the completing record's bits
  // the entry offsets are scanned straight into the output's ent_off (runs_expand reads them there);
  // runs_order writes the sorted runs' lengths itself
  if (nm > 0 && res[4] <= 1024 && !getenv_flag("KCEP_RUNS_RADIX")) {
    HIPCHECK(runs_order_launch(s->rk.as<unsigned long long>(), nm, int(res[4]), s->rk_sorted.as<unsigned long long>(),
                               s->r_len.as<int64_t>(), st));
    HIPCHECK(exclusive_scan(s->r_len.as<int64_t>(), nm, s->o_entoff.as<int64_t>(), scal + 4, s->scan_tmp.as<int64_t>(), st));
  } else {
    if (nm > 0)
      HIPCHECK(runs_sort(s->rk.as<unsigned long long>(), s->rk_sorted.as<unsigned long long>(), nm, bits, s->rk_tmp.p,
                         &tmp_bytes, st));
    HIPCHECK(runs_write_launch(A, s->rk_sorted.as<unsigned long long>(), nm, s->r_len.as<int64_t>(),
                               s->o_entoff.as<int64_t>(), scal + 4, s->scan_tmp.as<int64_t>(), nullptr, nullptr,
                               nullptr, nullptr, nullptr, st, true,
                               s->jit ? s->jit->runs_write : nullptr));
  }
  if (!res[3]) {
    // the traversals from the stage segments runs_sim recorded
    HIPCHECK(runs_expand_launch(A, s->rk_sorted.as<unsigned long long>(), nm, s->o_entoff.as<int64_t>(), ne,
                                s->o_record.as<int64_t>(), s->o_key.as<int32_t>(), s->o_entoff.as<int64_t>(),
                                s->o_name.as<int32_t>(), s->o_entrec.as<int64_t>(), st));
  } else {                                         // a run beyond RUNS_MAX_SEGS segments: walk every run again
    A.segs = nullptr;
    HIPCHECK(runs_write_launch(A, s->rk_sorted.as<unsigned long long>(), nm, s->r_len.as<int64_t>(),
                               s->o_entoff.as<int64_t>(), scal + 4, s->scan_tmp.as<int64_t>(), s->o_record.as<int64_t>(),
                               s->o_key.as<int32_t>(), s->o_entoff.as<int64_t>(), s->o_name.as<int32_t>(),
                               s->o_entrec.as<int64_t>(), st, false,
                               s->jit ? s->jit->runs_write : nullptr));
  }
  HIPCHECK(hipEventRecord(s->eb1, st));
  s->g_matches = nm;
  s->g_entries = ne;
  return CEP_OK;
}

int push_general(cep_session* s, const cep_batch* b, hipStream_t st) {
  const Program& P = s->pat->prog;
  const int64_t n = b->n;
  if (s->jit_on && !s->jitg_tried) {           // a stencil / runs session's first batch that needs the NFA
    s->jitg = jit_general(P, s->jit_why, s->opts.flags & CEP_SESSION_PROFILE);
    s->jitg_tried = true;
  }
  NfaArgs A{};
  A.P = s->dprog.as<DevProgram>();
  A.n = n;
  A.mode = s->opts.mode;
  int rc = stage_inputs(s, b, st, A);
  if (rc) return rc;
  s->d_key = A.key;
  s->g_err = CEP_OK;
  s->g_err_rec = -1;
  s->e_rec.clear();
  s->e_code.clear();
  s->g_matches = s->g_entries = 0;
  s->nseg = 0;
  A.base = s->carry ? s->base : 0;
  A.pos = s->cur_pos;
  if (n == 0) {                                   // cep_device_match_count reads scal[3]: zero it
    if (s->scal.ensure(64)) return fail(CEP_E_HIP, "allocation failed");
    HIPCHECK(hipMemsetAsync(s->scal.as<int64_t>() + 3, 0, 16, st));
    HIPCHECK(hipEventRecord(s->ev0, st));
    HIPCHECK(hipEventRecord(s->ev1, st));
    HIPCHECK(hipEventRecord(s->eb1, st));
    return CEP_OK;
  }
  // segments: one per key run of the grouped batch.  A wave-kernel batch of a session that has run one
  // before leaves the count on the device (NfaArgs.nseg_dev, read by the kernel and the scans): no host
  // round trip before the kernel -- per-segment buffers are sized for n segments, the pool estimate is the
  // last batch's (a pool overflow re-runs the batch with a larger one, as always)
  const bool dev_count = s->wave && !s->carry && s->nseg_hint > 0 && n < (int64_t(1) << 31);
  const size_t nb = size_t(n / 1024 + 2) * 16;
  if (s->seg.ensure(size_t(n + 1) * 8) || s->scan_tmp.ensure(nb) || s->scal.ensure(64) || s->ctl.ensure(64))
    return fail(CEP_E_HIP, "allocation failed");
  int64_t* scal = s->scal.as<int64_t>();
  HIPCHECK(nfa_segments(A.key, n, nullptr, nullptr, s->seg.as<int64_t>(), scal, s->scan_tmp.as<int64_t>(), st));
  int64_t nseg = n;                               // (an upper bound until the kernel's results are read)
  if (!dev_count) {
    int64_t segs[2] = {0, 0};                     // segment count, carry key-check flags
    if (s->carry) {
      HIPCHECK(hipMemsetAsync(scal + 1, 0, 8, st));
      HIPCHECK(carry_keycheck_launch(n, scal, A.key, s->seg.as<int64_t>(), int32_t(std::min<int64_t>(s->opts.max_keys, INT32_MAX)),
                                     s->kstamp.as<int32_t>(), ++s->batch_no, reinterpret_cast<unsigned long long*>(scal + 1),
                                     st));
    }
    HIPCHECK(hipMemcpyAsync(segs, scal, sizeof segs, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipStreamSynchronize(st));
    nseg = segs[0];
    if (segs[1] & 1) return fail(CEP_E_ARG, "carry sessions need key ids in [0, max_keys)");
    if (segs[1] & 2) return fail(CEP_E_ARG, "carry batch is not grouped by key: a key has two segments");
    if (nseg >= (int64_t(1) << 31)) return fail(CEP_E_ARG, "too many keys in one batch");
  }
  const int64_t nseg_est = dev_count ? s->nseg_hint : nseg;
  s->nseg = nseg;
  A.nseg = int32_t(nseg);
  A.nseg_dev = dev_count ? scal : nullptr;
  A.seg_start = s->seg.as<int64_t>();
  const DevProgram& D = P.dev;
  NfaCaps cap = kCaps;
  const double scale = s->opts.arena_scale > 0 ? s->opts.arena_scale : 1.0;
  cap.heap_mult = std::max<int32_t>(1, int32_t(cap.heap_mult * scale));
  cap.out_mult = std::max<int32_t>(1, int32_t(cap.out_mult * scale));
  const size_t sb = size_t(nseg) * 8;
  if (s->r_matches.ensure(sb) || s->r_words.ensure(sb) || s->r_out.ensure(sb) || s->r_ent.ensure(sb) || s->r_err.ensure(sb) ||
      s->r_errrec.ensure(sb) || s->r_carry.ensure(sb) || s->moff.ensure(sb) || s->eoff.ensure(sb))
    return fail(CEP_E_HIP, "allocation failed");
  // first-allocation words of every key (NfaCaps) plus the events carried into the batch
  const int64_t per_key = 48 + 16 * cap.q0 + 3 * D.nstates * (cap.seq_base + 1) + cap.heap_base + cap.out_base + 16;
  const int64_t per_ev = 4 * D.nslots + cap.heap_mult + cap.out_mult + 4 + 3 * D.nstates;
  int64_t est = nseg_est * per_key + (n + (s->carry ? s->cpool_used / 4 : 0)) * per_ev;
  s->pool_est = std::max<int64_t>(s->pool_est, est + est / 2 + (int64_t(1) << 20));
  // a workload that needed a regrown pool starts from that size (no re-run per batch), until kPoolQuiet
  // batches in a row fit the estimate again
  s->pool_words = std::max(s->pool_est, s->pool_learned);
  A.cap = cap;
  A.carry = s->carry ? 1 : 0;
  A.max_keys = int32_t(std::min<int64_t>(s->opts.max_keys, INT32_MAX));
  A.res_matches = s->r_matches.as<int64_t>();
  A.res_words = s->r_words.as<int64_t>();
  A.res_out = s->r_out.as<int64_t>();
  A.res_ent = s->r_ent.as<int64_t>();
  A.res_err = s->r_err.as<int32_t>();
  A.res_err_rec = s->r_errrec.as<int64_t>();
  A.res_carry = s->r_carry.as<int64_t>();
  unsigned long long* ctl = s->ctl.as<unsigned long long>();
  A.pool_top = ctl;
  A.cpool_top = ctl + 1;
  A.flags = reinterpret_cast<int32_t*>(ctl + 2);
  A.err_any = ctl + 4;
  // lane kernel: 64 key segments per wave (fewer diverge less but leave the chip emptier: C4 gained 5 %
  // at 8 per wave, light keys lost 2x, profiles/r01_s5_nfa_spread_*.log)
  A.wave_agg = (wave_stateful(D) ? 1 : 0) | (P.has_seq ? 2 : 0);
  A.spread = 64;
  if (s->opts.flags & CEP_SESSION_PROFILE) {
    if (s->r_prof.ensure(sb * NFA_PROFILE_W)) return fail(CEP_E_HIP, "allocation failed");
    A.profile = s->r_prof.as<int64_t>();
  }
  // the wave kernel's persistent grid and its workgroups' scratch regions (nfa_wave.h): 16 K words
  // each by default (KCEP_WAVE_SCRATCH words, 0: none -- every workspace from the pool)
  int64_t wgrid = 0;
  if (s->wave) {
    const char* scr_env = getenv("KCEP_WAVE_SCRATCH");
    const int64_t scr_words = scr_env ? std::max<int64_t>(0, atoll(scr_env)) & ~int64_t(3) : int64_t(1) << 14;
    wgrid = nfa_wave_grid(nseg, A.wave_agg != 0, s->jitg.get());
    A.scratch_words = scr_words;
    if (scr_words > 0) {
      if (s->wscratch.ensure(size_t(wgrid * scr_words) * 4)) return fail(CEP_E_HIP, "allocation failed");
      A.scratch = s->wscratch.as<int32_t>();
    }
  }
  // the wave kernel's schedule: segments by estimated cost, heaviest first (nfa_dev.h stage_may_take;
  // KCEP_NFA_ORDER=0: as they come, the tests' hook onto that order)
  if (s->wave && !getenv_flag_off("KCEP_NFA_ORDER")) {
    // ord_bucket: a byte per segment, then a byte per record (the per-record estimate bits)
    // ord_cnt: 16 bucket sizes per 256 segments
    if (s->ord.ensure(size_t(nseg) * 4) || s->ord_bucket.ensure(size_t(nseg) + size_t(n)) ||
        s->ord_cnt.ensure(size_t((nseg + 255) / 256) * 64))
      return fail(CEP_E_HIP, "allocation failed");
    A.seg_bucket = s->ord_bucket.as<uint8_t>();
    HIPCHECK(nfa_order_launch(A, nseg, s->ord_bucket.as<uint8_t>() + nseg, s->ord_cnt.as<unsigned>(), s->ord.as<int32_t>(),
                              st, s->jitg.get(), NFA_ORDER_LO));
    A.seg_order = s->ord.as<int32_t>();
  }
  bool timed = false;
  bool grew = false;                               // the pool was regrown for this batch: given back after it
  bool pool_at_limit = false;                      // the pool cannot grow further: overflowing keys are handed back
  int64_t tots[2] = {0, 0};                        // matches, entries of the batch
  // the CSR's arrays as the earlier batches left them: a first attempt that fits them is compacted
  // before the host reads its totals (one synchronisation per batch instead of two)
  const int64_t cap_m = int64_t(std::min({s->o_record.cap / 8, s->o_key.cap / 4, s->o_entoff.cap / 8}));
  const int64_t cap_e = int64_t(std::min(s->o_name.cap / 4, s->o_entrec.cap / 8));
  bool spec = false;                               // the first attempt's compaction is enqueued
  int attempts = 0;
  for (int attempt = 0;; attempt++) {
    attempts = attempt + 1;
    if (s->pool.ensure(size_t(s->pool_words) * 4)) {
      if (s->pool_words <= s->pool_est) return fail(CEP_E_RUN_CAPACITY, "cannot allocate the NFA pool");
      (void)hipGetLastError();                     // the learned size no longer fits: back to the estimate
      s->pool_learned = 0;
      s->pool_words = s->pool_est;
      if (s->pool.ensure(size_t(s->pool_words) * 4)) return fail(CEP_E_RUN_CAPACITY, "cannot allocate the NFA pool");
    }
    if (s->carry && s->cpool_used + nseg * 64 > s->cpool_words) {
      if ((rc = carry_gc(s, 2 * (s->cpool_used + nseg * 64), st))) return rc;
    }
    A.pool = s->pool.as<int32_t>();
    A.pool_cap = s->pool_words;
    A.ctab = s->carry ? s->ctab.as<int64_t>() : nullptr;
    A.cpool = s->carry ? s->cpool.as<int32_t>() : nullptr;
    A.cpool_cap = s->carry ? s->cpool_words : 0;
    A.last_attempt = attempt >= kMaxRetry || pool_at_limit ? 1 : 0;   // then an overflowing key is handed back per key
    A.max_key_words = s->opts.max_key_words;
    // ctl: pool top, carry-pool top, flags (2 words), err_any, next segment (a kernel, not a copy command)
    HIPCHECK(set_words_launch(reinterpret_cast<int64_t*>(ctl), 6, 1, s->cpool_used, st));
    if (!timed) HIPCHECK(hipEventRecord(s->ev0, st));
    A.seg_next = reinterpret_cast<int32_t*>(ctl + 5);
    if (s->wave) HIPCHECK(nfa_wave_launch(A, wgrid, st, s->jitg.get()));
    else HIPCHECK(nfa_launch(A, st, s->jitg ? s->jitg->nfa : nullptr));
    if (!timed) HIPCHECK(hipEventRecord(s->ev1, st));
    timed = true;
    // the CSR's match / entry counts are scanned right away, so that one synchronisation reads them
    // with the pool flags (a retried attempt scans again)
    HIPCHECK(exclusive_scan_pair(s->r_matches.as<int64_t>(), s->r_words.as<int64_t>(), nseg, A.nseg_dev,
                                 s->moff.as<int64_t>(), s->eoff.as<int64_t>(), scal + 3, scal + 4,
                                 s->scan_tmp.as<int64_t>(), st));
    if (attempt == 0 && cap_m > 0 && cap_e > 0) {
      HIPCHECK(nfa_compact_launch(nseg, A.nseg_dev, cap_m, cap_e, scal + 3, A.key, A.seg_start, s->r_out.as<int64_t>(),
                                  s->r_ent.as<int64_t>(), s->moff.as<int64_t>(), s->eoff.as<int64_t>(),
                                  s->o_record.as<int64_t>(), s->o_key.as<int32_t>(), s->o_entoff.as<int64_t>(),
                                  s->o_name.as<int32_t>(), s->o_entrec.as<int64_t>(), st));
      spec = true;
    }
    // the flags and counts into pinned host memory by one small kernel (two copy commands cost ~25 us
    // of gaps), then the batch's one synchronisation
    if (!s->h_res) HIPCHECK(hipHostMalloc(reinterpret_cast<void**>(&s->h_res), 128, hipHostMallocMapped | hipHostMallocCoherent));
    int64_t* h_res_dev = nullptr;
    HIPCHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&h_res_dev), s->h_res, 0));
    HIPCHECK(gather_words_launch(reinterpret_cast<const int64_t*>(ctl), 5, scal, 5, h_res_dev, st));
    HIPCHECK(hipStreamSynchronize(st));
    unsigned long long res[5];
    int64_t sc[5];                                 // [0] segments, [3] matches, [4] entries
    for (int q = 0; q < 5; q++) {
      res[q] = (unsigned long long)s->h_res[q];
      sc[q] = s->h_res[5 + q];
    }
    tots[0] = sc[3];
    tots[1] = sc[4];
    if (dev_count && attempt == 0) {               // the exact count from here on
      nseg = sc[0];
      s->nseg = nseg;
      A.nseg = int32_t(nseg);
    }
    s->g_any_err = res[4] != 0;
    const int32_t* fl = reinterpret_cast<const int32_t*>(res + 2);
    if (fl[2]) return fail(CEP_E_ARG, "carry sessions need key ids in [0, max_keys)");
    s->live_hwm = fl[3];
    if (!fl[0] && !fl[1]) {
      if (s->carry) s->cpool_used = int64_t(res[1]);
      break;
    }
    if ((attempt >= kMaxRetry || pool_at_limit) && fl[0])
      return fail(CEP_E_RUN_CAPACITY, "the NFA workspace pool cannot grow");
    if (attempt >= kMaxRetry && fl[1]) return fail(CEP_E_RUN_CAPACITY, "the carried-state pool cannot grow");
    if (fl[0]) {                                   // workspace pool exhausted: twice the pool, same inputs,
      s->pool.release();                           // within the session's budget (cep_opts.max_pool_bytes,
      size_t free_b = 0, total_b = 0;              // default a quarter of the HBM) and the free HBM (keeping
      HIPCHECK(hipMemGetInfo(&free_b, &total_b));  // 1/16 of it): past that a key is handed back per key
      // (the wave kernel's scratch regions count against the budget too)
      const int64_t budget = ((s->opts.max_pool_bytes > 0 ? s->opts.max_pool_bytes : int64_t(total_b / 4)) -
                              int64_t(s->wscratch.cap)) / 4;
      const int64_t room = std::min<int64_t>(int64_t(free_b / 4) - int64_t(free_b / 64), budget);
      const int64_t want = std::min<int64_t>(s->pool_words * 2, room);
      if (want <= s->pool_words) pool_at_limit = true;
      else s->pool_words = want;
      grew = true;
    }
    if (fl[1]) {                                   // carry pool exhausted: compact into a larger one
      if ((rc = carry_gc(s, 2 * s->cpool_words, st))) return rc;
    }
  }
  // compaction into the CSR (counts scanned with the last attempt)
  s->nseg_hint = nseg;
  s->last_attempts = attempts;
  const int64_t pool_used = s->h_res[0];           // the successful attempt's pool top
  s->g_matches = tots[0];
  s->g_entries = tots[1];
  if (!(spec && attempts == 1 && tots[0] <= cap_m && tots[1] <= cap_e)) {
    // (arrays grown with a quarter of headroom, so that the next batches compact speculatively)
    const size_t nm = size_t(std::max<int64_t>(tots[0], 1)), ne = size_t(std::max<int64_t>(tots[1], 1));
    const size_t hm = nm + nm / 4 + 256, he = ne + ne / 4 + 256;
    if ((s->o_record.cap < nm * 8 && s->o_record.ensure(hm * 8)) || (s->o_key.cap < nm * 4 && s->o_key.ensure(hm * 4)) ||
        (s->o_entoff.cap < nm * 8 && s->o_entoff.ensure(hm * 8)) || (s->o_name.cap < ne * 4 && s->o_name.ensure(he * 4)) ||
        (s->o_entrec.cap < ne * 8 && s->o_entrec.ensure(he * 8)))
      return fail(CEP_E_HIP, "allocation failed");
    HIPCHECK(nfa_compact_launch(nseg, nullptr, tots[0], tots[1], nullptr, A.key, A.seg_start, s->r_out.as<int64_t>(),
                                s->r_ent.as<int64_t>(), s->moff.as<int64_t>(), s->eoff.as<int64_t>(),
                                s->o_record.as<int64_t>(), s->o_key.as<int32_t>(), s->o_entoff.as<int64_t>(),
                                s->o_name.as<int32_t>(), s->o_entrec.as<int64_t>(), st));
  }
  if (s->carry) {                                  // NFAStore.put of every key of the batch
    HIPCHECK(carry_commit_launch(nseg, A.key, A.seg_start, s->r_carry.as<int64_t>(), s->r_err.as<int32_t>(),
                                 s->ctab.as<int64_t>(), st));
    s->base += n;
  }
  HIPCHECK(hipEventRecord(s->eb1, st));
  if (grew) {                                      // the next batches start from the grown size
    s->pool_learned = s->pool_words;
    s->pool_quiet = 0;
  } else if (s->pool_learned > 0) {
    s->pool_quiet = pool_used > s->pool_est ? 0 : s->pool_quiet + 1;
    if (s->pool_quiet >= kPoolQuiet) {
      // kPoolQuiet batches in a row within the estimate: the grown pool is given back, so one heavy stretch
      // does not hold the device for the session's lifetime (the compaction has read the matches out of it)
      HIPCHECK(hipStreamSynchronize(st));
      s->pool.release();
      s->wscratch.release();
      s->pool_learned = 0;
      s->pool_quiet = 0;
    }
  }
  // the reference fails the task at its first exception: report the earliest failing record
  if (!s->g_any_err) {                             // no key raised: nothing to read back
    if (s->carry && s->cpool_used > s->cpool_words / 4 * 3) {
      if ((rc = carry_gc(s, 0, st))) return rc;
    }
    return CEP_OK;
  }
  std::vector<int32_t> err(static_cast<size_t>(nseg));
  std::vector<int64_t> erec(static_cast<size_t>(nseg));
  HIPCHECK(hipMemcpyAsync(err.data(), s->r_err.p, size_t(nseg) * 4, hipMemcpyDeviceToHost, st));
  HIPCHECK(hipMemcpyAsync(erec.data(), s->r_errrec.p, size_t(nseg) * 8, hipMemcpyDeviceToHost, st));
  HIPCHECK(hipStreamSynchronize(st));
  for (int64_t i = 0; i < nseg; i++)
    if (err[size_t(i)]) {
      if (s->g_err_rec < 0 || erec[size_t(i)] < s->g_err_rec) {
        s->g_err = err[size_t(i)];
        s->g_err_rec = erec[size_t(i)];
      }
      s->e_rec.push_back(erec[size_t(i)]);         // segments are in stream order, so e_rec ascends
      s->e_code.push_back(err[size_t(i)]);
    }
  if (s->carry && s->cpool_used > s->cpool_words / 4 * 3) {   // keep room for the next batch
    if ((rc = carry_gc(s, 0, st))) return rc;
  }
  return CEP_OK;
}

}  // namespace

extern "C" {

const char* cep_last_error(void) { return g_err.c_str(); }
const char* cep_version(void) { return "kcep 0.1 (gfx950) build " KCEP_BUILD_ID; }

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
  o->runs_ok = P.runs_ok ? 1 : 0;
  return CEP_OK;
}

const char* cep_pattern_name(const cep_pattern* p, int32_t id) {
  if (!p || id < 0 || id >= int32_t(p->prog.names.size())) return nullptr;
  return p->prog.names[id].c_str();
}

int cep_pattern_check(const cep_pattern* p, int32_t session_flags) {
  if (!p) return fail(CEP_E_ARG, "null argument");
  const Program& P = p->prog;
  // a carry session keeps its keys' full NFA state on the general path whenever a batch needs it
  if ((session_flags & CEP_SESSION_CARRY) && !P.general_ok)
    return fail(CEP_E_UNSUPPORTED, "pattern cannot be lowered to the device NFA: " + P.general_why);
  if (!P.stencil_ok && !P.runs_ok && !P.general_ok)
    return fail(CEP_E_UNSUPPORTED, "no device path: " + P.general_why);
  return CEP_OK;
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
  if (path == 0) path = P.stencil_ok ? fast : P.runs_ok ? CEP_PATH_RUNS : CEP_PATH_GENERAL;
  if (path == CEP_PATH_RUNS && !P.runs_ok) return fail(CEP_E_UNSUPPORTED, "runs path does not apply: " + P.runs_why);
  if ((path == CEP_PATH_STENCIL || path == CEP_PATH_CHAIN) && !P.stencil_ok)
    return fail(CEP_E_UNSUPPORTED, "stencil path does not apply: " + P.stencil_why);
  if (path == CEP_PATH_STENCIL || path == CEP_PATH_CHAIN) path = fast;
  if (path == CEP_PATH_GENERAL && !P.general_ok)
    return fail(CEP_E_UNSUPPORTED, "pattern cannot be lowered to the device NFA: " + P.general_why);
  if (path != CEP_PATH_STENCIL && path != CEP_PATH_CHAIN && path != CEP_PATH_GENERAL && path != CEP_PATH_RUNS)
    return fail(CEP_E_ARG, "bad path");
  const bool carry = opts->flags & CEP_SESSION_CARRY;
  if (carry && (opts->max_keys <= 0 || opts->max_keys > INT32_MAX))
    return fail(CEP_E_ARG, "carry sessions need max_keys (dense key ids in [0, max_keys))");
  if (carry && !P.general_ok)
    return fail(CEP_E_UNSUPPORTED, "pattern cannot be lowered to the device NFA: " + P.general_why);
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
    const int64_t nt = stencil_tiles(cap);
    // a run ends at most once, so a batch has at most one match per start: its records, plus on chain
    // carry sessions the (at most K-1) starts in each batch key's halo
    const int64_t out_cap = carry && P.stencil.chain ? cap + std::min<int64_t>(cap, opts->max_keys) * (k - 1) : cap;
    if (s->prog.ensure(sizeof(StencilProgram)) || s->status.ensure(sizeof(int64_t) * size_t(2 * nt + 2)) ||
        s->counter.ensure(sizeof(int64_t) * size_t(nt / 1024 + 4)) || s->total.ensure(64) || s->sum.ensure(64) ||
        s->out.ensure(sizeof(int32_t) * size_t(k) * size_t(out_cap)) ||
        // (+ one super-tile of ints: a last, partial super-tile's aux bytes lie past its tiles' ints;
        // + the plain kernel's dense region, ST_DENSE ints per super-tile)
        s->slots.ensure(sizeof(int32_t) * ((size_t(k) * size_t(nt) + 4) * 4096 +
                                           size_t(nt) * std::max<size_t>(ST_DENSE, ST_DENSE_KEYED * 5 / 4))))
      return cleanup(fail(CEP_E_HIP, "device allocation failed"));
    s->out_cap = out_cap;
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
  if (carry && (path == CEP_PATH_STENCIL || path == CEP_PATH_CHAIN)) {   // per key two halo slots, none written yet
    s->carry = true;
    if (s->halo.ensure(size_t(opts->max_keys) * sizeof(HaloHdr)) || s->hflags.ensure(16) ||
        s->hpos.ensure(size_t(opts->max_keys) * 2 * size_t(std::max(1, P.stencil.k - 1)) * 8) ||
        hipMemset(s->halo.p, 0, size_t(opts->max_keys) * sizeof(HaloHdr)) || hipMemset(s->hflags.p, 0, 16))
      return cleanup(fail(CEP_E_HIP, "device allocation failed"));
  } else if (carry && path == CEP_PATH_RUNS) {    // per key a carried tail, none yet (runs.hip)
    s->carry = true;
    if (s->rtab.ensure(size_t(opts->max_keys) * 16) || s->rtop.ensure(8) || s->kstamp.ensure(size_t(opts->max_keys) * 4) ||
        hipMemset(s->rtab.p, 0, size_t(opts->max_keys) * 16) || hipMemset(s->rtop.p, 0, 8) ||
        hipMemset(s->kstamp.p, 0, size_t(opts->max_keys) * 4))
      return cleanup(fail(CEP_E_HIP, "device allocation failed"));
    if (tail_reserve(s, std::min<int64_t>(cap, int64_t(1) << 20), nullptr)) return cleanup(CEP_E_HIP);
  } else if (carry) {                            // NFAStore: no key has state yet
    s->carry = true;
    s->cpool_words = std::max<int64_t>(int64_t(1) << 20, opts->max_keys * 64);
    if (s->ctab.ensure(size_t(opts->max_keys) * 8) || s->cpool.ensure(size_t(s->cpool_words) * 4) ||
        hipMemset(s->ctab.p, 0xFF, size_t(opts->max_keys) * 8) || s->kstamp.ensure(size_t(opts->max_keys) * 4) ||
        hipMemset(s->kstamp.p, 0, size_t(opts->max_keys) * 4))
      return cleanup(fail(CEP_E_HIP, "device allocation failed"));
  }
  if (hipEventCreate(&s->ev0) || hipEventCreate(&s->ev1) || hipEventCreate(&s->eb0) || hipEventCreate(&s->eb1))
    return cleanup(fail(CEP_E_HIP, "event create failed"));
  // general path kernel: one key per wave (nfa_wave.h) where a key's live runs can multiply -- a stage
  // with an IGNORE edge (skip-till-next / skip-till-any, the C4 run explosion) -- else one key per
  // lane: keys of strict patterns hold a few runs, and a wave round costs a light key more than a
  // lane's walk (C3 on the general path: 342 vs 107 ms, profiles/r03_ab_c3_general_wave_lane.log).
  // CEP_SESSION_LANE_NFA / CEP_SESSION_WAVE_NFA choose explicitly.
  bool grows = false;
  for (const auto& st : P.stages)
    for (const auto& e : st.edges) grows = grows || e.op == E_IGNORE;
  bool wave = grows;
  if (opts->flags & CEP_SESSION_LANE_NFA) wave = false;
  else if (opts->flags & CEP_SESSION_WAVE_NFA) wave = true;
  s->wave = P.general_ok && wave;
  const char* env_jit = getenv("KCEP_JIT");
  s->jit_on = !(opts->flags & CEP_SESSION_INTERPRET) && !(env_jit && !strcmp(env_jit, "0"));
  if (s->jit_on && path == CEP_PATH_RUNS) s->jit = jit_runs(P, s->jit_why);   // on failure: built-in kernels
  if (s->jit_on && path == CEP_PATH_GENERAL) {
    s->jitg = jit_general(P, s->jit_why, s->opts.flags & CEP_SESSION_PROFILE);
    s->jitg_tried = true;
  }
  *out = s;
  return CEP_OK;
}

void cep_session_close(cep_session* s) {
  if (!s) return;
  for (DBuf* b : {&s->g_key, &s->g_arr, &s->g_pos, &s->g_valid, &s->g_topic, &s->g_part, &s->g_off, &s->g_ts, &s->g_head,
                  &s->g_top, &s->g_nodes, &s->g_start, &s->a_cnt, &s->a_ecnt, &s->a_head, &s->a_moff,
                  &s->a_moffe, &s->a_tmp, &s->a_record, &s->a_key, &s->a_entoff, &s->a_name, &s->a_entrec})
    b->release();
  for (auto& c : s->g_cols) c.release();
  for (DBuf* b : {&s->prog, &s->out, &s->status, &s->counter, &s->total, &s->sum, &s->mkey, &s->slots, &s->wscratch, &s->dstage, &s->dl_ticket,
                  &s->h_topic, &s->dprog, &s->flag, &s->idx, &s->seg, &s->scan_tmp,
                  &s->scal, &s->ctl, &s->pool, &s->r_matches, &s->r_words, &s->r_out, &s->r_err, &s->r_errrec,
                  &s->r_carry, &s->r_ent, &s->ord, &s->ord_bucket, &s->ord_cnt, &s->moff, &s->eoff, &s->o_record, &s->o_key, &s->o_entoff, &s->o_name,
                  &s->o_entrec, &s->ctab, &s->cpool, &s->kstamp, &s->halo, &s->hpos, &s->hflags, &s->opos, &s->rk, &s->rk_sorted, &s->rk_tmp, &s->r_segs, &s->r_blk, &s->r_len, &s->r_entoff,
                  &s->r_errcode, &s->r_errlist, &s->r_endof, &s->r_prof, &s->rtab, &s->rpool, &s->rpool2, &s->rtop, &s->e_key,
                  &s->e_topic, &s->e_part, &s->e_seg, &s->e_off, &s->e_ts, &s->e_pos, &s->rc_a, &s->rc_b, &s->rc_c,
                  &s->rc_d, &s->gc_len, &s->gc_off})
    b->release();
  for (auto& c : s->e_cols) c.release();
  for (int j = 0; j < 2; j++) {
    if (s->ring_ev[j]) (void)hipEventSynchronize(s->ring_ev[j]);
    if (s->ring_ev[j]) (void)hipEventDestroy(s->ring_ev[j]);
    if (s->ring[j]) (void)hipHostFree(s->ring[j]);
  }
  if (s->h2d_ev) (void)hipEventDestroy(s->h2d_ev);
  if (s->h_res) (void)hipHostFree(s->h_res);
  if (s->dl[0] || s->dl[1]) (void)hipDeviceSynchronize();   // a delivery may still be writing into them
  for (int j = 0; j < 2; j++)
    if (s->dl[j]) (void)hipHostFree(s->dl[j]);
  if (s->ev0) (void)hipEventDestroy(s->ev0);
  if (s->ev1) (void)hipEventDestroy(s->ev1);
  if (s->eb0) (void)hipEventDestroy(s->eb0);
  if (s->eb1) (void)hipEventDestroy(s->eb1);
  delete s;
}

int cep_session_path(const cep_session* s) { return s ? s->path : 0; }

int cep_live_run_hwm(const cep_session* s, int64_t* hwm) {
  if (!s || !hwm) return fail(CEP_E_ARG, "null argument");
  *hwm = s->last_path == CEP_PATH_GENERAL ? s->live_hwm : -1;
  return CEP_OK;
}

int cep_batch_errors(const cep_session* s, int64_t* records, int32_t* codes, int64_t cap, int64_t* n) {
  if (!s || !n) return fail(CEP_E_ARG, "null argument");
  *n = int64_t(s->e_rec.size());
  if (!records && !codes) return CEP_OK;
  if (cap < *n) return fail(CEP_E_ARG, "capacity below the error count");
  for (size_t i = 0; i < s->e_rec.size(); i++) {
    if (records) records[i] = s->e_rec[i];
    if (codes) codes[i] = s->e_code[i];
  }
  return CEP_OK;
}

int cep_key_profile(cep_session* s, int64_t* out, int64_t cap, int64_t* n_keys) {
  if (!s || !n_keys) return fail(CEP_E_ARG, "null argument");
  if (!(s->opts.flags & CEP_SESSION_PROFILE) || s->last_path != CEP_PATH_GENERAL)
    return fail(CEP_E_UNSUPPORTED, "key profiles need CEP_SESSION_PROFILE and a general-path batch");
  *n_keys = s->nseg;
  if (!out) return CEP_OK;
  constexpr int W = 1 + NFA_PROFILE_W;
  if (cap < W * s->nseg) return fail(CEP_E_ARG, "buffer too small");
  std::vector<int64_t> p(size_t(NFA_PROFILE_W * s->nseg)), start(size_t(s->nseg));
  std::vector<int32_t> keys(size_t(std::max<int64_t>(s->n, 1)));
  HIPCHECK(hipMemcpy(p.data(), s->r_prof.p, p.size() * 8, hipMemcpyDeviceToHost));
  HIPCHECK(hipMemcpy(start.data(), s->seg.p, start.size() * 8, hipMemcpyDeviceToHost));
  if (s->n > 0) HIPCHECK(hipMemcpy(keys.data(), s->d_key, size_t(s->n) * 4, hipMemcpyDeviceToHost));
  for (int64_t i = 0; i < s->nseg; i++) {
    out[W * i] = keys[size_t(start[size_t(i)])];
    for (int j = 0; j < NFA_PROFILE_W; j++) out[W * i + 1 + j] = p[size_t(NFA_PROFILE_W * i + j)];
  }
  return CEP_OK;
}

int cep_session_jit(const cep_session* s) {
  if (!s) return 0;
  return (s->path == CEP_PATH_RUNS && s->jit) || (s->path == CEP_PATH_GENERAL && s->jitg) ? 1 : 0;
}

int cep_session_wave(const cep_session* s) { return s && s->path == CEP_PATH_GENERAL && s->wave ? 1 : 0; }

int cep_batch_attempts(const cep_session* s) { return s && s->last_path == CEP_PATH_GENERAL ? s->last_attempts : 0; }

int cep_pattern_kernel_source(const cep_pattern* p, int path, char* buf, size_t cap, size_t* needed) {
  if (!p || !needed) return fail(CEP_E_ARG, "null argument");
  const bool runs = path == CEP_PATH_RUNS && p->prog.runs_ok, general = path == CEP_PATH_GENERAL && p->prog.general_ok;
  if (!runs && !general) return fail(CEP_E_UNSUPPORTED, "no compiled kernels for this path");
  std::string why;
  const std::string src = runs ? jit_source_runs(p->prog, why) : jit_source_general(p->prog, why);
  if (src.empty()) return fail(CEP_E_UNSUPPORTED, "kernel generation failed: " + why);
  *needed = src.size() + 1;
  if (!buf) return CEP_OK;
  if (cap < *needed) return fail(CEP_E_ARG, "buffer too small");
  memcpy(buf, src.c_str(), src.size() + 1);
  return CEP_OK;
}

int cep_pattern_build_kernels(const cep_pattern* p, int path) {
  if (!p) return fail(CEP_E_ARG, "null argument");
  const bool runs = path == CEP_PATH_RUNS && p->prog.runs_ok, general = path == CEP_PATH_GENERAL && p->prog.general_ok;
  if (!runs && !general) return fail(CEP_E_UNSUPPORTED, "no compiled kernels for this path");
  std::string why;
  if (!(runs ? jit_check_runs(p->prog, why) : jit_check_general(p->prog, why)))
    return fail(CEP_E_UNSUPPORTED, "kernel build failed: " + why);
  return CEP_OK;
}

static int push_dispatch(cep_session* s, const cep_batch* b, hipStream_t st, bool stencil_batch);

// CEP_BATCH_ARRIVAL_ORDER: the batch (records in arrival order, host or device) grouped by key on the device
// (group.hip) into the session's grouped columns; gb describes them (device memory, flags without
// CEP_BATCH_ARRIVAL_ORDER, CEP_BATCH_DELIVER added for the stencil / chain paths, whose rows the delivery
// then writes in arrival order); s->cur_pos = every grouped record's stream position (base + arrival index)
static int group_batch(cep_session* s, const cep_batch* b, hipStream_t st, cep_batch& gb, const void** gcols) {
  const Program& P = s->pat->prog;
  const int64_t n = b->n;
  NfaArgs in{};                                    // the batch's columns on the device (host ones staged)
  in.key = b->key_id; in.valid = b->valid; in.topic = b->topic; in.partition = b->partition;
  in.offset = b->offset; in.ts = b->ts;
  for (int c = 0; c < b->n_cols; c++) in.cols[c] = b->cols[c];
  if (b->mem == CEP_MEM_HOST) {
    HostArr arrs[6 + 16] = {{in.key, size_t(n) * 4, reinterpret_cast<const void**>(&in.key)},
                            {in.valid, size_t(n), reinterpret_cast<const void**>(&in.valid)},
                            {in.topic, size_t(n) * 4, reinterpret_cast<const void**>(&in.topic)},
                            {in.partition, size_t(n) * 4, reinterpret_cast<const void**>(&in.partition)},
                            {in.offset, size_t(n) * 8, reinterpret_cast<const void**>(&in.offset)},
                            {in.ts, size_t(n) * 8, reinterpret_cast<const void**>(&in.ts)}};
    for (int c = 0; c < b->n_cols; c++)
      arrs[6 + c] = HostArr{in.cols[c], size_t(n) * type_size(P.coltypes[c]), &in.cols[c]};
    // small batches are read over the link in place (staged by DMA instead, the grouping kernels took 12 us
    // less but the flush 16 us more: the copy sits on the stream in front of them)
    int rc = stage_host(s, arrs, 6 + b->n_cols, st, true);
    if (rc) return rc;
  }
  const size_t n4 = size_t(n) * 4, n8 = size_t(n) * 8;
  const size_t heads = size_t(s->opts.max_keys + 1) * 8;
  if (!s->g_head.p || !s->g_top.p) {               // epoch-tagged list heads and the node counter: zeroed once
    if (s->g_head.ensure(heads) || s->g_top.ensure(16) || hipMemsetAsync(s->g_head.p, 0, heads, st) ||
        hipMemsetAsync(s->g_top.p, 0, 16, st))
      return fail(CEP_E_HIP, "allocation failed");
  }
  if (s->g_key.ensure(n4) || s->g_arr.ensure(n4) || s->g_pos.ensure(n8) || s->g_nodes.ensure(8 * n4) ||
      s->g_start.ensure(n8) || s->scal.ensure(64) ||
      s->a_cnt.ensure(n8) || s->a_ecnt.ensure(n8) || s->a_head.ensure(n4) || (in.valid && s->g_valid.ensure(size_t(n))) ||
      (in.topic && s->g_topic.ensure(n4)) || (in.partition && s->g_part.ensure(n4)) || (in.offset && s->g_off.ensure(n8)) ||
      (in.ts && s->g_ts.ensure(n8)))
    return fail(CEP_E_HIP, "allocation failed");
  GroupArgs G{};
  G.max_keys = int32_t(std::min<int64_t>(s->opts.max_keys, INT32_MAX - 1));
  G.stamp = ++s->group_stamp;
  G.head = s->g_head.as<unsigned long long>();
  G.node_top = s->g_top.as<int32_t>();
  int32_t* nodes = s->g_nodes.as<int32_t>();
  G.node_key = nodes; G.node_chunk = nodes + n; G.node_cnt = nodes + 2 * n; G.node_next = nodes + 3 * n;
  G.node_prefix = nodes + 4 * n; G.node_leader = nodes + 5 * n; G.rec_node = nodes + 6 * n; G.rec_rank = nodes + 7 * n;
  G.start = s->g_start.as<int64_t>();
  G.cursor = s->g_top.as<unsigned long long>() + 1;
  G.key = in.key; G.g_key = s->g_key.as<int32_t>(); G.arr = s->g_arr.as<int32_t>(); G.pos = s->g_pos.as<int64_t>();
  G.base = s->base;
  G.valid = in.valid; G.g_valid = in.valid ? s->g_valid.as<uint8_t>() : nullptr;
  G.topic = in.topic; G.g_topic = in.topic ? s->g_topic.as<int32_t>() : nullptr;
  G.partition = in.partition; G.g_partition = in.partition ? s->g_part.as<int32_t>() : nullptr;
  G.offset = in.offset; G.g_offset = in.offset ? s->g_off.as<int64_t>() : nullptr;
  G.ts = in.ts; G.g_ts = in.ts ? s->g_ts.as<int64_t>() : nullptr;
  G.ncols = b->n_cols;
  for (int c = 0; c < b->n_cols; c++) {
    if (s->g_cols[c].ensure(size_t(n) * type_size(P.coltypes[c]))) return fail(CEP_E_HIP, "allocation failed");
    G.cols[c] = in.cols[c];
    G.g_cols[c] = s->g_cols[c].p;
    G.coltype[c] = P.coltypes[c];
    gcols[c] = s->g_cols[c].p;
  }
  G.cnt = s->a_cnt.as<int64_t>();
  G.ecnt = s->a_ecnt.as<int64_t>();
  HIPCHECK(group_launch(G, n, st));
  gb = *b;
  gb.key_id = G.g_key; gb.valid = G.g_valid; gb.topic = G.g_topic; gb.partition = G.g_partition;
  gb.offset = G.g_offset; gb.ts = G.g_ts;
  gb.cols = gcols;
  gb.mem = CEP_MEM_DEVICE;
  gb.flags = (b->flags & ~uint32_t(CEP_BATCH_ARRIVAL_ORDER)) | CEP_BATCH_DELIVER;
  s->cur_pos = G.pos;
  return CEP_OK;
}

// the general / runs CSR of an arrival-order batch into arrival order of the completing record (group.hip);
// base: the batch's first stream position
static int arrival_csr(cep_session* s, int64_t base, int64_t n, hipStream_t st) {
  if (!s->e_rec.empty()) {                         // exceptions: ascending position, the first one reported
    std::vector<std::pair<int64_t, int32_t>> e;
    for (size_t i = 0; i < s->e_rec.size(); i++) e.emplace_back(s->e_rec[i], s->e_code[i]);
    std::sort(e.begin(), e.end());
    for (size_t i = 0; i < e.size(); i++) {
      s->e_rec[i] = e[i].first;
      s->e_code[i] = e[i].second;
    }
    s->g_err_rec = e[0].first;
    s->g_err = e[0].second;
  }
  const int64_t nm = s->g_matches, ne = s->g_entries;
  if (nm <= 0) return CEP_OK;
  const size_t hm = size_t(nm + nm / 4 + 256), he = size_t(ne + ne / 4 + 256);
  if ((s->a_record.cap < size_t(nm) * 8 && s->a_record.ensure(hm * 8)) ||
      (s->a_key.cap < size_t(nm) * 4 && s->a_key.ensure(hm * 4)) ||
      (s->a_entoff.cap < size_t(nm) * 8 && s->a_entoff.ensure(hm * 8)) ||
      (s->a_name.cap < size_t(ne) * 4 && s->a_name.ensure(he * 4)) ||
      (s->a_entrec.cap < size_t(ne) * 8 && s->a_entrec.ensure(he * 8)) || s->a_moff.ensure(size_t(n) * 8) ||
      s->a_moffe.ensure(size_t(n) * 8) || s->a_tmp.ensure(size_t(n / 1024 + 4) * 16) || s->scal.ensure(64))
    return fail(CEP_E_HIP, "allocation failed");
  HIPCHECK(arrival_reorder(s->o_record.as<int64_t>(), s->o_key.as<int32_t>(), s->o_entoff.as<int64_t>(),
                           s->o_name.as<int32_t>(), s->o_entrec.as<int64_t>(), nm, ne, base, n, s->a_cnt.as<int64_t>(),
                           s->a_ecnt.as<int64_t>(), s->a_head.as<int32_t>(), s->a_moff.as<int64_t>(),
                           s->a_moffe.as<int64_t>(), s->scal.as<int64_t>() + 6, s->a_tmp.as<int64_t>(),
                           s->a_record.as<int64_t>(), s->a_key.as<int32_t>(), s->a_entoff.as<int64_t>(),
                           s->a_name.as<int32_t>(), s->a_entrec.as<int64_t>(), st));
  std::swap(s->o_record, s->a_record);
  std::swap(s->o_key, s->a_key);
  std::swap(s->o_entoff, s->a_entoff);
  std::swap(s->o_name, s->a_name);
  std::swap(s->o_entrec, s->a_entrec);
  return CEP_OK;
}

int cep_push_batch(cep_session* s, const cep_batch* b, void* stream) {
  if (!s || !b) return fail(CEP_E_ARG, "null argument");
  static const char* const kRange[] = {"cep_push_batch", "cep_push_batch:stencil", "cep_push_batch:general",
                                       "cep_push_batch:chain", "cep_push_batch:runs"};
  RoctxRange range(kRange[s->path >= 1 && s->path <= 4 ? s->path : 0]);
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
  s->push_id++;
  s->pending = true;
  s->collected = false;
  s->e_rec.clear();
  s->e_code.clear();
  if (s->timing) HIPCHECK(hipEventRecord(s->eb0, st));
  // records the processor would drop (null key/value, re-delivered offsets)
  // break contiguity: the stencil only takes batches without them
  const bool stencil_batch = !b->valid && !(s->opts.mode == CEP_MODE_PROCESSOR && b->offset &&
                                            !(b->flags & CEP_BATCH_OFFSETS_MONOTONE));
  s->h2d_wait = false;
  s->delivered = false;
  s->zc_slot = -1;
  s->cur_pos = nullptr;
  s->last_gpos = nullptr;
  int rc = CEP_OK;
  const bool arrival = (b->flags & CEP_BATCH_ARRIVAL_ORDER) && b->n > 0;
  if ((b->flags & CEP_BATCH_ARRIVAL_ORDER) && !s->carry)
    return fail(CEP_E_UNSUPPORTED, "CEP_BATCH_ARRIVAL_ORDER needs a CEP_SESSION_CARRY session");
  cep_batch gb;
  const void* gcols[16] = {};
  const int64_t base0 = s->base;
  if (arrival) {
    rc = group_batch(s, b, st, gb, gcols);
    if (!rc) rc = push_dispatch(s, &gb, st, stencil_batch);
    if (!rc && (s->last_path == CEP_PATH_GENERAL || s->last_path == CEP_PATH_RUNS)) rc = arrival_csr(s, base0, b->n, st);
    s->cur_pos = nullptr;
  } else {
    rc = push_dispatch(s, b, st, stencil_batch);
  }
  if (s->zc_slot >= 0) {                           // the ring slot is free again once the kernels are done
    HIPCHECK(hipEventRecord(s->ring_ev[s->zc_slot], st));
    s->zc_slot = -1;
  }
  if (s->h2d_wait) {                               // the caller's pinned columns are borrowed only for the call
    s->h2d_wait = false;
    HIPCHECK(hipEventSynchronize(s->h2d_ev));
  }
  return rc;
}

static int push_dispatch(cep_session* s, const cep_batch* b, hipStream_t st, bool stencil_batch) {
  const Program& P = s->pat->prog;
  if (s->path == CEP_PATH_RUNS && stencil_batch) {
    s->last_path = CEP_PATH_RUNS;
    return push_runs(s, b, st);
  }
  if (s->path != CEP_PATH_GENERAL && s->path != CEP_PATH_RUNS && stencil_batch) {
    s->last_path = s->path;
    return push_stencil(s, b, st);
  }
  if (s->carry && (s->path == CEP_PATH_STENCIL || s->path == CEP_PATH_CHAIN))   // the halo cannot be carried through the general path
    return fail(CEP_E_UNSUPPORTED, "a stencil carry session takes batches without null records (valid) and with "
                                   "per-key increasing offsets (CEP_BATCH_OFFSETS_MONOTONE)");
  if (s->carry && s->path == CEP_PATH_RUNS)      // nor the runs path's carried tails
    return fail(CEP_E_UNSUPPORTED, "a runs carry session takes batches without null records (valid) and with "
                                   "per-key increasing offsets (CEP_BATCH_OFFSETS_MONOTONE)");
  if (!P.general_ok)
    return fail(CEP_E_UNSUPPORTED, "batch needs the general NFA path, which this pattern cannot use: " + P.general_why);
  s->last_path = CEP_PATH_GENERAL;
  return push_general(s, b, st);
}

const int64_t* cep_device_match_count(const cep_session* s) {
  if (!s) return nullptr;
  // general and runs batches keep the count where their compaction scan left it
  return s->last_path == CEP_PATH_GENERAL || s->last_path == CEP_PATH_RUNS ? s->scal.as<int64_t>() + 3
                                                                            : s->total.as<int64_t>();
}

int cep_match_count_to(const cep_session* s, int64_t* dst, void* stream) {
  if (!s || !dst) return fail(CEP_E_ARG, "null argument");
  hipStream_t st = static_cast<hipStream_t>(stream);
  HIPCHECK(hipSetDevice(s->device));
  if (s->n == 0 || s->last_path == 0) HIPCHECK(hipMemsetAsync(dst, 0, 8, st));
  else HIPCHECK(hipMemcpyAsync(dst, cep_device_match_count(s), 8, hipMemcpyDeviceToDevice, st));
  return CEP_OK;
}

int cep_session_set_timing(cep_session* s, int on) {
  if (!s) return fail(CEP_E_ARG, "null argument");
  s->timing = on != 0;
  return CEP_OK;
}

int cep_last_kernel_ms(cep_session* s, float* ms) {
  if (!s || !ms) return fail(CEP_E_ARG, "null argument");
  if (!s->timing) return fail(CEP_E_UNSUPPORTED, "timing is off (cep_session_set_timing)");
  HIPCHECK(hipEventSynchronize(s->ev1));
  HIPCHECK(hipEventElapsedTime(ms, s->ev0, s->ev1));
  return CEP_OK;
}

int cep_last_batch_ms(cep_session* s, float* ms) {
  if (!s || !ms) return fail(CEP_E_ARG, "null argument");
  if (!s->timing) return fail(CEP_E_UNSUPPORTED, "timing is off (cep_session_set_timing)");
  HIPCHECK(hipEventSynchronize(s->eb1));
  HIPCHECK(hipEventElapsedTime(ms, s->eb0, s->eb1));
  return CEP_OK;
}

// A device-written CSR is checked before any host code walks it: a device bug then fails the call with
// CEP_E_HIP instead of crashing the JVM or Python process (the reference fails the task with an exception,
// SharedVersionedBufferStoreImpl.java:113-115, never with a crash).
int cep_csr_check(const cep_matches* m, int64_t n_records, int32_t n_names) {
  if (!m) return fail(CEP_E_ARG, "null argument");
  const int64_t nm = m->n_matches, ne = m->n_entries;
  if (nm < 0 || ne < 0) return fail(CEP_E_HIP, "device CSR inconsistent: negative counts");
  if (nm == 0) return ne == 0 && (!m->ent_off || m->ent_off[0] == 0) ? CEP_OK
                                                                   : fail(CEP_E_HIP, "device CSR inconsistent: entries without matches");
  if (!m->match_record || !m->ent_off || (ne > 0 && (!m->ent_name || !m->ent_record)))
    return fail(CEP_E_HIP, "device CSR inconsistent: missing arrays");
  if (m->ent_off[0] != 0 || m->ent_off[nm] != ne) return fail(CEP_E_HIP, "device CSR inconsistent: entry offsets' ends");
  bool bad = false;
  for (int64_t i = 0; i < nm; i++)
    bad |= m->ent_off[i + 1] < m->ent_off[i] || uint64_t(m->match_record[i]) >= uint64_t(n_records);
  if (bad) return fail(CEP_E_HIP, "device CSR inconsistent: entry offsets or match records out of range");
  for (int64_t e = 0; e < ne; e++)
    bad |= uint64_t(m->ent_record[e]) >= uint64_t(n_records) || uint32_t(m->ent_name[e]) >= uint32_t(n_names);
  if (bad) return fail(CEP_E_HIP, "device CSR inconsistent: entry records or stage names out of range");
  return CEP_OK;
}

// A delivered batch (CEP_BATCH_DELIVER) from host buffer `slot`, stamped `want`: spin until the delivery
// kernel has stamped it, then the host CSR.  latest: the last pushed batch (matches past the host buffer are
// still in the device arrays)
static int collect_delivered(cep_session* s, int slot, int64_t want, bool latest, cep_matches* o) {
  {
    const StencilProgram& SP = s->pat->prog.stencil;
    const int k = SP.k;
    int64_t* hdr;
    int32_t* hkey;
    int64_t* hpos;
    dl_layout(s, slot, hdr, hkey, hpos);
    // the delivery kernel's last workgroup stamps hdr[2] once every row is in host memory: spin on it (a
    // stream wait sleeps and wakes microseconds late); a stamp that does not come -- a fault -- is left
    // to the stream wait, which reports it
    const volatile int64_t* stamp = hdr + 2;
    const auto t0 = std::chrono::steady_clock::now();
    while (*stamp != want) {
      if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(200)) {
        HIPCHECK(hipStreamSynchronize(s->stream));
        if (*stamp != want) return fail(CEP_E_HIP, "the delivery kernel did not complete");
        break;
      }
      __builtin_ia32_pause();
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    const int64_t nm = hdr[0];
    const uint64_t hf = uint64_t(hdr[1]);
    if (hf & 1) return fail(CEP_E_ARG, "carry sessions need key ids in [0, max_keys)");
    if (hf & 2) return fail(CEP_E_ARG, "carry batch is not grouped by key: a key has two segments");
    if (hf & 4) return fail(CEP_E_RUN_CAPACITY, "chain carry batch: more runs completing in one tile than its match space");
    if (nm > s->out_cap) return fail(CEP_E_RUN_CAPACITY, "match output exceeded the session capacity");
    const int64_t nh = std::min(nm, s->dl_cap);
    if (nm > nh && !latest)                        // the rest was on the device, which a later push reused
      return fail(CEP_E_UNSUPPORTED, "a batch with more matches than the host delivery buffer is collected only "
                                     "before the next push");
    std::vector<int64_t> rest_pos;
    std::vector<int32_t> rest_key;
    if (nm > nh) {                                 // past the host buffer: from the device arrays
      rest_pos.resize(size_t(nm - nh) * k);
      rest_key.resize(size_t(nm - nh));
      HIPCHECK(hipMemcpy(rest_pos.data(), s->opos.as<int64_t>() + nh * k, rest_pos.size() * 8, hipMemcpyDeviceToHost));
      HIPCHECK(hipMemcpy(rest_key.data(), s->mkey.as<int32_t>() + nh, rest_key.size() * 4, hipMemcpyDeviceToHost));
    }
    s->match_record.resize(size_t(nm));
    s->match_key.resize(size_t(nm));
    s->ent_off.resize(size_t(nm) + 1);
    s->ent_name.resize(size_t(nm) * k);
    s->ent_record.resize(size_t(nm) * k);
    int64_t ne = 0;
    for (int64_t m = 0; m < nm; m++) {             // peek traversal order: final stage first
      const int64_t* p = m < nh ? hpos + m * k : rest_pos.data() + (m - nh) * k;
      s->match_key[size_t(m)] = m < nh ? hkey[m] : rest_key[size_t(m - nh)];
      s->match_record[size_t(m)] = p[k - 1];
      s->ent_off[size_t(m)] = ne;
      for (int i = k - 1; i >= 0; i--) {
        if (p[i] == -1) continue;                   // a skipped optional stage
        s->ent_name[size_t(ne)] = SP.name[i];
        s->ent_record[size_t(ne)] = p[i];
        ne++;
      }
    }
    s->ent_off[size_t(nm)] = ne;
    s->ent_name.resize(size_t(ne));
    s->ent_record.resize(size_t(ne));
    o->n_matches = nm;
    o->n_entries = ne;
    o->path = s->last_path;
    o->err = CEP_OK;
    o->err_record = -1;
  }
  return CEP_OK;
}

int cep_collect(cep_session* s, cep_matches* o) {
  if (!s || !o) return fail(CEP_E_ARG, "null argument");
  RoctxRange range("cep_collect");
  memset(o, 0, sizeof *o);
  if (s->collected) {                              // nothing pushed since: the host CSR is current
    *o = s->last;
    if (o->err) g_err = "the reference NFA raises an exception on this batch";
    return CEP_OK;
  }
  HIPCHECK(hipSetDevice(s->device));
  if (s->last_path == CEP_PATH_GENERAL || s->last_path == CEP_PATH_RUNS) {
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
    o->path = s->last_path;
    o->err = s->g_err;
    o->err_record = s->g_err_rec;
    o->match_record = s->match_record.data();
    o->ent_off = s->ent_off.data();
    o->ent_name = s->ent_name.data();
    o->ent_record = s->ent_record.data();
    // records: the batch's (stream positions on carry sessions: everything pushed so far)
    int rc = cep_csr_check(o, s->carry ? s->base : s->n, int32_t(s->pat->prog.names.size()));
    if (rc) return rc;
    if (s->g_err) g_err = "the reference NFA raises an exception on this batch";
  } else if (s->delivered) {                       // CEP_BATCH_DELIVER: the device wrote the CSR's inputs
    int rc = collect_delivered(s, int(s->dl_stamp & 1), s->dl_stamp, true, o);
    if (rc) return rc;
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
    // carry sessions: every entry as a stream position (halo entries from the keys' halos)
    std::vector<int64_t> pos_host;
    if (s->carry) {
      unsigned long long hf = 0;
      HIPCHECK(hipMemcpy(&hf, s->hflags.as<unsigned long long>() + (s->halo_stamp & 1), 8, hipMemcpyDeviceToHost));
      if (hf & 1) return fail(CEP_E_ARG, "carry sessions need key ids in [0, max_keys)");
      if (hf & 2) return fail(CEP_E_ARG, "carry batch is not grouped by key: a key has two segments");
      if (hf & 4) return fail(CEP_E_RUN_CAPACITY, "chain carry batch: more runs completing in one tile than its match space");
    }
    if (s->carry && nm > 0) {
      if (s->opos.ensure(size_t(nm) * k * 8)) return fail(CEP_E_HIP, "allocation failed");
      HIPCHECK(stencil_resolve_launch(s->d_key, s->out.as<int32_t>(), k, nm, carry_args(s), s->opos.as<int64_t>(),
                                      nullptr, nullptr, s->stream));
      pos_host.resize(size_t(nm) * k);
      HIPCHECK(hipMemcpyAsync(pos_host.data(), s->opos.p, pos_host.size() * 8, hipMemcpyDeviceToHost, s->stream));
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
      s->match_record[m] = s->carry ? pos_host[m * k + k - 1] : s->out_host[m * k + k - 1];
      s->ent_off[m] = ne;
      for (int i = 0; i < k; i++) {
        const int st = k - 1 - i;
        const int32_t r = s->out_host[m * k + st];
        if (r == -1) continue;
        s->ent_name[ne] = SP.name[st];
        s->ent_record[ne] = s->carry ? pos_host[m * k + st] : r;
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
  s->collected = true;
  s->last = *o;
  return CEP_OK;
}

int64_t cep_batch_id(const cep_session* s) { return s ? s->push_id : -1; }

// the delivery buffer holding batch `id`, or -1
static int delivered_slot(const cep_session* s, int64_t id) {
  for (int j = 0; j < 2; j++)
    if (s->dl[j] && s->dl_pid[j] == id) return j;
  return -1;
}

int cep_batch_ready(cep_session* s, int64_t id) {
  if (!s) return fail(CEP_E_ARG, "null argument");
  if (id < 1 || id > s->push_id) return fail(CEP_E_ARG, "no such batch");
  const int slot = delivered_slot(s, id);
  if (slot >= 0) {                                 // delivered: its stamp is in host memory once complete
    const int64_t want = s->dl_stamp - ((s->dl_stamp & 1) == slot ? 0 : 1);
    return *reinterpret_cast<const volatile int64_t*>(static_cast<int64_t*>(s->dl[slot]) + 2) == want ? 1 : 0;
  }
  if (id < s->push_id) return 1;                   // (an earlier batch: the stream has moved past it, or will)
  const hipError_t e = hipStreamQuery(s->stream);
  if (e == hipErrorNotReady) return 0;
  if (e != hipSuccess) return fail(CEP_E_HIP, std::string("hipStreamQuery: ") + hipGetErrorString(e));
  return 1;
}

int cep_collect_batch(cep_session* s, int64_t id, cep_matches* o) {
  if (!s || !o) return fail(CEP_E_ARG, "null argument");
  if (id == s->push_id) return cep_collect(s, o);
  const int slot = delivered_slot(s, id);
  if (slot < 0 || id != s->push_id - 1)
    return fail(CEP_E_ARG, "only the last batch, or the delivered batch before it, can be collected");
  RoctxRange range("cep_collect");
  memset(o, 0, sizeof *o);
  HIPCHECK(hipSetDevice(s->device));
  const int64_t want = s->dl_stamp - ((s->dl_stamp & 1) == slot ? 0 : 1);
  int rc = collect_delivered(s, slot, want, false, o);
  if (rc) return rc;
  o->match_record = s->match_record.data();
  o->match_key = s->match_key.data();
  o->ent_off = s->ent_off.data();
  o->ent_name = s->ent_name.data();
  o->ent_record = s->ent_record.data();
  s->collected = false;                            // the host CSR now holds the older batch
  return CEP_OK;
}

int cep_checksum(cep_session* s, uint64_t* sum, int64_t* n_matches) {
  if (!s || !sum) return fail(CEP_E_ARG, "null argument");
  HIPCHECK(hipSetDevice(s->device));
  if (s->last_path == CEP_PATH_GENERAL || s->last_path == CEP_PATH_RUNS) {
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
  if (s->carry) {                                  // over stream positions
    if (s->opos.ensure(size_t(std::max<int64_t>(nm, 1)) * SP.k * 8)) return fail(CEP_E_HIP, "allocation failed");
    HIPCHECK(stencil_resolve_launch(s->d_key, s->out.as<int32_t>(), SP.k, nm, carry_args(s), s->opos.as<int64_t>(),
                                    s->prog.as<StencilProgram>(), s->sum.as<unsigned long long>(), s->stream));
  } else {
    HIPCHECK(stencil_post(s->d_key, s->out.as<int32_t>(), SP.k, nm, nullptr, s->prog.as<StencilProgram>(),
                          s->sum.as<unsigned long long>(), s->stream));
  }
  uint64_t h = 0;
  HIPCHECK(hipMemcpyAsync(&h, s->sum.p, 8, hipMemcpyDeviceToHost, s->stream));
  HIPCHECK(hipStreamSynchronize(s->stream));
  *sum = h;
  if (n_matches) *n_matches = nm;
  return CEP_OK;
}

// ---- carried state (CEP_SESSION_CARRY) ----
// export format: "KCST", version 1, int64 next stream position, int32 key count,
// then per key: int32 key id, int32 words, the blob (kcep_internal.h CB_*)
namespace {
constexpr uint32_t kStateMagic = 0x5453434Bu;   // "KCST"
int need_carry(cep_session* s) {
  if (!s) return fail(CEP_E_ARG, "null argument");
  if (!s->carry) return fail(CEP_E_ARG, "the session was not opened with CEP_SESSION_CARRY");
  return CEP_OK;
}
}  // namespace

// stencil carry sessions: "KCSH", version 1, int64 next stream position, int32 key count, then per key
// with a halo: int32 key id, int32 records, uint64 stage masks, int64 stream positions[records]
constexpr uint32_t kHaloMagic = 0x4853434Bu;   // "KCSH"
bool halo_session(const cep_session* s) { return s->carry && (s->path == CEP_PATH_STENCIL || s->path == CEP_PATH_CHAIN); }
int halo_newest(const HaloHdr& h) { return h.stamp[1] > h.stamp[0] ? 1 : 0; }

int halo_export(cep_session* s, int32_t key_lo, int32_t key_hi, void* buf, size_t cap, size_t* needed) {
  const int km1 = s->pat->prog.stencil.k - 1;
  const size_t nk = size_t(std::max(0, key_hi - key_lo));
  std::vector<HaloHdr> tab(nk);
  std::vector<int64_t> pos(nk * 2 * size_t(km1));
  if (nk) {
    HIPCHECK(hipMemcpy(tab.data(), s->halo.as<HaloHdr>() + key_lo, nk * sizeof(HaloHdr), hipMemcpyDeviceToHost));
    if (km1)
      HIPCHECK(hipMemcpy(pos.data(), s->hpos.as<int64_t>() + 2 * int64_t(key_lo) * km1, pos.size() * 8,
                         hipMemcpyDeviceToHost));
  }
  size_t bytes = 20;
  int32_t nkeys = 0;
  for (size_t i = 0; i < nk; i++) {
    const int sl = halo_newest(tab[i]);
    if (tab[i].stamp[sl] > 0 && tab[i].cnt[sl] > 0) { bytes += 16 + 8 * size_t(tab[i].cnt[sl]); nkeys++; }
  }
  *needed = bytes;
  if (!buf) return CEP_OK;
  if (cap < bytes) return fail(CEP_E_ARG, "export buffer too small");
  uint8_t* p = static_cast<uint8_t*>(buf);
  const uint32_t ver = 1;
  memcpy(p, &kHaloMagic, 4); memcpy(p + 4, &ver, 4); memcpy(p + 8, &s->base, 8); memcpy(p + 16, &nkeys, 4);
  p += 20;
  for (size_t i = 0; i < nk; i++) {
    const int sl = halo_newest(tab[i]);
    const int32_t cnt = tab[i].cnt[sl];
    if (tab[i].stamp[sl] <= 0 || cnt <= 0) continue;
    const int32_t k = key_lo + int32_t(i);
    memcpy(p, &k, 4); memcpy(p + 4, &cnt, 4); memcpy(p + 8, &tab[i].masks[sl], 8);
    memcpy(p + 16, &pos[(2 * i + size_t(sl)) * size_t(km1)], 8 * size_t(cnt));
    p += 16 + 8 * size_t(cnt);
  }
  return CEP_OK;
}

int halo_import(cep_session* s, const uint8_t* p, size_t len) {
  int64_t base;
  int32_t nkeys;
  memcpy(&base, p + 8, 8); memcpy(&nkeys, p + 16, 4);
  const int K = s->pat->prog.stencil.k;
  struct Row { int32_t k, cnt; uint64_t masks; int64_t pos[STENCIL_MAX_K - 1]; };
  std::vector<Row> rows;
  size_t at = 20;
  if (s->halo_stamp == 0) s->halo_stamp = 1;     // imported slots count as written before the next batch
  for (int32_t i = 0; i < nkeys; i++) {
    if (at + 16 > len) return fail(CEP_E_ARG, "truncated state blob");
    Row r{};
    memcpy(&r.k, p + at, 4); memcpy(&r.cnt, p + at + 4, 4); memcpy(&r.masks, p + at + 8, 8);
    if (r.k < 0 || r.k >= s->opts.max_keys || r.cnt < 0 || r.cnt > K - 1 || at + 16 + 8 * size_t(r.cnt) > len)
      return fail(CEP_E_ARG, "bad key entry in the state blob");
    memcpy(r.pos, p + at + 16, 8 * size_t(r.cnt));
    rows.push_back(r);
    at += 16 + 8 * size_t(r.cnt);
  }
  HIPCHECK(hipSetDevice(s->device));
  if (s->stream) HIPCHECK(hipStreamSynchronize(s->stream));
  for (auto& r : rows) {                         // slot 0 holds the halo, slot 1 is empty
    HaloHdr h{};
    h.stamp[0] = s->halo_stamp;
    h.claim = s->halo_stamp;
    h.cnt[0] = uint8_t(r.cnt);
    h.masks[0] = r.masks;
    HIPCHECK(hipMemcpy(s->halo.as<HaloHdr>() + r.k, &h, sizeof h, hipMemcpyHostToDevice));
    if (K > 1)
      HIPCHECK(hipMemcpy(s->hpos.as<int64_t>() + 2 * int64_t(r.k) * (K - 1), r.pos, 8 * size_t(K - 1),
                         hipMemcpyHostToDevice));
  }
  s->base = std::max(s->base, base);
  return CEP_OK;
}

// runs carry sessions: "KCSR", version 1, int64 next stream position, int32 key count, then per key with
// a tail: int32 key id, int32 records, int32 words per record (5 + ncols), int32 0, then the records
// (runs.hip tail records: stream position first)
constexpr uint32_t kTailMagic = 0x5253434Bu;   // "KCSR"
int tail_download(cep_session* s, std::vector<int64_t>& tab, std::vector<int64_t>& pool) {
  tab.resize(size_t(s->opts.max_keys) * 2);
  pool.resize(size_t(s->rpool_used) * size_t(tail_rw(s)));
  HIPCHECK(hipMemcpy(tab.data(), s->rtab.p, tab.size() * 8, hipMemcpyDeviceToHost));
  if (!pool.empty()) HIPCHECK(hipMemcpy(pool.data(), s->rpool.p, pool.size() * 8, hipMemcpyDeviceToHost));
  return CEP_OK;
}
// appends key k's tail entry (key, records, words) to out; returns its record count
int64_t tail_entry(const cep_session* s, const std::vector<int64_t>& tab, const std::vector<int64_t>& pool, int32_t k,
                   std::vector<uint8_t>& out) {
  const int64_t L = tab[2 * size_t(k) + 1];
  if (L <= 0) return 0;
  const size_t RW = size_t(tail_rw(s)), at = out.size();
  const int32_t cnt = int32_t(L), rw = int32_t(RW), zero = 0;
  out.resize(at + 16 + size_t(L) * RW * 8);
  memcpy(&out[at], &k, 4); memcpy(&out[at + 4], &cnt, 4); memcpy(&out[at + 8], &rw, 4); memcpy(&out[at + 12], &zero, 4);
  memcpy(&out[at + 16], pool.data() + size_t(tab[2 * size_t(k)]) * RW, size_t(L) * RW * 8);
  return L;
}
int tail_export(cep_session* s, int32_t key_lo, int32_t key_hi, void* buf, size_t cap, size_t* needed) {
  std::vector<int64_t> tab, pool;
  int rc = tail_download(s, tab, pool);
  if (rc) return rc;
  std::vector<uint8_t> out(20);
  int32_t nkeys = 0;
  for (int32_t k = key_lo; k < key_hi; k++) nkeys += tail_entry(s, tab, pool, k, out) > 0;
  const uint32_t ver = 1;
  memcpy(&out[0], &kTailMagic, 4); memcpy(&out[4], &ver, 4); memcpy(&out[8], &s->base, 8); memcpy(&out[16], &nkeys, 4);
  *needed = out.size();
  if (!buf) return CEP_OK;
  if (cap < out.size()) return fail(CEP_E_ARG, "export buffer too small");
  memcpy(buf, out.data(), out.size());
  return CEP_OK;
}
int tail_import(cep_session* s, const uint8_t* p, size_t len) {
  int64_t base;
  int32_t nkeys;
  memcpy(&base, p + 8, 8); memcpy(&nkeys, p + 16, 4);
  const size_t RW = size_t(tail_rw(s));
  std::vector<std::pair<int32_t, size_t>> ents;
  size_t at = 20, recs = 0;
  for (int32_t i = 0; i < nkeys; i++) {
    if (at + 16 > len) return fail(CEP_E_ARG, "truncated state blob");
    int32_t k, cnt, rw;
    memcpy(&k, p + at, 4); memcpy(&cnt, p + at + 4, 4); memcpy(&rw, p + at + 8, 4);
    if (rw != int32_t(RW)) return fail(CEP_E_ARG, "state blob does not match this pattern");
    if (k < 0 || k >= s->opts.max_keys || cnt <= 0 || at + 16 + size_t(cnt) * RW * 8 > len)
      return fail(CEP_E_ARG, "bad key entry in the state blob");
    ents.push_back({k, at});
    recs += size_t(cnt);
    at += 16 + size_t(cnt) * RW * 8;
  }
  HIPCHECK(hipSetDevice(s->device));
  if (s->stream) HIPCHECK(hipStreamSynchronize(s->stream));
  int rc = tail_reserve(s, int64_t(recs), s->stream);
  if (rc) return rc;
  std::vector<int64_t> tab(size_t(s->opts.max_keys) * 2);
  HIPCHECK(hipMemcpy(tab.data(), s->rtab.p, tab.size() * 8, hipMemcpyDeviceToHost));
  std::vector<int64_t> words(recs * RW);
  int64_t w0 = 0;
  for (auto& e : ents) {
    int32_t cnt;
    memcpy(&cnt, p + e.second + 4, 4);
    memcpy(words.data() + size_t(w0) * RW, p + e.second + 16, size_t(cnt) * RW * 8);
    tab[2 * size_t(e.first)] = s->rpool_used + w0;
    tab[2 * size_t(e.first) + 1] = cnt;
    w0 += cnt;
  }
  if (recs) HIPCHECK(hipMemcpy(s->rpool.as<int64_t>() + size_t(s->rpool_used) * RW, words.data(), words.size() * 8,
                               hipMemcpyHostToDevice));
  HIPCHECK(hipMemcpy(s->rtab.p, tab.data(), tab.size() * 8, hipMemcpyHostToDevice));
  s->rpool_used += int64_t(recs);
  HIPCHECK(hipMemcpy(s->rtop.p, &s->rpool_used, 8, hipMemcpyHostToDevice));
  s->base = std::max(s->base, base);
  return CEP_OK;
}

int cep_state_export(cep_session* s, int32_t key_lo, int32_t key_hi, void* buf, size_t cap, size_t* needed) {
  int rc = need_carry(s);
  if (rc) return rc;
  if (!needed) return fail(CEP_E_ARG, "null argument");
  HIPCHECK(hipSetDevice(s->device));
  if (s->stream) HIPCHECK(hipStreamSynchronize(s->stream));
  key_lo = std::max<int32_t>(key_lo, 0);
  key_hi = int32_t(std::min<int64_t>(key_hi, s->opts.max_keys));
  if (halo_session(s)) return halo_export(s, key_lo, key_hi, buf, cap, needed);
  if (tail_session(s)) return tail_export(s, key_lo, key_hi, buf, cap, needed);
  std::vector<int64_t> tab(size_t(std::max(0, key_hi - key_lo)));
  if (!tab.empty()) HIPCHECK(hipMemcpy(tab.data(), s->ctab.as<int64_t>() + key_lo, tab.size() * 8, hipMemcpyDeviceToHost));
  std::vector<int32_t> pool(size_t(s->cpool_used));
  if (!pool.empty()) HIPCHECK(hipMemcpy(pool.data(), s->cpool.p, pool.size() * 4, hipMemcpyDeviceToHost));
  size_t bytes = 20;
  int32_t nkeys = 0;
  for (int64_t o : tab)
    if (o >= 0) { bytes += 8 + size_t(pool[size_t(o) + CB_WORDS]) * 4; nkeys++; }
  *needed = bytes;
  if (!buf) return CEP_OK;
  if (cap < bytes) return fail(CEP_E_ARG, "export buffer too small");
  uint8_t* p = static_cast<uint8_t*>(buf);
  const uint32_t ver = 1;
  memcpy(p, &kStateMagic, 4); memcpy(p + 4, &ver, 4); memcpy(p + 8, &s->base, 8); memcpy(p + 16, &nkeys, 4);
  p += 20;
  for (size_t i = 0; i < tab.size(); i++) {
    if (tab[i] < 0) continue;
    const int32_t k = key_lo + int32_t(i), w = pool[size_t(tab[i]) + CB_WORDS];
    memcpy(p, &k, 4); memcpy(p + 4, &w, 4);
    memcpy(p + 8, pool.data() + tab[i], size_t(w) * 4);
    p += 8 + size_t(w) * 4;
  }
  return CEP_OK;
}

int cep_state_import(cep_session* s, const void* buf, size_t len) {
  int rc = need_carry(s);
  if (rc) return rc;
  if (!buf || len < 20) return fail(CEP_E_ARG, "bad state blob");
  const uint8_t* p = static_cast<const uint8_t*>(buf);
  uint32_t magic, ver;
  int64_t base;
  int32_t nkeys;
  memcpy(&magic, p, 4); memcpy(&ver, p + 4, 4); memcpy(&base, p + 8, 8); memcpy(&nkeys, p + 16, 4);
  if (halo_session(s)) {
    if (magic != kHaloMagic || ver != 1 || nkeys < 0) return fail(CEP_E_ARG, "bad state blob (stencil sessions take KCSH)");
    return halo_import(s, p, len);
  }
  if (tail_session(s)) {
    if (magic != kTailMagic || ver != 1 || nkeys < 0) return fail(CEP_E_ARG, "bad state blob (runs sessions take KCSR)");
    return tail_import(s, p, len);
  }
  if (magic != kStateMagic || ver != 1 || nkeys < 0) return fail(CEP_E_ARG, "bad state blob");
  const DevProgram& D = s->pat->prog.dev;
  std::vector<std::pair<int32_t, size_t>> keys;    // key, byte offset of its blob
  size_t at = 20, words = 0;
  for (int32_t i = 0; i < nkeys; i++) {
    if (at + 8 > len) return fail(CEP_E_ARG, "truncated state blob");
    int32_t k, w;
    memcpy(&k, p + at, 4); memcpy(&w, p + at + 4, 4);
    if (k < 0 || k >= s->opts.max_keys || w < CB_HDR || at + 8 + size_t(w) * 4 > len)
      return fail(CEP_E_ARG, "bad key entry in the state blob");
    int32_t hdr[CB_HDR];
    memcpy(hdr, p + at + 8, sizeof hdr);
    if (hdr[CB_WORDS] != w || hdr[CB_NCOLS] != D.ncols || hdr[CB_NSTATES] != D.nstates)
      return fail(CEP_E_ARG, "state blob does not match this pattern");
    keys.push_back({k, at + 8});
    words += size_t(w);
    at += 8 + size_t(w) * 4;
  }
  HIPCHECK(hipSetDevice(s->device));
  if (s->stream) HIPCHECK(hipStreamSynchronize(s->stream));
  hipStream_t st = s->stream;
  if (s->cpool_used + int64_t(words) > s->cpool_words && (rc = carry_gc(s, 2 * (s->cpool_used + int64_t(words)), st)))
    return rc;
  std::vector<int32_t> blobs(words);
  std::vector<int64_t> tab(size_t(s->opts.max_keys));
  HIPCHECK(hipMemcpy(tab.data(), s->ctab.p, tab.size() * 8, hipMemcpyDeviceToHost));
  size_t w0 = 0;
  for (auto& kb : keys) {
    int32_t w;
    memcpy(&w, p + kb.second, 4);
    memcpy(blobs.data() + w0, p + kb.second, size_t(w) * 4);
    tab[size_t(kb.first)] = s->cpool_used + int64_t(w0);
    w0 += size_t(w);
  }
  if (words) HIPCHECK(hipMemcpy(s->cpool.as<int32_t>() + s->cpool_used, blobs.data(), words * 4, hipMemcpyHostToDevice));
  HIPCHECK(hipMemcpy(s->ctab.p, tab.data(), tab.size() * 8, hipMemcpyHostToDevice));
  s->cpool_used += int64_t(words);
  s->base = std::max(s->base, base);
  return CEP_OK;
}

int cep_state_clear(cep_session* s) {
  int rc = need_carry(s);
  if (rc) return rc;
  HIPCHECK(hipSetDevice(s->device));
  if (s->stream) HIPCHECK(hipStreamSynchronize(s->stream));
  s->base = 0;
  if (halo_session(s)) {
    HIPCHECK(hipMemset(s->halo.p, 0, size_t(s->opts.max_keys) * sizeof(HaloHdr)));
    HIPCHECK(hipMemset(s->hflags.p, 0, 16));       // both error-flag words (by stamp parity)
    s->halo_stamp = 0;
    return CEP_OK;
  }
  if (tail_session(s)) {
    HIPCHECK(hipMemset(s->rtab.p, 0, size_t(s->opts.max_keys) * 16));
    HIPCHECK(hipMemset(s->rtop.p, 0, 8));
    s->rpool_used = 0;
    return CEP_OK;
  }
  HIPCHECK(hipMemset(s->ctab.p, 0xFF, size_t(s->opts.max_keys) * 8));
  s->cpool_used = 0;
  return CEP_OK;
}

int cep_key_state(cep_session* s, int32_t key, int64_t* runs, int64_t* queue_len) {
  int rc = need_carry(s);
  if (rc) return rc;
  if (!runs || !queue_len || key < 0 || key >= s->opts.max_keys) return fail(CEP_E_ARG, "bad argument");
  if (halo_session(s))
    return fail(CEP_E_UNSUPPORTED, "a stencil carry session keeps each key's last records, not its NFA runs");
  if (tail_session(s))
    return fail(CEP_E_UNSUPPORTED, "a runs carry session keeps each key's records from its oldest open run, not its NFA queue");
  HIPCHECK(hipSetDevice(s->device));
  if (s->stream) HIPCHECK(hipStreamSynchronize(s->stream));
  int64_t off = -1;
  HIPCHECK(hipMemcpy(&off, s->ctab.as<int64_t>() + key, 8, hipMemcpyDeviceToHost));
  if (off < 0) { *runs = 0; *queue_len = -1; return CEP_OK; }
  int32_t hdr[CB_HDR];
  HIPCHECK(hipMemcpy(hdr, s->cpool.as<int32_t>() + off, sizeof hdr, hipMemcpyDeviceToHost));
  *runs = int64_t(uint32_t(hdr[CB_RUNS_LO])) | (int64_t(hdr[CB_RUNS_HI]) << 32);
  *queue_len = hdr[CB_QLEN];
  return CEP_OK;
}

int64_t cep_stream_position(const cep_session* s) { return s ? s->base : -1; }

int cep_state_evict(cep_session* s, const int32_t* keys, int64_t n, const uint8_t** blobs, int64_t* offs) {
  int rc = need_carry(s);
  if (rc) return rc;
  if (n < 0 || !blobs || !offs || (n > 0 && !keys)) return fail(CEP_E_ARG, "null argument");
  for (int64_t i = 0; i < n; i++)
    if (keys[i] < 0 || keys[i] >= s->opts.max_keys) return fail(CEP_E_ARG, "key id out of [0, max_keys)");
  HIPCHECK(hipSetDevice(s->device));
  if (s->stream) HIPCHECK(hipStreamSynchronize(s->stream));
  // one download of the key tables (and the carried pool), then one self-contained blob per key
  std::vector<uint8_t>& out = s->evict_buf;
  out.clear();
  offs[0] = 0;
  const uint32_t ver = 1;
  auto header = [&](uint32_t magic, int32_t nk) {
    const size_t at = out.size();
    out.resize(at + 20);
    memcpy(&out[at], &magic, 4); memcpy(&out[at + 4], &ver, 4); memcpy(&out[at + 8], &s->base, 8);
    memcpy(&out[at + 16], &nk, 4);
  };
  if (halo_session(s)) {
    const int km1 = s->pat->prog.stencil.k - 1;
    const int64_t nk = s->opts.max_keys;
    std::vector<HaloHdr> tab(static_cast<size_t>(nk));
    std::vector<int64_t> pos(static_cast<size_t>(nk) * 2 * size_t(km1));
    HIPCHECK(hipMemcpy(tab.data(), s->halo.p, tab.size() * sizeof(HaloHdr), hipMemcpyDeviceToHost));
    if (km1) HIPCHECK(hipMemcpy(pos.data(), s->hpos.p, pos.size() * 8, hipMemcpyDeviceToHost));
    for (int64_t i = 0; i < n; i++) {
      HaloHdr& h = tab[size_t(keys[i])];
      const int sl = halo_newest(h);
      const int32_t cnt = h.cnt[sl];
      if (h.stamp[sl] > 0 && cnt > 0) {
        header(kHaloMagic, 1);
        const size_t at = out.size();
        out.resize(at + 16 + 8 * size_t(cnt));
        memcpy(&out[at], &keys[i], 4); memcpy(&out[at + 4], &cnt, 4); memcpy(&out[at + 8], &h.masks[sl], 8);
        memcpy(&out[at + 16], &pos[(2 * size_t(keys[i]) + size_t(sl)) * size_t(km1)], 8 * size_t(cnt));
      }
      h = HaloHdr{};                                 // no halo: the next batch starts the key afresh
      offs[i + 1] = int64_t(out.size());
    }
    HIPCHECK(hipMemcpy(s->halo.p, tab.data(), tab.size() * sizeof(HaloHdr), hipMemcpyHostToDevice));
  } else if (tail_session(s)) {
    std::vector<int64_t> tab, pool;
    int rc2 = tail_download(s, tab, pool);
    if (rc2) return rc2;
    for (int64_t i = 0; i < n; i++) {
      if (tab[2 * size_t(keys[i]) + 1] > 0) {
        header(kTailMagic, 1);
        tail_entry(s, tab, pool, keys[i], out);
      }
      tab[2 * size_t(keys[i]) + 1] = 0;              // (the pool records are reclaimed by the next compaction)
      offs[i + 1] = int64_t(out.size());
    }
    HIPCHECK(hipMemcpy(s->rtab.p, tab.data(), tab.size() * 8, hipMemcpyHostToDevice));
  } else {
    std::vector<int64_t> tab(size_t(s->opts.max_keys));
    HIPCHECK(hipMemcpy(tab.data(), s->ctab.p, tab.size() * 8, hipMemcpyDeviceToHost));
    std::vector<int32_t> pool(size_t(s->cpool_used));
    if (!pool.empty()) HIPCHECK(hipMemcpy(pool.data(), s->cpool.p, pool.size() * 4, hipMemcpyDeviceToHost));
    for (int64_t i = 0; i < n; i++) {
      int64_t& o = tab[size_t(keys[i])];
      if (o >= 0) {
        const int32_t w = pool[size_t(o) + CB_WORDS];
        header(kStateMagic, 1);
        const size_t at = out.size();
        out.resize(at + 8 + 4 * size_t(w));
        memcpy(&out[at], &keys[i], 4); memcpy(&out[at + 4], &w, 4);
        memcpy(&out[at + 8], pool.data() + o, 4 * size_t(w));
      }
      o = -1;                                        // the blob's pool words are reclaimed by the next carry_gc
      offs[i + 1] = int64_t(out.size());
    }
    HIPCHECK(hipMemcpy(s->ctab.p, tab.data(), tab.size() * 8, hipMemcpyHostToDevice));
  }
  *blobs = out.data();
  return CEP_OK;
}

// A key's carried NFA state (one "KCST" key) in the reference's own terms -- "KCRF", version 1, little
// endian, strings as i32 length + UTF-8 bytes:
//   u32 magic, u32 version, i32 key id, i32 n_cols, i64 runs                      NFAStates.runs (NFA.runs)
//   i32 n, n x {i32 topic id, i64 offset}              NFAStates.latestOffsets: the next record's minimum
//   i32 n, n x {i64 stream position, i32 topic id, i32 partition, i64 offset, i64 timestamp,
//               n_cols x i64 value bits}               the events the buffer still holds (MatchedEvent)
//   i32 n, n x {i32 stage id, i32 epsilon target (-1: the stage itself), i32 flags (1 isBranching,
//               2 isIgnored), i64 sequence, i32 last event (index above, -1 null), i64 timestamp (-1:
//               never read -- within() is inert), i32 n_digits, n_digits x i32}
//                                                      the run queue (ComputationStage, FIFO order)
//   i32 n, n x {str stage name, i32 stage type, i32 event, i64 refs, i32 n_preds, n_preds x {i32 n_digits,
//               n_digits x i32, i32 has predecessor, str predecessor stage name, i32 its type, i32 its
//               event}}                                 buffer nodes Matched -> MatchedEvent, preds in order
//   i32 n, n x {str state name, i64 sequence, i32 type (1 int, 2 long, 3 double), i64 value bits}
//                                                      aggregates (record key, state, sequence) -> value
// Sequences are renumbered densely from 0 (runs sharing one share its aggregates); every new run the
// reference creates gets ++runs, beyond them.
int cep_state_to_reference(const cep_pattern* p, const void* blob, size_t len, void* out, size_t cap,
                           size_t* needed) {
  if (!p || !blob || !needed) return fail(CEP_E_ARG, "null argument");
  const Program& P = p->prog;
  const uint8_t* in = static_cast<const uint8_t*>(blob);
  uint32_t magic = 0;
  int32_t nkeys = 0;
  if (len < 20) return fail(CEP_E_ARG, "bad state blob");
  memcpy(&magic, in, 4);
  memcpy(&nkeys, in + 16, 4);
  if (magic != kStateMagic) return fail(CEP_E_ARG, "not a general-path (KCST) state blob");
  if (nkeys != 1) return fail(CEP_E_ARG, "cep_state_to_reference takes a single-key blob (cep_state_evict)");
  if (len < 28) return fail(CEP_E_ARG, "truncated state blob");
  int32_t key = 0, w = 0;
  memcpy(&key, in + 20, 4);
  memcpy(&w, in + 24, 4);
  if (w < CB_HDR || 28 + size_t(w) * 4 > len) return fail(CEP_E_ARG, "truncated state blob");
  std::vector<int32_t> b(static_cast<size_t>(w));
  memcpy(b.data(), in + 28, size_t(w) * 4);
  const int nhwm = b[CB_NHWM], qlen = b[CB_QLEN], nev = b[CB_NEV], nnode = b[CB_NNODE], npred = b[CB_NPRED];
  const int nver = b[CB_NVER], nseq = b[CB_NSEQ], ncols = b[CB_NCOLS], nst = b[CB_NSTATES];
  if (nhwm < 0 || qlen < 0 || nev < 0 || nnode < 0 || npred < 0 || nver < 0 || nseq < 0 || ncols < 0 || nst < 0)
    return fail(CEP_E_ARG, "bad state blob");
  const int64_t evw = 8 + 2 * int64_t(ncols);
  const int64_t total = int64_t(CB_HDR) + 3 * int64_t(nhwm) + 4 * int64_t(qlen) + evw * nev + 4 * int64_t(nnode) +
                        4 * int64_t(npred) + nver + int64_t(3) * nst * nseq;
  if (ncols != int(P.coltypes.size()) || nst != P.dev.nstates || total != w) return fail(CEP_E_ARG, "state blob does not match the pattern");
  // buffer-node slot -> (stage name, stage type), as lower_general numbers them (Matched.java:31-35)
  std::vector<std::pair<int, int>> slot(size_t(P.dev.nslots), {0, 0});
  for (const auto& st : P.stages) slot[size_t(P.dev.st[st.id].slot)] = {st.name, st.type};
  const int32_t* hw = b.data() + CB_HDR;
  const int32_t* q = hw + 3 * nhwm;
  const int32_t* ev = q + 4 * qlen;
  const int32_t* nd = ev + int64_t(evw) * nev;
  const int32_t* pr = nd + 4 * nnode;
  const int32_t* vs = pr + 4 * npred;
  const int32_t* ag = vs + nver;
  auto w64 = [](const int32_t* x) { return int64_t(uint64_t(uint32_t(x[0])) | (uint64_t(uint32_t(x[1])) << 32)); };
  std::vector<uint8_t> o;
  auto i32 = [&](int32_t v) { const size_t at = o.size(); o.resize(at + 4); memcpy(o.data() + at, &v, 4); };
  auto i64 = [&](int64_t v) { const size_t at = o.size(); o.resize(at + 8); memcpy(o.data() + at, &v, 8); };
  auto str = [&](const std::string& t) { i32(int32_t(t.size())); o.insert(o.end(), t.begin(), t.end()); };
  auto version = [&](int at) {
    if (at < 0 || at >= nver || vs[at] < 0 || at + vs[at] >= nver) return false;
    i32(vs[at]);
    for (int d = 1; d <= vs[at]; d++) i32(vs[at + d]);
    return true;
  };
  i32(int32_t(0x4652434Bu));                        // "KCRF"
  i32(1);
  i32(key);
  i32(ncols);
  i64(w64(b.data() + CB_RUNS_LO));
  i32(nhwm);
  for (int h = 0; h < nhwm; h++) { i32(hw[3 * h]); i64(w64(hw + 3 * h + 1)); }
  i32(nev);
  for (int e = 0; e < nev; e++) {
    const int32_t* x = ev + int64_t(evw) * e;
    i64(w64(x)); i32(x[2]); i32(x[3]); i64(w64(x + 4)); i64(w64(x + 6));
    for (int c = 0; c < ncols; c++) i64(w64(x + 8 + 2 * c));
  }
  i32(qlen);
  for (int r = 0; r < qlen; r++) {
    const int32_t w0 = q[4 * r];
    const int sid = w0 & 0xFF, eps = (w0 >> 8) & 0xFF;
    if (sid >= int(P.stages.size()) || (eps != 0xFF && eps >= int(P.stages.size()))) return fail(CEP_E_ARG, "bad run in state blob");
    if (q[4 * r + 2] < -1 || q[4 * r + 2] >= nev) return fail(CEP_E_ARG, "bad run event in state blob");
    i32(sid);
    i32(eps == 0xFF ? -1 : eps);
    i32(((w0 >> 16) & 1) | (((w0 >> 17) & 1) << 1));
    i64(q[4 * r + 3]);
    i32(q[4 * r + 2]);
    i64(-1);
    if (!version(q[4 * r + 1])) return fail(CEP_E_ARG, "bad version in state blob");
  }
  i32(nnode);
  for (int i = 0; i < nnode; i++) {
    const int32_t* x = nd + 4 * i;
    if (x[0] < 0 || x[0] >= P.dev.nslots) return fail(CEP_E_ARG, "bad node in state blob");
    if (x[1] < 0 || x[1] >= nev) return fail(CEP_E_ARG, "bad node event in state blob");
    str(P.names[size_t(slot[size_t(x[0])].first)]);
    i32(slot[size_t(x[0])].second);
    i32(x[1]);
    i64(x[2]);
    int cnt = 0;
    bool bad = false;
    for (int pi = x[3]; pi >= 0; pi = pr[4 * pi + 3])   // a link out of the list, or a cycle: malformed
      if (pi >= npred || ++cnt > npred) { bad = true; break; }
    if (bad) return fail(CEP_E_ARG, "bad predecessor list in state blob");
    i32(cnt);
    for (int pi = x[3]; pi >= 0; pi = pr[4 * pi + 3]) {
      const int32_t* y = pr + 4 * pi;
      if (!version(y[0])) return fail(CEP_E_ARG, "bad version in state blob");
      const bool has = y[1] >= 0;
      if (y[1] >= P.dev.nslots) return fail(CEP_E_ARG, "bad predecessor in state blob");
      if (has && (y[2] < 0 || y[2] >= nev)) return fail(CEP_E_ARG, "bad predecessor event in state blob");
      i32(has ? 1 : 0);
      str(has ? P.names[size_t(slot[size_t(y[1])].first)] : std::string());
      i32(has ? slot[size_t(y[1])].second : 0);
      i32(has ? y[2] : -1);
    }
  }
  int32_t nagg = 0;
  for (int64_t i = 0; i < int64_t(nst) * nseq; i++) {
    if (ag[3 * i] < 0 || ag[3 * i] > 3) return fail(CEP_E_ARG, "bad aggregate type in state blob");   // 1 int, 2 long, 3 double
    nagg += ag[3 * i] != 0;
  }
  i32(nagg);
  for (int sq = 0; sq < nseq; sq++)
    for (int st = 0; st < nst; st++) {
      const int32_t* a = ag + (int64_t(sq) * nst + st) * 3;
      if (!a[0]) continue;                          // unset: States.get would throw
      str(P.states[size_t(st)]);
      i64(sq);
      i32(a[0]);
      i64(w64(a + 1));
    }
  *needed = o.size();
  if (!out) return CEP_OK;
  if (cap < o.size()) return fail(CEP_E_ARG, "buffer too small");
  memcpy(out, o.data(), o.size());
  return CEP_OK;
}

int cep_state_import_keys(cep_session* s, const void* const* blobs, const size_t* lens, const int32_t* keys,
                          int64_t n) {
  int rc = need_carry(s);
  if (rc) return rc;
  if (n < 0 || (n > 0 && (!blobs || !lens || !keys))) return fail(CEP_E_ARG, "null argument");
  // one multi-key blob with the keys renumbered, then the ordinary import
  std::vector<uint8_t> all(20);
  const uint32_t magic = halo_session(s) ? kHaloMagic : tail_session(s) ? kTailMagic : kStateMagic, ver = 1;
  int64_t base = 0;
  int32_t nk = 0;
  for (int64_t i = 0; i < n; i++) {
    const uint8_t* p = static_cast<const uint8_t*>(blobs[i]);
    if (!p || lens[i] < 20) return fail(CEP_E_ARG, "bad state blob");
    uint32_t m, v;
    int64_t b;
    int32_t cnt;
    memcpy(&m, p, 4); memcpy(&v, p + 4, 4); memcpy(&b, p + 8, 8); memcpy(&cnt, p + 16, 4);
    if (m != magic || v != 1 || cnt > 1) return fail(CEP_E_ARG, "cep_state_import_keys takes single-key blobs of this session's kind");
    if (keys[i] < 0 || keys[i] >= s->opts.max_keys) return fail(CEP_E_ARG, "key id out of [0, max_keys)");
    base = std::max(base, b);
    if (cnt == 0) continue;
    const size_t at = all.size();
    all.insert(all.end(), p + 20, p + lens[i]);
    memcpy(&all[at], &keys[i], 4);
    nk++;
  }
  memcpy(&all[0], &magic, 4); memcpy(&all[4], &ver, 4); memcpy(&all[8], &base, 8); memcpy(&all[16], &nk, 4);
  return cep_state_import(s, all.data(), all.size());
}

int cep_state_positions(const void* buf, size_t len, int64_t* out, int64_t cap, int64_t* n) {
  if (!buf || !n || len < 20) return fail(CEP_E_ARG, "bad state blob");
  const uint8_t* p = static_cast<const uint8_t*>(buf);
  uint32_t magic;
  int32_t nkeys;
  memcpy(&magic, p, 4); memcpy(&nkeys, p + 16, 4);
  if ((magic != kStateMagic && magic != kHaloMagic && magic != kTailMagic) || nkeys < 0) return fail(CEP_E_ARG, "bad state blob");
  int64_t cnt = 0;
  size_t at = 20;
  auto put = [&](int64_t v) { if (out && cnt < cap) out[cnt] = v; cnt++; };
  for (int32_t i = 0; i < nkeys; i++) {
    if (at + 8 > len) return fail(CEP_E_ARG, "truncated state blob");
    int32_t w;
    memcpy(&w, p + at + 4, 4);
    if (magic == kTailMagic) {                       // key, records, words per record, 0, records (pos first)
      int32_t rw;
      if (at + 16 > len) return fail(CEP_E_ARG, "truncated state blob");
      memcpy(&rw, p + at + 8, 4);
      if (w <= 0 || rw < 5 || at + 16 + size_t(w) * size_t(rw) * 8 > len) return fail(CEP_E_ARG, "truncated state blob");
      for (int32_t j = 0; j < w; j++) {
        int64_t v;
        memcpy(&v, p + at + 16 + size_t(j) * size_t(rw) * 8, 8);
        put(v);
      }
      at += 16 + size_t(w) * size_t(rw) * 8;
      continue;
    }
    if (magic == kHaloMagic) {                       // key, records, masks, positions[records]
      if (w < 0 || at + 16 + 8 * size_t(w) > len) return fail(CEP_E_ARG, "truncated state blob");
      for (int32_t j = 0; j < w; j++) {
        int64_t v;
        memcpy(&v, p + at + 16 + 8 * size_t(j), 8);
        put(v);
      }
      at += 16 + 8 * size_t(w);
      continue;
    }
    if (w < CB_HDR || at + 8 + 4 * size_t(w) > len) return fail(CEP_E_ARG, "truncated state blob");
    const int32_t* b = reinterpret_cast<const int32_t*>(p + at + 8);   // 4-byte aligned in every blob we write
    int32_t hdr[CB_HDR];
    memcpy(hdr, b, sizeof hdr);
    const int32_t nev = hdr[CB_NEV];
    if (nev > 0) {                                   // events: stream position (int64) first, carry_evw words each
      const int64_t evw = 8 + 2 * int64_t(hdr[CB_NCOLS]);
      const int64_t e0 = CB_HDR + 3 * int64_t(hdr[CB_NHWM]) + 4 * int64_t(hdr[CB_QLEN]);
      if (e0 + nev * evw > w) return fail(CEP_E_ARG, "bad state blob");
      for (int32_t e = 0; e < nev; e++) {
        uint32_t lo, hi;
        memcpy(&lo, b + e0 + e * evw, 4); memcpy(&hi, b + e0 + e * evw + 1, 4);
        put(int64_t(uint64_t(lo) | (uint64_t(hi) << 32)));
      }
    }
    at += 8 + 4 * size_t(w);
  }
  *n = cnt;
  return out && cnt > cap ? fail(CEP_E_ARG, "output too small") : CEP_OK;
}

int cep_session_set_max_key_words(cep_session* s, int64_t words) {
  if (!s || words < 0) return fail(CEP_E_ARG, "bad argument");
  s->opts.max_key_words = words;
  return CEP_OK;
}

}  // extern "C"

// runs_dev.h — device engine of the deterministic-runs path (see runs.hip for
// the algorithm).  Templated on the program table Tab:
//   InterpTab (interp.h)  the pattern's DevProgram in device memory, predicates
//                         and folds interpreted (libkcep.so's built-in kernels)
//   JitTab (jit.cpp)      the DevProgram as a compile-time constant and the
//                         predicates as straight-line code (per-pattern kernels)
#pragma once
#include "interp.h"

#ifndef KCEP_UNROLL
#ifdef KCEP_JIT
#define KCEP_UNROLL _Pragma("unroll")
#else
#define KCEP_UNROLL
#endif
#endif

namespace kcep {


constexpr int RT = 256;

// aggregates of one run: (boxed type, value bits) per state, 0 = null
struct RunState {
  int32_t tag[RUNS_MAX_STATES];
  int64_t val[RUNS_MAX_STATES];
};

constexpr int RUNS_COLCACHE = 4;   // columns of the current record held in registers

// Record indices are 32-bit in the engine (a runs batch holds < 2^31 records, abi.cpp push_runs): half
// the VALU work of 64-bit index arithmetic and comparisons in the per-record loop.
__device__ __forceinline__ int64_t load_col(const RunsArgs& A, int col, int type, int32_t g) {
  const void* c = A.cols[col];
  if (type == T_I32) return static_cast<const int32_t*>(c)[g];
  return static_cast<const int64_t*>(c)[g];
}

struct RunEnv {
  const RunsArgs& A;
  int32_t g;
  const RunState& rs;
  int err;
  bool in_fold;
  int32_t curr_tag;
  int64_t curr;
  const int64_t* cv;               // the record's first RUNS_COLCACHE columns, loaded once per step
  __device__ __forceinline__ int64_t field(int col, int t) {
    if (col < RUNS_COLCACHE) {
      int64_t v = 0;
#pragma unroll
      for (int i = 0; i < RUNS_COLCACHE; i++)
        if (i == col) v = cv[i];
      return v;
    }
    const void* c = A.cols[col];
    if (t == T_I32) return static_cast<const int32_t*>(c)[g];
    return static_cast<const int64_t*>(c)[g];
  }
  __device__ __forceinline__ int64_t key() { return A.key[g]; }
  __device__ __forceinline__ int64_t ts() { return A.ts ? A.ts[g] : A.pos ? A.pos[g] : A.base + g; }
  __device__ __forceinline__ int64_t off() { return A.offset ? A.offset[g] : A.pos ? A.pos[g] : A.base + g; }
  __device__ __forceinline__ int64_t part() { return A.partition ? A.partition[g] : 0; }
  __device__ __forceinline__ int32_t topic() { return A.topic ? A.topic[g] : 0; }
  __device__ __forceinline__ bool state(int idx, int32_t& tag, int64_t& v) {
    tag = 0;
    v = 0;
#pragma unroll
    for (int i = 0; i < RUNS_MAX_STATES; i++)                // registers: select, no dynamic index
      if (i == idx) { tag = rs.tag[i]; v = rs.val[i]; }
    return true;
  }
  __device__ __forceinline__ bool seq_avg(int, int64_t&) { err = CEP_E_UNSUPPORTED; return false; }
  __device__ __forceinline__ bool seq_agg(int, int, int, int64_t&) { err = CEP_E_UNSUPPORTED; return false; }
  __device__ __forceinline__ void fail(int code) { err = code; }
};

__device__ __forceinline__ bool wave_any(bool x) { return __builtin_amdgcn_ballot_w64(x) != 0; }

// Runs walked in lock-step by the whole wave: one record per step for every
// live lane, and per record the stages in descending id (PROCEED /
// SKIP_PROCEED always lead to a smaller id, so a recursion on the same record
// is met later in the same sweep).  For each stage every edge predicate is
// evaluated (matchEdgesAndGet, NFA.java:371-384) by the lanes waiting there,
// then the one consuming edge (BEGIN / TAKE, with the stage's folds,
// :319-321) or the one recursion edge applies.
//
// A wave owns a chunk of A.chunk items (start records, or completed runs to
// write); a lane whose run ends takes the next item of the chunk at the next
// step, so the wave does not idle behind its longest run.  Large batches take
// RUNS_CHUNK items per wave (fewer, longer-lived waves: r02 sweep 1.86 ms at
// 1024 vs 2.59 at 128 on C3); a batch too small to give every SIMD three waves
// that way takes smaller chunks (runs_chunk).

// the args a runs_sim launch runs on: the record count from the device when the host passed a bound
__device__ __forceinline__ RunsArgs runs_args_dev(const RunsArgs& A) {
  RunsArgs a = A;
  if (A.n_dev) a.n = *A.n_dev < A.n ? *A.n_dev : A.n;
  return a;
}

struct RunResult {
  int32_t end;        // record where the run consumed its last stage, -1 none
  int32_t fail_at;    // record whose evaluation raised, -1 none
  int err;
  bool open;          // the run consumed its key's last record of the batch and waits for the next
};

// item(i, &j, &stop): start record and last record to walk of item i (false: skip)
// done(i, RunResult); on_consume(i, record, stage)
template <class Tab, class Item, class Done, class Consume>
__device__ __forceinline__ void run_engine(const Tab& T, const RunsArgs& A, int32_t i0, int32_t i1, Item&& item, Done&& done,
                                           Consume&& on_consume) {
  const auto& P = T.prog();                               // stage ids are wave-uniform: scalar reads
  RunState rs;
#pragma unroll
  for (int q = 0; q < RUNS_MAX_STATES; q++) { rs.tag[q] = 0; rs.val[q] = 0; }
  RunResult res{-1, -1, 0, false};
  bool alive = false;
  int32_t idx = -1, r = 0, stop = 0;
  const int32_t n = int32_t(A.n);
  int ps = -1, cur = -1;
  int32_t k = 0;
  int32_t next = i0;                                          // wave-uniform: next unassigned item
  const int nst = P.nstages;
  const int ncc = P.ncols < RUNS_COLCACHE ? P.ncols : RUNS_COLCACHE;
  int64_t cv[RUNS_COLCACHE];
#pragma unroll
  for (int q = 0; q < RUNS_COLCACHE; q++) cv[q] = 0;
  // the record's key and cached columns, issued together (one memory latency per step)
  auto load_record = [&](int32_t g, int32_t* kk) {
    *kk = A.key[g];
#pragma unroll
    for (int q = 0; q < RUNS_COLCACHE; q++)
      if (q < ncc) cv[q] = load_col(A, q, P.coltype[q], g);
  };
  for (;;) {
    // refill idle lanes from the chunk, in lane order
    const uint64_t idle = __builtin_amdgcn_ballot_w64(!alive);
    if (idle && next < i1) {
      const int rank = __builtin_amdgcn_mbcnt_hi(uint32_t(idle >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(idle), 0));
      if (!alive) {
        const int32_t it = next + rank;
        int32_t j = 0;
        if (it < i1 && item(it, &j, &stop)) {
          idx = it;
          alive = true;
          r = j;
          ps = P.begin;                                      // the begin run's evaluation on record j
          cur = -1;
          load_record(j, &k);
          res = RunResult{-1, -1, 0, false};
#pragma unroll
          for (int q = 0; q < RUNS_MAX_STATES; q++) { rs.tag[q] = 0; rs.val[q] = 0; }
        }
      }
      next += __popcll(idle);
    }
    if (!__builtin_amdgcn_ballot_w64(alive)) {
      if (next >= i1) break;
      continue;
    }
    const int32_t gs = alive ? r : i0;                          // a loadable record for idle lanes (JitTab)
#ifdef KCEP_JIT
    // Every stage's edge predicates at once, on the record and the run state as the sweep finds them.  A
    // lane's state changes only when it consumes, after which it evaluates nothing more in the sweep, and a
    // PROCEED stays on the same record: these are the values the stage loop would compute where the run
    // goes, and in one basic block the compiler shares their subexpressions across stages (C3: the running
    // average's divide once per record instead of once per visited stage).  Predicates have no side
    // effects; a stage's first failing edge (later edges inactive, matchEdgesAndGet NFA.java:371-384)
    // raises only where the run visits the stage.
    uint32_t pre_m[NFA_MAX_STAGES];
    int pre_e[NFA_MAX_STAGES];
    KCEP_UNROLL
    for (int s = nst - 1; s >= 1; s--) {
      const auto& st = P.st[s];
      uint32_t matched = 0;
      int err = 0;
      KCEP_UNROLL
      for (int e = 0; e < st.nedges; e++) {
        if (st.pred[e] < 0) { matched |= 1u << e; continue; }
        RunEnv env{A, gs, rs, 0, false, 0, 0, cv};
        int64_t v;
        if (!T.eval(st.pred[e], env, true, v)) {
          if (!err) err = env.err ? env.err : CEP_E_BAD_IR;
        } else if (!err && v) {
          matched |= 1u << e;
        }
      }
      pre_m[s] = matched;
      pre_e[s] = err;
    }
#endif
    // the stage a lane consumed at in this sweep: it evaluates nothing more in the sweep, so on_consume
    // runs once after the stage loop (one copy of its branches instead of one per unrolled stage)
    int cstage = -1;
    KCEP_UNROLL
    for (int s = nst - 1; s >= 1; s--) {
      const bool here = alive && ps == s;
      if (!wave_any(here)) continue;
      const auto& st = P.st[s];
      uint32_t matched = 0;
      bool ok = true;
#ifdef KCEP_JIT
      matched = pre_m[s];
      if (here && pre_e[s]) { ok = false; res.err = pre_e[s]; }
#else
      KCEP_UNROLL
      for (int e = 0; e < st.nedges; e++) {
        if (st.pred[e] < 0) { matched |= 1u << e; continue; }
        RunEnv env{A, gs, rs, 0, false, 0, 0, cv};
        int64_t v;
        const bool act = here && ok;
        if (!T.eval(st.pred[e], env, act, v)) {
          if (act) { ok = false; res.err = env.err; }
        } else if (act && v) {
          matched |= 1u << e;
        }
      }
#endif
      // the last matching consuming edge's target and the last matching recursion edge's (-2: none),
      // as selects: the stage's edges and ops are constants in a per-pattern kernel
      int take = -1, tk_to = 0, rec_to = -2;
      KCEP_UNROLL
      for (int e = 0; e < st.nedges; e++) {
        const bool m = (matched >> e) & 1;
        const int op = st.op[e];
        if (op == E_BEGIN || op == E_TAKE) {
          const int to = op == E_TAKE ? s : st.target[e];
          take = m ? e : take;
          tk_to = m ? to : tk_to;
        } else if (op == E_PROCEED || op == E_SKIP_PROCEED) {
          rec_to = m ? st.target[e] : rec_to;
        }
      }
      const bool consume = here && ok && take >= 0;
      // evaluateAggregates (:362-369): a fold that raises stops the later ones; the state updates as selects
      if (st.nfolds > 0 && wave_any(consume)) {
        KCEP_UNROLL
        for (int f = 0; f < st.nfolds; f++) {
          const int sidx = st.fold_state[f];
          int32_t ct = 0;
          int64_t cvv = 0;
#pragma unroll
          for (int q = 0; q < RUNS_MAX_STATES; q++)
            if (q == sidx) { ct = rs.tag[q]; cvv = rs.val[q]; }
          RunEnv env{A, gs, rs, 0, true, ct, cvv, cv};
          int64_t v = 0;
          const bool act = consume && ok;
          const bool good = T.eval(st.fold_code[f], env, act, v);
          const bool put = act && good;
          res.err = act && !good ? env.err : res.err;
          ok = act && !good ? false : ok;
          const int32_t ft = st.fold_type[f];
#pragma unroll
          for (int q = 0; q < RUNS_MAX_STATES; q++)
            if (q == sidx) { rs.tag[q] = put ? ft : rs.tag[q]; rs.val[q] = put ? v : rs.val[q]; }
        }
      }
      // the lane's move, branch-free: failed -> finished; consumed -> the next record, or emitted when the
      // edge forwards to $final; a recursion edge -> its target on the same record; no edge -> removed
      const bool cons = here && ok && take >= 0;
      res.fail_at = here && !ok ? r : res.fail_at;
      res.end = cons && tk_to == 0 ? r : res.end;
      cstage = cons ? s : cstage;
      cur = cons ? tk_to : cur;
      ps = !here ? ps : !ok ? -2 : take >= 0 ? (tk_to == 0 ? -2 : -1) : rec_to;
    }
    if (cstage >= 0) on_consume(idx, r, cstage);
    if (alive) {
      if (ps == -1) {                                              // consumed: on to the next record
        r++;
        int32_t kr = k + 1;
        if (r < n && r <= stop) load_record(r, &kr);
        ps = kr == k ? cur : -2;
        if (ps == -2 && r <= stop) res.open = true;                // out of the key's records, not dead
      } else if (ps != -2) {
        ps = -2;                                                   // (a recursion that consumed nothing)
      }
      if (ps == -2) {
        done(idx, res);
        alive = false;
      }
    }
  }
}

// end_of[j] = completing record of the run started at record j (-1 none, -2 open at the key's last
// carried record), and per wave chunk w its completed runs and their total length, stat[w] and
// stat[W + w] (W = the launch's waves: runs_compact places the chunk's runs at the scan of the
// counts, so no per-record flag array and no device-wide scan over it); the same split by the chunk
// the run ENDS in -- this chunk, stat[2W + w] / stat[3W + w], or the next one, stat[4W + w] /
// stat[5W + w] (runs_emit, when every span is shorter than a chunk); the longest completed span
// into *A.max_span.  With A.segs, also the run's consumed stages as segments (so runs_expand writes
// the traversal without walking the run again).  Both are staged in LDS: a lane's segments while its
// run is open (stored once, as two 16-B vectors, when the run completes -- and not at all when it
// dies), the chunk's results until the wave has finished the chunk (then stored coalesced).  Stored
// as they came, every segment word and every result was a partial-line write of its own.
template <class Tab>
__device__ __forceinline__ void runs_sim_body(const Tab& T, const RunsArgs& A, int64_t* __restrict__ stat,
                                              int32_t* __restrict__ end_of) {
  __shared__ __attribute__((aligned(16))) uint16_t s_seg[RT][RUNS_MAX_SEGS];
  __shared__ int32_t s_end[RT / 64][RUNS_CHUNK];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t wave = (int64_t(blockIdx.x) * RT + threadIdx.x) >> 6;
  const int64_t i0l = wave * A.chunk;
  const int32_t i0 = int32_t(i0l < A.n ? i0l : A.n), i1 = int32_t(i0l + A.chunk < A.n ? i0l + A.chunk : A.n);
  uint16_t* const myseg = s_seg[threadIdx.x];
  if (i0 < A.n) {
    int32_t seg_item = -1;                                      // the lane's current start record
    int seg_last = -1, seg_n = 0;
    run_engine(
        T, A, i0, i1, [&](int32_t i, int32_t* j, int32_t* stop) { *j = i; *stop = INT32_MAX; return true; },
        [&](int32_t i, const RunResult& res) {
          // carry: a run that ended in the carried records was emitted by an earlier batch; -2 marks a
          // run still open at its key's last record (its start begins the key's next carried tail)
          const bool old_end = A.pos && res.end >= 0 && A.pos[res.end] < A.emit_from;
          s_end[wv][i - i0] = old_end ? -1 : res.open ? -2 : int32_t(res.end);
          if (res.fail_at >= 0 && !(A.pos && A.pos[res.fail_at] < A.emit_from)) {
            A.err_code[i] = res.err;
            atomicMin(A.err_min, (unsigned long long)(int64_t(res.fail_at) << 31 | i));
            if (A.err_list) {
              const unsigned long long q = atomicAdd(A.err_n, 1ull);
              if (int64_t(q) < A.err_cap) {
                unsigned long long* e = A.err_list + 3 * q;
                e[0] = (unsigned long long)(int64_t(res.fail_at) << 31 | i);
                e[1] = (unsigned long long)(A.pos ? A.pos[res.fail_at] : res.fail_at);
                e[2] = (unsigned long long)(uint32_t(A.key[i])) << 32 | uint32_t(res.err);
              }
            }
          }
          // (storing every item's slot, terminators for runs that did not complete, so that the segment
          // words go out in full lines: C3 runs_sim WRITE 178 -> 229 MB -- the completed runs' partial lines
          // cost less than the dense array)
          if (A.segs && res.end >= 0 && !old_end) {
            // the run's segments, the ones past its last as the terminator (and padding) 0xFFFF, in
            // registers (a fill loop over the lane's LDS words cost the wave a loop per finishing lane);
            // one 8- or 16-byte store per completed run (by start record)
            const int sn = seg_item == i ? seg_n : 0;
            uint4 w = *reinterpret_cast<const uint4*>(myseg);
            auto pad = [sn](uint32_t v, int q) {
              return v | (q < sn ? 0u : 0xFFFFu) | (q + 1 < sn ? 0u : 0xFFFF0000u);
            };
            w.x = pad(w.x, 0);
            w.y = pad(w.y, 2);
            w.z = pad(w.z, 4);
            w.w = pad(w.w, 6);
            if (A.segn == 4) *reinterpret_cast<uint2*>(A.segs + i * 4) = make_uint2(w.x, w.y);
            else *reinterpret_cast<uint4*>(A.segs + i * 8) = w;
          }
        },
        [&](int32_t i, int32_t r, int stage) {
          if (!A.segs) return;
          if (i != seg_item) { seg_item = i; seg_last = -1; seg_n = 0; }
          if (stage == seg_last) return;
          seg_last = stage;
          const int32_t off = r - i;
          if (seg_n >= A.segn || off >= 4096 || stage >= 16) { atomicOr(A.seg_over, 1ull); return; }
          myseg[seg_n++] = uint16_t(stage << 12 | off);
        });
  }
  __syncthreads();                                              // (every wave reaches it)
  int64_t cnt = 0, len = 0, span = 0, cnt_own = 0, len_own = 0;
  for (int64_t k = lane; k < i1 - i0; k += 64) {
    const int32_t e = s_end[wv][k];
    end_of[i0 + k] = e;                                         // (-2: open, carried)
    if (e >= 0) {
      const int64_t d = int64_t(e) - (i0 + k);
      cnt++;
      len += d + 1;
      span = d > span ? d : span;
      if (e < i1) { cnt_own++; len_own += d + 1; }
    }
  }
  if (i0 >= A.n) return;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    cnt += __shfl_xor(cnt, d, 64);
    len += __shfl_xor(len, d, 64);
    cnt_own += __shfl_xor(cnt_own, d, 64);
    len_own += __shfl_xor(len_own, d, 64);
    const int64_t y = __shfl_xor(span, d, 64);
    span = y > span ? y : span;
  }
  if (lane == 0) {
    const int64_t W = int64_t(gridDim.x) * (RT / 64);
    stat[wave] = cnt;
    stat[W + wave] = len;
    stat[2 * W + wave] = cnt_own;
    stat[3 * W + wave] = len_own;
    stat[4 * W + wave] = cnt - cnt_own;
    stat[5 * W + wave] = len - len_own;
    // the longest span: a plain read first, so that the chunks agreeing with it add no contended atomic
    // (one atomicMax per 256 records on one word cost runs_compact ~400 us at 10 M records)
    if (span > 0 && (unsigned long long)span > __hip_atomic_load(A.max_span, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
      atomicMax(A.max_span, (unsigned long long)span);
  }
}

struct WriteArgs {
  RunsArgs R;
  const unsigned long long* sorted;
  int64_t nm;
  const int64_t* ent_off;        // exclusive scan of lengths
  int64_t* match_record;
  int32_t* match_key;
  int64_t* ent_off_out;
  int32_t* ent_name;
  int64_t* ent_record;
};

template <class Tab>
__device__ __forceinline__ void put_entry(const Tab& T, const WriteArgs& W, int64_t at, int stage, int64_t r) {
  W.ent_name[at] = T.prog().st[stage].name;
  W.ent_record[at] = W.R.pos ? W.R.pos[r] : W.R.base + r;
}

// re-walk each completed run: traversal order is final stage first (peek :176-201)
template <class Tab>
__device__ __forceinline__ void runs_write_body(const Tab& T, const WriteArgs& W) {
  const int64_t wave = (int64_t(blockIdx.x) * RT + threadIdx.x) >> 6;
  if (wave * W.R.chunk >= W.nm) return;
  const int32_t i0 = int32_t(wave * W.R.chunk), i1 = int32_t(i0 + W.R.chunk < W.nm ? i0 + W.R.chunk : W.nm);
  run_engine(
      T, W.R, i0, i1,
      [&](int32_t m, int32_t* j, int32_t* stop) {
        const unsigned long long kv = W.sorted[m];
        *j = int32_t(kv & 0x7FFFFFFFull);
        *stop = int32_t(kv >> 31);
        W.match_record[m] = W.R.pos ? W.R.pos[*stop] : W.R.base + *stop;
        W.match_key[m] = W.R.key[*j];
        W.ent_off_out[m] = W.ent_off[m];
        return true;
      },
      [](int32_t, const RunResult&) {},
      [&](int32_t m, int32_t r, int stage) {
        const int64_t end = int64_t(W.sorted[m] >> 31);
        put_entry(T, W, W.ent_off[m] + (end - r), stage, r);
      });
}

}  // namespace kcep

// kcep_dev.h — the compiled pattern as the kernels see it, and the launch
// argument blocks of the general and runs kernels.  Plain C++ with fixed-size
// arrays only: the same text is compiled into libkcep.so by hipcc and into the
// per-pattern kernels by hiprtc (jit.cpp), so it includes nothing but <stdint.h>.
#pragma once
#include <stdint.h>

#if defined(__HIP__) || defined(__HIPCC_RTC__)
#define KCEP_HD __host__ __device__
#else
#define KCEP_HD
#endif

namespace kcep {

// ---- static types / opcodes of the expression IR (kcep/expr.py) ----
enum : uint8_t { T_BOOL = 0, T_I32 = 1, T_I64 = 2, T_F64 = 3 };
enum : uint8_t {
  OP_TRUE = 0x01, OP_FALSE = 0x02, OP_CONST_I32 = 0x03, OP_CONST_I64 = 0x04, OP_CONST_F64 = 0x05,
  OP_FIELD = 0x10, OP_EV_KEY = 0x11, OP_EV_TS = 0x12, OP_EV_TOPIC_EQ = 0x13, OP_EV_OFFSET = 0x14,
  OP_EV_PARTITION = 0x15, OP_STATE_GET = 0x20, OP_STATE_GET_OR_ELSE = 0x21, OP_FOLD_CURR = 0x22,
  OP_SEQ_AVG = 0x23, OP_SEQ_AGG = 0x24, OP_NOT = 0x30, OP_AND = 0x31, OP_OR = 0x32, OP_ADD = 0x40, OP_SUB = 0x41,
  OP_MUL = 0x42, OP_DIV = 0x43, OP_REM = 0x44, OP_NEG = 0x45, OP_EQ = 0x50, OP_NE = 0x51,
  OP_LT = 0x52, OP_LE = 0x53, OP_GT = 0x54, OP_GE = 0x55, OP_CAST = 0x60
};

// Stage.StateType (nfa/Stage.java:243-245) and EdgeOperation (nfa/EdgeOperation.java:20-46)
enum : uint8_t { ST_BEGIN = 0, ST_NORMAL = 1, ST_FINAL = 2 };
enum : uint8_t { E_BEGIN = 0, E_TAKE = 1, E_PROCEED = 2, E_SKIP_PROCEED = 3, E_IGNORE = 4 };
enum : uint8_t { S_STRICT = 0, S_NEXT = 1, S_ANY = 2, S_NULL = 0xFF };

// ---- general NFA path: flat device program ----
// Predicates and folds become postfix bytecode over 64-bit slots (ints kept
// sign-extended, doubles as bits); the compiler inserts Java's binary numeric
// promotions.  AND/OR short-circuit with conditional jumps so that exceptions
// (unknown state, / by zero, ...) are raised exactly when Java would.
enum : uint8_t {
  BC_END = 0, BC_PUSH, BC_FIELD, BC_EV_KEY, BC_EV_TS, BC_EV_OFFSET, BC_EV_PARTITION, BC_TOPIC_EQ,
  BC_STATE_GET, BC_STATE_GET_OR_ELSE, BC_FOLD_CURR, BC_SEQ_AVG, BC_SEQ_AGG, BC_NOT, BC_JZ_KEEP, BC_JNZ_KEEP, BC_POP,
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

// SequenceMatcher reductions (OP_SEQ_AGG kind): over the partial Sequence's events, or over one
// stage's (Sequence.getByName(stage).getEvents(), a TreeSet: Sequence.java:57-60, 130-167)
enum : int { SEQ_SUM = 1, SEQ_COUNT = 2, SEQ_MIN = 3, SEQ_MAX = 4, SEQ_FIRST = 5, SEQ_LAST = 6 };
constexpr int SEQ_ANY_STAGE = -1;     // BC_SEQ_AGG stage word: no stage filter (-2: a stage that does not exist)

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
// per key segment: live-run max, run evaluations, wall clock (100 MHz), then (profiling kernels; -1
// otherwise) shader clocks in evaluate / predicates / buffer put+branch / removePattern /
// matchConstruction / first_compatible / add_pred / version copies, and counts of first_compatible
// calls / pred entries examined / digit-by-digit checks, reserved (0), the key's workspace words (wave
// scratch + pool), then (profiling kernels) those words per allocation kind -- first workspace, match
// output, heap, run queues, private lists, aggregates, other (nfa_dev.h AK_*) -- and the batch pool's
// share of them (the rest came from the wave's recycled scratch region)
constexpr int NFA_PROFILE_W = 24;

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
KCEP_HD inline int32_t carry_evw(int32_t ncols) { return 8 + 2 * ncols; }

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
  int32_t nseg;                   // key segments (an upper bound when nseg_dev is set)
  const int64_t* nseg_dev;        // wave kernel: the segment count on the device (nullptr: nseg is exact)
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
  int64_t* res_words;             // per segment: its matches' entries
  int64_t* res_out;               // device address of the key's match headers (4 words per match, nfa_dev.h)
  int64_t* res_ent;               // ... and of their entries (3 words per entry)
  int32_t* res_err;
  int64_t* res_err_rec;
  int32_t* flags;                 // [0] pool overflow lanes, [1] carry-pool overflow lanes, [2] bad key ids,
                                  // [3] live-run high-water mark over the batch's keys
  int64_t* profile;               // CEP_SESSION_PROFILE: NFA_PROFILE_W words per segment (nfa_dev.h)
  int32_t spread;                 // key segments per wave (1..64)
  int32_t wave_agg;               // wave kernel: bit 0 the pattern folds / reads / copies aggregates (rounds
                                  // check for runs sharing a sequence), bit 1 it has SequenceMatchers
  int32_t last_attempt;           // 1: no pool regrowth follows -- an overflowing key reports CEP_E_RUN_CAPACITY
  int32_t* seg_next;              // wave kernel: the next key segment a persistent wave takes (zeroed before)
  const int32_t* seg_order;       // wave kernel: the segments in the order the waves take them (null: as they
                                  // come), heaviest estimated first (nfa_order_*)
  uint8_t* seg_bucket;            // nfa_order_count's estimate per segment (the placement reads it)
  int32_t* scratch;               // wave kernel: one recycled workspace region per workgroup (nfa_wave.h) ...
  int64_t scratch_words;          // ... of this many words (0: none)
  int64_t max_key_words;          // per-key workspace cap in words (0 = none): over it, CEP_E_RUN_CAPACITY
  unsigned long long* err_any;    // set when any key reports an exception (the host reads res_err only then)
  const int64_t* pos;             // stream position of each batch record (CEP_BATCH_ARRIVAL_ORDER: base + its
                                  // arrival index); null: base + record index
};
// a batch record's stream position (emitted entries, carried events, exception records)
__device__ __forceinline__ int64_t a_pos(const NfaArgs& A, int64_t g) { return A.pos ? A.pos[g] : A.base + g; }

// deterministic-runs path (runs.hip)
struct RunsArgs {
  const DevProgram* P;
  const int32_t* key;
  const int32_t* topic;
  const int32_t* partition;
  const int64_t* offset;
  const int64_t* ts;
  const void* cols[16];
  int64_t n;                      // records (the grid and the chunk statistics' layout follow it) ...
  const int64_t* n_dev;           // ... or, when set, an upper bound, the count itself on the device
  int64_t base;
  unsigned long long* nmatch;     // match counter (append position)
  unsigned long long* match_key;  // appended (end << 31 | start), sorted afterwards
  int64_t match_cap;
  unsigned long long* err_min;    // min over failing runs of (record << 31 | start)
  int32_t* err_code;              // per start record (valid where it failed)
  // every failing run, appended: {record << 31 | start, stream position of the record, key << 32 | code}
  // (the host keeps each key's first -- a batch grouped by key fails first in ARRIVAL order at the
  // smallest of the keys' first failures, cep_batch_errors); err_n counts them, err_cap bounds the list
  unsigned long long* err_list;
  unsigned long long* err_n;
  int64_t err_cap;
  // runs_sim: the stages a run consumed, as up to segn (4 or 8) segments per start record j:
  // segs[j * segn + i] = stage << 12 | offset of the segment's first record from j (stage < 16, offset
  // < 4096), terminated by 0xFFFF when shorter (a run's consumed stages never increase, runs.hip); null: off
  uint16_t* segs;
  int32_t segn;
  unsigned long long* seg_over;   // set when a run needs more segments, a stage >= 16 or an offset >= 4096
  // carry sessions (runs.hip, carried tails): stream position of every record (null: base + index);
  // runs ending or failing at a position < emit_from were handled by an earlier batch (not emitted)
  const int64_t* pos;
  int64_t emit_from;
  int32_t chunk;                  // items per wave (a power of two <= RUNS_CHUNK; runs_chunk)
  unsigned long long* max_span;   // runs_sim: the longest completed run's span (end - start), atomicMax
};
constexpr int RUNS_MAX_SEGS = 8;
constexpr int RUNS_CHUNK = 1024;
KCEP_HD inline int32_t runs_chunk(int64_t items) {
  int32_t c = RUNS_CHUNK;
  while (c > 128 && items < int64_t(c) * 3072) c >>= 1;          // 3 waves on each of 1024 SIMDs
  return c;
}


}  // namespace kcep

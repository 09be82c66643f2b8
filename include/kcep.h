/*
 * kcep.h — C-ABI of libkcep.so, the MI355X-native replacement for the
 * kafkastreams-cep NFA evaluation path.
 *
 * The reference evaluates one record at a time inside
 *   CEPProcessor.process(K,V)            core/.../cep/processor/CEPProcessor.java:134-150
 *     -> NFA.matchPattern(Event)         core/.../cep/nfa/NFA.java:134-149
 * with the pattern compiled once by
 *   new StagesFactory().make(pattern)    core/.../cep/pattern/StagesFactory.java:49-70
 * This library takes the same pattern (as the byte IR produced by the host DSL,
 * kcep/pattern.py) and whole batches of records laid out struct-of-arrays in
 * HBM, grouped by record key in arrival order, and returns the emitted
 * sequences as a CSR.  A JNI / FFM binding for a Java GpuCEPProcessor is shown
 * in INTEGRATION.md.
 *
 * Threading: a session is used by one thread at a time (the reference's
 * CEPProcessor is driven single-threaded by its stream task).  Sessions are
 * independent.  Errors are int status codes; cep_last_error() returns a
 * thread-local message.  Codes mirror the reference exceptions.
 */
#ifndef KCEP_H
#define KCEP_H
#ifndef __HIPCC_RTC__   /* per-pattern kernels (jit.cpp) include this header through hiprtc */
#include <stddef.h>
#endif
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes (the reference throws; we return) */
#define CEP_OK 0
#define CEP_E_INVALID_PATTERN 1   /* StagesFactory.InvalidPatternException  StagesFactory.java:182-191 */
#define CEP_E_UNKNOWN_AGGREGATE 2 /* States.UnknownAggregateException        States.java:80-89 */
#define CEP_E_ILLEGAL_STATE 3     /* missing buffer predecessor  SharedVersionedBufferStoreImpl.java:113-115 */
#define CEP_E_NPE 4               /* NullPointerException (null strategy, null previous stage, ...) */
#define CEP_E_ARITHMETIC 5        /* integer "/ by zero" inside a matcher or aggregator */
#define CEP_E_CLASS_CAST 6        /* state read with another boxed type than it was folded with */
#define CEP_E_INDEX 7             /* DeweyVersion.addRun out of bounds  DeweyVersion.java:62-67 */
#define CEP_E_BAD_IR 8            /* malformed pattern IR */
#define CEP_E_RUN_CAPACITY 9      /* a key exceeded the device run/buffer capacity (per key: cep_opts.max_key_words) */
#define CEP_E_HIP 10              /* HIP runtime error */
#define CEP_E_ARG 11              /* invalid argument */
#define CEP_E_UNSUPPORTED 12      /* pattern feature not lowered to the device */

/* evaluation modes */
#define CEP_MODE_NFA 0            /* in-memory NFA per key (NFATest.java:842-866 semantics) */
#define CEP_MODE_PROCESSOR 1      /* CEPProcessor semantics: null filter, per-topic high-water mark,
                                     run queue round-trips ComputationStageSerde (isIgnored dropped) */

/* column types of the value schema */
#define CEP_T_I32 1
#define CEP_T_I64 2
#define CEP_T_F64 3

/* execution path chosen by cep_session_open */
#define CEP_PATH_STENCIL 1        /* strict single-cardinality patterns: k-event stencil */
#define CEP_PATH_GENERAL 2        /* full NFA: runs, Dewey versions, shared versioned buffer */
#define CEP_PATH_RUNS 4           /* strict patterns whose runs never branch (stateful predicates, folds,
                                     oneOrMore with exclusive TAKE/PROCEED): one lane per start record */
#define CEP_PATH_CHAIN 3          /* strict single-cardinality patterns with optional() stages: the stencil
                                     kernel with deterministic per-start runs (variable-length matches) */

typedef struct cep_pattern cep_pattern;
typedef struct cep_session cep_session;

typedef struct {
  int32_t n_stages;        /* compiled stages incl. $final (Stages.getAllStages().size()) */
  int32_t n_names;         /* distinct stage names; name 0 is "$final" */
  int32_t n_patterns;      /* user stages (select() calls) */
  int32_t n_cols;
  int32_t stencil_ok;      /* 1 if the strict stencil path applies */
  int32_t stencil_k;       /* number of stages of a stencil/chain pattern */
  int32_t chain_ok;        /* 1 if the chain path (strict + optional stages) applies */
  int32_t runs_ok;         /* 1 if the deterministic-runs path applies */
} cep_pattern_info;

typedef struct {
  int32_t device;          /* HIP device ordinal */
  int32_t mode;            /* CEP_MODE_* */
  int32_t force_path;      /* 0 = auto, else CEP_PATH_* */
  int32_t flags;           /* CEP_SESSION_* */
  int64_t max_events;      /* capacity of one batch */
  int64_t max_keys;        /* CEP_SESSION_CARRY: key ids are dense in [0, max_keys) */
  double arena_scale;      /* general path: per-key workspace multiplier (0 = default 1.0) */
  int64_t max_key_words;   /* general path: device workspace words one key may take (0 = no limit but the
                              pool).  A key over it -- or still out of pool after the pool regrowths -- is
                              handed back per key: cep_batch_errors lists it with CEP_E_RUN_CAPACITY at the
                              record where it ran out, its matches before that record are emitted, a carry
                              session keeps its state as of the batch start, and every other key of the
                              batch completes normally.  The host routes that key to the reference CPU path
                              (a key over capacity falls back per key). */
  int64_t max_pool_bytes;  /* general path: device memory the session's NFA workspace may grow to when a batch
                              overflows its pool (0 = a quarter of the device's HBM): the pool plus the wave
                              kernel's per-workgroup scratch regions.  Past it the overflowing keys are handed
                              back per key as above.  The next batches start from the grown size (no re-run
                              per batch); after 4 batches in a row that fit the estimated pool it is given
                              back, so one heavy stretch does not hold the device for the session's lifetime
                              (several sessions share one GPU: one GpuCEPProcessor per stream task) */
} cep_opts;

/* Session flags */
#define CEP_SESSION_CARRY 1  /* keep every key's NFA state across batches, as CEPProcessor does through its
                                NFAStore/buffer/aggregate stores (CEPProcessor.java:111-124, 144-147): a batch
                                continues each key's runs, Dewey versions, buffer and folds where the previous
                                one stopped.  Record positions in cep_matches are then stream positions
                                (records pushed before the batch + index in the batch).  Strict fixed-length
                                patterns (with or without optional() stages) stay on the stencil / chain path,
                                which carries only each key's last K-1 records; patterns of the
                                deterministic-runs path stay on it and carry each key's records from its oldest
                                still-open run on (the runs are simulated again over them; a run that stays open
                                for R records therefore keeps R records of its key carried and re-simulated per
                                batch -- bounded only by the 2^31 records of an extended batch, past which the push
                                fails with CEP_E_RUN_CAPACITY; such patterns, e.g. an unbounded oneOrMore that keeps
                                matching, are better carried on the general path: cep_opts.force_path =
                                CEP_PATH_GENERAL).  Both then take
                                batches without null records (valid) and with per-key increasing offsets
                                (CEP_BATCH_OFFSETS_MONOTONE; the host applies the high-water-mark rule); every
                                other pattern carries its full NFA state on the general path. */

#define CEP_SESSION_INTERPRET 2  /* runs path: use the built-in kernels, which interpret the pattern's predicates
                                    and folds, instead of kernels compiled for the pattern at cep_session_open
                                    (hiprtc; also disabled by the environment variable KCEP_JIT=0) */

#define CEP_SESSION_PROFILE 4    /* general path: record per key segment its live-run high-water mark, run
                                    evaluations and kernel cycles (cep_key_profile) */

#define CEP_SESSION_LANE_NFA 8    /* general path: always one lane per key segment (nfa_kernel) */
#define CEP_SESSION_WAVE_NFA 16   /* general path: always one key per wave with one queued run per lane
                                    (nfa_wave).  By default the wave kernel runs patterns whose keys' runs
                                    can multiply (a skip-till-next / skip-till-any stage) and the lane kernel
                                    the strict ones */

#define CEP_MEM_HOST 0
#define CEP_MEM_DEVICE 1

/* Batch flags */
#define CEP_BATCH_OFFSETS_MONOTONE 1  /* per key and topic, offsets strictly increase (no re-delivery) */
#define CEP_BATCH_DELIVER 2           /* the caller collects this batch (a processor flush): on stencil / chain
                                         carry sessions the device hands the matches to pinned host memory as
                                         part of the push, so cep_collect only waits (one host round trip) */
#define CEP_BATCH_ARRIVAL_ORDER 4     /* CEP_SESSION_CARRY sessions: the records are in arrival order, as
                                         CEPProcessor.process sees them one by one (CEPProcessor.java:134-150),
                                         not grouped by key.  The library groups them by key on the device (a
                                         stable sort), record positions are arrival positions (stream position =
                                         records pushed before + arrival index), and cep_collect returns the
                                         matches in arrival order of their completing record -- per record in
                                         matchPattern's emission order: the order context.forward sends them
                                         (:148) -- with cep_batch_errors in ascending position.  No host sort */

/* One batch of records, struct-of-arrays, grouped by key (each key's records
 * contiguous and in arrival order; or in plain arrival order with CEP_BATCH_ARRIVAL_ORDER).  Replaces a sequence of
 * CEPProcessor.process(key, value) calls; the per-record Event fields of
 * Event.java:27-123 map to key_id/topic/partition/offset/ts, the value's typed
 * fields to cols.  Optional arrays may be NULL: valid -> all records valid,
 * topic/partition -> 0, offset -> record index, ts -> record index. */
typedef struct {
  int64_t n;
  const int32_t* key_id;
  const uint8_t* valid;       /* 0 = null key or value (CEPProcessor.java:136-138) */
  const int32_t* topic;
  const int32_t* partition;
  const int64_t* offset;
  const int64_t* ts;
  int32_t n_cols;
  int32_t mem;                /* CEP_MEM_HOST or CEP_MEM_DEVICE */
  const void* const* cols;    /* n_cols typed column pointers (host array of pointers) */
  uint32_t flags;
  uint32_t reserved;
} cep_batch;

/* Emitted sequences of one batch, library-owned, valid until the next
 * push/collect/close on the session.  Record positions are batch indices, or
 * stream positions on CEP_SESSION_CARRY sessions (an entry may then name a
 * record of an earlier batch).  Match m was emitted while processing
 * record match_record[m] (context.forward order of CEPProcessor.java:148),
 * for key match_key[m].  Its traversal of the shared buffer, final stage
 * first (SharedVersionedBufferStoreImpl.peek :176-201), is
 *   entries [ent_off[m], ent_off[m+1]) : (ent_name[i], ent_record[i])
 * i.e. stage-name id and batch record index.  Sequence.Builder.build(true)
 * (Sequence.java:210-223) groups these by name in reverse order; helpers in
 * kcep/sequence.py do it.  Matches are ordered by key (batch order), and per
 * key in emission order, which is the reference's per-key forward order. */
typedef struct {
  int64_t n_matches;
  int64_t n_entries;
  const int64_t* match_record;
  const int32_t* match_key;
  const int64_t* ent_off;     /* n_matches + 1 */
  const int32_t* ent_name;
  const int64_t* ent_record;
  int32_t path;               /* CEP_PATH_* that produced it */
  int32_t err;                /* first error (reference exception) of the batch, CEP_OK if none */
  int64_t err_record;         /* record that raised it (-1 if none) */
} cep_matches;

/* --- pattern: replaces StagesFactory.make (StagesFactory.java:49-70) --- */
int cep_compile(const uint8_t* ir, size_t len, cep_pattern** out);
void cep_pattern_free(cep_pattern* p);
int cep_pattern_get_info(const cep_pattern* p, cep_pattern_info* out);
const char* cep_pattern_name(const cep_pattern* p, int32_t name_id);
/* Compiled stage `sid` (Stages.getAllStages().get(sid), Stage.java:40-252):
 * name id, StateType (0 BEGIN, 1 NORMAL, 2 FINAL), window, and up to `cap`
 * edges as (EdgeOperation 0 BEGIN 1 TAKE 2 PROCEED 3 SKIP_PROCEED 4 IGNORE,
 * target stage id or -1).  Returns the edge count, or -1 for a bad id. */
int32_t cep_pattern_stage(const cep_pattern* p, int32_t sid, int32_t* name_id, int32_t* type, int64_t* window_ms,
                          int32_t* ops, int32_t* targets, int32_t cap);
/* CEP_OK if a session opened with `session_flags` (CEP_SESSION_CARRY for a processor) runs the pattern on
 * a device path, else CEP_E_UNSUPPORTED with the reason in cep_last_error.  Host-only: the per-query
 * routing decision of a host (lowerable -> GPU, else the reference CEPProcessor) needs no device. */
int cep_pattern_check(const cep_pattern* p, int32_t session_flags);

/* --- session: one per stream task (CEPProcessor.init :88-108) --- */
int cep_session_open(const cep_pattern* p, const cep_opts* opts, cep_session** out);
void cep_session_close(cep_session* s);
int cep_session_path(const cep_session* s);
/* 1 if the session runs kernels compiled for its pattern (see CEP_SESSION_INTERPRET), else 0 */
int cep_session_jit(const cep_session* s);
/* General path: 1 if the session runs one key per wave (kcep_nfa_wave, CEP_SESSION_WAVE_NFA), 0 if one
   key per lane (kcep_nfa_kernel) or another path */
int cep_session_wave(const cep_session* s);
/* General path: kernel attempts the last batch took (1, plus one per pool regrowth re-run); 0 if the last
   batch ran on another path.  cep_last_kernel_ms times the first attempt only. */
int cep_batch_attempts(const cep_session* s);
/* General path: the most live runs (NFA run queue length, NFAStates.java:33-37) any key held during the
   last batch -- C4's run-explosion high-water mark.  -1 if the last batch ran on another path. */
int cep_live_run_hwm(const cep_session* s, int64_t* hwm);
/* Per-batch HIP event timing (cep_last_kernel_ms / cep_last_batch_ms), on by default.  Off, the
   stencil and chain paths put no event packets into the stream; the two timing calls then fail
   with CEP_E_UNSUPPORTED.  A serving host that does not read the timings turns it off. */
int cep_session_set_timing(cep_session* s, int on);
/* Every exception of the last batch, one per failing key: (stream position, CEP_E_* code), in
   ascending position.  cep_collect reports only the earliest in the batch's key-grouped order; a
   host that re-orders a batch by key (GpuCEPProcessor) uses this list to find the first failure in
   arrival order, which is where the reference's process() throws (CEPProcessor.java:134-149).
   Call with records = codes = NULL for the count.  (The runs path lists up to 2^20 failing runs per batch;
   past that it reports the batch's first exception only.) */
int cep_batch_errors(const cep_session* s, int64_t* records, int32_t* codes, int64_t cap, int64_t* n);
/* CEP_SESSION_PROFILE sessions, after a general-path batch: per key segment {key id, live-run
   high-water mark, run evaluations, kernel wall clock (100 MHz ticks), then shader clocks spent in
   NFA.evaluate / edge predicates / buffer put+branch / removePattern / matchConstruction /
   getPointerByVersion scans / predecessor appends / Dewey version copies, then counts of scans /
   predecessor entries examined / digit-by-digit version checks (-1 each when the session runs the
   built-in kernel), then the key's start (wall clock, 100 MHz ticks), the workspace words the key took (wave scratch region + device
   pool), then those words per allocation kind -- first workspace, match output, heap, run queues,
   private run lists / logs, aggregates, other -- and the device pool's share of them (-1 each when the
   session runs the built-in kernel)}; 25 int64 per key;
   out == NULL sets only *n_keys. */
int cep_key_profile(cep_session* s, int64_t* out, int64_t cap, int64_t* n_keys);
/* The HIP source of the pattern's compiled kernels for a path (CEP_PATH_RUNS), NUL-terminated;
   with buf == NULL only *needed is set.  CEP_E_UNSUPPORTED if the path has none for this pattern. */
int cep_pattern_kernel_source(const cep_pattern* p, int path, char* buf, size_t cap, size_t* needed);
/* Generate and compile (gfx950 code object, no device needed) the pattern's kernels for a path. */
int cep_pattern_build_kernels(const cep_pattern* p, int path);

/* --- batch evaluation: replaces NFA.matchPattern per record (NFA.java:134-149) ---
 * Enqueues the match phase on `stream` (a hipStream_t, NULL = default stream)
 * and returns without waiting.  Device-resident batches are read in place.  Host batches (CEP_MEM_HOST)
 * are borrowed only for the call: pageable columns are copied into the session's pinned staging ring
 * before it returns; columns that are themselves pinned are copied from directly and the call returns
 * once that copy is done. */
int cep_push_batch(cep_session* s, const cep_batch* b, void* stream);

/* Number of matches of the last pushed batch, device-resident (int64 on the
 * device) so that a caller can chain work without a host sync. */
const int64_t* cep_device_match_count(const cep_session* s);

/* Waits for the last batch and materialises the host CSR.  A second call before the next push
 * returns the same CSR without touching the device. */
int cep_collect(cep_session* s, cep_matches* out);

/* Host-only consistency check of a CSR before it is walked: ent_off starts at 0, never decreases and ends
 * at n_entries; every match_record and ent_record lies in [0, n_records); every ent_name in [0, n_names).
 * cep_collect applies it to the device-written CSR of the general and runs paths (n_records = the batch,
 * or everything pushed so far on a carry session), so a device fault surfaces as CEP_E_HIP instead of a
 * host crash in the walk (the reference fails the task with an exception,
 * SharedVersionedBufferStoreImpl.java:113-115). */
int cep_csr_check(const cep_matches* m, int64_t n_records, int32_t n_names);

/* Pipelined flushes.  cep_batch_id: the number of the last pushed batch (1, 2, ...).  On stencil / chain carry
 * sessions a CEP_BATCH_DELIVER batch's matches go to one of two host buffers, so a host can push batch i + 1
 * before it collects batch i: cep_collect_batch(id) collects the last batch (as cep_collect) or the delivered
 * batch before it (CEP_E_UNSUPPORTED if that one had more matches than the host buffer holds, 2^20 rows, which
 * are collected only before the next push); cep_batch_ready(id) tells without waiting whether batch id's
 * matches are complete (1) or not yet (0).  The host CSR of cep_collect_batch is valid until the next collect. */
int64_t cep_batch_id(const cep_session* s);
int cep_batch_ready(cep_session* s, int64_t id);
int cep_collect_batch(cep_session* s, int64_t id, cep_matches* out);

/* Order-independent 64-bit checksum of the last batch's matches, computed on
 * the device (matches the oracle's orc_baseline checksum); waits. */
int cep_checksum(cep_session* s, uint64_t* sum, int64_t* n_matches);

/* Kernel timing of the last batch's dominant kernel (HIP events on the launch stream):
 * stencil_kernel on the stencil path, the first nfa_kernel launch on the general path. */
int cep_last_kernel_ms(cep_session* s, float* ms);

/* Device time of the whole last cep_push_batch (staging, segmentation, kernels,
 * regrowth re-runs and compaction), HIP events on the launch stream. */
int cep_last_batch_ms(cep_session* s, float* ms);

/* --- carried state (CEP_SESSION_CARRY): replaces NFAStoreImpl / NFAStates persistence
 * (state/internal/NFAStoreImpl.java:34-85, NFAStates.java:33-109, NFAStateValueSerde.java:77-147)
 * together with the buffer and aggregate stores the runs still reference. ---
 * Serialises the state of keys in [key_lo, key_hi) into buf (library format "KCST"):
 * with buf == NULL only *needed is set.  Fails with CEP_E_ARG if cap < *needed. */
int cep_state_export(cep_session* s, int32_t key_lo, int32_t key_hi, void* buf, size_t cap, size_t* needed);
/* Restores keys from an export (replacing their current state); the stream position
 * continues from the exported one if that is later. */
int cep_state_import(cep_session* s, const void* buf, size_t len);
/* Drops every key's state (a fresh NFAStore). */
int cep_state_clear(cep_session* s);
/* NFA.getRuns() and the run-queue length of a key (NFATest assertNFA, NFATest.java:836-840);
 * *queue_len = -1 if the key has no state yet. */
int cep_key_state(cep_session* s, int32_t key, int64_t* runs, int64_t* queue_len);
/* Stream position the next batch's record 0 gets (0 for sessions without CEP_SESSION_CARRY). */
int64_t cep_stream_position(const cep_session* s);
/* Spill keys to the host, freeing their ids (the reference's NFAStore is an unbounded KV store,
 * NFAStoreImpl.java:34-85; a session holds max_keys ids, so a host with more live keys keeps the cold
 * ones' state itself).  Key keys[i]'s state becomes the self-contained single-key blob
 * (*blobs)[offs[i] .. offs[i+1]) -- "KCST" or "KCSH" as cep_state_export writes it, empty if the key
 * has no state -- and is dropped from the device, so the id starts afresh.  The blobs are
 * library-owned, valid until the next cep_state_evict on the session.  offs has n + 1 entries. */
int cep_state_evict(cep_session* s, const int32_t* keys, int64_t n, const uint8_t** blobs, int64_t* offs);
/* Restores single-key blobs (from cep_state_evict, or a one-key cep_state_export) under the key ids
 * keys[i] -- a spilled key re-admitted under whatever id is free.  Empty blobs are skipped. */
int cep_state_import_keys(cep_session* s, const void* const* blobs, const size_t* lens, const int32_t* keys,
                          int64_t n);
/* The stream positions of every record a state blob (cep_state_export / cep_state_evict) still
 * references -- the records a host must keep to build the Sequences of carried runs (the reference
 * keeps them in its buffer store, MatchedEvent.java:29-34).  out == NULL: only *n. */
int cep_state_positions(const void* blob, size_t len, int64_t* out, int64_t cap, int64_t* n);
/* A key's carried NFA state -- a single-key "KCST" blob from cep_state_evict, typically of a key handed back
 * with CEP_E_RUN_CAPACITY -- written in the reference's own terms ("KCRF", layout in abi.cpp): NFA.runs,
 * the per-topic high-water marks, the run queue (stage, epsilon target, isBranching / isIgnored, sequence,
 * last event, Dewey digits; ComputationStage.java:30-185, NFAStates.java:33-109), the buffer nodes with
 * their refs and ordered predecessors (Matched.java:31-66, MatchedEvent.java:27-169) and the aggregates
 * (AggregatesStoreImpl.java:30-76), over the events the buffer holds.  A host builds the reference's
 * NFAStates / buffer / aggregate entries from it and continues the key on the reference NFA (SURVEY §8(b):
 * a key over capacity falls back per key).  Host-only; out == NULL: only *needed. */
int cep_state_to_reference(const cep_pattern* p, const void* blob, size_t len, void* out, size_t cap,
                           size_t* needed);
/* Changes cep_opts.max_key_words for the next batches: a host re-pushes the records of keys handed
 * back with CEP_E_RUN_CAPACITY with the limit lifted (0 = only the device pool bounds a key). */
int cep_session_set_max_key_words(cep_session* s, int64_t words);

/* --- key-hash sharding across the GPUs of one node ---
 * The reference gets per-key independence from Kafka: the producer partitions records by key
 * hash, so each key's NFA lives in exactly one stream task (README.md:348-355; per-key run
 * counter NFAStates.java:36, buffer nodes keyed by (stage, topic, partition, offset), aggregates
 * by (key, state, run)).  A node splits a batch the same way, one shard per GPU, and the shards
 * are matched with no exchange; only match counts and offsets cross GPUs (kcep/shard.py, RCCL). */
#define CEP_MAX_SHARDS 64
/* MurmurHash3 fmix32 of the key id, and the default shard fmix32(key_id) % n_shards. */
uint32_t cep_key_hash(int32_t key_id);
int32_t cep_key_shard(int32_t key_id, int32_t n_shards);
/* Shard plan for dense key ids [0, n_keys) with key_events[k] records each: key_shard[k] =
 * cep_key_shard(k); with rebalance != 0 keys then move from the fullest shard to the emptiest
 * (the largest key lighter than the gap, repeatedly) toward equal event counts.  A carry session's
 * keys must keep their shard across batches: compute the plan once and pass it to every
 * cep_partition.  shard_events (optional, n_shards entries) receives the planned loads. */
int cep_shard_plan(const int64_t* key_events, int64_t n_keys, int32_t n_shards, int32_t rebalance,
                   int32_t* key_shard, int64_t* shard_events);
/* Stable split of a batch by shard: shard(i) = key_shard[key_id[i]] when key_shard != NULL and
 * 0 <= key_id[i] < n_keys (entries outside [0, n_shards) fall back to the hash), else
 * cep_key_shard(key_id[i]).  perm[j] = source record of output position j; shard s owns positions
 * [shard_off[s], shard_off[s+1]) (n_shards + 1 entries), in batch order, so each shard keeps the
 * batch's key grouping and per-key arrival order.  mem = CEP_MEM_HOST (computed in the call) or
 * CEP_MEM_DEVICE (every array on the device, kernels enqueued on `stream`, no host sync).
 * n_shards <= CEP_MAX_SHARDS. */
int cep_partition(const int32_t* key_id, int64_t n, int32_t n_shards, const int32_t* key_shard, int64_t n_keys,
                  int64_t* perm, int64_t* shard_off, int32_t mem, void* stream);
/* dst[i] = src[perm[i]] for i < n, elements of elem_bytes (1, 4 or 8): a shard's columns from
 * perm + shard_off[s].  Same memory rules as cep_partition. */
int cep_gather(const void* src, int32_t elem_bytes, const int64_t* perm, int64_t n, void* dst, int32_t mem,
               void* stream);
/* Enqueue a copy of the last batch's device-resident match count (cep_device_match_count) to
 * dst (device memory) on `stream`: a per-step slot for an RCCL all-gather of counts that
 * overlaps the next batch (kcep/shard.py CountExchange). */
int cep_match_count_to(const cep_session* s, int64_t* dst, void* stream);

/* --- IR builder: the lowering of a reference Pattern to the IR cep_compile consumes ---
 * A host that walks the reference DSL (java/.../pattern/PatternIR.java, over JNI) issues one call per
 * element of the ancestor chain, first pattern to last, and gets the same bytes kcep/pattern.py
 * encode_pattern writes for the query:
 *   cep_irb_select      a Pattern (Pattern.java:42-62: name or NULL for the level's default name
 *                       Pattern.java:181-183, level, Selected strategy 0..2 or -1 for null
 *                       Selected.java:48-50, topic or NULL)
 *   cep_irb_quantifier  StageBuilder.oneOrMore / zeroOrMore / times, PredicateBuilder.optional
 *   cep_irb_within      PatternBuilder.within (TimeUnit.toMillis)
 *   cep_irb_where       PredicateBuilder.where / PatternBuilder.and (conj 1) / or (conj 0): pops the
 *                       top expression (Pattern.andPredicate / orPredicate, Pattern.java:157-169)
 *   cep_irb_fold        PatternBuilder.fold(state, aggregator): pops the aggregate expression; type 0
 *                       keeps its static type, else CEP_T_* is the boxed result type
 * Matcher / aggregator bodies go on an expression stack in postfix order (children first).  Java's
 * static typing is applied as it is pushed (binary numeric promotion i32 < i64 < f64; booleans only
 * from comparisons, logic and topic tests): a type error fails that call with CEP_E_BAD_IR.  A body
 * the host cannot express with these calls (an opaque lambda) never reaches the builder: that query
 * stays on the reference CPU path. */
#define CEP_T_BOOL 0
/* expression operators (cep_irb_op) and event accessors (cep_irb_event) */
#define CEP_OP_EV_KEY 0x11
#define CEP_OP_EV_TS 0x12
#define CEP_OP_EV_OFFSET 0x14
#define CEP_OP_EV_PARTITION 0x15
#define CEP_OP_NOT 0x30
#define CEP_OP_AND 0x31
#define CEP_OP_OR 0x32
#define CEP_OP_ADD 0x40
#define CEP_OP_SUB 0x41
#define CEP_OP_MUL 0x42
#define CEP_OP_DIV 0x43     /* Java '/': truncating for integers, ArithmeticException on / 0 */
#define CEP_OP_REM 0x44
#define CEP_OP_NEG 0x45
#define CEP_OP_EQ 0x50
#define CEP_OP_NE 0x51
#define CEP_OP_LT 0x52
#define CEP_OP_LE 0x53
#define CEP_OP_GT 0x54
#define CEP_OP_GE 0x55
/* SequenceMatcher reductions (cep_irb_seq) over the partial Sequence (SequenceMatcher.java:21-26) */
#define CEP_SEQ_AVG 0       /* IntSummaryStatistics.getAverage over every event */
#define CEP_SEQ_SUM 1       /* mapToLong(..).sum() / DoubleStream.sum() */
#define CEP_SEQ_COUNT 2
#define CEP_SEQ_MIN 3
#define CEP_SEQ_MAX 4
#define CEP_SEQ_FIRST 5     /* getByName(stage).getEvents(): the TreeSet's first / last event */
#define CEP_SEQ_LAST 6

typedef struct cep_irb cep_irb;
/* A builder over the value schema: n_cols column types (CEP_T_I32 / I64 / F64). */
int cep_irb_new(const int32_t* col_types, int32_t n_cols, cep_irb** out);
void cep_irb_free(cep_irb* b);
/* Interns a topic name (kcep/pattern.py Schema.topic_id: ids in first-use order); returns its id, the
 * id a host's records of that topic carry in cep_batch.topic.  Negative on error. */
int32_t cep_irb_topic(cep_irb* b, const char* topic);
int32_t cep_irb_topic_count(const cep_irb* b);
const char* cep_irb_topic_name(const cep_irb* b, int32_t id);
int cep_irb_select(cep_irb* b, const char* name, int32_t level, int32_t strategy, const char* topic);
int cep_irb_quantifier(cep_irb* b, int32_t one_or_more, int32_t optional, int32_t times);
int cep_irb_within(cep_irb* b, int64_t window_ms);
/* constants: type CEP_T_BOOL (i != 0 is true), CEP_T_I32 / CEP_T_I64 (i), CEP_T_F64 (d) */
int cep_irb_const(cep_irb* b, int32_t type, int64_t i, double d);
/* Event.value() / a named field: the schema's column `col` */
int cep_irb_field(cep_irb* b, int32_t col);
/* Event.timestamp() / offset() / partition() (CEP_OP_EV_*); CEP_OP_EV_KEY reads the batch's key id */
int cep_irb_event(cep_irb* b, int32_t what);
/* Event.topic().equals(topic) (Matcher.TopicPredicate, Matcher.java:104-120) */
int cep_irb_topic_eq(cep_irb* b, const char* topic);
/* States.get(name) as a boxed `type` (or_else = 0), or States.getOrElse(name, <popped default>)
 * (States.java:56-73) */
int cep_irb_state(cep_irb* b, const char* name, int32_t type, int32_t or_else);
/* the `curr` argument of Aggregator.aggregate (Aggregator.java:27-29) as a boxed `type` */
int cep_irb_curr(cep_irb* b, int32_t type);
/* a reduction CEP_SEQ_* over column `col` of the partial sequence, or of one stage's events (stage
 * NULL: every event; CEP_SEQ_COUNT ignores col) */
int cep_irb_seq(cep_irb* b, int32_t kind, int32_t col, const char* stage);
/* pops one (CEP_OP_NOT, CEP_OP_NEG) or two operands (left below right) and pushes the result */
int cep_irb_op(cep_irb* b, int32_t op);
/* Java's (int) / (long) / (double) cast of the top */
int cep_irb_cast(cep_irb* b, int32_t type);
int cep_irb_where(cep_irb* b, int32_t conj);
int cep_irb_fold(cep_irb* b, const char* state, int32_t type);
/* Serialises the chain (buf == NULL: only *needed).  The builder stays valid. */
int cep_irb_finish(cep_irb* b, uint8_t* buf, size_t cap, size_t* needed);

const char* cep_last_error(void);
const char* cep_version(void);

#ifdef __cplusplus
}
#endif
#endif

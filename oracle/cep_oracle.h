/*
 * cep_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C) of the kafkastreams-cep NFA evaluation path, used
 * as the parity checker for the HIP implementation and as the CPU baseline in
 * bench.py.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load it.  The product (libkcep.so) never links or calls it.
 *
 * Parity pinning: the reference is Java and cannot be built or run here (no
 * JDK, no Kafka/Kryo jars, no network).  This restatement is
 * pinned by the reference's own test vectors, transcribed as fixtures under
 * tests/golden/ (NFATest, DeweyVersionTest, SharedVersionedBufferTest,
 * StagesFactoryTest, CEPProcessorTest, CEPStreamIntegrationTest,
 * CEPStockDemoTest).
 */
#ifndef CEP_ORACLE_H
#define CEP_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* error codes: identical numbering to include/kcep.h CEP_E_* */
#define ORC_OK 0
#define ORC_E_INVALID_PATTERN 1   /* StagesFactory.InvalidPatternException */
#define ORC_E_UNKNOWN_AGGREGATE 2 /* States.UnknownAggregateException */
#define ORC_E_ILLEGAL_STATE 3     /* missing buffer predecessor */
#define ORC_E_NPE 4               /* NullPointerException */
#define ORC_E_ARITHMETIC 5        /* integer division by zero */
#define ORC_E_CLASS_CAST 6        /* boxed state type mismatch */
#define ORC_E_INDEX 7             /* DeweyVersion.addRun out of bounds */
#define ORC_E_BAD_IR 8
#define ORC_E_CAPACITY 9

/* run modes */
#define ORC_MODE_NFA_SINGLE 0   /* one NFA for every record (NFATest) */
#define ORC_MODE_PROCESSOR 1    /* CEPProcessor: per key, HWM, null filter, queue serde */
#define ORC_MODE_NFA_PER_KEY 2  /* one in-memory NFA per key, no processor rules */

/* column types */
#define ORC_T_BOOL 0
#define ORC_T_I32 1
#define ORC_T_I64 2
#define ORC_T_F64 3

typedef struct orc_pattern orc_pattern;
typedef struct orc_run orc_run;

typedef struct {
  int64_t n;
  const int32_t* key;       /* record key id (required) */
  const uint8_t* valid;     /* 0 = null key or value (CEPProcessor.java:136); NULL = all valid */
  const int32_t* topic;     /* NULL -> 0 */
  const int32_t* partition; /* NULL -> 0 */
  const int64_t* offset;    /* NULL -> record index */
  const int64_t* ts;        /* NULL -> record index */
  int32_t ncols;
  const void* const* cols;  /* typed per the pattern schema */
} orc_batch;

int orc_compile(const uint8_t* ir, size_t len, orc_pattern** out, char* err, size_t errlen);
void orc_pattern_free(orc_pattern* p);
int orc_n_stages(const orc_pattern* p);
int orc_n_names(const orc_pattern* p);
const char* orc_name(const orc_pattern* p, int name_id);
/* stage table (for StagesFactoryTest): returns number of edges */
int orc_stage_info(const orc_pattern* p, int sid, int* name_id, int* type, int64_t* window,
                   int* ops, int* targets);

orc_run* orc_run_new(const orc_pattern* p, int mode);
void orc_run_free(orc_run* r);
/* process the batch records in order; returns ORC_OK or an error code (processing
 * stops at the failing record, like the Java task) */
int orc_run_batch(orc_run* r, const orc_batch* b);
/* Continue one key from its carried state in the reference's own terms ("KCRF", written by libkcep's
 * cep_state_to_reference): the batch's first E records must be the state's E events (in order, same key,
 * topic, partition, offset, timestamp); records E..n-1 are then processed as orc_run_batch does. */
int orc_run_resume(orc_run* r, const orc_batch* b, const uint8_t* state, size_t len);
int64_t orc_err_record(const orc_run* r);
const char* orc_err_msg(const orc_run* r);

int64_t orc_n_matches(const orc_run* r);
/* match m: emitting record, key, traversal entries (final -> begin) */
void orc_match(const orc_run* r, int64_t m, int64_t* record, int32_t* key, int64_t* ent_begin,
               int64_t* ent_end);
void orc_entry(const orc_run* r, int64_t e, int32_t* name_id, int64_t* event_record);
/* materialised Sequence (reference Sequence.Builder.build(true) + TreeSet order):
 * groups in output order, each with its events */
int64_t orc_seq_groups(const orc_run* r, int64_t m, int32_t* names, int64_t* ev_counts, int64_t cap);
int64_t orc_seq_events(const orc_run* r, int64_t m, int64_t* events, int64_t cap);

/* instance state (assertNFA, NFATest.java:836-840) */
int orc_inst_state(const orc_run* r, int32_t key, int64_t* runs, int64_t* queue_size);
int orc_queue_entry(const orc_run* r, int32_t key, int64_t idx, int32_t* stage_id, int32_t* eps_target,
                    int64_t* seq, int64_t* last_event, char* version, size_t vcap);

/* CPU baseline: batch grouped by key; processed with nthreads workers over
 * contiguous whole-key shards (each shard its own processor-mode state).
 * Returns number of matches; *checksum = order-independent hash of matches. */
int64_t orc_baseline(const orc_pattern* p, const orc_batch* b, int mode, int nthreads,
                     uint64_t* checksum, int* err);

/* orc_baseline keeping every match: the CSR of the key-grouped batch, key order then per-key emission
 * order (what cep_collect returns), for element-wise comparison at full size */
typedef struct orc_csr orc_csr;
orc_csr* orc_baseline_csr(const orc_pattern* p, const orc_batch* b, int mode, int nthreads);
void orc_csr_sizes(const orc_csr* c, int64_t* n_matches, int64_t* n_entries, int* err);
void orc_csr_copy(const orc_csr* c, int64_t* match_record, int32_t* match_key, int64_t* ent_off, int32_t* ent_name,
                  int64_t* ent_record);
void orc_csr_free(orc_csr* c);

/* SharedVersionedBufferTest (SharedVersionedBufferTest.java:50-87): buffer puts and gets on the
 * events of a bound batch.  psid < 0 selects the 3-arg put.  orc_svb_get appends the traversal
 * (and its materialised Sequence) to the run's matches. */
void orc_svb_bind(orc_run* r, const orc_batch* b);
int orc_svb_put(orc_run* r, int stage_id, int64_t ev, int prev_stage_id, int64_t prev_ev, const char* version);
int orc_svb_get(orc_run* r, int stage_id, int64_t ev, const char* version, int remove);

/* DeweyVersion helpers exposed for DeweyVersionTest */
int orc_dewey_compatible(const char* a, const char* b);
int orc_dewey_add_run(const char* v, int offset, char* out, size_t cap);
int orc_dewey_add_stage(const char* v, char* out, size_t cap);

#ifdef __cplusplus
}
#endif
#endif

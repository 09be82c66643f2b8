// kcep_internal.h — compiled-pattern representation shared by the host
// compiler (compile.cpp) and the HIP kernels (stencil.hip, nfa.hip).
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include "kcep_dev.h"

#include <memory>
#include <string>
#include <vector>

namespace kcep {

struct Expr {
  uint8_t op = 0, t = 0, ct = 0;
  int32_t i32 = 0;
  int64_t i64 = 0;
  double f64 = 0;
  int col = 0, name = 0;
  std::string sname;                 // OP_SEQ_AGG: the stage name filter
  std::shared_ptr<Expr> a, b;
};
using ExprP = std::shared_ptr<Expr>;

struct Fold {
  int state;
  uint8_t type;
  ExprP expr;
};

struct PatternDef {                 // one select() of the DSL (pattern/Pattern.java)
  std::string name;
  int name_id = 0, level = 0;
  uint8_t strategy = S_STRICT;
  int32_t topic = -1;
  uint8_t one_or_more = 0, optional = 0;
  int32_t times = 1;
  int64_t window_ms = -1;
  ExprP pred;
  std::vector<Fold> folds;
};

struct EdgeDef {
  uint8_t op;
  ExprP pred;                       // nullptr = Matcher.TruePredicate
  int target;                       // stage id, -1 for IGNORE
};

struct StageDef {                   // nfa/Stage.java
  int id, name;
  uint8_t type;
  int64_t window_ms;
  int pattern;                      // index into patterns (aggregates), -1 for $final
  std::vector<EdgeDef> edges;
};

// ---- stencil (strict single-cardinality fast path) ----
constexpr int STENCIL_MAX_K = 8;
constexpr int STENCIL_MAX_TERMS = 6;
constexpr int STENCIL_MAX_ATOMS = 2;   // per term: one value-column range + one topic range

struct StencilAtomI { int64_t lo, hi; };
struct StencilAtomF { double lo, hi; };

// Predicate slot p (0..7): OR over terms of (value in [lo,hi] AND topic in [tlo,thi]).
// Slots 0..k-1 are the stage predicates (BEGIN edges, topic filter included).
// Chain patterns (strict with optional() stages, k <= 4) also use slot 4+i for
// the SKIP_PROCEED edge of optional stage i: the successor's predicate without
// its topic filter (StagesFactory.java:159-169); the edge is that AND NOT slot i.
constexpr int CHAIN_MAX_K = 4;
struct StencilProgram {
  int32_t k;
  int32_t col;                       // value column read by every predicate
  int32_t coltype;                   // T_I32 / T_I64 / T_F64
  int32_t use_topic;                 // 1 if any atom constrains the topic
  int32_t chain;                     // 1: some stage is optional (variable-length matches)
  int32_t optmask;                   // bit i: stage i is optional
  int32_t pslots;                    // bit p: predicate slot p is in use
  int32_t nterms[STENCIL_MAX_K];
  int32_t hasv[STENCIL_MAX_K][STENCIL_MAX_TERMS];   // 0: term does not constrain the value
  StencilAtomI vi[STENCIL_MAX_K][STENCIL_MAX_TERMS];
  StencilAtomF vf[STENCIL_MAX_K][STENCIL_MAX_TERMS];
  StencilAtomI tp[STENCIL_MAX_K][STENCIL_MAX_TERMS];
  int32_t name[STENCIL_MAX_K];       // stage name id of pattern s
  // Interval table: the breakpoints of every value/topic atom cut the value
  // (topic) axis into intervals on which each stage predicate is constant, so
  // a record's k-bit stage mask is table[it * 16 + iv] with iv = #{value
  // breakpoints <= v} and it = #{topic breakpoints <= topic}.
  int32_t nbp;                       // value breakpoints (<= 15), sorted ascending
  int32_t ntbp;                      // topic breakpoints (<= 3)
  int64_t bpi[15];                   // integer columns (clamped to int32 for i32 columns)
  double bpf[15];                    // double columns
  int32_t tbp[3];
  uint8_t table[64];
  uint8_t nan_mask[4];               // double columns: mask of a NaN value per topic interval
  // Dense form of the same table for integer columns without topic atoms with >= 6 breakpoints spanning
  // < 256 values: mask = lut[v - lut_lo] inside [lut_lo, lut_lo + lut_n), table[0] below,
  // table[nbp] above (one LDS read per record instead of nbp compares); lut_n = 0: not used
  int64_t lut_lo;
  int32_t lut_n;
  uint8_t lut[256];
};

struct Program {
  std::vector<uint8_t> coltypes;
  std::vector<PatternDef> pats;
  std::vector<StageDef> stages;
  std::vector<std::string> names;    // stage names, 0 = "$final"
  std::vector<std::string> states;   // aggregate state names
  std::vector<int> defined_states;   // Stages.getDefinedStates()
  int begin = -1;
  bool general_ok = false;
  std::string general_why;
  DevProgram dev{};
  bool stencil_ok = false;
  std::string stencil_why;           // reason the stencil path does not apply
  bool runs_ok = false;              // deterministic strict runs (compile.cpp analyse_runs)
  bool has_seq = false;              // some predicate or fold is a SequenceMatcher (OP_SEQ_*)
  std::string runs_why;
  StencilProgram stencil{};
};

// ---- carried state of the stencil / chain paths (CEP_SESSION_CARRY) ----
// A strict fixed-length match needs only the key's last K-1 records from earlier batches (SURVEY
// Q9): per key two slots (the batch that wrote it, its records oldest first: stage masks and
// stream positions).  A batch reads the newer slot written before it and writes the other one,
// so readers and the writer of one key never touch the same slot.  What a batch reads is one
// 32-byte header per key (both slots, dense by key id: consecutive keys of a batch share lines);
// the stream positions, written per batch and read only when a match reaches into the halo, sit
// in a separate dense array of (K-1) int64 per key and slot.
struct HaloHdr {
  int32_t stamp[2];                  // batch number that wrote slot s, 0 = never
  int32_t claim;                     // the last batch that had a segment of the key
  uint8_t cnt[2];                    // records held by slot s (<= K-1)
  uint8_t pad[2];
  uint64_t masks[2];                 // byte h of slot s: stage mask of its record h
};
static_assert(sizeof(HaloHdr) == 32, "HaloHdr is one 32-byte header per key");
struct StencilCarry {
  HaloHdr* hdr;                      // per key id
  int64_t* pos;                      // [(2 * key + slot) * km1 + h]: stream position of record h
  int32_t km1;                       // K - 1
  int32_t stamp;                     // this batch's number (>= 1)
  int32_t max_keys;
  int64_t base;                      // stream position of batch record 0
  unsigned long long* flags;         // bit 0: key id out of range, bit 1: a key in two segments,
                                     // bit 2: chain carry batch beyond a tile's match space
  const int64_t* gpos;               // stream position of each batch record (CEP_BATCH_ARRIVAL_ORDER: base + its
                                     // arrival index); null: base + record index
  int32_t grouped;                   // the device grouped the batch (CEP_BATCH_ARRIVAL_ORDER): each key is one
                                     // segment by construction, no claims (for an interleaved flush nearly every
                                     // record starts a segment, and its returning atomic was waited for in turn)
};
KCEP_HD inline int64_t halo_gpos(const StencilCarry& C, int64_t r) { return C.gpos ? C.gpos[r] : C.base + r; }
KCEP_HD inline int halo_old(const HaloHdr& h, int32_t stamp) {
  // the newer slot written before batch `stamp` (or an empty one)
  const int32_t a = h.stamp[0] < stamp ? h.stamp[0] : -1, b = h.stamp[1] < stamp ? h.stamp[1] : -1;
  return a >= b ? 0 : 1;
}

// ---- launch interfaces shared by abi.cpp and the .hip files ----
// CEP_BATCH_DELIVER on a carry session: where the device hands the batch's matches to the host
struct DeliverArgs {
  int64_t* hdr = nullptr;         // pinned host: {match count, this batch's error flags}; null: no delivery
  int32_t* hkey = nullptr;        // pinned host: key id per match (the first host_cap matches)
  int64_t* hpos = nullptr;        // pinned host: k stream positions per match
  int32_t* dkey = nullptr;        // device: the same past host_cap
  int64_t* dpos = nullptr;
  int64_t host_cap = 0;
  unsigned* ticket = nullptr;     // device: workgroups done (the last one stamps hdr[2] = stamp; reset to 0)
  int64_t stamp = 0;              // this delivery's number: cep_collect spins until hdr[2] holds it
  // CEP_BATCH_ARRIVAL_ORDER (group.hip): the rows delivered in arrival order of their completing record --
  // per arrival record its matches (a_cnt, zeroed by group_gather), their prefix (a_moff), its first match
  int64_t* a_cnt = nullptr;       // null: grouped order
  int32_t* a_head = nullptr;
  int64_t* a_moff = nullptr;
  int64_t* a_tot = nullptr;
  int64_t* a_tmp = nullptr;       // the scan's scratch
  int64_t a_n = 0;                // the batch's records
};
// CEP_BATCH_ARRIVAL_ORDER: an arrival-order batch grouped by key (group.hip)
struct GroupArgs {
  const int32_t* key;             // in: arrival order
  int32_t* g_key;                 // out: grouped (stable by key id)
  int32_t* arr;                   // out: arrival index of each grouped record
  int64_t* pos;                   // out: its stream position, base + arrival index
  int64_t base;
  const uint8_t* valid; uint8_t* g_valid;
  const int32_t* topic; int32_t* g_topic;
  const int32_t* partition; int32_t* g_partition;
  const int64_t* offset; int64_t* g_offset;
  const int64_t* ts; int64_t* g_ts;
  const void* cols[16]; void* g_cols[16];
  int32_t coltype[16];
  int32_t ncols;
  int64_t* cnt;                   // zeroed (n): the reorder's per-record match / entry counts
  int64_t* ecnt;
  // the grouping's state and scratch (group.hip)
  int32_t max_keys;
  uint32_t stamp;                 // this grouping's number (>= 1)
  unsigned long long* head;       // max_keys + 1 epoch-tagged list heads
  int32_t* node_top;
  int32_t *node_key, *node_chunk, *node_cnt, *node_next, *node_prefix, *node_leader, *rec_node, *rec_rank;
  int64_t* start;                 // per leader node: its key's first grouped position
  unsigned long long* cursor;     // the groups placed so far (zeroed once)
};
hipError_t group_launch(const GroupArgs& G, int64_t n, hipStream_t st);
hipError_t arrival_reorder(const int64_t* mrec, const int32_t* mkey, const int64_t* eoff, const int32_t* ename,
                           const int64_t* erec, int64_t nm, int64_t ne, int64_t base, int64_t n, int64_t* cnt,
                           int64_t* ecnt, int32_t* head, int64_t* moff, int64_t* moff_e, int64_t* tot, int64_t* tmp,
                           int64_t* o_rec, int32_t* o_key, int64_t* o_eoff, int32_t* o_name, int64_t* o_erec,
                           hipStream_t st);
hipError_t stencil_arrival_ranks(const int32_t* out, int k, const int64_t* total, int64_t out_cap, const int64_t* gpos,
                                 int64_t base, int64_t n, int64_t* cnt, int32_t* head, int64_t* moff, int64_t* tot,
                                 int64_t* tmp, hipStream_t st);
// The plain stencil kernel without carry stores a super-tile's first ST_DENSE matches (one int each)
// in a dense region at the head of the slot buffer (super-tile t at t * ST_DENSE) and the rest in
// the super-tile's own region after it (nsuper * ST_DENSE + t * sub * 4096 + m): the dense runs sit
// a few KB apart instead of 196 KB, C2 kernel -7.5 us (profiles/r04_ab_stencil_stores.txt).
#ifndef KCEP_ST_DENSE
#define KCEP_ST_DENSE 512                  // (<= 512: the session allocates 512 per tile; A/B builds only)
#endif
constexpr int ST_DENSE = KCEP_ST_DENSE;
// The keyed kernel without carry (C5's chain) the same way, with its aux bytes: a super-tile's first
// ST_DENSE_KEYED matches at t * ST_DENSE_KEYED ints and, after nsuper of those, their aux bytes at
// t * ST_DENSE_KEYED; the rest in the super-tile's own region (ints, then aux bytes) after both.
constexpr int ST_DENSE_KEYED = 1024;
#ifndef ST_KEYED_DENSE
#define ST_KEYED_DENSE 0                   // A/B knob (builds only; off: kernel -16 us, step +5 us on C5)
#endif

struct StencilLaunch {
  const int32_t* key;
  const void* val;
  const int32_t* topic;
  int64_t n;
  const StencilProgram* prog_dev;
  int k, coltype, use_topic, chain;
  int32_t* slots;                 // per-tile match slots, ST_TILE * k ints each (+ ST_DENSE per tile, see below)
  int64_t* tile_count;            // matches per tile
  int64_t* tile_pre;              // their exclusive prefix
  int64_t* scan_tmp;
  int32_t* out;                   // contiguous output, k ints per match
  int64_t out_cap;                // matches
  int64_t* total;                 // device: number of matches
  StencilCarry carry;             // halo != nullptr: carry session
  int plain;                      // plain stencil (no carry, no chain, k <= 7): the keyless kernel (KCEP_STENCIL_KEYED=1: off)
  unsigned long long* clear_flag; // carry: the next batch's error-flag word, zeroed by the scan kernel (or null)
  DeliverArgs deliver;            // carry sessions' CEP_BATCH_DELIVER batches
};

// compile.cpp
int lower_general(Program& P, std::string& why);
bool wave_stateful(const DevProgram& D);
int compile_ir(const uint8_t* ir, size_t len, Program& out, std::string& err);

// ---- carried tails of the runs path (CEP_SESSION_CARRY, runs.hip) ----
// the batch's columns as runs_carry_build reads them (device pointers; optional ones may be null)
struct RcIn {
  const int64_t* pos;                // stream positions of the batch's records (null: base + index)
  const int32_t* key;
  const int32_t* topic;
  const int32_t* partition;
  const int64_t* offset;
  const int64_t* ts;
  const void* cols[16];
};
// the extended batch: each key's carried tail, then its records of the batch; seg = batch segment
struct RcExt {
  int32_t *key, *topic, *partition, *seg;
  int64_t *offset, *ts, *pos;
  void* cols[16];
  int32_t coltype[16];
  int32_t ncols;
  int64_t cap;                       // records the arrays hold: writes past it are dropped (a batch with a key
                                     // in two segments gives that key's tail to both; it is rejected anyway)
};
hipError_t runs_carry_build(const RcIn& B, int64_t n, int64_t base, const int64_t* seg_flag, const int64_t* seg_idx,
                            const int64_t* seg_start, const int64_t* nseg, const int64_t* rtab, const int64_t* rpool,
                            int64_t* tlen, int64_t* toff, int64_t* total, int64_t* scan_tmp, const RcExt& X,
                            hipStream_t st, bool lens_only, int32_t max_keys);
hipError_t runs_carry_count(int64_t* out, int64_t nb, const int64_t* tails, int64_t cap, hipStream_t st);
hipError_t runs_carry_tails(const RcExt& X, int64_t ext_n, int64_t n, const int64_t* nseg, const int64_t* seg_start,
                            const int32_t* key, const int64_t* toff, const int32_t* end_of, unsigned long long* tstart,
                            int64_t* newlen, int64_t* noff, int64_t* new_total, int64_t* scan_tmp, int64_t* top,
                            int64_t* rpool, int64_t* rtab, hipStream_t st, const int64_t* ext_n_dev, const int64_t* bad);
hipError_t runs_carry_gc(int64_t* rtab, int64_t nkeys, int RW, const int64_t* src, int64_t* dst, int64_t* len,
                         int64_t* off, int64_t* total, int64_t* scan_tmp, hipStream_t st);

}  // namespace kcep

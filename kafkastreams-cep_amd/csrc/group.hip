// group.hip -- CEP_BATCH_ARRIVAL_ORDER: a batch handed over in arrival order, as CEPProcessor.process
// sees its records one by one (CEPProcessor.java:134-150), grouped by key on the device, and the
// matches put back into arrival order of their completing record -- the order context.forward
// emits them (:148).  Neither the JVM nor the Python host sorts anything.
//
//   grouping: a stable grouping by key id without a sort, in three kernels and a scan (group_launch):
//     group_chunks  one wave per chunk of 256 / 1024 consecutive records: an LDS hash table of the chunk's keys
//                   gives every record its rank among the chunk's earlier records of its key (rounds of
//                   64 records; a round's lanes of one key found by an LDS bit mask, not by lane order), and
//                   every (chunk, key) pair becomes a node pushed onto the key's list (an epoch-tagged head
//                   per key id: nothing is cleared between batches)
//     group_nodes   per node: the key's records in earlier chunks (its prefix), the key's total and its
//                   leader (the node of the key's first chunk); each leader takes its key's group from a
//                   cursor (one atomic per workgroup)
//     group_gather  per record: grouped position = start(leader) + prefix + rank; every column moved there,
//                   and its stream position written (base + arrival index)
//   The paths take the grouped positions as NfaArgs.pos / RcIn.pos / StencilCarry.gpos, so carried state and
//   emitted entries speak arrival positions.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kcep_internal.h"

namespace kcep {

hipError_t exclusive_scan(const int64_t* in, int64_t n, int64_t* out, int64_t* total, int64_t* tmp, hipStream_t st);
hipError_t exclusive_scan_pair(const int64_t* in0, const int64_t* in1, int64_t n, const int64_t* n_dev, int64_t* out0,
                               int64_t* out1, int64_t* total0, int64_t* total1, int64_t* tmp, hipStream_t st);

static unsigned blocks256(int64_t n) { return unsigned((std::max<int64_t>(n, 1) + 255) / 256); }

namespace {

__device__ __forceinline__ void copy_col(const void* src, void* dst, int type, int64_t from, int64_t to) {
  if (type == T_I32) static_cast<int32_t*>(dst)[to] = static_cast<const int32_t*>(src)[from];
  else static_cast<int64_t*>(dst)[to] = static_cast<const int64_t*>(src)[from];
}

// records per wave (a chunk): 1024, or 256 for batches up to 2^18 records (four times the waves: a 64 k-record
// flush took 27 us with 64 of them); a key's node list is at most the batch's chunks long
constexpr int32_t GR_EMPTY = -2;                 // (invalid key ids are all -1: one group, the batch fails later)

__device__ __forceinline__ uint32_t gr_hash(int32_t k) {
  uint32_t h = uint32_t(k);
  h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
  return h;
}

template <int GR_CHUNK>
__global__ __launch_bounds__(64) void group_chunks(const int32_t* __restrict__ key, int64_t n, int32_t max_keys,
                                                   uint32_t stamp, unsigned long long* __restrict__ head,
                                                   int32_t* __restrict__ node_top, int32_t* __restrict__ node_key,
                                                   int32_t* __restrict__ node_chunk, int32_t* __restrict__ node_cnt,
                                                   int32_t* __restrict__ node_next, int32_t* __restrict__ rec_node,
                                                   int32_t* __restrict__ rec_rank) {
  constexpr int GR_TAB = 2 * GR_CHUNK;           // LDS hash slots (at most half full)
  __shared__ int32_t tkey[GR_TAB];
  __shared__ int32_t tcnt[GR_TAB];               // the key's records so far; at the end: its node
  __shared__ unsigned long long tmask[GR_TAB];   // the round's lanes of the key
  __shared__ uint16_t rslot[GR_CHUNK];
  __shared__ uint16_t rrank[GR_CHUNK];
  __shared__ int32_t s_base;
  const int lane = threadIdx.x;
  const int64_t r0 = int64_t(blockIdx.x) * GR_CHUNK;
  for (int i = lane; i < GR_TAB; i += 64) {
    tkey[i] = GR_EMPTY;
    tcnt[i] = 0;
    tmask[i] = 0;
  }
  // the chunk's keys, all loads in flight at once (a batch read over the link in place costs a link
  // round trip per dependent load: 16 of them took 55 us per 64 k-record flush)
  int32_t kr[GR_CHUNK / 64];
#pragma unroll
  for (int round = 0; round < GR_CHUNK / 64; round++) {
    const int64_t r = r0 + round * 64 + lane;
    kr[round] = r < n ? key[r] : 0;
  }
  __syncthreads();
#pragma unroll
  for (int round = 0; round < GR_CHUNK / 64; round++) {
    const int64_t r = r0 + round * 64 + lane;
    if (r0 + round * 64 >= n) break;             // (uniform)
    const bool act = r < n;
    int h = 0;
    if (act) {
      const int32_t k0 = kr[round];
      const int32_t k = k0 >= 0 && k0 < max_keys ? k0 : -1;
      h = int(gr_hash(k) & (GR_TAB - 1));
      for (;;) {
        const int32_t old = atomicCAS(&tkey[h], GR_EMPTY, k);
        if (old == GR_EMPTY || old == k) break;
        h = (h + 1) & (GR_TAB - 1);
      }
      atomicOr(&tmask[h], 1ull << lane);
    }
    __syncthreads();
    const unsigned long long m = act ? tmask[h] : 0ull;
    const int rk = __popcll(m & ((1ull << lane) - 1ull));
    __syncthreads();                             // every lane has read its mask
    if (act && rk == 0) {                        // the round's first lane of the key
      tcnt[h] += __popcll(m);
      tmask[h] = 0;
    }
    __syncthreads();
    if (act) {
      rslot[round * 64 + lane] = uint16_t(h);
      rrank[round * 64 + lane] = uint16_t(tcnt[h] - __popcll(m) + rk);
    }
  }
  __syncthreads();
  // the chunk's keys become nodes (consecutive ids), pushed onto their keys' lists
  int d = 0;
  for (int i = lane; i < GR_TAB; i += 64) d += __popcll(__ballot(tkey[i] != GR_EMPTY));
  if (lane == 0) s_base = d ? atomicAdd(node_top, d) : 0;
  __syncthreads();
  // every head exchange of the chunk in flight before the first result is used (one list push per node;
  // waited one by one they cost a memory round trip each: 32 per wave)
  int nd = s_base;
  unsigned long long old[GR_TAB / 64];
  int xs[GR_TAB / 64];
#pragma unroll
  for (int j = 0; j < GR_TAB / 64; j++) {
    const int i = j * 64 + lane;
    const bool occ = tkey[i] != GR_EMPTY;
    const unsigned long long b = __ballot(occ);
    xs[j] = -1;
    old[j] = 0;
    if (occ) {
      const int x = nd + __popcll(b & ((1ull << lane) - 1ull));
      const int32_t k = tkey[i];
      xs[j] = x;
      old[j] = atomicExch(&head[k >= 0 ? k : max_keys], (static_cast<unsigned long long>(stamp) << 32) | uint32_t(x));
    }
    nd += __popcll(b);
  }
#pragma unroll
  for (int j = 0; j < GR_TAB / 64; j++) {
    const int i = j * 64 + lane;
    const int x = xs[j];
    if (x >= 0) {
      node_key[x] = tkey[i];
      node_chunk[x] = int32_t(blockIdx.x);
      node_cnt[x] = tcnt[i];
      node_next[x] = uint32_t(old[j] >> 32) == stamp ? int32_t(uint32_t(old[j])) : -1;
      tcnt[i] = x;
    }
  }
  __syncthreads();
  for (int j = lane; j < GR_CHUNK; j += 64) {
    const int64_t r = r0 + j;
    if (r >= n) break;
    rec_node[r] = tcnt[rslot[j]];
    rec_rank[r] = rrank[j];
  }
}

// per node: its key's records in earlier chunks, and the key's leader node (first chunk); a leader takes
// the key's group -- its total records -- from a cursor (any order of the groups will do: one atomic per
// workgroup, lanes placed by a scan)
__global__ __launch_bounds__(256) void group_nodes(int64_t cap, const int32_t* __restrict__ node_top, int32_t max_keys,
                                                   const unsigned long long* __restrict__ head,
                                                   const int32_t* __restrict__ node_key, const int32_t* __restrict__ node_chunk,
                                                   const int32_t* __restrict__ node_cnt, const int32_t* __restrict__ node_next,
                                                   int32_t* __restrict__ node_prefix, int32_t* __restrict__ node_leader,
                                                   int64_t* __restrict__ start, unsigned long long* __restrict__ cursor) {
  const int64_t x = int64_t(blockIdx.x) * 256 + threadIdx.x;
  const int lane = threadIdx.x & 63;
  int64_t total = 0;
  bool leader = false;
  if (x < cap && x < *node_top) {
    const int32_t k = node_key[x], c = node_chunk[x];
    int32_t y = int32_t(uint32_t(head[k >= 0 ? k : max_keys]));   // (this batch's: x is on the list)
    int64_t prefix = 0;
    int32_t lead = int32_t(x), leadc = c;
    while (y >= 0) {
      const int32_t cc = node_chunk[y], cn = node_cnt[y];
      total += cn;
      if (cc < c) prefix += cn;
      if (cc < leadc) { leadc = cc; lead = y; }
      y = node_next[y];
    }
    node_prefix[x] = int32_t(prefix);
    node_leader[x] = lead;
    leader = lead == int32_t(x);
  }
  __shared__ int64_t s_w[4];
  __shared__ unsigned long long s_base;
  const int wid = threadIdx.x >> 6;
  int64_t v = leader ? total : 0, incl = v;      // the workgroup's leaders' groups: one cursor add
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int64_t t = __shfl_up(incl, d, 64);
    if (lane >= d) incl += t;
  }
  if (lane == 63) s_w[wid] = incl;
  __syncthreads();
  if (threadIdx.x == 0) {
    const int64_t sum = s_w[0] + s_w[1] + s_w[2] + s_w[3];
    s_base = sum ? atomicAdd(cursor, (unsigned long long)sum) : 0;
  }
  __syncthreads();
  int64_t before = int64_t(s_base);
  for (int w = 0; w < wid; w++) before += s_w[w];
  if (leader) start[x] = before + incl - v;
}

// grouped record g = start(leader) + prefix + rank <- arrival record i; zeroes the reorder's per-record counts
__global__ __launch_bounds__(256) void group_gather(GroupArgs G, int64_t n) {
  const int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (i == 0) {                                   // (read by group_nodes only, which is done)
    *G.node_top = 0;
    *G.cursor = 0;
  }
  if (i >= n) return;
  const int32_t x = G.rec_node[i];
  const int64_t g = G.start[G.node_leader[x]] + G.node_prefix[x] + G.rec_rank[i];
  G.g_key[g] = G.key[i];
  G.arr[g] = int32_t(i);
  G.pos[g] = G.base + i;
  if (G.valid) G.g_valid[g] = G.valid[i];
  if (G.topic) G.g_topic[g] = G.topic[i];
  if (G.partition) G.g_partition[g] = G.partition[i];
  if (G.offset) G.g_offset[g] = G.offset[i];
  if (G.ts) G.g_ts[g] = G.ts[i];
  for (int c = 0; c < G.ncols; c++) copy_col(G.cols[c], G.g_cols[c], G.coltype[c], i, g);
  G.cnt[i] = 0;
  G.ecnt[i] = 0;
}

// CSR in grouped order (match_record = stream positions, already arrival-based) -> per arrival record its
// matches and entries, and the first of its matches
__global__ __launch_bounds__(256) void arrival_count(const int64_t* __restrict__ mrec, const int64_t* __restrict__ eoff,
                                                     int64_t nm, int64_t ne, int64_t base, int64_t n,
                                                     unsigned long long* __restrict__ cnt,
                                                     unsigned long long* __restrict__ ecnt, int32_t* __restrict__ head) {
  const int64_t m = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (m >= nm) return;
  const int64_t a = mrec[m] - base;
  if (a < 0 || a >= n) return;                    // (cep_csr_check reports it at collect)
  atomicAdd(&cnt[a], 1ull);
  atomicAdd(&ecnt[a], (unsigned long long)((m + 1 < nm ? eoff[m + 1] : ne) - eoff[m]));
  if (m == 0 || mrec[m - 1] != mrec[m]) head[a] = int32_t(m);
}

__global__ __launch_bounds__(256) void arrival_scatter(const int64_t* __restrict__ mrec, const int32_t* __restrict__ mkey,
                                                       const int64_t* __restrict__ eoff, const int32_t* __restrict__ ename,
                                                       const int64_t* __restrict__ erec, int64_t nm, int64_t ne,
                                                       int64_t base, int64_t n, const int64_t* __restrict__ moff,
                                                       const int64_t* __restrict__ moff_e, const int32_t* __restrict__ head,
                                                       int64_t* __restrict__ o_rec, int32_t* __restrict__ o_key,
                                                       int64_t* __restrict__ o_eoff, int32_t* __restrict__ o_name,
                                                       int64_t* __restrict__ o_erec) {
  const int64_t m = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (m >= nm) return;
  const int64_t a = mrec[m] - base;
  if (a < 0 || a >= n) return;
  const int64_t h = head[a];
  const int64_t j = moff[a] + (m - h);
  const int64_t e0 = eoff[m], e1 = m + 1 < nm ? eoff[m + 1] : ne;
  const int64_t d = moff_e[a] + (e0 - eoff[h]);
  o_rec[j] = mrec[m];
  o_key[j] = mkey[m];
  o_eoff[j] = d;
  for (int64_t e = e0; e < e1; e++) {
    o_name[d + (e - e0)] = ename[e];
    o_erec[d + (e - e0)] = erec[e];
  }
}

// stencil / chain rows (k ints per match, grouped order; the completing record is stage k-1 and always in
// the batch): per arrival record its matches and the first of them
__global__ __launch_bounds__(256) void stencil_arrival_count(const int32_t* __restrict__ out, int k,
                                                             const int64_t* __restrict__ total, int64_t out_cap,
                                                             const int64_t* __restrict__ gpos, int64_t base,
                                                             unsigned long long* __restrict__ cnt,
                                                             int32_t* __restrict__ head) {
  const int64_t t = *total, nm = t < out_cap ? t : out_cap;
  for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < nm; i += int64_t(gridDim.x) * 256) {
    const int32_t last = out[i * k + k - 1];
    const int64_t a = gpos[last] - base;
    atomicAdd(&cnt[a], 1ull);
    if (i == 0 || out[(i - 1) * k + k - 1] != last) head[a] = int32_t(i);
  }
}

}  // namespace

// key ids -> the grouped batch (G.g_key, G.arr, G.pos, the columns); G.head: max_keys + 1 epoch-tagged list
// heads (zeroed once), G.stamp: this call's number (>= 1, never repeated); scratch: n entries each of the
// node and record arrays, G.node_top and G.cursor zeroed once (group_gather re-zeroes them)
hipError_t group_launch(const GroupArgs& G, int64_t n, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (n <= (int64_t(1) << 18)) {
    hipLaunchKernelGGL(group_chunks<256>, dim3(unsigned((n + 255) / 256)), dim3(64), 0, st, G.key, n, G.max_keys, G.stamp,
                       G.head, G.node_top, G.node_key, G.node_chunk, G.node_cnt, G.node_next, G.rec_node, G.rec_rank);
  } else {
    hipLaunchKernelGGL(group_chunks<1024>, dim3(unsigned((n + 1023) / 1024)), dim3(64), 0, st, G.key, n, G.max_keys,
                       G.stamp, G.head, G.node_top, G.node_key, G.node_chunk, G.node_cnt, G.node_next, G.rec_node,
                       G.rec_rank);
  }
  hipLaunchKernelGGL(group_nodes, dim3(blocks256(n)), dim3(256), 0, st, n, G.node_top, G.max_keys, G.head, G.node_key,
                     G.node_chunk, G.node_cnt, G.node_next, G.node_prefix, G.node_leader, G.start, G.cursor);
  hipLaunchKernelGGL(group_gather, dim3(blocks256(n)), dim3(256), 0, st, G, n);
  return hipGetLastError();
}

// the general / runs CSR (grouped order, in) into arrival order (out); cnt / ecnt were zeroed by
// group_gather, moff / moff_e: n entries of scratch, tmp: the scans' scratch
hipError_t arrival_reorder(const int64_t* mrec, const int32_t* mkey, const int64_t* eoff, const int32_t* ename,
                           const int64_t* erec, int64_t nm, int64_t ne, int64_t base, int64_t n, int64_t* cnt,
                           int64_t* ecnt, int32_t* head, int64_t* moff, int64_t* moff_e, int64_t* tot, int64_t* tmp,
                           int64_t* o_rec, int32_t* o_key, int64_t* o_eoff, int32_t* o_name, int64_t* o_erec,
                           hipStream_t st) {
  if (nm <= 0) return hipSuccess;
  hipLaunchKernelGGL(arrival_count, dim3(blocks256(nm)), dim3(256), 0, st, mrec, eoff, nm, ne, base, n,
                     reinterpret_cast<unsigned long long*>(cnt), reinterpret_cast<unsigned long long*>(ecnt), head);
  hipError_t e = exclusive_scan_pair(cnt, ecnt, n, nullptr, moff, moff_e, tot, tot + 1, tmp, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(arrival_scatter, dim3(blocks256(nm)), dim3(256), 0, st, mrec, mkey, eoff, ename, erec, nm, ne, base,
                     n, moff, moff_e, head, o_rec, o_key, o_eoff, o_name, o_erec);
  return hipGetLastError();
}

// stencil / chain rows: per arrival record its matches (cnt, zeroed by group_gather), their exclusive
// prefix into moff -- the delivery then writes match i at moff[a] + (i - head[a])
hipError_t stencil_arrival_ranks(const int32_t* out, int k, const int64_t* total, int64_t out_cap, const int64_t* gpos,
                                 int64_t base, int64_t n, int64_t* cnt, int32_t* head, int64_t* moff, int64_t* tot,
                                 int64_t* tmp, hipStream_t st) {
  const int64_t blocks = std::min<int64_t>((out_cap + 255) / 256, 1024);
  hipLaunchKernelGGL(stencil_arrival_count, dim3(unsigned(std::max<int64_t>(blocks, 1))), dim3(256), 0, st, out, k, total,
                     out_cap, gpos, base, reinterpret_cast<unsigned long long*>(cnt), head);
  return exclusive_scan(cnt, n, moff, tot, tmp, st);
}

}  // namespace kcep

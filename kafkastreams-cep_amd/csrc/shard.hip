// shard.hip — key-hash sharding of record batches across the GPUs of a node
// (SURVEY §8(e)).
//
// The reference never shares a key between stream tasks: Kafka's producer
// partitions records by key hash (README.md:348-355) and each task owns the
// NFAs of its keys (per-key run counter NFAStates.java:36, buffer nodes keyed
// by (stage, topic, partition, offset), aggregates by (key, state, run)).  The
// node-level equivalent assigns every key to one GPU: shard(k) = a plan table
// entry when the caller has one (sticky across batches, optionally rebalanced
// to equal event counts by cep_shard_plan), else fmix32(k) % n_shards.  A
// batch is split by a stable counting sort on the shard, so every shard keeps
// the batch's key grouping and per-key arrival order.
//
// Device path (mem = CEP_MEM_DEVICE, enqueued on the caller's stream with
// stream-ordered scratch, no host sync): tiles of 4096 records (256 threads x 16 consecutive records); pass 1
// counts each tile's records per shard, an exclusive scan over the
// shard-major [shard][tile] counts gives every (shard, tile) its output
// offset, pass 2 recomputes the shards and writes the permutation with the
// per-shard ranks of a block scan in thread order (stable).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <set>
#include <string>
#include <utility>
#include <vector>

#include "../../include/kcep.h"

namespace kcep {
int set_error(int code, const std::string& msg);   // abi.cpp: cep_last_error()
hipError_t exclusive_scan(const int64_t* in, int64_t n, int64_t* out, int64_t* total, int64_t* tmp, hipStream_t st);

constexpr int PT_THREADS = 256;
constexpr int PT_PER = 16;                       // consecutive records per thread
constexpr int PT_TILE = PT_THREADS * PT_PER;

__host__ __device__ __forceinline__ uint32_t fmix32(uint32_t h) {   // MurmurHash3 finaliser
  h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
  return h;
}
__host__ __device__ __forceinline__ int32_t shard_of(int32_t k, const int32_t* table, int64_t nkeys, int32_t G) {
  if (table && k >= 0 && k < nkeys) {
    const int32_t s = table[k];
    if (s >= 0 && s < G) return s;
  }
  return int32_t(fmix32(uint32_t(k)) % uint32_t(G));
}

// LDS: cnt[s][t] = records of shard s among thread t's 16
__device__ __forceinline__ void tile_counts(const int32_t* __restrict__ key, int64_t n, const int32_t* __restrict__ table,
                                            int64_t nkeys, int32_t G, int32_t* cnt, int64_t r0) {
  const int t = threadIdx.x;
  for (int s = 0; s < G; s++) cnt[s * PT_THREADS + t] = 0;
  for (int j = 0; j < PT_PER; j++) {
    const int64_t r = r0 + j;
    if (r < n) cnt[shard_of(key[r], table, nkeys, G) * PT_THREADS + t]++;
  }
}

__global__ __launch_bounds__(PT_THREADS) void part_count(const int32_t* __restrict__ key, int64_t n,
                                                         const int32_t* __restrict__ table, int64_t nkeys, int32_t G,
                                                         int64_t nb, int64_t* __restrict__ counts) {
  extern __shared__ int32_t cnt[];
  const int64_t r0 = int64_t(blockIdx.x) * PT_TILE + int64_t(threadIdx.x) * PT_PER;
  tile_counts(key, n, table, nkeys, G, cnt, r0);
  __syncthreads();
  for (int s = threadIdx.x >> 6; s < G; s += PT_THREADS / 64) {     // one wave per shard row
    int32_t v = 0;
    for (int t = threadIdx.x & 63; t < PT_THREADS; t += 64) v += cnt[s * PT_THREADS + t];
    for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d);
    if ((threadIdx.x & 63) == 0) counts[int64_t(s) * nb + blockIdx.x] = v;
  }
}

__global__ __launch_bounds__(PT_THREADS) void part_scatter(const int32_t* __restrict__ key, int64_t n,
                                                           const int32_t* __restrict__ table, int64_t nkeys, int32_t G,
                                                           int64_t nb, const int64_t* __restrict__ offs,
                                                           int64_t* __restrict__ perm) {
  extern __shared__ int32_t cnt[];
  __shared__ int32_t wsum[PT_THREADS / 64];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t r0 = int64_t(blockIdx.x) * PT_TILE + int64_t(t) * PT_PER;
  tile_counts(key, n, table, nkeys, G, cnt, r0);
  __syncthreads();
  // per shard: exclusive scan of the thread counts in thread order
  for (int s = 0; s < G; s++) {
    const int32_t v = cnt[s * PT_THREADS + t];
    int32_t x = v;
    for (int d = 1; d < 64; d <<= 1) {
      const int32_t y = __shfl_up(x, d);
      if (lane >= d) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    int32_t before = 0;
    for (int i = 0; i < w; i++) before += wsum[i];
    cnt[s * PT_THREADS + t] = before + x - v;
    __syncthreads();
  }
  for (int j = 0; j < PT_PER; j++) {
    const int64_t r = r0 + j;
    if (r >= n) break;
    const int s = shard_of(key[r], table, nkeys, G);
    const int32_t rank = cnt[s * PT_THREADS + t]++;
    perm[offs[int64_t(s) * nb + blockIdx.x] + rank] = r;
  }
}

__global__ void part_bounds(const int64_t* __restrict__ offs, int64_t nb, int32_t G, int64_t n,
                            int64_t* __restrict__ shard_off) {
  const int s = threadIdx.x;
  if (s < G) shard_off[s] = offs[int64_t(s) * nb];
  if (s == 0) shard_off[G] = n;
}

template <class T>
__global__ void gather_kernel(const T* __restrict__ src, const int64_t* __restrict__ perm, int64_t n,
                              T* __restrict__ dst) {
  const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[perm[i]];
}

}  // namespace kcep

using namespace kcep;

namespace {
int sfail(int code, const char* msg) { return set_error(code, msg); }
}  // namespace

extern "C" {

uint32_t cep_key_hash(int32_t key_id) { return fmix32(uint32_t(key_id)); }

int32_t cep_key_shard(int32_t key_id, int32_t n_shards) {
  return n_shards > 0 ? int32_t(fmix32(uint32_t(key_id)) % uint32_t(n_shards)) : -1;
}

int cep_shard_plan(const int64_t* key_events, int64_t n_keys, int32_t n_shards, int32_t rebalance,
                   int32_t* key_shard, int64_t* shard_events) {
  if (!key_shard || n_keys < 0 || n_shards <= 0 || (n_keys > 0 && !key_events))
    return sfail(CEP_E_ARG, "cep_shard_plan: bad argument");
  std::vector<int64_t> load(size_t(n_shards), 0);
  for (int64_t k = 0; k < n_keys; k++) {
    if (key_events[k] < 0) return sfail(CEP_E_ARG, "cep_shard_plan: negative event count");
    key_shard[k] = int32_t(fmix32(uint32_t(k)) % uint32_t(n_shards));
    load[size_t(key_shard[k])] += key_events[k];
  }
  if (rebalance && n_shards > 1 && n_keys > 0) {
    // equal-event rebalance: move a key from the fullest shard to the emptiest one -- the
    // largest key lighter than their gap, so both end below the old maximum -- until no key fits.
    // Every move lowers the sum of squared loads, so the loop ends.
    std::vector<std::set<std::pair<int64_t, int64_t>>> keys;
    keys.resize(size_t(n_shards));
    for (int64_t k = 0; k < n_keys; k++)
      if (key_events[k] > 0) keys[size_t(key_shard[k])].insert({key_events[k], k});
    for (int64_t it = 0; it < 4 * n_keys + 16; it++) {
      const auto mx = std::max_element(load.begin(), load.end()) - load.begin();
      const auto mn = std::min_element(load.begin(), load.end()) - load.begin();
      const int64_t gap = load[size_t(mx)] - load[size_t(mn)];
      auto& from = keys[size_t(mx)];
      auto itk = from.lower_bound({gap, -1});          // first key with events >= gap
      if (itk == from.begin()) break;
      --itk;                                           // the largest key lighter than the gap
      const auto kv = *itk;
      from.erase(itk);
      keys[size_t(mn)].insert(kv);
      key_shard[kv.second] = int32_t(mn);
      load[size_t(mx)] -= kv.first;
      load[size_t(mn)] += kv.first;
    }
  }
  if (shard_events)
    for (int32_t s = 0; s < n_shards; s++) shard_events[s] = load[size_t(s)];
  return CEP_OK;
}

int cep_partition(const int32_t* key_id, int64_t n, int32_t n_shards, const int32_t* key_shard, int64_t n_keys,
                  int64_t* perm, int64_t* shard_off, int32_t mem, void* stream) {
  if (n < 0 || n_shards <= 0 || n_shards > CEP_MAX_SHARDS || !shard_off || (n > 0 && (!key_id || !perm)))
    return sfail(CEP_E_ARG, "cep_partition: bad argument");
  if (mem == CEP_MEM_HOST) {
    std::vector<int64_t> cnt(size_t(n_shards) + 1, 0);
    for (int64_t i = 0; i < n; i++) cnt[size_t(shard_of(key_id[i], key_shard, n_keys, n_shards)) + 1]++;
    for (int32_t s = 0; s < n_shards; s++) cnt[size_t(s) + 1] += cnt[size_t(s)];
    for (int32_t s = 0; s <= n_shards; s++) shard_off[s] = cnt[size_t(s)];
    for (int64_t i = 0; i < n; i++) perm[cnt[size_t(shard_of(key_id[i], key_shard, n_keys, n_shards))]++] = i;
    return CEP_OK;
  }
  if (mem != CEP_MEM_DEVICE) return sfail(CEP_E_ARG, "cep_partition: bad mem");
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int64_t nb = std::max<int64_t>(1, (n + PT_TILE - 1) / PT_TILE);
  const int64_t m = nb * n_shards;
  // stream-ordered scratch: [shard][tile] counts, their offsets, scan partials (+ the total)
  const int64_t nt = m / 1024 + 4;
  int64_t* scratch = nullptr;
  if (hipMallocAsync(reinterpret_cast<void**>(&scratch), size_t(2 * m + nt) * 8, st) != hipSuccess)
    return sfail(CEP_E_HIP, "cep_partition: device allocation failed");
  int64_t *counts = scratch, *offs = scratch + m, *tmp = scratch + 2 * m;
  const size_t lds = size_t(n_shards) * PT_THREADS * 4;
  hipLaunchKernelGGL(part_count, dim3(unsigned(nb)), dim3(PT_THREADS), lds, st, key_id, n, key_shard, n_keys, n_shards,
                     nb, counts);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = exclusive_scan(counts, m, offs, tmp + nt - 1, tmp, st);
  if (e == hipSuccess && n > 0) {
    hipLaunchKernelGGL(part_scatter, dim3(unsigned(nb)), dim3(PT_THREADS), lds, st, key_id, n, key_shard, n_keys,
                       n_shards, nb, offs, perm);
    e = hipGetLastError();
  }
  if (e == hipSuccess) {
    hipLaunchKernelGGL(part_bounds, dim3(1), dim3(64), 0, st, offs, nb, n_shards, n, shard_off);
    e = hipGetLastError();
  }
  (void)hipFreeAsync(scratch, st);
  return e == hipSuccess ? CEP_OK : sfail(CEP_E_HIP, "cep_partition: launch failed");
}

int cep_gather(const void* src, int32_t elem_bytes, const int64_t* perm, int64_t n, void* dst, int32_t mem,
               void* stream) {
  if (n < 0 || (n > 0 && (!src || !perm || !dst)) || (elem_bytes != 1 && elem_bytes != 4 && elem_bytes != 8))
    return sfail(CEP_E_ARG, "cep_gather: bad argument");
  if (n == 0) return CEP_OK;
  if (mem == CEP_MEM_HOST) {
    for (int64_t i = 0; i < n; i++)
      memcpy(static_cast<char*>(dst) + i * elem_bytes, static_cast<const char*>(src) + perm[i] * elem_bytes,
             size_t(elem_bytes));
    return CEP_OK;
  }
  if (mem != CEP_MEM_DEVICE) return sfail(CEP_E_ARG, "cep_gather: bad mem");
  hipStream_t st = static_cast<hipStream_t>(stream);
  const dim3 g(unsigned((n + 255) / 256)), b(256);
  if (elem_bytes == 1)
    hipLaunchKernelGGL(gather_kernel<uint8_t>, g, b, 0, st, static_cast<const uint8_t*>(src), perm, n,
                       static_cast<uint8_t*>(dst));
  else if (elem_bytes == 4)
    hipLaunchKernelGGL(gather_kernel<uint32_t>, g, b, 0, st, static_cast<const uint32_t*>(src), perm, n,
                       static_cast<uint32_t*>(dst));
  else
    hipLaunchKernelGGL(gather_kernel<uint64_t>, g, b, 0, st, static_cast<const uint64_t*>(src), perm, n,
                       static_cast<uint64_t*>(dst));
  return hipGetLastError() == hipSuccess ? CEP_OK : sfail(CEP_E_HIP, "cep_gather: launch failed");
}

}  // extern "C"

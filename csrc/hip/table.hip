// Bucketized two-choice cuckoo hash table for the GPU sparse parameter server.
//
// Layout (SoA): keys[nb][16] (one 128-B line per bucket, kEmptyKey = free),
// fill[nb] (occupied prefix length), values[(nb*16 + stash) * stride] fp32 rows
// indexed by slot position.  Keys stored are h = mix64(feasign).
//
// Probe: one wave handles 4 queries; a 16-lane group loads one bucket line
// (16 x 8 B, fully coalesced), matches with a ballot, then the second bucket on
// a miss, then the (normally empty) stash.  The block's queries are staged in
// LDS first.  Inserts never race on a slot: a key claims slot
// atomicAdd(&fill[b], 1) of the emptier of its two buckets; the rare keys that
// find both buckets full go through a serial cuckoo displacement pass.
//
// Semantics reproduced: BoxPS FeedPass/BeginPass working-set build and
// PullSparseGPU/PushSparseGPU lookups (reference contract in
// paddle/fluid/framework/fleet/box_wrapper.cc:120-210,
// box_wrapper_impl.h:152-155,476-480); shrink/decay per
// distributed/ps/table/ctr_accessor.cc:63-80.
#include <hip/hip_runtime.h>

#include "kernels.h"
#include "table_probe.h"

namespace pbx {

namespace {

__device__ __forceinline__ uint64_t bucket1(uint64_t h, uint64_t nb) { return fast_range64(h, nb); }
__device__ __forceinline__ uint64_t bucket2(uint64_t h, uint64_t nb) {
  uint64_t b = fast_range64(rehash64(h), nb);
  return b;
}

__device__ void init_row(const TableDev& t, int64_t row, uint64_t key, const SparseSGDConfig& cfg,
                         uint64_t seed, int init_embedx) {
  const RowLayout l = make_row_layout(t.dim);
  float* v = t.values + row * (int64_t)t.stride;
  for (int c = 0; c < t.stride; ++c) v[c] = 0.f;
  if (cfg.initial_range > 0.f) v[kEmbedW] = (hash_uniform(key, seed) * 2.f - 1.f) * cfg.initial_range;
  if (init_embedx) {
    for (int d = 0; d < t.dim; ++d) v[kEmbedx + d] = hash_uniform(key, seed + 1 + d) * cfg.mf_initial_range;
    v[l.mf_size] = 1.f;
  }
}

// Row of mixed key `key` (kEmptyKey: -1) for the 16-lane group (sub, j) of
// the wave: bucket 1, bucket 2, then the (normally empty) stash.
__device__ __forceinline__ int64_t probe_group(const TableDev& t, uint64_t key, int sub, int j) {
  int64_t r = -1;
  if (key != kEmptyKey) {
    const uint64_t b1 = bucket1(key, t.nb);
    const uint64_t k1 = t.keys[b1 * kBucketSlots + j];
    uint64_t m = (__ballot(k1 == key) >> (sub * 16)) & 0xFFFFull;
    if (m) {
      r = (int64_t)(b1 * kBucketSlots) + (__ffsll((long long)m) - 1);
    } else {
      const uint64_t b2 = bucket2(key, t.nb);
      const uint64_t k2 = t.keys[b2 * kBucketSlots + j];
      m = (__ballot(k2 == key) >> (sub * 16)) & 0xFFFFull;
      if (m) {
        r = (int64_t)(b2 * kBucketSlots) + (__ffsll((long long)m) - 1);
      } else {
        const uint32_t sn = t.stash_n ? *t.stash_n : 0u;
        const uint32_t lim = sn < t.stash_cap ? sn : t.stash_cap;
        int64_t found = -1;
        for (uint32_t s = j; s < lim; s += 16)
          if (t.stash_keys[s] == key) found = (int64_t)(t.nb * kBucketSlots) + s;
        // reduce within the 16-lane group
        for (int off = 8; off > 0; off >>= 1) {
          long long o = __shfl_xor((long long)found, off, 16);
          found = found > o ? found : o;
        }
        r = found;
      }
    }
  }
  return r;
}

// MIX: the queries are raw feasigns (-1 = padding) mixed here, so a batch's
// occurrences are probed straight from its key buffer (no-dedup pull).
template <bool MIX>
__global__ __launch_bounds__(256) void k_probe(TableDev t, const uint64_t* __restrict__ h, int64_t n,
                                               const int32_t* n_dev, int64_t* __restrict__ rows) {
  __shared__ uint64_t q[16];
  const int64_t nn = n_dev ? (int64_t)*n_dev : n;
  const int64_t blk = (int64_t)blockIdx.x * 16;
  if (blk >= nn) return;
  if (threadIdx.x < 16) {
    uint64_t k = (blk + threadIdx.x < nn) ? h[blk + threadIdx.x] : kEmptyKey;
    if (MIX && k != kEmptyKey) k = mix64(k);
    q[threadIdx.x] = k;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int j = lane & 15;
  const int g = threadIdx.x >> 4;
  const int64_t r = probe_group(t, q[g], lane >> 4, j);
  if (j == 0 && blk + g < nn) rows[blk + g] = r;
}

// Per-thread probe: table_probe.h (shared with the fused probe of the seqpool).
__device__ __forceinline__ int64_t probe_thread(const TableDev& t, uint64_t key) { return table_probe_thread(t, key); }

// Table dedup of a single-shard batch (the pass-resident table row IS the
// unique id): one launch probes every occurrence and ranks it
// within its row -- per block, occurrences are counted per row in an LDS
// hash, then ONE global atomicAdd per distinct row per block on cnt_row[row]
// returns the block's base; the block that finds the count at 0 owns the
// row's unique id (one global atomic per block allocates the block's new
// ids).  k_table_seg turns the counts into run starts (and re-zeroes them),
// k_table_scatter writes perm.  Replaces the scratch-hash insert, rank and
// cleanup plus the separate probe of the unique keys.
// The counters [U, n_valid, -, segment cursor] accumulate in a private block
// (acc) that k_table_scatter publishes to u_count and re-zeroes, so a dedup
// needs no fill launch before it (acc is zero between dedups by construction).
// PROBE = false: rows_occ already holds every occurrence's row (the split
// pull probed it on the critical stream; this dedup runs on a side stream
// under the dense forward).
template <bool PROBE, int kTdItems, int kTdLds = 512 * kTdItems>  // LDS hash at load factor <= 1/2
__global__ __launch_bounds__(256) void k_table_rank(TableDev t, const uint64_t* __restrict__ keys, int64_t n,
                                                    int64_t* __restrict__ rows_occ, int32_t* __restrict__ rank,
                                                    int32_t* __restrict__ cnt_row, int64_t cnt_rs,
                                                    int32_t* __restrict__ uid_row,
                                                    int64_t* __restrict__ rows_u, int32_t* __restrict__ u_count) {
  __shared__ int32_t lkey[kTdLds];
  __shared__ int32_t lcnt[kTdLds];
  __shared__ int32_t lnew[kTdLds];
  __shared__ int32_t nvalid_blk, nnew_blk, base_blk;
  for (int e = threadIdx.x; e < kTdLds; e += blockDim.x) {
    lkey[e] = -1;
    lcnt[e] = 0;
  }
  if (threadIdx.x == 0) {
    nvalid_blk = 0;
    nnew_blk = 0;
  }
  __syncthreads();
  const int64_t i0 = (int64_t)blockIdx.x * (blockDim.x * kTdItems);
  int64_t row[kTdItems];
  int pos[kTdItems], lr[kTdItems];
  int nv = 0;
  if (PROBE) {
    // every item's bucket lines in flight together (table_probe_thread_n)
    uint64_t q[kTdItems];
#pragma unroll
    for (int it = 0; it < kTdItems; ++it) {
      const int64_t i = i0 + it * blockDim.x + threadIdx.x;
      const uint64_t k = i < n ? keys[i] : kEmptyKey;
      q[it] = k == kEmptyKey ? kEmptyKey : mix64(k);
    }
    table_probe_thread_n<kTdItems>(t, q, row);
  }
#pragma unroll
  for (int it = 0; it < kTdItems; ++it) {
    if (!PROBE) {
      const int64_t i = i0 + it * blockDim.x + threadIdx.x;
      row[it] = i < n ? rows_occ[i] : -1;
    }
    nv += row[it] >= 0;  // n_valid = occurrences placed in perm (absent keys are skipped like padding)
  }
#pragma unroll
  for (int it = 0; it < kTdItems; ++it) {
    pos[it] = -1;
    if (row[it] < 0) continue;
    const int32_t r = (int32_t)row[it];
    unsigned e = ((unsigned)r * 2654435761u) & (kTdLds - 1);
    for (;;) {
      const int32_t old = atomicCAS(&lkey[e], -1, r);
      if (old == -1 || old == r) break;
      e = (e + 1) & (kTdLds - 1);
    }
    pos[it] = (int)e;
    lr[it] = atomicAdd(&lcnt[e], 1);
  }
  if (nv) atomicAdd(&nvalid_blk, nv);
  __syncthreads();
  for (int e = threadIdx.x; e < kTdLds; e += blockDim.x) {
    const int32_t r = lkey[e];
    lnew[e] = -1;
    if (r < 0) continue;
    const int32_t base = atomicAdd(&cnt_row[(int64_t)r * cnt_rs], lcnt[e]);
    lcnt[e] = base;  // the block's base rank within row r
    if (base == 0) lnew[e] = atomicAdd(&nnew_blk, 1);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    base_blk = nnew_blk ? atomicAdd(&u_count[0], nnew_blk) : 0;
    if (nvalid_blk) atomicAdd(&u_count[1], nvalid_blk);
  }
  __syncthreads();
  for (int e = threadIdx.x; e < kTdLds; e += blockDim.x) {
    if (lnew[e] < 0) continue;
    const int32_t u = base_blk + lnew[e];
    uid_row[lkey[e]] = u;
    rows_u[u] = lkey[e];
  }
#pragma unroll
  for (int it = 0; it < kTdItems; ++it) {
    const int64_t i = i0 + it * blockDim.x + threadIdx.x;
    if (i >= n) continue;
    if (PROBE) rows_occ[i] = row[it];
    rank[i] = pos[it] >= 0 ? lcnt[pos[it]] + lr[it] : -1;
  }
}

// run starts: block exclusive scan of the per-row counts of the block's
// unique ids + one cursor atomic per block (runs contiguous, not id-ordered);
// the row counts are re-zeroed for the next batch
template <int kTdSegItems>
__global__ __launch_bounds__(256) void k_table_seg(const int64_t* __restrict__ rows_u, int32_t* __restrict__ cnt_row,
                                                   int64_t cnt_rs, int32_t* __restrict__ u_count,
                                                   int32_t* __restrict__ seg) {
  __shared__ int32_t wsum[4];
  __shared__ int32_t base;
  const int64_t U = u_count[0];
  const int64_t b0 = (int64_t)blockIdx.x * (blockDim.x * kTdSegItems);
  if (b0 >= U) return;  // block-uniform
  const int64_t u0 = b0 + (int64_t)threadIdx.x * kTdSegItems;
  int c[kTdSegItems];
  int tot = 0;
#pragma unroll
  for (int it = 0; it < kTdSegItems; ++it) {
    c[it] = 0;
    if (u0 + it < U) {
      const int64_t r = rows_u[u0 + it] * cnt_rs;
      c[it] = cnt_row[r];
      cnt_row[r] = 0;
    }
    tot += c[it];
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int x = tot;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(x, off);
    if (lane >= off) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  if (threadIdx.x == 0) base = atomicAdd(&u_count[3], wsum[0] + wsum[1] + wsum[2] + wsum[3]);
  __syncthreads();
  int p = base + x - tot;
  for (int i = 0; i < w; ++i) p += wsum[i];
#pragma unroll
  for (int it = 0; it < kTdSegItems; ++it) {
    if (u0 + it < U) seg[u0 + it] = p;
    p += c[it];
  }
}

// reset_rows: rows_occ is handed back all -1 (the split pull's fused probe
// writes only the occurrences inside the lod, so the padding must read -1)
__global__ void k_table_scatter(int64_t* __restrict__ rows_occ, const int32_t* __restrict__ rank,
                                const int32_t* __restrict__ uid_row, const int32_t* __restrict__ seg, int64_t n,
                                int32_t* __restrict__ uid, int32_t* __restrict__ perm, int reset_rows,
                                int32_t* __restrict__ acc, int32_t* __restrict__ u_count,
                                const int64_t* __restrict__ rows_u, int32_t* err) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < 4) {  // publish the counters, leave the accumulator zero for the next dedup
    u_count[i] = acc[i];
    acc[i] = 0;
  }
  if (i >= n) return;
  const int64_t r = rows_occ[i];
  if (reset_rows && r >= 0) rows_occ[i] = -1;
  if (r < 0) {
    uid[i] = -1;
    return;
  }
  const int32_t u = uid_row[r];
  // a row whose dedup counter was not zero at the dedup's start has no unique
  // id of this batch (its uid_row entry is stale): skipped and recorded
  if (u < 0 || u >= n) {
    uid[i] = -1;
    if (err) atomicOr(err, 2);
    return;
  }
  const int64_t q = (int64_t)seg[u] + rank[i];
  if (q < 0 || q >= n || rows_u[u] != r) {
    uid[i] = -1;
    if (err) atomicOr(err, 4);
    return;
  }
  uid[i] = u;
  perm[q] = (int32_t)i;
}

// Owner side of the sharded pull in one launch: probe every received key (one
// 16-lane group per key, as k_probe) and copy its pull record (P floats,
// zero padded to out_stride) straight into the answer buffer -- no dedup of
// the received keys (a key asked by several peers is simply read twice).
__global__ __launch_bounds__(256) void k_probe_gather(TableDev t, const uint64_t* __restrict__ h, int64_t n,
                                                      int64_t* __restrict__ rows, float* __restrict__ out,
                                                      int out_stride) {
  __shared__ uint64_t q[16];
  const int64_t blk = (int64_t)blockIdx.x * 16;
  if (blk >= n) return;
  if (threadIdx.x < 16) q[threadIdx.x] = (blk + threadIdx.x < n) ? h[blk + threadIdx.x] : kEmptyKey;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int sub = lane >> 4;
  const int j = lane & 15;
  const int g = threadIdx.x >> 4;
  const uint64_t key = q[g];
  const int64_t r = probe_group(t, key, sub, j);
  const int64_t e = blk + g;
  if (e >= n) return;
  if (j == 0) rows[e] = r;
  if (key == kEmptyKey) return;  // exchange padding: nobody reads its record
  // the group's 16 lanes copy the record (pull head = the row's first P floats)
  const int P = kPullHead + t.dim;
  float* o = out + e * (int64_t)out_stride;
  for (int c = j; c < out_stride; c += 16) o[c] = (r >= 0 && c < P) ? t.values[r * (int64_t)t.stride + c] : 0.f;
}

__global__ void k_insert(TableDev t, const uint64_t* __restrict__ h, int64_t n, const int32_t* n_dev,
                         const int64_t* __restrict__ rows, SparseSGDConfig cfg, uint64_t seed,
                         int init_embedx, uint64_t* ovf, uint32_t* ovf_n) {
  const int64_t nn = n_dev ? (int64_t)*n_dev : n;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nn) return;
  if (rows && rows[i] >= 0) return;
  const uint64_t key = h[i];
  if (key == kEmptyKey) return;
  const uint64_t b1 = bucket1(key, t.nb), b2 = bucket2(key, t.nb);
  const uint32_t f1 = __hip_atomic_load(&t.fill[b1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t f2 = __hip_atomic_load(&t.fill[b2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint64_t first = f1 <= f2 ? b1 : b2;
  const uint64_t second = f1 <= f2 ? b2 : b1;
  uint64_t cand[2] = {first, second};
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const uint32_t s = atomicAdd(&t.fill[cand[c]], 1u);
    if (s < kBucketSlots) {
      const int64_t row = (int64_t)cand[c] * kBucketSlots + s;
      init_row(t, row, key, cfg, seed, init_embedx);
      t.keys[row] = key;
      return;
    }
  }
  const uint32_t o = atomicAdd(ovf_n, 1u);
  ovf[o] = key;
}

__global__ void k_clamp_fill(TableDev t) {
  const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= t.nb) return;
  if (t.fill[b] > kBucketSlots) t.fill[b] = kBucketSlots;
}

// Serial random-walk cuckoo displacement; one thread (overflow is rare: a
// handful of keys per billion at the sizing load factor).
__global__ void k_resolve_overflow(TableDev t, const uint64_t* ovf, const uint32_t* ovf_n,
                                   SparseSGDConfig cfg, uint64_t seed, int init_embedx,
                                   uint32_t* fail_n) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  constexpr int kMaxStride = 160;
  float hand[kMaxStride];
  float tmp[kMaxStride];
  const uint32_t n = *ovf_n;
  const int64_t stash_row0 = (int64_t)(t.nb * kBucketSlots);
  for (uint32_t i = 0; i < n; ++i) {
    uint64_t cur = ovf[i];
    // build the fresh row in "hand" via a scratch row: reuse init_row on stash
    // row cap-1 is unsafe; compute inline instead.
    for (int c = 0; c < t.stride; ++c) hand[c] = 0.f;
    {
      const RowLayout l = make_row_layout(t.dim);
      if (cfg.initial_range > 0.f) hand[kEmbedW] = (hash_uniform(cur, seed) * 2.f - 1.f) * cfg.initial_range;
      if (init_embedx) {
        for (int d = 0; d < t.dim; ++d) hand[kEmbedx + d] = hash_uniform(cur, seed + 1 + d) * cfg.mf_initial_range;
        hand[l.mf_size] = 1.f;
      }
    }
    uint64_t prev_bucket = ~0ull;
    bool placed = false;
    for (int step = 0; step < 512 && !placed; ++step) {
      const uint64_t b1 = bucket1(cur, t.nb), b2 = bucket2(cur, t.nb);
      const uint64_t bs[2] = {b1, b2};
      for (int c = 0; c < 2 && !placed; ++c) {
        if (t.fill[bs[c]] < kBucketSlots) {
          const int64_t row = (int64_t)bs[c] * kBucketSlots + t.fill[bs[c]];
          t.fill[bs[c]] += 1;
          float* v = t.values + row * (int64_t)t.stride;
          for (int k = 0; k < t.stride; ++k) v[k] = hand[k];
          t.keys[row] = cur;
          placed = true;
        }
      }
      if (placed) break;
      // evict from the bucket we did not just come from
      uint64_t vb = (b1 == prev_bucket) ? b2 : (b2 == prev_bucket ? b1 : ((mix64(cur + step) & 1) ? b2 : b1));
      const int vs = (int)(mix64(cur ^ (seed + step)) & 15);
      const int64_t vrow = (int64_t)vb * kBucketSlots + vs;
      float* v = t.values + vrow * (int64_t)t.stride;
      for (int k = 0; k < t.stride; ++k) { tmp[k] = v[k]; v[k] = hand[k]; hand[k] = tmp[k]; }
      const uint64_t victim = t.keys[vrow];
      t.keys[vrow] = cur;
      cur = victim;
      prev_bucket = vb;
    }
    if (!placed) {
      const uint32_t s = *t.stash_n;
      if (s < t.stash_cap) {
        t.stash_keys[s] = cur;
        float* v = t.values + (stash_row0 + s) * (int64_t)t.stride;
        for (int k = 0; k < t.stride; ++k) v[k] = hand[k];
        *t.stash_n = s + 1;
      } else {
        atomicAdd(fail_n, 1u);
      }
    }
  }
}

__global__ void k_count(TableDev t, unsigned long long* count) {
  unsigned long long local = 0;
  for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < t.nb;
       b += (uint64_t)gridDim.x * blockDim.x)
    local += t.fill[b];
  for (int off = 32; off > 0; off >>= 1) local += __shfl_down(local, off);
  if ((threadIdx.x & 63) == 0) atomicAdd(count, local);
}

__global__ void k_export(TableDev t, uint64_t* out_keys, float* out_vals, unsigned long long* cursor) {
  const int64_t total = (int64_t)t.nb * kBucketSlots;
  const uint32_t sn = t.stash_n ? (*t.stash_n < t.stash_cap ? *t.stash_n : t.stash_cap) : 0;
  for (int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; row < total + sn;
       row += (int64_t)gridDim.x * blockDim.x) {
    uint64_t key;
    if (row < total) {
      const uint64_t b = row / kBucketSlots;
      if ((uint32_t)(row % kBucketSlots) >= t.fill[b]) continue;
      key = t.keys[row];
    } else {
      key = t.stash_keys[row - total];
    }
    if (key == kEmptyKey) continue;
    const unsigned long long o = atomicAdd(cursor, 1ull);
    out_keys[o] = key;
    if (out_vals) {
      const float* v = t.values + row * (int64_t)t.stride;
      float* dst = out_vals + (int64_t)o * t.stride;
      for (int k = 0; k < t.stride; ++k) dst[k] = v[k];
    }
  }
}

__global__ void k_assign(TableDev t, const int64_t* rows, const float* vals, int64_t n, int vs) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t r = rows[i];
  if (r < 0) return;
  float* dst = t.values + r * (int64_t)t.stride;
  const float* src = vals + i * (int64_t)vs;
  const int w = vs < t.stride ? vs : t.stride;
  for (int k = 0; k < w; ++k) dst[k] = src[k];
}

// One thread per bucket: decay, age, delete, compact to a prefix.
__global__ void k_shrink(TableDev t, ShrinkConfig c, unsigned long long* deleted) {
  const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= t.nb) return;
  const RowLayout l = make_row_layout(t.dim);
  const uint32_t f = t.fill[b];
  uint32_t w = 0;
  unsigned long long del = 0;
  for (uint32_t s = 0; s < f; ++s) {
    const int64_t row = (int64_t)b * kBucketSlots + s;
    float* v = t.values + row * (int64_t)t.stride;
    v[kShow] *= c.show_click_decay_rate;
    v[kClick] *= c.show_click_decay_rate;
    v[l.unseen_days] += 1.f;
    const float score = (v[kShow] - v[kClick]) * c.nonclk_coeff + v[kClick] * c.clk_coeff;
    const bool drop = score < c.delete_threshold || v[l.unseen_days] > c.delete_after_unseen_days;
    if (drop) { ++del; continue; }
    if (w != s) {
      const int64_t wr = (int64_t)b * kBucketSlots + w;
      float* dv = t.values + wr * (int64_t)t.stride;
      for (int k = 0; k < t.stride; ++k) dv[k] = v[k];
      t.keys[wr] = t.keys[row];
    }
    ++w;
  }
  for (uint32_t s = w; s < f; ++s) t.keys[(int64_t)b * kBucketSlots + s] = kEmptyKey;
  t.fill[b] = w;
  if (del) atomicAdd(deleted, del);
}

// Stash rows get the same decay / age / delete pass; the stash is compacted
// in order by one thread (it holds the rare keys whose cuckoo walk failed,
// normally none).
__global__ void k_shrink_stash(TableDev t, ShrinkConfig c, unsigned long long* deleted) {
  if (threadIdx.x != 0 || blockIdx.x != 0 || !t.stash_n) return;
  const RowLayout l = make_row_layout(t.dim);
  const int64_t row0 = (int64_t)(t.nb * kBucketSlots);
  const uint32_t n = *t.stash_n < t.stash_cap ? *t.stash_n : t.stash_cap;
  uint32_t w = 0;
  unsigned long long del = 0;
  for (uint32_t s = 0; s < n; ++s) {
    float* v = t.values + (row0 + s) * (int64_t)t.stride;
    v[kShow] *= c.show_click_decay_rate;
    v[kClick] *= c.show_click_decay_rate;
    v[l.unseen_days] += 1.f;
    const float score = (v[kShow] - v[kClick]) * c.nonclk_coeff + v[kClick] * c.clk_coeff;
    if (score < c.delete_threshold || v[l.unseen_days] > c.delete_after_unseen_days) {
      ++del;
      continue;
    }
    if (w != s) {
      float* dv = t.values + (row0 + w) * (int64_t)t.stride;
      for (int k = 0; k < t.stride; ++k) dv[k] = v[k];
      t.stash_keys[w] = t.stash_keys[s];
    }
    ++w;
  }
  for (uint32_t s = w; s < n; ++s) t.stash_keys[s] = kEmptyKey;
  *t.stash_n = w;
  if (del) atomicAdd(deleted, del);
}

}  // namespace

static inline unsigned int blocks_for(int64_t n, int per) {
  int64_t b = (n + per - 1) / per;
  return (unsigned int)(b < 1 ? 1 : b);
}

void launch_table_probe(const TableDev& t, const uint64_t* h, int64_t n, const int32_t* n_dev,
                        int64_t* rows, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_probe<false>, dim3(blocks_for(n, 16)), dim3(256), 0, s, t, h, n, n_dev, rows);
}

void launch_probe_raw(const TableDev& t, const int64_t* keys, int64_t n, int64_t* rows, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_probe<true>, dim3(blocks_for(n, 16)), dim3(256), 0, s, t,
                     reinterpret_cast<const uint64_t*>(keys), n, nullptr, rows);
}

void launch_table_dedup(const TableDev& t, const int64_t* keys, int64_t n, int64_t* rows_occ, int32_t* rank,
                        int32_t* cnt_row, int64_t cnt_rs, int32_t* uid_row, int64_t* rows_u, int32_t* uid,
                        int32_t* perm, int32_t* seg, int32_t* u_count, int32_t* acc, bool rows_given,
                        hipStream_t s, bool do_scatter, int stage) {
  if (n <= 0) {  // no scatter to publish the counters: [U, n_valid, -, cursor] = 0
    if (stage != 1) launch_fill32(reinterpret_cast<uint32_t*>(u_count), 0u, 4, s);
    return;
  }
  // occurrences per thread (PBX_TD_ITEMS 1 / 2 / 4): more probes in flight
  // per thread and fewer workgroups (fewer same-address u_count atomics);
  // same-box A/B 0.252-0.257 (2) vs 0.258-0.262 (1) vs 0.262-0.267 (4) ms/step
  static const int items = [] {
    const char* e = getenv("PBX_TD_ITEMS");
    const int v = e ? atoi(e) : 2;
    return (v == 1 || v == 4) ? v : 2;
  }();
#define PBX_TD_LAUNCH(PR, IT)                                                                                  \
  hipLaunchKernelGGL((k_table_rank<PR, IT>), dim3(blocks_for(n, 256 * IT)), dim3(256), 0, s, t,              \
                     reinterpret_cast<const uint64_t*>(keys), n, rows_occ, rank, cnt_row, cnt_rs, uid_row, rows_u, acc)
  if (stage != 2) {
    if (rows_given) {
      if (items == 4) PBX_TD_LAUNCH(false, 4);
      else if (items == 2) PBX_TD_LAUNCH(false, 2);
      else PBX_TD_LAUNCH(false, 1);
    } else {
      if (items == 4) PBX_TD_LAUNCH(true, 4);
      else if (items == 2) PBX_TD_LAUNCH(true, 2);
      else PBX_TD_LAUNCH(true, 1);
    }
  }
#undef PBX_TD_LAUNCH
  if (stage == 1) return;
  // unique ids per thread of the run-start scan (PBX_TD_SEG_ITEMS 1 / 2 / 4);
  // same-box A/B: 0.250-0.259 ms/step at 1 vs 0.255-0.262 at 4
  static const int seg_items = [] {
    const char* e = getenv("PBX_TD_SEG_ITEMS");
    const int v = e ? atoi(e) : 1;
    return (v == 2 || v == 4) ? v : 1;
  }();
  if (seg_items == 1)
    hipLaunchKernelGGL(k_table_seg<1>, dim3(blocks_for(n, 256)), dim3(256), 0, s, rows_u, cnt_row, cnt_rs, acc, seg);
  else if (seg_items == 2)
    hipLaunchKernelGGL(k_table_seg<2>, dim3(blocks_for(n, 512)), dim3(256), 0, s, rows_u, cnt_row, cnt_rs, acc, seg);
  else
    hipLaunchKernelGGL(k_table_seg<4>, dim3(blocks_for(n, 1024)), dim3(256), 0, s, rows_u, cnt_row, cnt_rs, acc, seg);
  if (!do_scatter) return;  // the caller's seqpool launch scatters (SeqpoolCvmArgs.sc_*)
  hipLaunchKernelGGL(k_table_scatter, dim3(blocks_for(n, 256)), dim3(256), 0, s, rows_occ, rank, uid_row, seg, n, uid,
                     perm, rows_given ? 1 : 0, acc, u_count, rows_u, t.err);
}

void launch_probe_gather(const TableDev& t, const uint64_t* h, int64_t n, int64_t* rows, float* out, int out_stride,
                         hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_probe_gather, dim3(blocks_for(n, 16)), dim3(256), 0, s, t, h, n, rows, out, out_stride);
}

void launch_table_insert(const TableDev& t, const uint64_t* h, int64_t n, const int32_t* n_dev,
                         const int64_t* rows, const SparseSGDConfig& cfg, uint64_t seed,
                         int init_embedx, uint64_t* ovf_keys, uint32_t* ovf_n, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_insert, dim3(blocks_for(n, 256)), dim3(256), 0, s, t, h, n, n_dev, rows, cfg,
                     seed, init_embedx, ovf_keys, ovf_n);
}

void launch_table_clamp_fill(const TableDev& t, hipStream_t s) {
  hipLaunchKernelGGL(k_clamp_fill, dim3(blocks_for((int64_t)t.nb, 256)), dim3(256), 0, s, t);
}

void launch_table_resolve_overflow(const TableDev& t, const uint64_t* ovf_keys,
                                   const uint32_t* ovf_n, const SparseSGDConfig& cfg, uint64_t seed,
                                   int init_embedx, uint32_t* fail_n, hipStream_t s) {
  hipLaunchKernelGGL(k_resolve_overflow, dim3(1), dim3(64), 0, s, t, ovf_keys, ovf_n, cfg, seed,
                     init_embedx, fail_n);
}

void launch_table_count(const TableDev& t, unsigned long long* count, hipStream_t s) {
  hipLaunchKernelGGL(k_count, dim3(1024), dim3(256), 0, s, t, count);
}

void launch_table_export(const TableDev& t, uint64_t* out_keys, float* out_vals,
                         unsigned long long* cursor, hipStream_t s) {
  hipLaunchKernelGGL(k_export, dim3(2048), dim3(256), 0, s, t, out_keys, out_vals, cursor);
}

void launch_table_assign(const TableDev& t, const int64_t* rows, const float* vals, int64_t n,
                         int vals_stride, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_assign, dim3(blocks_for(n, 256)), dim3(256), 0, s, t, rows, vals, n, vals_stride);
}

void launch_table_shrink(const TableDev& t, const ShrinkConfig& c, unsigned long long* deleted,
                         hipStream_t s) {
  hipLaunchKernelGGL(k_shrink, dim3(blocks_for((int64_t)t.nb, 256)), dim3(256), 0, s, t, c, deleted);
  if (t.stash_cap > 0) hipLaunchKernelGGL(k_shrink_stash, dim3(1), dim3(64), 0, s, t, c, deleted);
}

}  // namespace pbx

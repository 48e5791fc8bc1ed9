// Device-side probe of the bucketized cuckoo table (table.hip layout), shared
// by the table kernels and the fused probe of the split pull's seqpool.
#pragma once
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace pbx {

// Per-thread probe of one mixed key (8 x 16-B loads per bucket line, all in
// flight at once): used where every thread owns one occurrence (the table
// dedup, the split pull's seqpool), so many independent bucket reads overlap
// instead of one 16-lane group per key.
__device__ __forceinline__ int64_t table_probe_thread(const TableDev& t, uint64_t key) {
  if (key == kEmptyKey) return -1;
#pragma unroll
  for (int which = 0; which < 2; ++which) {
    const uint64_t b = which == 0 ? fast_range64(key, t.nb) : fast_range64(rehash64(key), t.nb);
    const uint4* p = reinterpret_cast<const uint4*>(t.keys + b * kBucketSlots);
    uint4 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = p[j];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint64_t k0 = (uint64_t)v[j].x | ((uint64_t)v[j].y << 32);
      const uint64_t k1 = (uint64_t)v[j].z | ((uint64_t)v[j].w << 32);
      if (k0 == key) return (int64_t)(b * kBucketSlots) + 2 * j;
      if (k1 == key) return (int64_t)(b * kBucketSlots) + 2 * j + 1;
    }
  }
  const uint32_t sn = t.stash_n ? *t.stash_n : 0u;
  const uint32_t lim = sn < t.stash_cap ? sn : t.stash_cap;
  for (uint32_t s = 0; s < lim; ++s)
    if (t.stash_keys[s] == key) return (int64_t)(t.nb * kBucketSlots) + s;
  return -1;
}

// Batched per-thread probe of N keys: every key's first bucket line is
// loaded before any is scanned, then the misses' second lines together -- at
// most two dependent memory round trips per thread instead of 2N (same result
// as table_probe_thread per key: a key sits in one slot at most).
__device__ __forceinline__ void table_load_line(const TableDev& t, uint64_t b, uint4 (&v)[8]) {
  const uint4* p = reinterpret_cast<const uint4*>(t.keys + b * kBucketSlots);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = p[j];
}
__device__ __forceinline__ int64_t table_scan_line(const uint4 (&v)[8], uint64_t b, uint64_t key) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint64_t k0 = (uint64_t)v[j].x | ((uint64_t)v[j].y << 32);
    const uint64_t k1 = (uint64_t)v[j].z | ((uint64_t)v[j].w << 32);
    if (k0 == key) return (int64_t)(b * kBucketSlots) + 2 * j;
    if (k1 == key) return (int64_t)(b * kBucketSlots) + 2 * j + 1;
  }
  return -1;
}
template <int N>
__device__ __forceinline__ void table_probe_thread_n(const TableDev& t, const uint64_t (&key)[N], int64_t (&r)[N]) {
  uint4 v[N][8];
  uint64_t b[N];
#pragma unroll
  for (int n = 0; n < N; ++n) {
    b[n] = key[n] == kEmptyKey ? 0 : fast_range64(key[n], t.nb);
    if (key[n] != kEmptyKey) table_load_line(t, b[n], v[n]);
  }
  bool miss[N];
  bool any = false;
#pragma unroll
  for (int n = 0; n < N; ++n) {
    r[n] = key[n] == kEmptyKey ? -1 : table_scan_line(v[n], b[n], key[n]);
    miss[n] = key[n] != kEmptyKey && r[n] < 0;
    any = any || miss[n];
  }
  if (!any) return;
#pragma unroll
  for (int n = 0; n < N; ++n)
    if (miss[n]) {
      b[n] = fast_range64(rehash64(key[n]), t.nb);
      table_load_line(t, b[n], v[n]);
    }
  const uint32_t sn = t.stash_n ? *t.stash_n : 0u;
  const uint32_t lim = sn < t.stash_cap ? sn : t.stash_cap;
#pragma unroll
  for (int n = 0; n < N; ++n) {
    if (!miss[n]) continue;
    r[n] = table_scan_line(v[n], b[n], key[n]);
    if (r[n] >= 0) continue;
    for (uint32_t s = 0; s < lim; ++s)
      if (t.stash_keys[s] == key[n]) r[n] = (int64_t)(t.nb * kBucketSlots) + s;
  }
}

// The key stored at row r (bucket slots, then the stash).  Lazy embedx
// creation draws a row's initial values from its key, not its row index, so a
// key gets the same values whichever shard and row hold it (an N-rank run
// equals the one-rank run on the union batch).
__device__ __forceinline__ uint64_t table_row_key(const TableDev& t, int64_t r) {
  const int64_t total = (int64_t)t.nb * kBucketSlots;
  return r < total ? t.keys[r] : t.stash_keys[r - total];
}

}  // namespace pbx

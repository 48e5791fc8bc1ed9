// Batch feature dedup (BoxPS DedupKeysAndFillIdx contract: reference call sites
// paddle/fluid/framework/fleet/box_wrapper_impl.h:128-136,292-300; open
// analogue heter_ps/heter_comm_inl.h:2231-2343).
//
// Keys are mixed (h = mix64(key), a bijection) and radix-sorted together with
// their original positions.  Because the owner shard is a monotone function of
// h, the unique list comes out already grouped by owner GPU, which is what the
// key all-to-all needs -- no separate partition pass.
//
// Outputs: uniq_h[U] (sorted), seg[U+1] segment starts into perm (sorted
// position -> original index), uid[i] (original index -> unique id), U on the
// device (no host sync, graph-capturable; padding keys == kEmptyKey sort last
// and are excluded).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <hipcub/hipcub.hpp>

#include "kernels.h"

namespace pbx {
namespace {

__global__ void k_mix(const uint64_t* __restrict__ keys, int64_t n, int mixed, uint64_t* __restrict__ h,
                      int32_t* __restrict__ idx) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t k = keys[i];
  h[i] = (k == kEmptyKey) ? kEmptyKey : (mixed ? k : mix64(k));
  idx[i] = (int32_t)i;
}

__global__ void k_heads(const uint64_t* __restrict__ hs, int64_t n, int32_t* __restrict__ flags) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t v = hs[i];
  flags[i] = (v != kEmptyKey && (i == 0 || hs[i - 1] != v)) ? 1 : 0;
}

// scan = inclusive prefix of head flags -> unique id = scan - 1
__global__ void k_emit(const uint64_t* __restrict__ hs, const int32_t* __restrict__ perm,
                       const int32_t* __restrict__ flags, const int32_t* __restrict__ scan, int64_t n,
                       int32_t* __restrict__ uid, uint64_t* __restrict__ uniq_h, int32_t* __restrict__ seg,
                       int32_t* __restrict__ u_count) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t v = hs[i];
  const int32_t o = perm[i];
  if (v == kEmptyKey) {
    uid[o] = -1;
    // first padding element closes the last segment
    if (i == 0 || hs[i - 1] != kEmptyKey) {
      const int32_t u = (i == 0) ? 0 : scan[i - 1];
      seg[u] = (int32_t)i;
      u_count[0] = u;
      u_count[1] = (int32_t)i;  // number of valid occurrences
    }
    return;
  }
  const int32_t u = scan[i] - 1;
  uid[o] = u;
  if (flags[i]) {
    uniq_h[u] = v;
    seg[u] = (int32_t)i;
  }
  if (i == n - 1) {
    seg[u + 1] = (int32_t)n;
    u_count[0] = u + 1;
    u_count[1] = (int32_t)n;
  }
}


// ---------------------------------------------------------------- hash dedup
// Sort-free variant (no consumer needs the unique list in any order: the
// single-shard engine, the sender before the owner pack, and the owner side
// of the key all-to-all):
//   insert   : block-local pre-dedup in an LDS hash, then one open-addressing
//              insert per distinct key into a scratch table (read before CAS);
//              the block's winners take their unique ids with ONE global
//              atomic (a single counter word saturates near 90 returning
//              atomics/us, so per-wave allocation was the bottleneck)
//   rank     : per block, occurrences are counted per unique id in an LDS
//              hash (LDS atomics), then ONE global atomicAdd per distinct id per
//              block returns the block's base -> rank of every occurrence
//              within its id (Zipf-hot ids see <= #blocks global atomics);
//              cnt[u] ends as the occurrence count of u
//   seg      : block exclusive scan of cnt + one atomic per block on a cursor:
//              seg[u] = start of u's run in perm.  Runs are contiguous but not
//              in id order (nobody needs that), which replaces a device-wide
//              scan (two launches) with one short kernel
//   scatter  : perm[seg[u] + rank] = occurrence
// The used table slots are released by k_seg_alloc (the table is not read
// after k_hash_rank) and the per-id counts at the start of the next run, so
// there is no per-batch memset of the table.
// u_count = [U, n_valid, U of the previous run, segment cursor]
// occurrences per thread in k_hash_rank (LDS hash at load <= 0.5) and unique
// ids per thread in k_seg_alloc: template parameters, picked at launch
// (PBX_HASH_RANK_ITEMS 1/2/4, PBX_HASH_SEG_ITEMS 1/2/4)

__global__ void k_hash_cleanup(int32_t* __restrict__ u_count, int32_t* __restrict__ cnt, int64_t cap,
                               int32_t* __restrict__ zero_extra, int zero_n) {
  // the previous run's scatter kernel saved its U into [2], so [0], [1] and
  // the cursor [3] can be reset here; its table slots were already released
  // by its k_seg_alloc, so only the (coalesced) per-id counts remain
  const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u == 0) {
    u_count[0] = 0;
    u_count[1] = 0;
    u_count[3] = 0;
  }
  if (u < zero_n) zero_extra[u] = 0;  // a consumer's counters, zeroed here instead of by a launch of their own
  if (u >= cap || u >= u_count[2]) return;
  cnt[u] = 0;
}

// Block-level pre-dedup in LDS (64-bit CAS) so a Zipf-hot key costs at most
// one global table operation per block, and a read-before-CAS so keys that
// are already present take no atomic at all.
constexpr int kInsItems = 2;
constexpr int kInsLds = 1024;
__global__ __launch_bounds__(256) void k_hash_insert(const uint64_t* __restrict__ keys, int64_t n, int mixed,
                                                     uint64_t* __restrict__ tk, int32_t* __restrict__ tu,
                                                     uint64_t tmask, int32_t* __restrict__ slot,
                                                     int32_t* __restrict__ slot_of_u, uint64_t* __restrict__ uniq_h,
                                                     int32_t* __restrict__ u_count) {
  __shared__ unsigned long long lk[kInsLds];
  __shared__ int32_t lslot[kInsLds];
  __shared__ int32_t nvalid_blk, nwon_blk, base_blk;
  for (int e = threadIdx.x; e < kInsLds; e += blockDim.x) lk[e] = (unsigned long long)kEmptyKey;
  if (threadIdx.x == 0) {
    nvalid_blk = 0;
    nwon_blk = 0;
  }
  __syncthreads();
  const int64_t i0 = (int64_t)blockIdx.x * (blockDim.x * kInsItems);
  int pos[kInsItems];
  bool own[kInsItems];
  uint64_t hv[kInsItems];
  int nv = 0;
  // 1) block-local dedup
#pragma unroll
  for (int t = 0; t < kInsItems; ++t) {
    const int64_t i = i0 + t * blockDim.x + threadIdx.x;
    pos[t] = -1;
    own[t] = false;
    if (i >= n) continue;
    const uint64_t k = keys[i];
    if (k == kEmptyKey) {
      slot[i] = -1;
      continue;
    }
    ++nv;
    const uint64_t h = mixed ? k : mix64(k);
    hv[t] = h;
    unsigned e = (unsigned)(rehash64(h) >> 40) & (kInsLds - 1);
    for (;;) {
      const unsigned long long old = atomicCAS(&lk[e], (unsigned long long)kEmptyKey, (unsigned long long)h);
      if (old == (unsigned long long)kEmptyKey) { own[t] = true; break; }
      if (old == (unsigned long long)h) break;
      e = (e + 1) & (kInsLds - 1);
    }
    pos[t] = (int)e;
  }
  if (nv) atomicAdd(&nvalid_blk, nv);
  // 2) one global insert per distinct key of the block
  bool won[kInsItems];
  uint64_t gp[kInsItems];
#pragma unroll
  for (int t = 0; t < kInsItems; ++t) {
    won[t] = false;
    if (!own[t]) continue;
    const uint64_t h = hv[t];
    uint64_t p = rehash64(h) & tmask;
    for (;;) {
      unsigned long long cur = *reinterpret_cast<volatile unsigned long long*>(&tk[p]);
      if (cur == (unsigned long long)h) break;
      if (cur == (unsigned long long)kEmptyKey) {
        cur = atomicCAS(reinterpret_cast<unsigned long long*>(&tk[p]), (unsigned long long)kEmptyKey,
                        (unsigned long long)h);
        if (cur == (unsigned long long)kEmptyKey) { won[t] = true; break; }
        if (cur == (unsigned long long)h) break;
      }
      p = (p + 1) & tmask;
    }
    gp[t] = p;
    lslot[pos[t]] = (int32_t)p;
  }
  // new ids: block-local ranks (LDS atomics), one global atomic per block
  int lid[kInsItems];
#pragma unroll
  for (int t = 0; t < kInsItems; ++t) lid[t] = won[t] ? atomicAdd(&nwon_blk, 1) : -1;
  __syncthreads();
  if (threadIdx.x == 0) {
    base_blk = nwon_blk ? atomicAdd(&u_count[0], nwon_blk) : 0;
    if (nvalid_blk) atomicAdd(&u_count[1], nvalid_blk);
  }
  __syncthreads();
#pragma unroll
  for (int t = 0; t < kInsItems; ++t) {
    if (!won[t]) continue;
    const int u = base_blk + lid[t];
    tu[gp[t]] = u;
    uniq_h[u] = hv[t];
    slot_of_u[u] = (int32_t)gp[t];
  }
  // 3) every occurrence takes its key's global slot (lslot is complete
  // after the barriers above)
#pragma unroll
  for (int t = 0; t < kInsItems; ++t) {
    const int64_t i = i0 + t * blockDim.x + threadIdx.x;
    if (pos[t] >= 0) slot[i] = lslot[pos[t]];
  }
}

template <int kRankItems, int kRankLds = 512 * kRankItems>
__global__ __launch_bounds__(256) void k_hash_rank(const int32_t* __restrict__ slot, const int32_t* __restrict__ tu,
                                                   int64_t n, int32_t* __restrict__ uid, int32_t* __restrict__ cnt,
                                                   int32_t* __restrict__ rank) {
  __shared__ int32_t lkey[kRankLds];
  __shared__ int32_t lcnt[kRankLds];
  for (int e = threadIdx.x; e < kRankLds; e += blockDim.x) {
    lkey[e] = -1;
    lcnt[e] = 0;
  }
  __syncthreads();
  const int64_t i0 = (int64_t)blockIdx.x * (blockDim.x * kRankItems);
  int pos[kRankItems], lr[kRankItems];
#pragma unroll
  for (int t = 0; t < kRankItems; ++t) {
    const int64_t i = i0 + t * blockDim.x + threadIdx.x;
    pos[t] = -1;
    if (i >= n) continue;
    const int32_t sl = slot[i];
    const int32_t u = sl >= 0 ? tu[sl] : -1;
    uid[i] = u;
    if (u < 0) continue;
    unsigned e = ((unsigned)u * 2654435761u) & (kRankLds - 1);
    for (;;) {
      const int32_t old = atomicCAS(&lkey[e], -1, u);
      if (old == -1 || old == u) break;
      e = (e + 1) & (kRankLds - 1);
    }
    pos[t] = (int)e;
    lr[t] = atomicAdd(&lcnt[e], 1);
  }
  __syncthreads();
  for (int e = threadIdx.x; e < kRankLds; e += blockDim.x) {
    const int32_t u = lkey[e];
    if (u >= 0) lcnt[e] = atomicAdd(&cnt[u], lcnt[e]);  // block base within id u
  }
  __syncthreads();
#pragma unroll
  for (int t = 0; t < kRankItems; ++t) {
    const int64_t i = i0 + t * blockDim.x + threadIdx.x;
    if (pos[t] >= 0) rank[i] = lcnt[pos[t]] + lr[t];
  }
}

// Also releases the run's hash-set slots (tk / tu are not read after
// k_hash_rank): the random slot writes ride on this kernel's pass over the
// ids instead of a separate cleanup pass at the start of the next run.
template <int kSegItems>
__global__ __launch_bounds__(256) void k_seg_alloc(const int32_t* __restrict__ cnt, int32_t* __restrict__ u_count,
                                                   int32_t* __restrict__ seg, const int32_t* __restrict__ slot_of_u,
                                                   uint64_t* __restrict__ tk, int32_t* __restrict__ tu) {
  __shared__ int32_t wsum[4];
  __shared__ int32_t base;
  const int64_t U = u_count[0];
  const int64_t u0 = (int64_t)blockIdx.x * (blockDim.x * kSegItems) + (int64_t)threadIdx.x * kSegItems;
  if ((int64_t)blockIdx.x * (blockDim.x * kSegItems) >= U) return;  // block-uniform
  int c[kSegItems];
  int tot = 0;
#pragma unroll
  for (int t = 0; t < kSegItems; ++t) {
    c[t] = (u0 + t < U) ? cnt[u0 + t] : 0;
    tot += c[t];
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int x = tot;  // inclusive wave scan of the per-thread totals
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
  for (int t = 0; t < kSegItems; ++t) {
    if (u0 + t < U) {
      seg[u0 + t] = p;
      const int32_t sl = slot_of_u[u0 + t];
      tk[sl] = kEmptyKey;
      tu[sl] = -1;
    }
    p += c[t];
  }
}

__global__ void k_hash_scatter(const int32_t* __restrict__ uid, const int32_t* __restrict__ rank,
                               const int32_t* __restrict__ seg, int64_t n, int32_t* __restrict__ perm,
                               int32_t* __restrict__ u_count) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) u_count[2] = u_count[0];  // for the next run's cleanup
  if (i >= n) return;
  const int32_t u = uid[i];
  if (u >= 0) perm[seg[u] + rank[i]] = (int32_t)i;
}

}  // namespace

size_t dedup_temp_bytes(int64_t n) {
  size_t a = 0, b = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, a, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                     (const int32_t*)nullptr, (int32_t*)nullptr, (int)n);
  (void)hipcub::DeviceScan::InclusiveSum(nullptr, b, (const int32_t*)nullptr, (int32_t*)nullptr, (int)n);
  return (a > b ? a : b) + 256;
}

void launch_dedup(const uint64_t* keys, int64_t n, bool keys_are_mixed, uint64_t* h_tmp,
                  uint64_t* h_sorted, int32_t* idx_tmp, int32_t* perm, int32_t* flags,
                  int32_t* scan, int32_t* uid, uint64_t* uniq_h, int32_t* seg, int32_t* u_count,
                  void* temp, size_t temp_bytes, hipStream_t s) {
  if (n <= 0) {
    launch_fill32(u_count, 0u, 2, s);
    launch_fill32(seg, 0u, 1, s);
    return;
  }
  const unsigned int g = (unsigned int)((n + 255) / 256);
  hipLaunchKernelGGL(k_mix, dim3(g), dim3(256), 0, s, keys, n, keys_are_mixed ? 1 : 0, h_tmp, idx_tmp);
  size_t tb = temp_bytes;
  (void)hipcub::DeviceRadixSort::SortPairs(temp, tb, h_tmp, h_sorted, idx_tmp, perm, (int)n, 0, 64, s);
  hipLaunchKernelGGL(k_heads, dim3(g), dim3(256), 0, s, h_sorted, n, flags);
  tb = temp_bytes;
  (void)hipcub::DeviceScan::InclusiveSum(temp, tb, flags, scan, (int)n, s);
  hipLaunchKernelGGL(k_emit, dim3(g), dim3(256), 0, s, h_sorted, perm, flags, scan, n, uid, uniq_h,
                     seg, u_count);
}

size_t hash_dedup_temp_bytes(int64_t cap) {
  (void)cap;
  return 256;
}

void launch_dedup_hash(const HashDedupArgs& a, void* temp, size_t temp_bytes, hipStream_t s) {
  const int64_t cap = a.cap;
  const unsigned gc = (unsigned)((cap + 255) / 256);
  hipLaunchKernelGGL(k_hash_cleanup, dim3(gc), dim3(256), 0, s, a.u_count, a.cnt, cap, a.zero_extra, a.zero_n);
  if (a.n <= 0) {
    launch_fill32(a.seg, 0u, 1, s);
    launch_fill32(a.u_count + 2, 0u, 1, s);
    return;
  }
  const unsigned g = (unsigned)((a.n + 255) / 256);
  const unsigned gi = (unsigned)((a.n + 256 * kInsItems - 1) / (256 * kInsItems));
  hipLaunchKernelGGL(k_hash_insert, dim3(gi), dim3(256), 0, s, a.keys, a.n, a.mixed, a.tk, a.tu, a.tmask, a.slot,
                     a.slot_of_u, a.uniq_h, a.u_count);
  auto env_items = [](const char* name, int dflt) {
    const char* e = getenv(name);
    const int v = e ? atoi(e) : dflt;
    return (v == 1 || v == 2 || v == 4) ? v : dflt;
  };
  static const int ri = env_items("PBX_HASH_RANK_ITEMS", 4), si = env_items("PBX_HASH_SEG_ITEMS", 4);
  const unsigned gr = (unsigned)((a.n + 256 * ri - 1) / (256 * ri));
  if (ri == 1) hipLaunchKernelGGL(k_hash_rank<1>, dim3(gr), dim3(256), 0, s, a.slot, a.tu, a.n, a.uid, a.cnt, a.rank);
  else if (ri == 2) hipLaunchKernelGGL(k_hash_rank<2>, dim3(gr), dim3(256), 0, s, a.slot, a.tu, a.n, a.uid, a.cnt, a.rank);
  else hipLaunchKernelGGL(k_hash_rank<4>, dim3(gr), dim3(256), 0, s, a.slot, a.tu, a.n, a.uid, a.cnt, a.rank);
  (void)temp;
  (void)temp_bytes;
  const unsigned gs = (unsigned)((a.n + 256 * si - 1) / (256 * si));  // U <= n
  if (si == 1)
    hipLaunchKernelGGL(k_seg_alloc<1>, dim3(gs), dim3(256), 0, s, a.cnt, a.u_count, a.seg, a.slot_of_u, a.tk, a.tu);
  else if (si == 2)
    hipLaunchKernelGGL(k_seg_alloc<2>, dim3(gs), dim3(256), 0, s, a.cnt, a.u_count, a.seg, a.slot_of_u, a.tk, a.tu);
  else
    hipLaunchKernelGGL(k_seg_alloc<4>, dim3(gs), dim3(256), 0, s, a.cnt, a.u_count, a.seg, a.slot_of_u, a.tk, a.tu);
  hipLaunchKernelGGL(k_hash_scatter, dim3(g), dim3(256), 0, s, a.uid, a.rank, a.seg, a.n, a.perm, a.u_count);
}

}  // namespace pbx

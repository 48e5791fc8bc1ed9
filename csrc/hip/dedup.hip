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
    (void)hipMemsetAsync(u_count, 0, 2 * sizeof(int32_t), s);
    (void)hipMemsetAsync(seg, 0, sizeof(int32_t), s);
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

}  // namespace pbx

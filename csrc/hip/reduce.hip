// Column reduction of per-block partial slabs: out[c] += sum_r part[r, c].
// grid (ceil(W/64), ceil(R/64)); lane -> column, the 4 waves split a 64-row
// chunk, LDS combine, one atomic per column per block (R/64 adders per
// address -- no hot-address serialisation; the one-thread-per-column form
// walked all R rows serially and took 60-130 us on a 512 x 600 slab).
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace pbx {
namespace {

__global__ __launch_bounds__(256) void k_colsum(const float* __restrict__ part, int R, int W, float* __restrict__ out,
                                                int split_col, float* __restrict__ out2) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const int r0 = blockIdx.y * 64;
  const int r1 = min(R, r0 + 64);
  float s = 0.f;
  if (c < W)
    for (int r = r0 + w; r < r1; r += 4) s += part[(int64_t)r * W + c];
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && c < W) {
    const float t = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
    if (c < split_col) atomicAdd(&out[c], t);
    else atomicAdd(&out2[c - split_col], t);
  }
}

// 32-bit fill.  Replaces hipMemsetAsync inside captured steps: a memset
// node of a HIP graph was observed to leave the last bytes of a buffer whose
// size is not a multiple of 16 unwritten on replay (data_norm statistics of
// the last columns went stale in tests/test_gpu_fluid.py).
__global__ void k_fill32(uint32_t* __restrict__ p, uint32_t v, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

}  // namespace

void launch_fill32(void* p, uint32_t v, int64_t n_words, hipStream_t s) {
  if (n_words <= 0) return;
  hipLaunchKernelGGL(k_fill32, dim3((unsigned)((n_words + 255) / 256)), dim3(256), 0, s,
                     reinterpret_cast<uint32_t*>(p), v, n_words);
}

void launch_colsum_acc(const float* part, int R, int W, float* out, int split_col, float* out2, hipStream_t s) {
  if (R == 0 || W == 0) return;
  const dim3 g((W + 63) / 64, (R + 63) / 64);
  hipLaunchKernelGGL(k_colsum, g, dim3(256), 0, s, part, R, W, out, split_col < 0 ? W : split_col, out2);
}

}  // namespace pbx

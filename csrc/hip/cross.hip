// DCN-V2 cross network helpers (the GEMMs themselves run on gemm.hip's MFMA
// kernel with the EPI_CROSS_* epilogues):
//   k_cross_dot      s[m] = x_L[m, :] . w_c            (wave per row)
//   k_cross_top_bwd  top of the backward: g_L = ds (x) w_c, u = bf16(x0 * g_L),
//                    acc = z_{L-1} * g_L, per-block partials of dw_c
// Reference: the cross layer is a fluid program composition in PaddleBox
// (SURVEY §7.4 M6 / BASELINE config 5); here it is one op per direction.
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace pbx {
namespace {

constexpr int kTopRows = 32;

__device__ __forceinline__ unsigned short f2bf_c(float f) {
  unsigned int u = __float_as_uint(f);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (unsigned short)(u >> 16);
}

__global__ __launch_bounds__(256) void k_cross_dot(const float* __restrict__ x, int M, int N, int ld,
                                                   const float* __restrict__ w, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int m = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= M) return;
  float s = 0.f;
  for (int n = lane; n < N; n += 64) s += x[(int64_t)m * ld + n] * w[n];
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
  if (lane == 0) out[m] = s;
}

__global__ __launch_bounds__(256) void k_cross_top_bwd(const float* __restrict__ x, const unsigned short* __restrict__ x0,
                                                       int ldx0, const float* __restrict__ z,
                                                       const float* __restrict__ w, const float* __restrict__ ds, int M,
                                                       int N, int ld, float* __restrict__ g,
                                                       unsigned short* __restrict__ u, float* __restrict__ acc,
                                                       float* __restrict__ part) {
  const int m0 = blockIdx.x * kTopRows, m1 = min(M, m0 + kTopRows);
  for (int n = threadIdx.x; n < N; n += blockDim.x) {
    const float wn = w[n];
    float p = 0.f;
    for (int m = m0; m < m1; ++m) {
      const int64_t o = (int64_t)m * ld + n;
      const float d = ds[m];
      const float gv = d * wn;
      const float x0v = __uint_as_float(((unsigned)x0[(int64_t)m * ldx0 + n]) << 16);
      g[o] = gv;
      u[o] = f2bf_c(x0v * gv);
      acc[o] = z[o] * gv;
      p += d * x[o];
    }
    part[(int64_t)blockIdx.x * N + n] = p;
  }
}

}  // namespace

void launch_cross_dot(const float* x, int M, int N, int ld, const float* w, float* out, hipStream_t s) {
  if (M <= 0) return;
  hipLaunchKernelGGL(k_cross_dot, dim3((M + 3) / 4), dim3(256), 0, s, x, M, N, ld, w, out);
}

int cross_top_blocks(int M) { return (M + kTopRows - 1) / kTopRows; }

void launch_cross_top_bwd(const float* x, const unsigned short* x0, int ldx0, const float* z, const float* w,
                          const float* ds, int M, int N, int ld, float* g, unsigned short* u, float* acc, float* part,
                          float* dw, hipStream_t s) {
  if (M <= 0) return;
  const int nb = cross_top_blocks(M);
  hipLaunchKernelGGL(k_cross_top_bwd, dim3(nb), dim3(256), 0, s, x, x0, ldx0, z, w, ds, M, N, ld, g, u, acc, part);
  launch_colsum_acc(part, nb, N, dw, -1, nullptr, s);
}

}  // namespace pbx

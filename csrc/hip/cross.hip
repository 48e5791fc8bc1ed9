// DCN-V2 cross network helpers (the GEMMs themselves run on the LDS-DMA MFMA
// engine, mlp.hip, with the MLP_EPI_CROSS_* epilogues):
//   k_cross_dot      s[m] = x_L[m, :] . w_c            (wave per row)
//   k_cross_top_bwd  top of the backward: g_L = ds (x) w_c, u = bf16(x0 * g_L)
//                    and u^T, acc = z_{L-1} * g_L, per-tile partials of dw_c
// Reference: the cross layer is a fluid program composition in PaddleBox
// (SURVEY §7.4 M6 / BASELINE config 5); here it is one op per direction.
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace pbx {
namespace {

constexpr int kTile = 64;

__device__ __forceinline__ unsigned short f2bf_c(float f) {
  return __builtin_bit_cast(unsigned short, static_cast<__bf16>(f));  // v_cvt_pk_bf16_f32, RNE
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

// 64 x 64 tile per block: thread (tx = column, ty = row phase).  u goes to LDS
// for the transposed store (u^T rows are the A operand of the dW GEMM).
__global__ __launch_bounds__(256) void k_cross_top_bwd(const float* __restrict__ x, const unsigned short* __restrict__ x0,
                                                       const float* __restrict__ z, const float* __restrict__ w,
                                                       const float* __restrict__ ds, int M, int N, int ld,
                                                       float* __restrict__ g, unsigned short* __restrict__ u,
                                                       unsigned short* __restrict__ ut, int ldt,
                                                       float* __restrict__ acc, float* __restrict__ part) {
  __shared__ unsigned short tu[kTile][kTile + 2];
  __shared__ float red[4][kTile];
  const int m0 = blockIdx.y * kTile, n0 = blockIdx.x * kTile;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int n = n0 + tx;
  const bool nv = n < N;
  const float wn = nv ? w[n] : 0.f;
  float p = 0.f;
  for (int i = ty; i < kTile; i += 4) {
    const int m = m0 + i;
    unsigned short uv = 0;
    if (m < M && nv) {
      const int64_t o = (int64_t)m * ld + n;
      const float d = ds[m];
      const float gv = d * wn;
      uv = f2bf_c(__uint_as_float(((unsigned)x0[o]) << 16) * gv);
      g[o] = gv;
      u[o] = uv;
      acc[o] = z[o] * gv;
      p += d * x[o];
    }
    tu[i][tx] = uv;
  }
  red[ty][tx] = p;
  __syncthreads();
  if (ty == 0 && nv) part[(int64_t)blockIdx.y * N + n] = red[0][tx] + red[1][tx] + red[2][tx] + red[3][tx];
  // u^T[n][m0 + tx] for the tile's 64 columns, 4 rows of u^T per pass
  for (int j = ty; j < kTile; j += 4) {
    const int nn = n0 + j, m = m0 + tx;
    if (nn < N && m < M) ut[(int64_t)nn * ldt + m] = tu[tx][j];
  }
}

}  // namespace

void launch_cross_dot(const float* x, int M, int N, int ld, const float* w, float* out, hipStream_t s) {
  if (M <= 0) return;
  hipLaunchKernelGGL(k_cross_dot, dim3((M + 3) / 4), dim3(256), 0, s, x, M, N, ld, w, out);
}

int cross_top_blocks(int M) { return (M + kTile - 1) / kTile; }

void launch_cross_top_bwd(const float* x, const unsigned short* x0, const float* z, const float* w, const float* ds,
                          int M, int N, int ld, float* g, unsigned short* u, unsigned short* ut, int ldt, float* acc,
                          float* part, float* dw, hipStream_t s) {
  if (M <= 0) return;
  const dim3 grid((N + kTile - 1) / kTile, cross_top_blocks(M));
  hipLaunchKernelGGL(k_cross_top_bwd, grid, dim3(256), 0, s, x, x0, z, w, ds, M, N, ld, g, u, ut, ldt, acc, part);
  launch_colsum_acc(part, cross_top_blocks(M), N, dw, -1, nullptr, s);
}

}  // namespace pbx

// CTR op family beyond the DeepFM hot path, hand-written for gfx950.
//
//   k_sgemm          fp32 batched GEMM with arbitrary operand strides, bias
//                    (+scale) and accumulate epilogues: batch_fc (all three
//                    layouts), scaled_fc, and their backward GEMMs.
//                    (reference: batch_fc_op.cu:34-567, scaled_fc_op.cu:39-342
//                    -- cuBLAS batched/fp16 GEMMs plus separate bias kernels)
//   k_i8_quant / k_i8_gemm
//                    scaled_int8fc: clip/expand quantisation and an int8 MFMA
//                    GEMM (v_mfma_i32_32x32x32_i8, exact int32 accumulation)
//                    with the dequantising epilogue (scaled_int8fc_op.cu:38-440)
//   k_ra_*           rank_attention forward, the reference's gather-form input
//                    gradient and the per-block parameter gradient
//                    (rank_attention.cu.h:28-190, rank_attention_op.cu:30-392)
//   k_cvm_*          cvm op (cvm_op.cu:29-70)
//   k_mdn_*          masked_data_norm (masked_data_norm_op.cu:39-290)
//   k_cnh_*          cross_norm_hadamard (cross_norm_hadamard.cu.h:44-240)
//   k_colsum_rows    ordered column reduction of per-block partial rows
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace pbx {
namespace {

inline unsigned nblk(int64_t n, int per = 256) {
  const int64_t b = (n + per - 1) / per;
  return (unsigned)(b < 1 ? 1 : b);
}

// ---------------------------------------------------------------- fp32 batched GEMM
// 64x64 output tile per 256-thread block, K step 16, each thread a 4x4 block.
__global__ __launch_bounds__(256) void k_sgemm(SgemmArgs g) {
  __shared__ float As[16][64 + 4];
  __shared__ float Bs[16][64 + 4];
  const int b = blockIdx.z;
  const int m0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
  const int t = threadIdx.x, tx = t & 15, ty = t >> 4;
  const float* A = g.A + (int64_t)b * g.sA;
  const float* Bm = g.B + (int64_t)b * g.sB;
  float acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = 0.f;
  for (int k0 = 0; k0 < g.K; k0 += 16) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int e = t + 256 * j;
      const int mm = e & 63, kk = e >> 6;
      const int gm = m0 + mm, gk = k0 + kk;
      As[kk][mm] = (gm < g.M && gk < g.K) ? A[(int64_t)gm * g.rsA + (int64_t)gk * g.csA] : 0.f;
      const int gn = n0 + mm;
      Bs[kk][mm] = (gn < g.N && gk < g.K) ? Bm[(int64_t)gk * g.rsB + (int64_t)gn * g.csB] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      const float4 av = *reinterpret_cast<const float4*>(&As[kk][ty * 4]);
      const float4 bv = *reinterpret_cast<const float4*>(&Bs[kk][tx * 4]);
      const float a4[4] = {av.x, av.y, av.z, av.w};
      const float b4[4] = {bv.x, bv.y, bv.z, bv.w};
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] += a4[i] * b4[j];
    }
    __syncthreads();
  }
  float* C = g.C + (int64_t)b * g.sC;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + ty * 4 + i;
    if (m >= g.M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + tx * 4 + j;
      if (n >= g.N) continue;
      float v = g.alpha * acc[i][j];
      if (g.bias) v += g.bias[(int64_t)b * g.sBias + n] * g.bias_scale;
      float* dst = C + (int64_t)m * g.ldc + n;
      if (g.accumulate) v += *dst;
      *dst = v;
    }
  }
}

// column sums of a [batch][M][N] strided matrix into out[batch][N] (+=): bias
// gradients of batch_fc / scaled_fc.  One thread per (batch, column).
__global__ void k_colsum_strided(const float* __restrict__ x, int batch, int M, int N, int64_t sb, int64_t ld,
                                 float* __restrict__ out, int64_t so, int accumulate) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)batch * N) return;
  const int b = (int)(t / N), n = (int)(t % N);
  const float* p = x + (int64_t)b * sb + n;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int m = 0;
  for (; m + 3 < M; m += 4) {
    s0 += p[(int64_t)m * ld];
    s1 += p[(int64_t)(m + 1) * ld];
    s2 += p[(int64_t)(m + 2) * ld];
    s3 += p[(int64_t)(m + 3) * ld];
  }
  for (; m < M; ++m) s0 += p[(int64_t)m * ld];
  const float s = (s0 + s1) + (s2 + s3);
  float* o = out + (int64_t)b * so + n;
  *o = accumulate ? *o + s : s;
}

// ---------------------------------------------------------------- int8 fc
// clip(v * expand, +-clip) quantised with interval 2*clip/range:
// trunc(e / interval + 0.5), clamped to int8.  transpose: write [C][R].
__global__ void k_i8_quant(const float* __restrict__ x, int R, int C, int ldo, float expand, float clip,
                           float range, int transpose, signed char* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)R * C) return;
  const int r = (int)(t / C), c = (int)(t % C);
  float e = x[t] * expand;
  if (e >= 1e-6f) {
    if (e - clip > 1e-6f) e = clip;
  } else if (e + clip < 1e-6f) {
    e = -clip;
  }
  const float interval = 2.f * clip / range;
  float q = truncf(e / interval + 0.5f);
  q = q < -128.f ? -128.f : (q > 127.f ? 127.f : q);
  const int64_t o = transpose ? (int64_t)c * ldo + r : (int64_t)r * ldo + c;
  out[o] = (signed char)q;
}

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

// y[m][n] = acc(qx[m] . qwt[n]) * scale + bias[n]; qx [M][Kp], qwt [N][Kp]
// int8 with Kp % 32 == 0 (zero padded).  One wave per 32x32 tile, 4 waves
// per block (64x64); lane l feeds 16 consecutive k of row/col l%32.
__global__ __launch_bounds__(256) void k_i8_gemm(const signed char* __restrict__ qx,
                                                 const signed char* __restrict__ qwt, int M, int N, int Kp,
                                                 float scale, const float* __restrict__ bias, float* __restrict__ y,
                                                 int ldy) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int m0 = blockIdx.y * 64 + (w >> 1) * 32, n0 = blockIdx.x * 64 + (w & 1) * 32;
  const int r = lane & 31, h = lane >> 5;
  const int am = min(m0 + r, M - 1), bn = min(n0 + r, N - 1);
  const signed char* ap = qx + (int64_t)am * Kp + 16 * h;
  const signed char* bp = qwt + (int64_t)bn * Kp + 16 * h;
  i32x16 acc = {0};
  for (int k = 0; k < Kp; k += 32) {
    const i32x4 a = *reinterpret_cast<const i32x4*>(ap + k);
    const i32x4 b = *reinterpret_cast<const i32x4*>(bp + k);
    acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, acc, 0, 0, 0);
  }
  const int n = n0 + r;
  if (n >= N) return;
  const float bv = bias ? bias[n] : 0.f;
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) {
    const int m = m0 + 8 * (reg >> 2) + 4 * h + (reg & 3);
    if (m < M) y[(int64_t)m * ldy + n] = (float)acc[reg] * scale + bv;
  }
}

// ---------------------------------------------------------------- rank_attention
// rank_offset row i: [rank_i, (rank_k, index_k) for k < R]; a pair (i, k) is
// valid when rank_i >= 1 and rank_k >= 1; its parameter block is
// (rank_i - 1) * R + (rank_k - 1) of W [R*R][C][P].
__device__ __forceinline__ int ra_block(const int* ro, int ld, int i, int k, int R, int* idx) {
  const int lower = ro[(int64_t)i * ld] - 1;
  const int faster = ro[(int64_t)i * ld + 2 * k + 1] - 1;
  *idx = ro[(int64_t)i * ld + 2 * k + 2];
  if (lower < 0 || faster < 0 || *idx < 0) return -1;
  return lower * R + faster;
}

// out[i][p] = sum_k x[idx_k] . W[blk_k][:, p].  Block: 64 instances x 64
// columns; W_b is staged through LDS 32 rows at a time for every block b
// that occurs in the tile; each thread holds 16 outputs of one instance.
template <int R>
__global__ __launch_bounds__(256) void k_ra_fwd(const float* __restrict__ x, const int* __restrict__ ro, int ld,
                                                const float* __restrict__ W, int B, int C, int P,
                                                float* __restrict__ out) {
  __shared__ float Ws[32][64];
  __shared__ int used[64];
  const int t = threadIdx.x, ii = t & 63, g = t >> 6;
  const int i = blockIdx.x * 64 + ii;
  const int p0 = blockIdx.y * 64 + g * 16;
  float acc[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) acc[j] = 0.f;
  int blk[R], idx[R];
#pragma unroll
  for (int k = 0; k < R; ++k) blk[k] = (i < B) ? ra_block(ro, ld, i, k, R, &idx[k]) : -1;
  if (t < 64) used[t] = 0;
  __syncthreads();
  if (g == 0)
#pragma unroll
    for (int k = 0; k < R; ++k)
      if (blk[k] >= 0) used[blk[k]] = 1;
  __syncthreads();
  for (int b = 0; b < R * R; ++b) {
    if (!used[b]) continue;  // block-uniform
    for (int c0 = 0; c0 < C; c0 += 32) {
      __syncthreads();
      for (int e = t; e < 32 * 64; e += 256) {
        const int cc = e >> 6, pp = e & 63;
        const int c = c0 + cc, p = blockIdx.y * 64 + pp;
        Ws[cc][pp] = (c < C && p < P) ? W[((int64_t)b * C + c) * P + p] : 0.f;
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < R; ++k) {
        if (blk[k] != b) continue;
        const float* xr = x + (int64_t)idx[k] * C + c0;
        const int cn = min(32, C - c0);
        for (int cc = 0; cc < cn; ++cc) {
          const float xv = xr[cc];
#pragma unroll
          for (int j = 0; j < 16; ++j) acc[j] += xv * Ws[cc][g * 16 + j];
        }
      }
    }
  }
  if (i >= B) return;
#pragma unroll
  for (int j = 0; j < 16; ++j)
    if (p0 + j < P) out[(int64_t)i * P + p0 + j] = acc[j];
}

// dexp[j][k][c] = valid(j,k) ? sum_p dout[j][p] W[blk(j,k)][c][p] : 0
template <int R>
__global__ __launch_bounds__(256) void k_ra_dexp(const float* __restrict__ dout, const int* __restrict__ ro, int ld,
                                                 const float* __restrict__ W, int B, int C, int P,
                                                 float* __restrict__ dexp) {
  __shared__ float Ws[64][33];  // [c][p chunk]
  __shared__ int used[64];
  const int t = threadIdx.x, jj = t & 63, g = t >> 6;
  const int j = blockIdx.x * 64 + jj;
  const int c0 = blockIdx.y * 64 + g * 16;
  int blk[R], idx[R];
#pragma unroll
  for (int k = 0; k < R; ++k) blk[k] = (j < B) ? ra_block(ro, ld, j, k, R, &idx[k]) : -1;
  if (t < 64) used[t] = 0;
  __syncthreads();
  if (g == 0)
#pragma unroll
    for (int k = 0; k < R; ++k)
      if (blk[k] >= 0) used[blk[k]] = 1;
  __syncthreads();
  float acc[R][16];
#pragma unroll
  for (int k = 0; k < R; ++k)
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[k][q] = 0.f;
  for (int b = 0; b < R * R; ++b) {
    if (!used[b]) continue;
    for (int pc = 0; pc < P; pc += 32) {
      __syncthreads();
      for (int e = t; e < 64 * 32; e += 256) {
        const int cc = e >> 5, pp = e & 31;
        const int c = blockIdx.y * 64 + cc, p = pc + pp;
        Ws[cc][pp] = (c < C && p < P) ? W[((int64_t)b * C + c) * P + p] : 0.f;
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < R; ++k) {
        if (blk[k] != b) continue;
        const float* dr = dout + (int64_t)j * P + pc;
        const int pn = min(32, P - pc);
        for (int pp = 0; pp < pn; ++pp) {
          const float dv = dr[pp];
#pragma unroll
          for (int q = 0; q < 16; ++q) acc[k][q] += dv * Ws[g * 16 + q][pp];
        }
      }
    }
  }
  if (j >= B) return;
#pragma unroll
  for (int k = 0; k < R; ++k)
#pragma unroll
    for (int q = 0; q < 16; ++q)
      if (c0 + q < C) dexp[((int64_t)j * R + k) * C + c0 + q] = acc[k][q];
}

// dx[i][c] = sum_t dexp[ro[i][2t+2]][rank_i - 1][c]   (reference gather form,
// merge_input_gradient_kernel: exact for consistent page-view rank data)
__global__ void k_ra_dx(const float* __restrict__ dexp, const int* __restrict__ ro, int ld, int B, int C, int R,
                        float* __restrict__ dx) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)B * C) return;
  const int i = (int)(t / C), c = (int)(t % C);
  const int rank = ro[(int64_t)i * ld];
  float s = 0.f;
  if (rank >= 1 && rank <= R) {
    for (int q = 0; q < R; ++q) {
      const int j = ro[(int64_t)i * ld + 2 * q + 2];
      if (j < 0 || j >= B) continue;
      s += dexp[((int64_t)j * R + (rank - 1)) * C + c];
    }
  }
  dx[t] = s;
}

// dW[b][c][p] += sum over valid pairs (j,k) with blk = b of x[idx][c] dout[j][p].
// Grid: (c tiles of 64, p tiles of 64, R*R * splits).  Pairs of the split's
// instance range are scanned in chunks of 32, staged through LDS.
__global__ __launch_bounds__(256) void k_ra_dw(const float* __restrict__ x, const float* __restrict__ dout,
                                               const int* __restrict__ ro, int ld, int B, int C, int P, int R,
                                               int per_split, float* __restrict__ dW) {
  __shared__ float xs[32][64];
  __shared__ float ds[32][64];
  __shared__ int cnt;
  const int b = blockIdx.z % (R * R), split = blockIdx.z / (R * R);
  const int c0 = blockIdx.x * 64, p0 = blockIdx.y * 64;
  const int t = threadIdx.x, tc = t & 15, tp = t >> 4;  // 4 c x 4 p per thread
  float acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[a][q] = 0.f;
  const int j_beg = split * per_split, j_end = min(B, j_beg + per_split);
  __shared__ int pj[32], px[32];
  for (int jb = j_beg; jb < j_end; jb += 32 / R > 0 ? 32 / R : 1) {
    const int jn = min(j_end, jb + (32 / R > 0 ? 32 / R : 1));
    if (t == 0) {
      int n = 0;
      for (int j = jb; j < jn; ++j)
        for (int k = 0; k < R; ++k) {
          int idx;
          if (ra_block(ro, ld, j, k, R, &idx) == b && idx < B) {
            pj[n] = j;
            px[n] = idx;
            ++n;
          }
        }
      cnt = n;
    }
    __syncthreads();
    const int n = cnt;
    for (int e = t; e < n * 64; e += 256) {
      const int r = e >> 6, q = e & 63;
      xs[r][q] = (c0 + q < C) ? x[(int64_t)px[r] * C + c0 + q] : 0.f;
      ds[r][q] = (p0 + q < P) ? dout[(int64_t)pj[r] * P + p0 + q] : 0.f;
    }
    __syncthreads();
    for (int r = 0; r < n; ++r) {
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const float xv = xs[r][tc * 4 + a];
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[a][q] += xv * ds[r][tp * 4 + q];
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const int c = c0 + tc * 4 + a;
    if (c >= C) continue;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int p = p0 + tp * 4 + q;
      if (p < P && acc[a][q] != 0.f) atomicAdd(&dW[((int64_t)b * C + c) * P + p], acc[a][q]);
    }
  }
}

// ---------------------------------------------------------------- cvm op
// y = [log(show+1), log(clk+1) - log(show+1), rest] (use_cvm) or rest
__global__ void k_cvm_fwd(const float* __restrict__ x, int64_t n, int W, int use_cvm, float* __restrict__ y) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int Wo = use_cvm ? W : W - 2;
  if (t >= n * Wo) return;
  const int64_t r = t / Wo;
  const int c = (int)(t % Wo);
  const float* xr = x + r * W;
  float v;
  if (!use_cvm) v = xr[c + 2];
  else if (c == 0) v = logf(xr[0] + 1.f);
  else if (c == 1) v = logf(xr[1] + 1.f) - logf(xr[0] + 1.f);
  else v = xr[c];
  y[t] = v;
}

// dx = [cvm input (show, click), dy body]  (the CVM gradient trick)
__global__ void k_cvm_bwd(const float* __restrict__ dy, const float* __restrict__ cvm, int64_t n, int W, int use_cvm,
                          int cvm_rows, float* __restrict__ dx) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * W) return;
  const int64_t r = t / W;
  const int c = (int)(t % W);
  const int Wo = use_cvm ? W : W - 2;
  float v;
  if (c < 2) v = cvm[(cvm_rows == 1 ? 0 : r) * 2 + c];
  else v = dy[r * Wo + (use_cvm ? c : c - 2)];
  dx[t] = v;
}

// ---------------------------------------------------------------- masked data_norm
// fwd: y = mask ? (x - mean) * scale (* sw + bias) : 0, plus per-block masked
// statistic partials part[block][3][C] = (count, sum x, sum (x-mean)^2).
constexpr int kMdnRows = 64;
__global__ __launch_bounds__(256) void k_mdn_fwd(const float* __restrict__ x, const float* __restrict__ mask, int N,
                                                 int C, const float* __restrict__ bsize,
                                                 const float* __restrict__ bsum, const float* __restrict__ bsq,
                                                 const float* __restrict__ sw, const float* __restrict__ bias,
                                                 float* __restrict__ y, float* __restrict__ part) {
  const int r0 = blockIdx.y * kMdnRows;
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int w = threadIdx.x >> 6;
  __shared__ float s[3][4][64];
  float n = 0.f, sx = 0.f, sq = 0.f;
  if (c < C) {
    const float mean = bsum[c] / bsize[c], scale = sqrtf(bsize[c] / bsq[c]);
    for (int r = r0 + w; r < min(N, r0 + kMdnRows); r += 4) {
      const int64_t o = (int64_t)r * C + c;
      const bool m = mask[r] > 0.f;
      const float xv = x[o];
      float v = 0.f;
      if (m) {
        v = (xv - mean) * scale;
        if (sw) v = v * sw[c] + bias[c];
        n += 1.f;
        sx += xv;
        sq += (xv - mean) * (xv - mean);
      }
      y[o] = v;
    }
  }
  s[0][w][threadIdx.x & 63] = n;
  s[1][w][threadIdx.x & 63] = sx;
  s[2][w][threadIdx.x & 63] = sq;
  __syncthreads();
  if (w == 0 && c < C) {
    const int l = threadIdx.x;
    for (int q = 0; q < 3; ++q)
      part[((int64_t)blockIdx.y * 3 + q) * C + c] = (s[q][0][l] + s[q][1][l]) + (s[q][2][l] + s[q][3][l]);
  }
}

// bwd: dx = mask ? dy * sw * scale : 0; optional per-block partials of
// dsw = sum dy * xn and dbias = sum dy * mask
__global__ __launch_bounds__(256) void k_mdn_bwd(const float* __restrict__ x, const float* __restrict__ dy,
                                                 const float* __restrict__ mask, int N, int C,
                                                 const float* __restrict__ bsize, const float* __restrict__ bsum,
                                                 const float* __restrict__ bsq, const float* __restrict__ sw,
                                                 float* __restrict__ dx, float* __restrict__ part) {
  const int r0 = blockIdx.y * kMdnRows;
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int w = threadIdx.x >> 6;
  __shared__ float s[2][4][64];
  float dsw = 0.f, db = 0.f;
  if (c < C) {
    const float mean = bsum[c] / bsize[c], scale = sqrtf(bsize[c] / bsq[c]);
    const float swc = sw ? sw[c] : 1.f;
    for (int r = r0 + w; r < min(N, r0 + kMdnRows); r += 4) {
      const int64_t o = (int64_t)r * C + c;
      const bool m = mask[r] > 0.f;
      const float g = dy[o];
      dx[o] = m ? g * swc * scale : 0.f;
      if (m) {
        dsw += g * (x[o] - mean) * scale;
        db += g;
      }
    }
  }
  if (!part) return;
  s[0][w][threadIdx.x & 63] = dsw;
  s[1][w][threadIdx.x & 63] = db;
  __syncthreads();
  if (w == 0 && c < C) {
    const int l = threadIdx.x;
    for (int q = 0; q < 2; ++q)
      part[((int64_t)blockIdx.y * 2 + q) * C + c] = (s[q][0][l] + s[q][1][l]) + (s[q][2][l] + s[q][3][l]);
  }
}

// ---------------------------------------------------------------- cross_norm_hadamard
// x [B][F][2][E] -> raw [B][F][3E+1] = [a, b, a*b, <a,b>], normalised with the
// running summary (means = s1/s0, scales = sqrt(s0/s2)).  One thread per
// (row, field); per-block partial column sums of raw and (raw - mean)^2.
constexpr int kCnhRows = 32;
__global__ __launch_bounds__(256) void k_cnh_fwd(const float* __restrict__ x, int B, int F, int E,
                                                 const float* __restrict__ summary, float* __restrict__ y,
                                                 float* __restrict__ part) {
  const int W = F * (3 * E + 1);
  extern __shared__ float red[];  // [2][W] block partials
  for (int i = threadIdx.x; i < 2 * W; i += blockDim.x) red[i] = 0.f;
  __syncthreads();
  const float* s0 = summary;
  const float* s1 = summary + W;
  const float* s2 = summary + 2 * W;
  const int r0 = blockIdx.x * kCnhRows;
  for (int u = threadIdx.x; u < kCnhRows * F; u += blockDim.x) {
    const int r = r0 + u / F, f = u % F;
    if (r >= B) continue;
    const float* a = x + ((int64_t)r * F + f) * 2 * E;
    const float* bb = a + E;
    float* out = y + (int64_t)r * W + f * (3 * E + 1);
    const int cb = f * (3 * E + 1);
    float dot = 0.f;
    for (int e = 0; e < 3 * E; ++e) {
      const int ee = e % E;
      const float v = e < E ? a[ee] : (e < 2 * E ? bb[ee] : a[ee] * bb[ee]);
      if (e >= 2 * E) dot += v;
      const int col = cb + e;
      const float mean = s1[col] / s0[col];
      out[e] = (v - mean) * sqrtf(s0[col] / s2[col]);
      atomicAdd(&red[col], v);
      atomicAdd(&red[W + col], (v - mean) * (v - mean));
    }
    const int col = cb + 3 * E;
    const float mean = s1[col] / s0[col];
    out[3 * E] = (dot - mean) * sqrtf(s0[col] / s2[col]);
    atomicAdd(&red[col], dot);
    atomicAdd(&red[W + col], (dot - mean) * (dot - mean));
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * W; i += blockDim.x) part[(int64_t)blockIdx.x * 2 * W + i] = red[i];
}

// exact input gradient of the forward (see ops/ctr_ext.py _CrossNormHadamard)
__global__ void k_cnh_bwd(const float* __restrict__ x, const float* __restrict__ dy, int B, int F, int E,
                          const float* __restrict__ summary, float* __restrict__ dx) {
  const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= (int64_t)B * F) return;
  const int W = F * (3 * E + 1);
  const int64_t r = u / F;
  const int f = (int)(u % F);
  const float* a = x + u * 2 * E;
  const float* bb = a + E;
  const int cb = f * (3 * E + 1);
  const float* g = dy + r * W + cb;
  auto sc = [&](int col) { return sqrtf(summary[col] / summary[2 * W + col]); };
  const float gdot = g[3 * E] * sc(cb + 3 * E);
  float* da = dx + u * 2 * E;
  float* db = da + E;
  for (int e = 0; e < E; ++e) {
    const float ga = g[e] * sc(cb + e);
    const float gb = g[E + e] * sc(cb + E + e);
    const float gab = g[2 * E + e] * sc(cb + 2 * E + e);
    da[e] = ga + gab * bb[e] + gdot * bb[e];
    db[e] = gb + gab * a[e] + gdot * a[e];
  }
}

// out[q][c] = sum_r part[r][q][c] * mul[q] + add[q] (ordered, deterministic)
__global__ void k_colsum_rows(const float* __restrict__ part, int rows, int Q, int C, ColAffine f,
                              float* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)Q * C) return;
  const int q = (int)(t / C), c = (int)(t % C);
  float s = 0.f;
  for (int r = 0; r < rows; ++r) s += part[((int64_t)r * Q + q) * C + c];
  out[t] = s * f.mul[q] + f.add[q];
}

// masked data_norm statistics from the partials: n = masked rows,
// stats = [n > 0, sum x / n, sum (x-mean)^2 / n + eps [n > 0]]
__global__ void k_mdn_stats(const float* __restrict__ part, int rows, int C, float eps, float* __restrict__ stats) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float n = 0.f, sx = 0.f, sq = 0.f;
  for (int r = 0; r < rows; ++r) {
    n += part[((int64_t)r * 3 + 0) * C + c];
    sx += part[((int64_t)r * 3 + 1) * C + c];
    sq += part[((int64_t)r * 3 + 2) * C + c];
  }
  const float has = n > 0.f ? 1.f : 0.f, d = n > 1.f ? n : 1.f;
  stats[c] = has;
  stats[C + c] = sx / d;
  stats[2 * C + c] = sq / d + eps * has;
}

}  // namespace

void launch_sgemm(const SgemmArgs& g, hipStream_t s) {
  if (g.M == 0 || g.N == 0 || g.batch == 0) return;
  dim3 grid((g.N + 63) / 64, (g.M + 63) / 64, g.batch);
  hipLaunchKernelGGL(k_sgemm, grid, dim3(256), 0, s, g);
}

void launch_colsum_strided(const float* x, int batch, int M, int N, int64_t sb, int64_t ld, float* out, int64_t so,
                           bool accumulate, hipStream_t s) {
  if (batch * N == 0) return;
  hipLaunchKernelGGL(k_colsum_strided, dim3(nblk((int64_t)batch * N)), dim3(256), 0, s, x, batch, M, N, sb, ld, out,
                     so, accumulate ? 1 : 0);
}

void launch_i8_quant(const float* x, int R, int C, int ldo, float expand, float clip, float range, bool transpose,
                     signed char* out, hipStream_t s) {
  if ((int64_t)R * C == 0) return;
  hipLaunchKernelGGL(k_i8_quant, dim3(nblk((int64_t)R * C)), dim3(256), 0, s, x, R, C, ldo, expand, clip, range,
                     transpose ? 1 : 0, out);
}

void launch_i8_gemm(const signed char* qx, const signed char* qwt, int M, int N, int Kp, float scale,
                    const float* bias, float* y, int ldy, hipStream_t s) {
  if (M == 0 || N == 0) return;
  hipLaunchKernelGGL(k_i8_gemm, dim3((N + 63) / 64, (M + 63) / 64), dim3(256), 0, s, qx, qwt, M, N, Kp, scale, bias,
                     y, ldy);
}

#define PBX_RA_DISPATCH(KER, GRID, ...)                                       \
  switch (R) {                                                                \
    case 1: hipLaunchKernelGGL(KER<1>, GRID, dim3(256), 0, s, __VA_ARGS__); break; \
    case 2: hipLaunchKernelGGL(KER<2>, GRID, dim3(256), 0, s, __VA_ARGS__); break; \
    case 3: hipLaunchKernelGGL(KER<3>, GRID, dim3(256), 0, s, __VA_ARGS__); break; \
    case 4: hipLaunchKernelGGL(KER<4>, GRID, dim3(256), 0, s, __VA_ARGS__); break; \
    case 5: hipLaunchKernelGGL(KER<5>, GRID, dim3(256), 0, s, __VA_ARGS__); break; \
    case 6: hipLaunchKernelGGL(KER<6>, GRID, dim3(256), 0, s, __VA_ARGS__); break; \
    case 7: hipLaunchKernelGGL(KER<7>, GRID, dim3(256), 0, s, __VA_ARGS__); break; \
    default: hipLaunchKernelGGL(KER<8>, GRID, dim3(256), 0, s, __VA_ARGS__); break; \
  }

void launch_rank_attention_fwd(const float* x, const int* ro, int ld, const float* W, int B, int C, int P, int R,
                               float* out, hipStream_t s) {
  if (B == 0) return;
  PBX_RA_DISPATCH(k_ra_fwd, dim3((B + 63) / 64, (P + 63) / 64), x, ro, ld, W, B, C, P, out);
}

void launch_rank_attention_bwd(const float* x, const float* dout, const int* ro, int ld, const float* W, int B, int C,
                               int P, int R, float* dexp, float* dx, float* dW, hipStream_t s) {
  if (B == 0) return;
  PBX_RA_DISPATCH(k_ra_dexp, dim3((B + 63) / 64, (C + 63) / 64), dout, ro, ld, W, B, C, P, dexp);
  hipLaunchKernelGGL(k_ra_dx, dim3(nblk((int64_t)B * C)), dim3(256), 0, s, dexp, ro, ld, B, C, R, dx);
  const int splits = B > 4096 ? 8 : (B > 512 ? 4 : 1);
  const int per = (B + splits - 1) / splits;
  hipLaunchKernelGGL(k_ra_dw, dim3((C + 63) / 64, (P + 63) / 64, R * R * splits), dim3(256), 0, s, x, dout, ro, ld, B,
                     C, P, R, per, dW);
}

void launch_cvm_fwd(const float* x, int64_t n, int W, bool use_cvm, float* y, hipStream_t s) {
  const int64_t tot = n * (use_cvm ? W : W - 2);
  if (tot == 0) return;
  hipLaunchKernelGGL(k_cvm_fwd, dim3(nblk(tot)), dim3(256), 0, s, x, n, W, use_cvm ? 1 : 0, y);
}

void launch_cvm_bwd(const float* dy, const float* cvm, int64_t n, int W, bool use_cvm, int cvm_rows, float* dx,
                    hipStream_t s) {
  if (n * W == 0) return;
  hipLaunchKernelGGL(k_cvm_bwd, dim3(nblk(n * W)), dim3(256), 0, s, dy, cvm, n, W, use_cvm ? 1 : 0, cvm_rows, dx);
}

int mdn_blocks(int N) { return (N + kMdnRows - 1) / kMdnRows; }

void launch_masked_dn_fwd(const float* x, const float* mask, int N, int C, const float* bsize, const float* bsum,
                          const float* bsq, const float* sw, const float* bias, float* y, float* part, hipStream_t s) {
  if ((int64_t)N * C == 0) return;
  hipLaunchKernelGGL(k_mdn_fwd, dim3((C + 63) / 64, mdn_blocks(N)), dim3(256), 0, s, x, mask, N, C, bsize, bsum, bsq,
                     sw, bias, y, part);
}

void launch_masked_dn_bwd(const float* x, const float* dy, const float* mask, int N, int C, const float* bsize,
                          const float* bsum, const float* bsq, const float* sw, float* dx, float* part,
                          hipStream_t s) {
  if ((int64_t)N * C == 0) return;
  hipLaunchKernelGGL(k_mdn_bwd, dim3((C + 63) / 64, mdn_blocks(N)), dim3(256), 0, s, x, dy, mask, N, C, bsize, bsum,
                     bsq, sw, dx, part);
}

int cnh_blocks(int B) { return (B + kCnhRows - 1) / kCnhRows; }

void launch_cnh_fwd(const float* x, int B, int F, int E, const float* summary, float* y, float* part, hipStream_t s) {
  if (B == 0) return;
  const int W = F * (3 * E + 1);
  hipLaunchKernelGGL(k_cnh_fwd, dim3(cnh_blocks(B)), dim3(256), (size_t)2 * W * sizeof(float), s, x, B, F, E, summary,
                     y, part);
}

void launch_cnh_bwd(const float* x, const float* dy, int B, int F, int E, const float* summary, float* dx,
                    hipStream_t s) {
  if (B == 0) return;
  hipLaunchKernelGGL(k_cnh_bwd, dim3(nblk((int64_t)B * F)), dim3(256), 0, s, x, dy, B, F, E, summary, dx);
}

void launch_colsum_rows(const float* part, int rows, int Q, int C, const ColAffine& f, float* out, hipStream_t s) {
  if ((int64_t)Q * C == 0) return;
  hipLaunchKernelGGL(k_colsum_rows, dim3(nblk((int64_t)Q * C)), dim3(256), 0, s, part, rows, Q, C, f, out);
}

void launch_mdn_stats(const float* part, int rows, int C, float eps, float* stats, hipStream_t s) {
  if (C == 0) return;
  hipLaunchKernelGGL(k_mdn_stats, dim3(nblk(C)), dim3(256), 0, s, part, rows, C, eps, stats);
}

}  // namespace pbx

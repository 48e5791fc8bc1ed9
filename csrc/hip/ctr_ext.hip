// CTR op family beyond the DeepFM hot path, hand-written for gfx950.
//
//   k_mgemm          fp32 batched GEMM on v_mfma_f32_16x16x4_f32 (exact fp32
//                    products, the reference fc precision) with arbitrary
//                    operand strides staged through LDS, bias (+scale) and
//                    accumulate epilogues: batch_fc (all three layouts),
//                    scaled_fc, and their backward GEMMs.
//                    (reference: batch_fc_op.cu:34-567, scaled_fc_op.cu:39-342
//                    -- cuBLAS batched/fp16 GEMMs plus separate bias kernels)
//   k_i8_quant / k_i8_gemm
//                    scaled_int8fc: clip/expand quantisation and an int8 MFMA
//                    GEMM (v_mfma_i32_32x32x32_i8, exact int32 accumulation)
//                    with the dequantising epilogue (scaled_int8fc_op.cu:38-440)
//   k_ra_*           rank_attention as grouped MFMA GEMMs over the R*R
//                    parameter blocks with gather-on-load: forward, the
//                    reference's gather-form input gradient and the per-block
//                    parameter gradient (pairs found by a parallel ballot scan)
//                    (rank_attention.cu.h:28-190, rank_attention_op.cu:30-392)
//   k_cvm_*          cvm op (cvm_op.cu:29-70)
//   k_mdn_*          masked_data_norm (masked_data_norm_op.cu:39-290)
//   k_cnh_*          cross_norm_hadamard (cross_norm_hadamard.cu.h:44-240)
//   k_colsum_rows    ordered column reduction of per-block partial rows
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>

#include "kernels.h"

namespace pbx {
namespace {

inline unsigned nblk(int64_t n, int per = 256) {
  const int64_t b = (n + per - 1) / per;
  return (unsigned)(b < 1 ? 1 : b);
}

// ---------------------------------------------------------------- fp32 batched GEMM
typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
// One 64x64 output tile per 256-thread block: 4 waves of 32x32, each 2x2
// v_mfma_f32_16x16x4 tiles; K staged through LDS 16 at a time (k-major, rows
// padded to 68 floats).  16x16x4 operand layout: lane l feeds A[l%16][l/16]
// and B[l/16][l%16]; accumulator register r is C[4(l/16)+r][l%16].
// Split-K (g.ksplit > 1, small M x N with long K such as the dW GEMMs of
// batch_fc): blockIdx.z = batch * ksplit + slice, each slice adds its partial
// product with fp32 atomics into C (zeroed by the launcher unless
// accumulating); slice 0 adds the bias.
__global__ __launch_bounds__(256) void k_mgemm(SgemmArgs g) {
  __shared__ float As[16][68];
  __shared__ float Bs[16][68];
  const int b = blockIdx.z / g.ksplit, ks = blockIdx.z % g.ksplit;
  const int kper = ((g.K + g.ksplit - 1) / g.ksplit + 15) / 16 * 16;
  const int kbeg = ks * kper, kend = min(g.K, kbeg + kper);
  const int m0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wm = (w >> 1) * 32, wn = (w & 1) * 32;
  const int fr = lane & 15, fk = lane >> 4;
  const float* A = g.A + (int64_t)b * g.sA;
  const float* Bm = g.B + (int64_t)b * g.sB;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  // staging follows each operand's unit stride so a wave's loads coalesce:
  // k-contiguous operands (x / dy rows of batch_fc, W^T of its dx GEMM) read
  // one 16-float k run per row -- one float4 per thread when aligned -- and
  // m/n-contiguous ones 64 consecutive columns per k.  LDS writes of either
  // mapping hit 64 distinct banks (rows padded to 68).
  const bool a_kc = g.csA == 1 && g.rsA != 1, b_kc = g.rsB == 1 && g.csB != 1;
  const bool a_v4 = a_kc && (g.rsA & 3) == 0 && ((uintptr_t)A & 15) == 0;
  const bool b_v4 = b_kc && (g.csB & 3) == 0 && ((uintptr_t)Bm & 15) == 0;
  auto stage = [&](const float* X, int64_t rs, int64_t cs, int lim, int base, bool kc, bool v4, int k0,
                   float (*S)[68]) {
    if (v4) {
      const int mm = t >> 2, kq = (t & 3) * 4;
      const int gm = base + mm, gk = k0 + kq;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (gm < lim) {
        const float* src = X + (int64_t)gm * rs + gk;
        if (gk + 3 < kend) {
          v = *reinterpret_cast<const float4*>(src);
        } else {
          v.x = gk < kend ? src[0] : 0.f;
          v.y = gk + 1 < kend ? src[1] : 0.f;
          v.z = gk + 2 < kend ? src[2] : 0.f;
        }
      }
      S[kq][mm] = v.x;
      S[kq + 1][mm] = v.y;
      S[kq + 2][mm] = v.z;
      S[kq + 3][mm] = v.w;
      return;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int e = t + 256 * j;
      const int mm = kc ? (e >> 4) : (e & 63), kk = kc ? (e & 15) : (e >> 6);
      const int gm = base + mm, gk = k0 + kk;
      S[kk][mm] = (gm < lim && gk < kend) ? X[(int64_t)gm * rs + (int64_t)gk * cs] : 0.f;
    }
  };
  for (int k0 = kbeg; k0 < kend; k0 += 16) {
    stage(A, g.rsA, g.csA, g.M, m0, a_kc, a_v4, k0, As);
    // B indexed [k][n]: as an "m-major" operand its row stride is csB
    stage(Bm, g.csB, g.rsB, g.N, n0, b_kc, b_v4, k0, Bs);
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < 16; kk += 4) {
      const float a0 = As[kk + fk][wm + fr], a1 = As[kk + fk][wm + 16 + fr];
      const float b0 = Bs[kk + fk][wn + fr], b1 = Bs[kk + fk][wn + 16 + fr];
      acc[0][0] = mfma4(a0, b0, acc[0][0]);
      acc[0][1] = mfma4(a0, b1, acc[0][1]);
      acc[1][0] = mfma4(a1, b0, acc[1][0]);
      acc[1][1] = mfma4(a1, b1, acc[1][1]);
    }
    __syncthreads();
  }
  float* C = g.C + (int64_t)b * g.sC;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wn + j * 16 + fr;
      if (n >= g.N) continue;
      const float bv = (g.bias && ks == 0) ? g.bias[(int64_t)b * g.sBias + n] * g.bias_scale : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm + i * 16 + 4 * fk + r;
        if (m >= g.M) continue;
        float v = g.alpha * acc[i][j][r] + bv;
        float* dst = C + (int64_t)m * g.ldc + n;
        if (g.ksplit > 1) {
          atomicAdd(dst, v);
        } else {
          if (g.accumulate) v += *dst;
          *dst = v;
        }
      }
    }
}

// ---------------------------------------------------------------- batch_fc (<= 64 x 64 per slot)
// Tiles live in LDS row-major ([row][col], rows padded to 68 floats, 16-B
// aligned for float4 writes); a 16x16x4 MFMA fragment reads either T[m][k]
// (bank 4m + k: conflict-free) or T[k][m] (2-way).  4 waves each own a 32x32
// quadrant of every 64x64 product.  The next tile's float4 loads are issued
// before the current tile's MFMAs.
constexpr int kBfcLd = 68;
typedef float BfcTile[64][kBfcLd];

// one 64 x 64 tile (rows r0.., cols < ncol, unit column stride) into
// 1024 / NT float4 registers per thread: thread t covers rows (t >> 4) +
// (NT / 16) j, cols 4 (t & 15)
template <int NT>
__device__ __forceinline__ void bfc_fetch(const float* __restrict__ X, int64_t rs, int r0, int nrow, int ncol,
                                          float4 (&v)[1024 / NT]) {
  const int t = threadIdx.x, c = (t & 15) * 4;
#pragma unroll
  for (int j = 0; j < 1024 / NT; ++j) {
    const int r = (t >> 4) + (NT / 16) * j;
    v[j] = (r0 + r < nrow && c < ncol) ? *reinterpret_cast<const float4*>(X + (int64_t)(r0 + r) * rs + c)
                                       : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}
template <int NT>
__device__ __forceinline__ void bfc_put(BfcTile& T, const float4 (&v)[1024 / NT]) {
  const int t = threadIdx.x, c = (t & 15) * 4;
#pragma unroll
  for (int j = 0; j < 1024 / NT; ++j) *reinterpret_cast<float4*>(&T[(t >> 4) + (NT / 16) * j][c]) = v[j];
}

// forward: 256 threads; the next x tile's loads are issued before this
// tile's MFMAs (a two-ahead ring measured slower: 35.8 vs 33.2 us)
__global__ __launch_bounds__(256) void k_bfc_fwd(BfcArgs a) {
  __shared__ __attribute__((aligned(16))) BfcTile Ws;
  __shared__ __attribute__((aligned(16))) BfcTile Xs;
  const int p = blockIdx.y;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wm = (w >> 1) * 32, wn = (w & 1) * 32, fr = lane & 15, fk = lane >> 4;
  const float* x = a.x + (int64_t)p * a.sx;
  float* y = a.y + (int64_t)p * a.sy;
  float4 v[4];
  bfc_fetch<256>(a.W + (int64_t)p * a.sw, a.rw, 0, a.I, a.O, v);
  bfc_put<256>(Ws, v);
  float bv[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = wn + 16 * j + fr;
    bv[j] = (a.b != nullptr && n < a.O) ? a.b[(int64_t)p * a.sb + n] : 0.f;
  }
  const int tile0 = blockIdx.x * a.tiles;
  bfc_fetch<256>(x, a.rx, tile0 * 64, a.N, a.I, v);
  for (int it = 0; it < a.tiles; ++it) {
    const int r0 = (tile0 + it) * 64;
    if (r0 >= a.N) break;
    bfc_put<256>(Xs, v);
    __syncthreads();
    if (it + 1 < a.tiles) bfc_fetch<256>(x, a.rx, r0 + 64, a.N, a.I, v);
    f32x4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < a.I; k += 4) {  // A[m][k] = Xs[m][k], B[k][n] = Ws[k][n]
      const float a0 = Xs[wm + fr][k + fk], a1 = Xs[wm + 16 + fr][k + fk];
      const float b0 = Ws[k + fk][wn + fr], b1 = Ws[k + fk][wn + 16 + fr];
      acc[0][0] = mfma4(a0, b0, acc[0][0]);
      acc[0][1] = mfma4(a0, b1, acc[0][1]);
      acc[1][0] = mfma4(a1, b0, acc[1][0]);
      acc[1][1] = mfma4(a1, b1, acc[1][1]);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int n = wn + 16 * j + fr;
        if (n >= a.O) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = r0 + wm + 16 * i + 4 * fk + r;
          if (m < a.N) y[(int64_t)m * a.ry + n] = acc[i][j][r] + bv[j];
        }
      }
    __syncthreads();
  }
}

// backward: 256 threads, every wave owns a 32 x 32 quadrant of both the dx
// tile and the dW partial (kept in registers across the block's tiles);
// splitting dx / dW over 8 waves measured slower (67.5 vs 62.9 us)
__global__ __launch_bounds__(256) void k_bfc_bwd(BfcArgs a) {
  __shared__ __attribute__((aligned(16))) BfcTile Ws;
  __shared__ __attribute__((aligned(16))) BfcTile Ds;
  __shared__ __attribute__((aligned(16))) BfcTile Xs;
  const int p = blockIdx.y;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wm = (w >> 1) * 32, wn = (w & 1) * 32, fr = lane & 15, fk = lane >> 4;
  const float* x = a.x + (int64_t)p * a.sx;
  const float* dy = a.dy + (int64_t)p * a.sy;
  float* dx = a.dx + (int64_t)p * a.sx;
  float4 vd[4], vx[4];
  bfc_fetch<256>(a.W + (int64_t)p * a.sw, a.rw, 0, a.I, a.O, vd);
  bfc_put<256>(Ws, vd);
  f32x4 aw[2][2];  // dW quadrant (rows i = wm.., cols o = wn..) over this block's rows
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) aw[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float dbp = 0.f;  // column t & 63 over rows 16 (t >> 6) .. + 15 of every tile
  const int tile0 = blockIdx.x * a.tiles;
  bfc_fetch<256>(dy, a.ry, tile0 * 64, a.N, a.O, vd);
  bfc_fetch<256>(x, a.rx, tile0 * 64, a.N, a.I, vx);
  for (int it = 0; it < a.tiles; ++it) {
    const int r0 = (tile0 + it) * 64;
    if (r0 >= a.N) break;
    bfc_put<256>(Ds, vd);
    bfc_put<256>(Xs, vx);
    __syncthreads();
    if (it + 1 < a.tiles) {
      bfc_fetch<256>(dy, a.ry, r0 + 64, a.N, a.O, vd);
      bfc_fetch<256>(x, a.rx, r0 + 64, a.N, a.I, vx);
    }
    // dx tile [rows][i] = Ds [rows][o] . W^T: A[m][k] = Ds[m][k], B[k][n] = Ws[n][k]
    f32x4 ax[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) ax[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < a.O; k += 4) {
      const float a0 = Ds[wm + fr][k + fk], a1 = Ds[wm + 16 + fr][k + fk];
      const float b0 = Ws[wn + fr][k + fk], b1 = Ws[wn + 16 + fr][k + fk];
      ax[0][0] = mfma4(a0, b0, ax[0][0]);
      ax[0][1] = mfma4(a0, b1, ax[0][1]);
      ax[1][0] = mfma4(a1, b0, ax[1][0]);
      ax[1][1] = mfma4(a1, b1, ax[1][1]);
    }
    // dW [i][o] += Xs^T . Ds over the tile's rows: A[m][k] = Xs[k][m], B[k][n] = Ds[k][n]
    // (rows past N were staged as zeros)
#pragma unroll 4
    for (int k = 0; k < 64; k += 4) {
      const float a0 = Xs[k + fk][wm + fr], a1 = Xs[k + fk][wm + 16 + fr];
      const float b0 = Ds[k + fk][wn + fr], b1 = Ds[k + fk][wn + 16 + fr];
      aw[0][0] = mfma4(a0, b0, aw[0][0]);
      aw[0][1] = mfma4(a0, b1, aw[0][1]);
      aw[1][0] = mfma4(a1, b0, aw[1][0]);
      aw[1][1] = mfma4(a1, b1, aw[1][1]);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) dbp += Ds[16 * w + r][lane];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int n = wn + 16 * j + fr;
        if (n >= a.I) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = r0 + wm + 16 * i + 4 * fk + r;
          if (m < a.N) dx[(int64_t)m * a.rx + n] = ax[i][j][r];
        }
      }
    __syncthreads();
  }
  // this block's dW [64][64] and db [64] partials, read back in block order by
  // the reduce
  float* part = a.ws + ((int64_t)p * gridDim.x + blockIdx.x) * kBfcPart;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) part[(wm + 16 * i + 4 * fk + r) * 64 + wn + 16 * j + fr] = aw[i][j][r];
  // the 4 row-quarter partials of each column through LDS (Xs is free now)
  Xs[w][lane] = dbp;
  __syncthreads();
  if (t < 64) part[64 * 64 + t] = Xs[0][t] + Xs[1][t] + Xs[2][t] + Xs[3][t];
}

// dW[p][i][o] / db[p][o] = sum over the G block partials, in block order
__global__ void k_bfc_reduce(BfcArgs a, int G) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)a.P * kBfcPart) return;
  const int p = (int)(e / kBfcPart), q = (int)(e % kBfcPart);
  const bool isb = q >= 64 * 64;
  const int i = isb ? 0 : q >> 6, o = isb ? q - 64 * 64 : q & 63;
  if (i >= a.I || o >= a.O) return;
  const float* src = a.ws + (int64_t)p * G * kBfcPart + q;
  float v = 0.f;
  for (int g = 0; g < G; ++g) v += src[(int64_t)g * kBfcPart];
  if (isb) {
    a.db[(int64_t)p * a.sb + o] = v;
  } else {
    a.dW[(int64_t)p * a.sw + (int64_t)i * a.rw + o] = v;
  }
}

// ---------------------------------------------------------------- scaled_fc fp16 GEMM
typedef _Float16 h16x8 __attribute__((ext_vector_type(8)));
// One 64x64 output tile per 256-thread block: 4 waves of 32x32, each 2x2
// v_mfma_f32_16x16x32_f16 tiles.  K steps of 32: the fp32 operands are read
// with arbitrary strides, scaled, rounded to fp16 and written to LDS k-minor
// ([row][k], rows padded to 40 halves) so every lane reads its 8-element
// fragment with one 16-B LDS read; the next K step's operands are loaded into
// registers while the current one is multiplied.  16x16x32 layout: lane l
// feeds A[l%16][8(l/16)+j] and B[8(l/16)+j][l%16]; accumulator register r is
// C[4(l/16)+r][l%16].
constexpr int kHPad = 40;
__device__ __forceinline__ float h16_epi(float acc, float bv, const HgemmArgs& g) {
  _Float16 v = (_Float16)((float)(_Float16)g.alpha * acc);
  if (g.bias) v = (_Float16)((float)v + (float)(_Float16)((float)(_Float16)bv * (float)(_Float16)g.bias_scale));
  float y = (float)v * g.out_scale;
  return __builtin_isinf(y) ? __int_as_float(0x7fc00000) : y;
}

__global__ __launch_bounds__(256) void k_hgemm(HgemmArgs g) {
  __shared__ __attribute__((aligned(16))) _Float16 As[64 * kHPad];
  __shared__ __attribute__((aligned(16))) _Float16 Bs[64 * kHPad];
  const int ks = blockIdx.z;
  const int kper = ((g.K + g.ksplit - 1) / g.ksplit + 31) / 32 * 32;
  const int kbeg = ks * kper, kend = min(g.K, kbeg + kper);
  const int m0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wm = (w >> 1) * 32, wn = (w & 1) * 32;
  const int fr = lane & 15, fk = lane >> 4;
  // staging: thread t covers row / column (t & 63), k = 8 (t >> 6) .. + 7
  const int sr = t & 63, sk = (t >> 6) * 8;
  float ra[8], rb[8];
  auto load = [&](int k0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int gk = k0 + sk + j;
      const int gm = m0 + sr, gn = n0 + sr;
      ra[j] = (gm < g.M && gk < kend) ? g.A[(int64_t)gm * g.rsA + (int64_t)gk * g.csA] : 0.f;
      rb[j] = (gn < g.N && gk < kend) ? g.B[(int64_t)gk * g.rsB + (int64_t)gn * g.csB] : 0.f;
    }
  };
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  if (kbeg < kend) load(kbeg);
  for (int k0 = kbeg; k0 < kend; k0 += 32) {
    h16x8 ha, hb;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      ha[j] = (_Float16)(ra[j] * g.a_scale);
      hb[j] = (_Float16)(rb[j] * g.b_scale);
    }
    __syncthreads();  // the previous step's reads of As / Bs are done
    *reinterpret_cast<h16x8*>(&As[sr * kHPad + sk]) = ha;
    *reinterpret_cast<h16x8*>(&Bs[sr * kHPad + sk]) = hb;
    __syncthreads();
    if (k0 + 32 < kend) load(k0 + 32);  // next step in flight under the MFMAs
    const h16x8 a0 = *reinterpret_cast<const h16x8*>(&As[(wm + fr) * kHPad + 8 * fk]);
    const h16x8 a1 = *reinterpret_cast<const h16x8*>(&As[(wm + 16 + fr) * kHPad + 8 * fk]);
    const h16x8 b0 = *reinterpret_cast<const h16x8*>(&Bs[(wn + fr) * kHPad + 8 * fk]);
    const h16x8 b1 = *reinterpret_cast<const h16x8*>(&Bs[(wn + 16 + fr) * kHPad + 8 * fk]);
    acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, b0, acc[0][0], 0, 0, 0);
    acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, b1, acc[0][1], 0, 0, 0);
    acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, b0, acc[1][0], 0, 0, 0);
    acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, b1, acc[1][1], 0, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wn + j * 16 + fr;
      if (n >= g.N) continue;
      const float bv = g.bias ? g.bias[n] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm + i * 16 + 4 * fk + r;
        if (m >= g.M) continue;
        if (g.ksplit > 1)
          atomicAdd(&g.ws[(int64_t)m * g.N + n], acc[i][j][r]);
        else
          g.C[(int64_t)m * g.ldc + n] = h16_epi(acc[i][j][r], bv, g);
      }
    }
}

// the fp16 epilogue over an fp32 accumulator matrix [M][N] (ld N) -- the
// library-GEMM path of scaled_fc, and the split-K second pass below
__global__ void k_h16_epi(const float* acc, const float* __restrict__ bias, int M, int N, float alpha,
                          float bias_scale, float out_scale, float* out) {  // out may alias acc
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)M * N) return;
  const int n = (int)(e % N);
  HgemmArgs g;
  g.alpha = alpha;
  g.bias = bias;
  g.bias_scale = bias_scale;
  g.out_scale = out_scale;
  out[e] = h16_epi(acc[e], bias ? bias[n] : 0.f, g);
}

// vector form (N % 4 == 0, M * N < 2^31): four columns per thread, 32-bit
// index math (the 64-bit modulo per element dominated the scalar form)
__global__ __launch_bounds__(256) void k_h16_epi4(const float* acc, const float* __restrict__ bias, int M, int N,
                                                  float alpha, float bias_scale, float out_scale, float* out) {
  const int e4 = blockIdx.x * blockDim.x + threadIdx.x;
  const int total4 = (M * N) >> 2;
  if (e4 >= total4) return;
  const int n = (e4 << 2) % N;
  HgemmArgs g;
  g.alpha = alpha;
  g.bias = bias;
  g.bias_scale = bias_scale;
  g.out_scale = out_scale;
  const float4 a = reinterpret_cast<const float4*>(acc)[e4];
  float4 b = make_float4(0.f, 0.f, 0.f, 0.f);
  if (bias) b = *reinterpret_cast<const float4*>(bias + n);
  reinterpret_cast<float4*>(out)[e4] =
      make_float4(h16_epi(a.x, b.x, g), h16_epi(a.y, b.y, g), h16_epi(a.z, b.z, g), h16_epi(a.w, b.w, g));
}

// ---------------------------------------------------------------- scaled_fc fused fp16 GEMM
// out[M][Nd] = h16_epi( fp16(A * a_scale) [M][Kd] @ Bk^T ) with Bk fp16 [Nd][Kd]
// (k-minor: the weight's cached fp16 copy) -- scaled_fc's forward (A = x,
// Bk = W16^T) and its dx (A = dy, a_scale = grad_scale / in_scale, Bk = W16)
// in ONE launch: the fp32 -> fp16 cast happens in the A staging and the
// reference's fp16 epilogue in the store, so no fp16 copy of A and no fp32
// accumulator matrix go through HBM.  64 x 80 tiles (80 = 5 x 16 divides the
// 400-wide CTR layers), 4 waves of 16 rows x 80 columns, v_mfma_f32_16x16x32_f16;
// K in chunks of 64, double-buffered in LDS (41 KB: 3 workgroups per CU), the
// next chunk's global loads in flight under the current chunk's MFMAs.  The
// tiles of one row block are consecutive work ids of one XCD, so the A rows
// come from HBM once and from that XCD's L2 for the other 4 column tiles.
constexpr int kSfcBM = 64, kSfcBN = 80, kSfcKC = 64, kSfcPad = 72;  // LDS row: 64 k + 8 (bank spread)
__device__ __forceinline__ int sfc_xcd_id(int block, int n) {
  const int q = n / 8, rr = n % 8, xcd = block % 8;
  return (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + block / 8;
}
__global__ __launch_bounds__(256) void k_sfc(const float* __restrict__ A, const _Float16* __restrict__ Bk, int M,
                                             int Nd, int Kd, float a_scale, const float* __restrict__ bias,
                                             float alpha, float bias_scale, float out_scale, float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) _Float16 As[2][kSfcBM * kSfcPad];
  __shared__ __attribute__((aligned(16))) _Float16 Bs[2][kSfcBN * kSfcPad];
  const int ntn = (Nd + kSfcBN - 1) / kSfcBN, ntiles = ntn * ((M + kSfcBM - 1) / kSfcBM);
  const int wid = sfc_xcd_id((int)blockIdx.x, ntiles);
  const int m0 = (wid / ntn) * kSfcBM, n0 = (wid % ntn) * kSfcBN;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int fr = lane & 15, fk = lane >> 4;
  // A staging: row t >> 2, k 16 (t & 3) .. + 15 (four float4, two 16-B LDS writes)
  const int ar = t >> 2, ak = (t & 3) * 16;
  const int64_t arow = (int64_t)min(m0 + ar, M - 1) * Kd;
  const bool arow_ok = m0 + ar < M;
  float4 ra[4];
  _Float16 __attribute__((ext_vector_type(8))) rb[3];
  auto load = [&](int k0) {
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int k = k0 + ak + 4 * v;
      ra[v] = (arow_ok && k < Kd) ? *reinterpret_cast<const float4*>(A + arow + k) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int idx = t + 256 * i, n = idx >> 3, k = k0 + (idx & 7) * 8;
      h16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
      if (idx < kSfcBN * 8 && n0 + n < Nd && k < Kd) z = *reinterpret_cast<const h16x8*>(Bk + (int64_t)(n0 + n) * Kd + k);
      rb[i] = z;
    }
  };
  auto stage = [&](int buf) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      h16x8 v;
      const float4 x0 = ra[2 * h], x1 = ra[2 * h + 1];
      v[0] = (_Float16)(x0.x * a_scale); v[1] = (_Float16)(x0.y * a_scale);
      v[2] = (_Float16)(x0.z * a_scale); v[3] = (_Float16)(x0.w * a_scale);
      v[4] = (_Float16)(x1.x * a_scale); v[5] = (_Float16)(x1.y * a_scale);
      v[6] = (_Float16)(x1.z * a_scale); v[7] = (_Float16)(x1.w * a_scale);
      *reinterpret_cast<h16x8*>(&As[buf][ar * kSfcPad + ak + 8 * h]) = v;
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int idx = t + 256 * i;
      if (idx < kSfcBN * 8) *reinterpret_cast<h16x8*>(&Bs[buf][(idx >> 3) * kSfcPad + (idx & 7) * 8]) = rb[i];
    }
  };
  f32x4 acc[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) acc[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int nch = (Kd + kSfcKC - 1) / kSfcKC;
  load(0);
  stage(0);
  __syncthreads();
  for (int c = 0; c < nch; ++c) {
    const int buf = c & 1;
    if (c + 1 < nch) load((c + 1) * kSfcKC);  // in flight under this chunk's MFMAs
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const h16x8 a = *reinterpret_cast<const h16x8*>(&As[buf][(16 * w + fr) * kSfcPad + 32 * s2 + 8 * fk]);
#pragma unroll
      for (int j = 0; j < 5; ++j) {
        const h16x8 b = *reinterpret_cast<const h16x8*>(&Bs[buf][(16 * j + fr) * kSfcPad + 32 * s2 + 8 * fk]);
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc[j], 0, 0, 0);
      }
    }
    if (c + 1 < nch) stage(buf ^ 1);  // the other buffer was last read before the previous barrier
    __syncthreads();
  }
  HgemmArgs g;
  g.alpha = alpha;
  g.bias = bias;
  g.bias_scale = bias_scale;
  g.out_scale = out_scale;
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    const int n = n0 + 16 * j + fr;
    if (n >= Nd) continue;
    const float bv = bias ? bias[n] : 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + 16 * w + 4 * fk + r;
      if (m < M) out[(int64_t)m * Nd + n] = h16_epi(acc[j][r], bv, g);
    }
  }
}

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
// round-to-nearest-even fp32 -> bf16 bits, and back
__device__ __forceinline__ unsigned short f3_bf(float f) {
  unsigned int u = __float_as_uint(f);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (unsigned short)(u >> 16);
}
__device__ __forceinline__ float f3_f(unsigned short h) { return __uint_as_float(((unsigned int)h) << 16); }
// x = hi + lo + r, |r| <~ 2^-17 |x|: the split of the fp32 x 3 bf16 GEMMs (four values)
__device__ __forceinline__ void f3_split4(const float4& x, s16x4& hi, s16x4& lo) {
  const float v[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const unsigned short h = f3_bf(v[j]);
    hi[j] = (short)h;
    lo[j] = (short)f3_bf(v[j] - f3_f(h));
  }
}

// ---------------------------------------------------------------- fp32 GEMM as three bf16 products
// out[M][Nd] = A[M][Kd] (fp32) @ B^T, B given as its bf16 split Bh + Bl
// ([Nd][Kd], k-minor: a weight split once per optimizer step), A split in the
// staging pass: out = Ah Bh + Ah Bl + Al Bh with fp32 accumulation -- the
// product error of the dropped Al Bl and the split residuals is ~2^-16
// relative, i.e. tighter than the TF32 the reference's cuBLAS applies to its
// fp32 GEMMs in training (gpu_context.cc:61-67 enable_cublas_tf32_op_math,
// CublasCall), at 3 bf16 MFMAs (v_mfma_f32_16x16x32_bf16) instead of 8 fp32
// ones.  scaled_int8fc's straight-through dx.  Tiles as k_sfc (64 x 80, 4
// waves of 16 x 80, XCD-grouped row blocks); K in chunks of 32, double
// buffered: 4 LDS images (A hi / lo, B hi / lo) of 80-B rows (conflict-free
// 16-B fragment reads), 46 KB, 3 workgroups per CU.
constexpr int kF3KC = 32, kF3Pad = 40;
__global__ __launch_bounds__(256) void k_f3gemm_nt(const float* __restrict__ A, const short* __restrict__ Bh,
                                                   const short* __restrict__ Bl, int M, int Nd, int Kd,
                                                   float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) short As[2][2][kSfcBM * kF3Pad];  // [buffer][hi / lo]
  __shared__ __attribute__((aligned(16))) short Bs[2][2][kSfcBN * kF3Pad];
  typedef short s8v __attribute__((ext_vector_type(8)));
  const int ntn = (Nd + kSfcBN - 1) / kSfcBN, ntiles = ntn * ((M + kSfcBM - 1) / kSfcBM);
  const int wid = sfc_xcd_id((int)blockIdx.x, ntiles);
  const int m0 = (wid / ntn) * kSfcBM, n0 = (wid % ntn) * kSfcBN;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int fr = lane & 15, fk = lane >> 4;
  // A staging: row t >> 2, k 8 (t & 3) .. + 7 (two float4 -> one 16-B write per
  // image); B: 640 16-B chunks, image idx / 320, row (idx % 320) / 4, chunk idx % 4.
  // Range-checked buffer loads (rows past M / Nd and k past Kd read zeros), so
  // the loads are unconditional and a 3-deep register ring keeps 2 chunks of
  // loads in flight under the MFMAs.
  constexpr int D = 3;
  const int ar = t >> 2, ak = (t & 3) * 8;
  typedef unsigned u32x4v __attribute__((ext_vector_type(4)));
  const __amdgpu_buffer_rsrc_t as = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(A + (int64_t)m0 * Kd), 0, (int)((int64_t)min(kSfcBM, M - m0) * Kd * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t bhs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<short*>(Bh + (int64_t)n0 * Kd), 0, (int)((int64_t)min(kSfcBN, Nd - n0) * Kd * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t bls = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<short*>(Bl + (int64_t)n0 * Kd), 0, (int)((int64_t)min(kSfcBN, Nd - n0) * Kd * 2), 0x00020000);
  float4 ra[D][2];
  s8v rb[D][3];
  auto load = [&](auto jc, int k0) {
    constexpr int J = decltype(jc)::value;
#pragma unroll
    for (int v = 0; v < 2; ++v) {
      const int k = k0 + ak + 4 * v;
      ra[J][v] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(as, k < Kd ? (ar * Kd + k) * 4 : 0x7ffffff0, 0, 0));
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int idx = t + 256 * i, im = idx >= 320, r = (idx - 320 * im) >> 2, k = k0 + (idx & 3) * 8;
      const int off = (idx < 640 && k < Kd) ? (r * Kd + k) * 2 : 0x7ffffff0;
      rb[J][i] = __builtin_bit_cast(s8v, __builtin_amdgcn_raw_buffer_load_b128(im ? bls : bhs, off, 0, 0));
    }
  };
  auto stage = [&](auto jc, int buf) {
    constexpr int J = decltype(jc)::value;
    s16x4 h0, l0, h1, l1;
    f3_split4(ra[J][0], h0, l0);
    f3_split4(ra[J][1], h1, l1);
    *reinterpret_cast<s8v*>(&As[buf][0][ar * kF3Pad + ak]) = (s8v){h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
    *reinterpret_cast<s8v*>(&As[buf][1][ar * kF3Pad + ak]) = (s8v){l0[0], l0[1], l0[2], l0[3], l1[0], l1[1], l1[2], l1[3]};
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int idx = t + 256 * i, im = idx >= 320, r = (idx - 320 * im) >> 2;
      if (idx < 640) *reinterpret_cast<s8v*>(&Bs[buf][im][r * kF3Pad + (idx & 3) * 8]) = rb[J][i];
    }
  };
  f32x4 acc[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) acc[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  auto compute = [&](int buf) {
    const s8v ah = *reinterpret_cast<const s8v*>(&As[buf][0][(16 * w + fr) * kF3Pad + 8 * fk]);
    const s8v al = *reinterpret_cast<const s8v*>(&As[buf][1][(16 * w + fr) * kF3Pad + 8 * fk]);
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      const s8v bh = *reinterpret_cast<const s8v*>(&Bs[buf][0][(16 * j + fr) * kF3Pad + 8 * fk]);
      const s8v bl = *reinterpret_cast<const s8v*>(&Bs[buf][1][(16 * j + fr) * kF3Pad + 8 * fk]);
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, acc[j], 0, 0, 0);
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, acc[j], 0, 0, 0);
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, acc[j], 0, 0, 0);
    }
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  auto body = [&](auto jc, int c) {  // chunk c lives in ring set c % D = J
    constexpr int J = decltype(jc)::value;
    load(jc, (c + D) * kF3KC);  // set J was staged at chunk c - 1
    compute(c & 1);
    stage(std::integral_constant<int, (J + 1) % D>{}, (c + 1) & 1);
    __syncthreads();
  };
  // chunks rounded up to whole rings: the extra chunks load and multiply zeros
  const int nch = (Kd + kF3KC * D - 1) / (kF3KC * D) * D;
  load(I0{}, 0);
  load(I1{}, kF3KC);
  load(I2{}, 2 * kF3KC);
  stage(I0{}, 0);
  __syncthreads();
  for (int c0 = 0; c0 < nch; c0 += D) {
    body(I0{}, c0);
    body(I1{}, c0 + 1);
    body(I2{}, c0 + 2);
  }
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    const int n = n0 + 16 * j + fr;
    if (n >= Nd) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + 16 * w + 4 * fk + r;
      if (m < M) out[(int64_t)m * Nd + n] = acc[j][r];
    }
  }
}

// split-K second pass: the fp16 epilogue over the fp32 sums
__global__ void k_hgemm_epi(HgemmArgs g) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)g.M * g.N) return;
  const int m = (int)(e / g.N), n = (int)(e % g.N);
  g.C[(int64_t)m * g.ldc + n] = h16_epi(g.ws[e], g.bias ? g.bias[n] : 0.f, g);
}

// ---------------------------------------------------------------- scaled_fc weight gradient
// dW [K][O] = h16_epi( sum_n fp16(x[n][k] * a_scale) fp16(d[n][o] * b_scale) ) and
// db [O] = sum_n d[n][o] (fp32, unscaled) in ONE launch (scaled_fc_op.cu:232-330's
// dW GEMM + bias column sum).  Both operands are row-major over the reduction
// index n, so a workgroup stages 32 rows of x[n][k0 .. k0 + 79] and d[n][o0 ..
// o0 + 79] as fp16 into LDS exactly as they lie ([n][col] images, one 8-B
// write per float4) and the MFMA fragments, which want 8 consecutive n per
// lane, come out of ds_read_b64_tr_b16 (two per fragment: rows 8g .. 8g + 3
// and 8g + 4 .. 8g + 7 of the 16-lane group g).  Image rows are 256 B with
// the five 32-B column groups XOR-swizzled by (r & 3) | ((r >> 3) & 1) << 2, so
// the 8 rows a 32-lane half reads land on 8 disjoint 8-bank windows.
// Tile 80 x 80 of dW, 5 waves: wave w owns columns 16w .. 16w + 15 and all
// five 16-row blocks (5 accumulators; one B fragment feeds 5 MFMAs).  The
// batch is split over S workgroups per tile (split-K over n); every split
// stores its partial to a slab, the last arriving split sums the slabs in
// split order and applies the fp16 epilogue -- deterministic, no fp32 atomics,
// no memset, no second launch.  Tiles with k0 == 0 also sum their d columns
// (a fixed-order reduce in LDS, then the same slab hand-off) for db.
constexpr int kSdwT = 80, kSdwNT = 320, kSdwRowB = 256;
typedef _Float16 h16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int sdw_off(int r, int c) {
  const int h = (r & 3) | (((r >> 3) & 1) << 2);
  return r * kSdwRowB + ((((c >> 4) ^ h)) << 5) + ((c & 15) << 1);
}

__device__ __forceinline__ s16x8 sdw_frag(const unsigned char* img, int r, int c) {
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + sdw_off(r, c)));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + sdw_off(r + 4, c)));
  return (s16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// MODE 0: scaled_fc (fp16 operands scaled by a_scale / b_scale, the fp16
// epilogue, two images).  MODE 1: fp32 x^T d as three bf16 MFMA products per
// pair (hi.hi + hi.lo + lo.hi of the operands' bf16 splits; scaled_int8fc's
// straight-through dW), fp32 result, four images (x hi, x lo, d hi, d lo).
// Steps of 32 rows, double-buffered in LDS, fed by a 4-deep register ring.
template <int MODE>
__global__ __launch_bounds__(kSdwNT) void k_sfc_dw(SfcDwArgs a) {
  constexpr int ROWS = 32, NIMG = MODE ? 4 : 2, IMG = ROWS * kSdwRowB, NI = ROWS / 16;
  __shared__ __attribute__((aligned(16))) unsigned char lds[2 * NIMG * IMG];  // [buffer][image]
  __shared__ int flag;
  auto img = [&](int buf, int m) { return lds + (buf * NIMG + m) * IMG; };
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int tiles = a.ntk * a.nto;
  const int wid = sfc_xcd_id((int)blockIdx.x, tiles * a.S);  // one XCD: consecutive splits, all tiles
  const int split = wid / tiles, tile = wid % tiles;
  const int tk = tile / a.nto, to = tile % a.nto;
  const int k0 = tk * kSdwT, o0 = to * kSdwT;
  const int nbeg = split * a.chunk, nend = min(a.N, nbeg + a.chunk);
  // staging: float4 column c4 = t % 20 of rows t / 20 + 16 i (i < NI) -- the
  // same column for every item, so the db partial is a per-thread float4
  const int c4 = t % 20, r0 = t / 20;
  const bool kx = k0 + 4 * c4 < a.K, ko = o0 + 4 * c4 < a.O;
  const bool do_db = a.db != nullptr && tk == 0;
  const float* xp = a.x + k0 + 4 * c4;
  const float* dp = a.d + o0 + 4 * c4;
  // register ring of D steps: the loads of step s + D are issued at the start
  // of step s, so D - 1 steps of loads stay in flight under the MFMAs (one step
  // in flight left every step waiting a full memory latency)
  constexpr int D = 4;
  float4 rx[D][NI], rd[D][NI];
  float4 dsum = make_float4(0.f, 0.f, 0.f, 0.f);
  // buffer loads over [nbeg, nend) only: rows past the split and columns past
  // K / O (voffset pushed out of range) read as zeros, so every load is
  // unconditional and the compiler's vmcnt tracking stays exact across steps
  typedef unsigned u32x4v __attribute__((ext_vector_type(4)));
  const int rows_here = nend > nbeg ? nend - nbeg : 0;
  const __amdgpu_buffer_rsrc_t xs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(a.x + (int64_t)nbeg * a.ldx), 0, (int)((int64_t)rows_here * a.ldx * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t ds = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(a.d + (int64_t)nbeg * a.ldd), 0, (int)((int64_t)rows_here * a.ldd * 4), 0x00020000);
  const int xcol = kx ? (k0 + 4 * c4) * 4 : 0x7ffffff0, dcol = ko ? (o0 + 4 * c4) * 4 : 0x7ffffff0;
  auto load = [&](auto jc, int rb) {  // rb: first row of the step, relative to nbeg
    constexpr int J = decltype(jc)::value;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int n = rb + r0 + 16 * i;
      rx[J][i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xs, kx ? n * (int)a.ldx * 4 + xcol : xcol, 0, 0));
      rd[J][i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(ds, ko ? n * (int)a.ldd * 4 + dcol : dcol, 0, 0));
    }
  };
  auto stage = [&](auto jc, int buf) {
    constexpr int J = decltype(jc)::value;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int off = sdw_off(r0 + 16 * i, 4 * c4);
      const float4 vx = rx[J][i], vd = rd[J][i];
      if (MODE == 0) {
        const h16x4 hx = {(_Float16)(vx.x * a.a_scale), (_Float16)(vx.y * a.a_scale), (_Float16)(vx.z * a.a_scale),
                          (_Float16)(vx.w * a.a_scale)};
        const h16x4 hd = {(_Float16)(vd.x * a.b_scale), (_Float16)(vd.y * a.b_scale), (_Float16)(vd.z * a.b_scale),
                          (_Float16)(vd.w * a.b_scale)};
        *reinterpret_cast<h16x4*>(img(buf, 0) + off) = hx;
        *reinterpret_cast<h16x4*>(img(buf, 1) + off) = hd;
      } else {
        s16x4 xh, xl, dh, dl;
        f3_split4(vx, xh, xl);
        f3_split4(vd, dh, dl);
        *reinterpret_cast<s16x4*>(img(buf, 0) + off) = xh;
        *reinterpret_cast<s16x4*>(img(buf, 1) + off) = xl;
        *reinterpret_cast<s16x4*>(img(buf, 2) + off) = dh;
        *reinterpret_cast<s16x4*>(img(buf, 3) + off) = dl;
      }
      if (do_db) {
        dsum.x += vd.x; dsum.y += vd.y; dsum.z += vd.z; dsum.w += vd.w;
      }
    }
  };
  f32x4 acc[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) acc[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  // tr-read addressing: lane 16g + 4q + p reads row 8g + q, columns 4p .. 4p + 3 of a 16-column block
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  auto compute = [&](int buf) {
#pragma unroll
    for (int s2 = 0; s2 < ROWS / 32; ++s2) {
      const int r = 32 * s2 + 8 * g + q;
      if (MODE == 0) {
        const h16x8 b = __builtin_bit_cast(h16x8, sdw_frag(img(buf, 1), r, 16 * w + 4 * p));
#pragma unroll
        for (int kb = 0; kb < 5; ++kb) {
          const h16x8 av = __builtin_bit_cast(h16x8, sdw_frag(img(buf, 0), r, 16 * kb + 4 * p));
          acc[kb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av, b, acc[kb], 0, 0, 0);
        }
      } else {
        const s16x8 bh = sdw_frag(img(buf, 2), r, 16 * w + 4 * p);
        const s16x8 bl = sdw_frag(img(buf, 3), r, 16 * w + 4 * p);
#pragma unroll
        for (int kb = 0; kb < 5; ++kb) {
          const s16x8 ah = sdw_frag(img(buf, 0), r, 16 * kb + 4 * p);
          const s16x8 al = sdw_frag(img(buf, 1), r, 16 * kb + 4 * p);
          acc[kb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, acc[kb], 0, 0, 0);
          acc[kb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, acc[kb], 0, 0, 0);
          acc[kb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, acc[kb], 0, 0, 0);
        }
      }
    }
  };
  // steps rounded up to whole rings: the extra steps load and multiply zeros
  const int nsteps = rows_here > 0 ? (rows_here + ROWS * D - 1) / (ROWS * D) * D : 0;
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3 % D>;
  auto body = [&](auto jc, int s) {  // step s lives in ring set s % D = J
    constexpr int J = decltype(jc)::value;
    load(jc, (s + D) * ROWS);  // set J was staged at step s - 1
    compute(s & 1);
    stage(std::integral_constant<int, (J + 1) % D>{}, (s + 1) & 1);
    __syncthreads();
  };
  if (nsteps > 0) {
    load(I0{}, 0);
    load(I1{}, ROWS);
    load(I2{}, 2 * ROWS);
    if (D > 3) load(I3{}, 3 * ROWS);
    stage(I0{}, 0);
    __syncthreads();
    for (int s0 = 0; s0 < nsteps; s0 += D) {
      body(I0{}, s0);
      body(I1{}, s0 + 1);
      body(I2{}, s0 + 2);
      if (D > 3) body(I3{}, s0 + 3);
    }
  }
  // db partial of this split: the 16 threads of one float4 column meet in LDS, summed in row order
  float* dpart = reinterpret_cast<float*>(lds);  // staging is done (barrier above)
  if (do_db) {
    reinterpret_cast<float4*>(dpart)[r0 * 20 + c4] = dsum;
    __syncthreads();
    if (t < kSdwT) {
      float v = 0.f;
      for (int rr = 0; rr < 16; ++rr) v += dpart[rr * kSdwT + t];
      dpart[16 * kSdwT + t] = v;
    }
    __syncthreads();
  }
  HgemmArgs ep;
  ep.alpha = a.alpha;
  ep.bias = nullptr;
  ep.out_scale = a.out_scale;
  const int c = lane & 15;
  auto store_out = [&](const f32x4 (&v)[5]) {
    const int o = o0 + 16 * w + c;
    if (o >= a.O) return;
#pragma unroll
    for (int kb = 0; kb < 5; ++kb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = k0 + 16 * kb + 4 * g + r;
        if (k < a.K) a.dW[(int64_t)k * a.O + o] = MODE == 0 ? h16_epi(v[kb][r], 0.f, ep) : v[kb][r];
      }
  };
  if (a.S == 1) {
    store_out(acc);
    if (do_db && t < kSdwT && o0 + t < a.O) a.db[o0 + t] = dpart[16 * kSdwT + t];
    return;
  }
  // hand-off: slab [tile][split][wave][kb][lane][4] (+ db slab [to][split][80]),
  // write-through stores, then one arrival per workgroup on the tile counter
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  float* tile_slab = a.slab + (int64_t)tile * a.S * (kSdwT * kSdwT);
  {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        tile_slab + (int64_t)split * (kSdwT * kSdwT), 0, kSdwT * kSdwT * 4, 0x00020000);
#pragma unroll
    for (int kb = 0; kb < 5; ++kb)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[kb]), rs, ((w * 5 + kb) * 64 + lane) * 16, 0,
                                             16 /* sc1 */);
    if (do_db && t < kSdwT / 4) {
      const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
          a.db_slab + ((int64_t)to * a.S + split) * kSdwT, 0, kSdwT * 4, 0x00020000);
      const f32x4 v = reinterpret_cast<const f32x4*>(dpart + 16 * kSdwT)[t];
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rb, t * 16, 0, 16 /* sc1 */);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) {
    const int old = __hip_atomic_fetch_add(&a.cnt[tile], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == a.S - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(&a.cnt[tile], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // ready for the next launch
    }
    flag = last;
  }
  __syncthreads();
  if (!flag) return;
  f32x4 sum[5];
#pragma unroll
  for (int kb = 0; kb < 5; ++kb) sum[kb] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const f32x4* base = reinterpret_cast<const f32x4*>(tile_slab) + w * 5 * 64 + lane;
  for (int sp = 0; sp < a.S; ++sp) {
    const f32x4* src = base + (int64_t)sp * (kSdwT * kSdwT / 4);
#pragma unroll
    for (int kb = 0; kb < 5; ++kb) sum[kb] += src[kb * 64];
  }
  store_out(sum);
  if (do_db && t < kSdwT && o0 + t < a.O) {
    const float* src = a.db_slab + (int64_t)to * a.S * kSdwT + t;
    float v = 0.f;
    for (int sp = 0; sp < a.S; ++sp) v += src[(int64_t)sp * kSdwT];
    a.db[o0 + t] = v;
  }
}

// column sums of a [batch][M][N] strided matrix into out[batch][N] (+=): bias
// gradients of batch_fc / scaled_fc.  Block = 64 columns x 4 row phases over
// a slice of kColSlice rows; the 4 phases meet in LDS and one fp32 atomic
// per column adds the slice (out zeroed first unless accumulating): enough
// workgroups for M in the thousands instead of one serial thread per column.
constexpr int kColSlice = 128;
__global__ __launch_bounds__(256) void k_colsum_strided(const float* __restrict__ x, int batch, int M, int N, int64_t sb,
                                                        int64_t ld, float* __restrict__ out, int64_t so) {
  __shared__ float part[4][64];
  const int b = blockIdx.z;
  const int n = blockIdx.x * 64 + (threadIdx.x & 63), ph = threadIdx.x >> 6;
  const int m0 = blockIdx.y * kColSlice, m1 = min(M, m0 + kColSlice);
  float s = 0.f;
  if (n < N) {
    // 8 independent row loads in flight per thread (a dependent chain of
    // single loads left this memory-bound kernel latency-bound)
    const float* p = x + (int64_t)b * sb + n;
    float a[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = 0.f;
    int m = m0 + ph;
    for (; m + 28 < m1; m += 32) {
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] += p[(int64_t)(m + 4 * j) * ld];
    }
    for (; m < m1; m += 4) a[0] += p[(int64_t)m * ld];
    s = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  }
  part[ph][threadIdx.x & 63] = s;
  __syncthreads();
  if (ph == 0 && n < N) {
    const float t = (part[0][threadIdx.x] + part[1][threadIdx.x]) + (part[2][threadIdx.x] + part[3][threadIdx.x]);
    atomicAdd(out + (int64_t)b * so + n, t);
  }
}

__global__ void k_zero_strided(float* __restrict__ out, int batch, int N, int64_t so) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)batch * N) return;
  out[(t / N) * so + (t % N)] = 0.f;
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
// int8 with Kp % 32 == 0 (zero padded).  64x64 tile per block, 4 waves of
// 32x32; the A and B panels move through LDS 64 k at a time (one 16-B load
// per lane per operand, rows padded to 80 B), then each wave feeds
// v_mfma_i32_32x32x32_i8 from LDS: lane l takes 16 consecutive k of row l%32.
__global__ __launch_bounds__(256) void k_i8_gemm(const signed char* __restrict__ qx,
                                                 const signed char* __restrict__ qwt, int M, int N, int Kp,
                                                 float scale, const float* __restrict__ bias, float* __restrict__ y,
                                                 int ldy) {
  constexpr int LDR = 80;  // bytes per LDS row (64 k + pad)
  __shared__ __attribute__((aligned(16))) signed char As[64 * LDR];
  __shared__ __attribute__((aligned(16))) signed char Bs[64 * LDR];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int bm = blockIdx.y * 64, bn = blockIdx.x * 64;
  const int wm = (w >> 1) * 32, wn = (w & 1) * 32;
  const int r = lane & 31, h = lane >> 5;
  // staging: thread t moves 16 B of row t/4, k bytes 16*(t%4)
  const int sr = t >> 2, sk = (t & 3) * 16;
  const int am = min(bm + sr, M - 1), an = min(bn + sr, N - 1);
  i32x16 acc = {0};
  for (int k0 = 0; k0 < Kp; k0 += 64) {
    i32x4 av = {0, 0, 0, 0}, bv = {0, 0, 0, 0};
    if (k0 + sk < Kp) {
      av = *reinterpret_cast<const i32x4*>(qx + (int64_t)am * Kp + k0 + sk);
      bv = *reinterpret_cast<const i32x4*>(qwt + (int64_t)an * Kp + k0 + sk);
    }
    __syncthreads();
    *reinterpret_cast<i32x4*>(As + sr * LDR + sk) = av;
    *reinterpret_cast<i32x4*>(Bs + sr * LDR + sk) = bv;
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < 64; ks += 32) {
      const i32x4 a = *reinterpret_cast<const i32x4*>(As + (wm + r) * LDR + ks + 16 * h);
      const i32x4 b = *reinterpret_cast<const i32x4*>(Bs + (wn + r) * LDR + ks + 16 * h);
      acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, acc, 0, 0, 0);
    }
  }
  const int n = bn + wn + r;
  if (n >= N) return;
  const float bvv = bias ? bias[n] : 0.f;
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) {
    const int m = bm + wm + 8 * (reg >> 2) + 4 * h + (reg & 3);
    if (m < M) y[(int64_t)m * ldy + n] = (float)acc[reg] * scale + bvv;
  }
}

// ---------------------------------------------------------------- rank_attention
// Rank-bucketed rank_attention.  An instance i of rank r = rank_i - 1 uses
// only the R parameter blocks W[r*R + f] (f = faster rank of a peer), and they
// sit contiguously: W_r = W[r*R*C : (r+1)*R*C] viewed as [R*C, P].  With
//   A_i[f*C + c] = sum over valid peers k of i with faster_k = f of x[idx_k][c]
// the op is, per rank r over the instances of that rank,
//   out_i = A_i W_r,   G_i = dout_i W_r^T (the input-gradient rows),   dW_r = sum_i A_i^T dout_i
// -- dense GEMMs (K = R*C for out / G, K = the rank's instances for dW) that
// never visit a block an instance does not use.  k_ra_bucket counting-sorts
// the instances by rank once (stable, one workgroup); the forward keeps the
// permutation + tile table for the backward.  Exact fp32 (v_mfma_f32_16x16x4_f32).
// A pair (i, k) is valid when rank_i in 1..R, faster_k + 1 in 1..R and
// 0 <= idx_k < B; invalid pairs contribute nothing (k_ra_dx skips them).
constexpr int kRaT = 32;  // instances per tile
constexpr int kRaBucketThreads = 1024;
constexpr int kRaSeg = 256;  // dW: peer tables staged per segment of instances

__device__ __forceinline__ int ra_bucket_of(int rank, int R) { return (rank >= 1 && rank <= R) ? rank - 1 : R; }

// meta (ints, after perm[B]): [0, R+1) count, [R+1, 2R+2) base, [2R+2, 3R+4) tile prefix
template <int R>
__global__ __launch_bounds__(kRaBucketThreads) void k_ra_bucket(const int* __restrict__ ro, int ld, int B,
                                                                int* __restrict__ perm, int* __restrict__ meta) {
  constexpr int Q = R + 1;
  __shared__ int wsum[kRaBucketThreads / 64][Q];
  __shared__ int tot[Q];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int chunk = (B + kRaBucketThreads - 1) / kRaBucketThreads;
  const int i0 = min(B, t * chunk), i1 = min(B, i0 + chunk);
  // up to kPre ranks per thread are loaded once, all in flight together, and
  // kept for the scatter pass (a serial load per instance and pass made this
  // one-workgroup kernel latency bound: ~11 us at B = 5k)
  constexpr int kPre = 8;
  const bool pre = chunk <= kPre;
  int bk[kPre];
#pragma unroll
  for (int j = 0; j < kPre; ++j) bk[j] = (pre && i0 + j < i1) ? ro[(int64_t)(i0 + j) * ld] : 0;
#pragma unroll
  for (int j = 0; j < kPre; ++j) bk[j] = ra_bucket_of(bk[j], R);
  int cnt[Q];
#pragma unroll
  for (int q = 0; q < Q; ++q) cnt[q] = 0;
  if (pre) {
#pragma unroll
    for (int j = 0; j < kPre; ++j)
      if (i0 + j < i1) {
#pragma unroll
        for (int q = 0; q < Q; ++q) cnt[q] += bk[j] == q;
      }
  } else {
    for (int i = i0; i < i1; ++i) {
      const int b = ra_bucket_of(ro[(int64_t)i * ld], R);
#pragma unroll
      for (int q = 0; q < Q; ++q) cnt[q] += b == q;
    }
  }
  int off[Q];
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    int v = cnt[q];
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int u = __shfl_up(v, d);
      if (lane >= d) v += u;
    }
    off[q] = v - cnt[q];
    if (lane == 63) wsum[w][q] = v;
  }
  __syncthreads();
  if (t < Q) {
    int s = 0;
    for (int ww = 0; ww < kRaBucketThreads / 64; ++ww) {
      const int v = wsum[ww][t];
      wsum[ww][t] = s;
      s += v;
    }
    tot[t] = s;
  }
  __syncthreads();
  int base = 0;
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    off[q] += wsum[w][q] + base;
    base += tot[q];
  }
  if (pre) {
#pragma unroll
    for (int j = 0; j < kPre; ++j) {
      if (i0 + j >= i1) continue;
      int pos = 0;
#pragma unroll
      for (int q = 0; q < Q; ++q)
        if (bk[j] == q) pos = off[q]++;
      perm[pos] = i0 + j;
    }
  } else {
    for (int i = i0; i < i1; ++i) {
      const int b = ra_bucket_of(ro[(int64_t)i * ld], R);
      int pos = 0;
#pragma unroll
      for (int q = 0; q < Q; ++q)
        if (b == q) pos = off[q]++;
      perm[pos] = i;
    }
  }
  if (t == 0) {
    int bs = 0, tp = 0;
    for (int q = 0; q < Q; ++q) {
      meta[q] = tot[q];
      meta[Q + q] = bs;
      meta[2 * Q + q] = tp;
      bs += tot[q];
      tp += (tot[q] + kRaT - 1) / kRaT;
    }
    meta[3 * Q] = tp;
  }
}

// tile x of the bucketed order -> (bucket, first sorted position, instances)
template <int R>
__device__ __forceinline__ bool ra_tile(const int* __restrict__ meta, int x, int* q, int* start, int* n) {
  constexpr int Q = R + 1;
  // the tile prefix is non-decreasing: the bucket is the number of prefix
  // entries <= x, every entry loaded at once (a search loop made each step a
  // dependent load)
  int pre[R + 1];
#pragma unroll
  for (int j = 0; j <= R; ++j) pre[j] = meta[2 * Q + 1 + j];
  if (x >= pre[R]) return false;
  int b = 0;
#pragma unroll
  for (int j = 0; j < R; ++j) b += x >= pre[j];
  const int lt = x - (b ? pre[b - 1] : 0);
  *q = b;
  *start = meta[Q + b] + lt * kRaT;
  *n = min(kRaT, meta[b] - lt * kRaT);
  return true;
}

// the valid peers of instance i as (faster, idx), faster = -1 if invalid
template <int R>
__device__ __forceinline__ void ra_peers(const int* __restrict__ ro, int ld, int i, int B, int* pf, int* px) {
#pragma unroll
  for (int k = 0; k < R; ++k) {
    int f = -1, id = 0;
    if (i >= 0) {
      f = ro[(int64_t)i * ld + 2 * k + 1] - 1;
      id = ro[(int64_t)i * ld + 2 * k + 2];
      if (f >= R || id < 0 || id >= B) f = -1;
    }
    pf[k] = f;
    px[k] = f >= 0 ? id : 0;
  }
}

// out rows of one tile (32 instances of rank q) x 64 outputs; K = R*C in
// chunks of KC, the next chunk's gathered A and W_q rows held in registers
// while the current one runs on MFMA.  KC = 128 when the gathers vectorise
// (half the chunk round trips of KC = 64: the loop is load-latency bound).
template <int R, int KC>
__global__ __launch_bounds__(256) void k_ra_fwd(const float* __restrict__ x, const int* __restrict__ ro, int ld,
                                                const float* __restrict__ W, int B, int C, int P,
                                                const int* __restrict__ perm, const int* __restrict__ meta,
                                                float* __restrict__ out) {
  constexpr int AK = KC / 8;   // A elements per thread: instance t & 31, k rows ka .. ka + AK - 1
  constexpr int WN = KC / 4;   // W elements per thread
  __shared__ float As[KC][kRaT + 4];  // [k][instance]
  __shared__ __attribute__((aligned(16))) float Ws[KC][68];  // [k][p]
  __shared__ int sperm[kRaT];
  int q, start, n;
  if (!ra_tile<R>(meta, blockIdx.x, &q, &start, &n)) return;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int p0 = blockIdx.y * 64;
  if (t < kRaT) sperm[t] = t < n ? perm[start + t] : -1;
  __syncthreads();
  if (q == R) {  // instances without a valid rank: zero rows
    for (int e = t; e < n * 64; e += 256) {
      const int p = p0 + (e & 63);
      if (p < P) out[(int64_t)sperm[e >> 6] * P + p] = 0.f;
    }
    return;
  }
  const int KT = R * C;
  const float* Wq = W + (int64_t)q * KT * P;
  const int ii = t & 31, ka = (t >> 5) * AK;
  int pf[R], px[R];
  ra_peers<R>(ro, ld, sperm[ii], B, pf, px);
  // W staging: column p = t & 63, k rows (t >> 6) + 4 j (scalar), or
  // columns 4 (t & 15) .. +3, k rows (t >> 4) + 16 j (float4)
  const int wp = t & 63, wr = t >> 6;
  const int wq = (t & 15) * 4, wr4 = t >> 4;
  // C % AK == 0: a thread's AK consecutive k rows lie in one peer block (one
  // faster rank f) and one aligned run of each matching peer's x row --
  // AK / 4 float4 loads per matching peer instead of R predicated scalar
  // loads per row.  P % 4 == 0: W rows by float4.
  const bool vec = (C % AK) == 0 && (P % 4) == 0 && ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(W)) & 15) == 0;
  float ra[AK], rw[WN];
  auto load = [&](int kc) {
    int kg = kc + ka;
    if (vec) {
      float4 av[AK / 4];
#pragma unroll
      for (int v = 0; v < AK / 4; ++v) av[v] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (kg < KT) {
        const int f = kg / C, c = kg - f * C;
#pragma unroll
        for (int k = 0; k < R; ++k)
          if (pf[k] == f) {
            const float4* xp = reinterpret_cast<const float4*>(x + (int64_t)px[k] * C + c);
#pragma unroll
            for (int v = 0; v < AK / 4; ++v) {
              const float4 xv = xp[v];
              av[v].x += xv.x; av[v].y += xv.y; av[v].z += xv.z; av[v].w += xv.w;
            }
          }
      }
#pragma unroll
      for (int v = 0; v < AK / 4; ++v) {
        ra[4 * v] = av[v].x; ra[4 * v + 1] = av[v].y; ra[4 * v + 2] = av[v].z; ra[4 * v + 3] = av[v].w;
      }
#pragma unroll
      for (int j = 0; j < WN / 4; ++j) {
        const int r = kc + wr4 + 16 * j;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (r < KT && p0 + wq < P) v = *reinterpret_cast<const float4*>(Wq + (int64_t)r * P + p0 + wq);
        rw[4 * j] = v.x; rw[4 * j + 1] = v.y; rw[4 * j + 2] = v.z; rw[4 * j + 3] = v.w;
      }
      return;
    }
    int f = kg / C, c = kg - f * C;
#pragma unroll
    for (int j = 0; j < AK; ++j) {
      float a = 0.f;
      if (kg < KT) {
#pragma unroll
        for (int k = 0; k < R; ++k)
          if (pf[k] == f) a += x[(int64_t)px[k] * C + c];
      }
      ra[j] = a;
      ++kg;
      if (++c == C) { c = 0; ++f; }
    }
#pragma unroll
    for (int j = 0; j < WN; ++j) {
      const int r = kc + wr + 4 * j;
      rw[j] = (r < KT && p0 + wp < P) ? Wq[(int64_t)r * P + p0 + wp] : 0.f;
    }
  };
  const int fr = lane & 15, fk = lane >> 4, mi = (w & 1) * 16, nb = (w >> 1) * 32;
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  load(0);
  for (int kc = 0; kc < KT; kc += KC) {
    __syncthreads();
#pragma unroll
    for (int j = 0; j < AK; ++j) As[ka + j][ii] = ra[j];
    if (vec) {
#pragma unroll
      for (int j = 0; j < WN / 4; ++j)
        *reinterpret_cast<float4*>(&Ws[wr4 + 16 * j][wq]) =
            make_float4(rw[4 * j], rw[4 * j + 1], rw[4 * j + 2], rw[4 * j + 3]);
    } else {
#pragma unroll
      for (int j = 0; j < WN; ++j) Ws[wr + 4 * j][wp] = rw[j];
    }
    __syncthreads();
    if (kc + KC < KT) load(kc + KC);
#pragma unroll
    for (int kk = 0; kk < KC; kk += 4) {
      const float a = As[kk + fk][mi + fr];
      acc0 = mfma4(a, Ws[kk + fk][nb + fr], acc0);
      acc1 = mfma4(a, Ws[kk + fk][nb + 16 + fr], acc1);
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int m = mi + 4 * fk + r;
    if (m >= n) continue;
    const int64_t row = (int64_t)sperm[m] * P;
    if (p0 + nb + fr < P) out[row + p0 + nb + fr] = acc0[r];
    if (p0 + nb + 16 + fr < P) out[row + p0 + nb + 16 + fr] = acc1[r];
  }
}

// G_j = dout_j W_q^T for every instance j of a valid rank q, dense [B][R*C]
// (row j, column f*C + c: the gradient reaching the peer of j whose faster
// rank is f).  Tile: 32 instances; a workgroup runs `cbs` 64-column blocks of
// R*C (blockIdx.y, + gridDim.y, ...), so the bucket lookup, the perm read and
// -- when P <= 64 -- the dout tile are paid once per tile, not once per
// column block; the next block's W_q^T chunk is loaded into registers while
// the current one runs on MFMA.  Invalid pairs are resolved by k_ra_dx (no
// zero rows, no per-peer scatter).
template <int R>
__global__ __launch_bounds__(256) void k_ra_g(const float* __restrict__ dout, const float* __restrict__ W, int B,
                                              int C, int P, const int* __restrict__ perm,
                                              const int* __restrict__ meta, float* __restrict__ G, int dbg) {
  constexpr int KC = 64;
  // staging: thread t reads 4 consecutive p (one float4 when P % 4 == 0) of
  // rows t / 16 + 16 j, so a wave instruction covers 4 whole 256 B rows --
  // coalesced (a lane-per-row mapping touched 64 segments per instruction
  // and made the kernel TA-bound: 21.5 us at B = 5k R = 8).  Row strides 33 /
  // 65: the transposed LDS stores hit 64 distinct banks.
  __shared__ float Ds[KC][kRaT + 1];  // [p][instance]
  __shared__ float Ws[KC][65];        // [p][column]
  __shared__ int sperm[kRaT];
  int q, start, n;
  if (!ra_tile<R>(meta, blockIdx.x, &q, &start, &n)) return;
  if (q == R) return;  // rank-less instances: no valid pair reads their G row
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int KT = R * C, ncb = (KT + 63) / 64, npc = (P + KC - 1) / KC;
  const int nmine = blockIdx.y < ncb ? (ncb - 1 - blockIdx.y) / gridDim.y + 1 : 0;
  const int nit = nmine * npc;  // (column block, p chunk) iterations, p fastest
  if (nit == 0) return;
  if (t < kRaT) sperm[t] = t < n ? perm[start + t] : -1;
  __syncthreads();
  const float* Wq = W + (int64_t)q * KT * P;
  const int sr = t >> 4, sp = (t & 15) * 4;
  const bool vec = (P % 4) == 0 && ((reinterpret_cast<uintptr_t>(dout) | reinterpret_cast<uintptr_t>(W)) & 15) == 0;
  int64_t drow[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) drow[j] = sperm[sr + 16 * j] >= 0 ? (int64_t)sperm[sr + 16 * j] * P : -1;
  const bool dout_once = npc == 1;  // the dout tile is the same for every column block
  float4 rd[2], rw[4];
  auto ld4 = [&](const float* row, int p, bool ok) {
    if (!ok || p >= P) return make_float4(0.f, 0.f, 0.f, 0.f);
    if (vec) return *reinterpret_cast<const float4*>(row + p);
    return make_float4(row[p], p + 1 < P ? row[p + 1] : 0.f, p + 2 < P ? row[p + 2] : 0.f,
                       p + 3 < P ? row[p + 3] : 0.f);
  };
  auto load = [&](int it) {
    const int n0 = (blockIdx.y + (it / npc) * gridDim.y) * 64, pc = (it % npc) * KC;
    if (!dout_once || it == 0) {
#pragma unroll
      for (int j = 0; j < 2; ++j) rd[j] = ld4(dout + (drow[j] >= 0 ? drow[j] : 0), pc + sp, drow[j] >= 0);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = n0 + sr + 16 * j;
      rw[j] = ld4(Wq + (int64_t)(col < KT ? col : 0) * P, pc + sp, col < KT);
    }
  };
  auto put4 = [](float* base, int stride, const float4& v) {
    base[0] = v.x;
    base[stride] = v.y;
    base[2 * stride] = v.z;
    base[3 * stride] = v.w;
  };
  const int fr = lane & 15, fk = lane >> 4, mi = (w & 1) * 16, nb = (w >> 1) * 32;
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  load(0);
  for (int it = 0; it < nit; ++it) {
    __syncthreads();
    if (!dout_once || it == 0) {
#pragma unroll
      for (int j = 0; j < 2; ++j) put4(&Ds[sp][sr + 16 * j], kRaT + 1, rd[j]);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) put4(&Ws[sp][sr + 16 * j], 65, rw[j]);
    __syncthreads();
    if (it + 1 < nit) load(it + 1);
#pragma unroll
    for (int kk = 0; kk < KC; kk += 4) {
      const float a = Ds[kk + fk][mi + fr];
      acc0 = mfma4(a, Ws[kk + fk][nb + fr], acc0);
      acc1 = mfma4(a, Ws[kk + fk][nb + 16 + fr], acc1);
    }
    if ((it + 1) % npc) continue;
    const int n0 = (blockIdx.y + (it / npc) * gridDim.y) * 64;
    if (dbg & 2) {  // timing experiment: keep the GEMM live, skip the stores
      if (acc0[0] + acc1[3] == 1234.5f) G[t] = acc0[1];
      acc0 = (f32x4){0.f, 0.f, 0.f, 0.f};
      acc1 = acc0;
      continue;
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int col = n0 + nb + 16 * h + fr;
      if (col >= KT) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = mi + 4 * fk + r;
        if (m < n) G[(int64_t)sperm[m] * KT + col] = h ? acc1[r] : acc0[r];
      }
    }
    acc0 = (f32x4){0.f, 0.f, 0.f, 0.f};
    acc1 = acc0;
  }
}

// dx[i][c] = sum over the peers j = ro[i][2t+2] of dexp[j][rank_i - 1][c]
// (the reference's gather form, merge_input_gradient_kernel), where
// dexp[j][k] = G_j[faster_{j,k} C : +C] when j's pair k is valid (rank_j,
// faster_{j,k} in 1..R, its index in [0, B)) and 0 otherwise -- resolved here
// from j's rank_offset row instead of materialising the zero rows
template <int R>
__global__ __launch_bounds__(256) void k_ra_dx(const float* __restrict__ G, const int* __restrict__ ro, int ld,
                                               int B, int C, float* __restrict__ dx) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)B * C) return;
  const int i = (int)(t / C), c = (int)(t % C);
  const int* ri = ro + (int64_t)i * ld;
  const int rank = ri[0];
  float s = 0.f;
  if (rank >= 1 && rank <= R) {
    // three rounds of independent loads (peer ids, their rank_offset
    // entries, the G values) instead of a dependent chain per peer
    const int k = rank - 1;
    int j[R], f[R];
#pragma unroll
    for (int u = 0; u < R; ++u) j[u] = ri[2 * u + 2];
#pragma unroll
    for (int u = 0; u < R; ++u) {
      f[u] = -1;
      if (j[u] < 0 || j[u] >= B) continue;
      const int* rj = ro + (int64_t)j[u] * ld;
      const int rkj = rj[0], ff = rj[2 * k + 1] - 1, id = rj[2 * k + 2];
      if (rkj >= 1 && rkj <= R && ff >= 0 && ff < R && id >= 0 && id < B) f[u] = ff;
    }
    float v[R];
#pragma unroll
    for (int u = 0; u < R; ++u) v[u] = f[u] >= 0 ? G[((int64_t)j[u] * R + f[u]) * C + c] : 0.f;
#pragma unroll
    for (int u = 0; u < R; ++u) s += v[u];
  }
  dx[t] = s;
}

// dW_q[m][p] += sum over a split of rank q's instances i of A_i[m] dout_i[p].
// Grid: (64-row tiles of R*C, 64-column tiles of P, R * splits).  Peer
// tables of kRaSeg instances at a time in LDS; the K loop takes 32 instances
// per stage, the next stage's gathered rows prefetched into registers.
template <int R>
__global__ __launch_bounds__(256) void k_ra_dw(const float* __restrict__ x, const float* __restrict__ dout,
                                               const int* __restrict__ ro, int ld, int B, int C, int P,
                                               const int* __restrict__ perm, const int* __restrict__ meta, int splits,
                                               float* __restrict__ dW, int dbg) {
  constexpr int Q = R + 1, KC = 32;
  __shared__ float Xs[KC][68];  // [instance][m]
  __shared__ float Ds[KC][68];  // [instance][p]
  __shared__ int sinst[kRaSeg], spf[R][kRaSeg], spx[R][kRaSeg];
  // per instance and faster rank f: the x row of its first peer of rank f
  // (-1: none), and a bit per f with further peers of that rank
  __shared__ int spm[R][kRaSeg];
  __shared__ unsigned sdup[kRaSeg];
  const int q = blockIdx.z / splits, s = blockIdx.z % splits;
  const int cnt = meta[q], per = (cnt + splits - 1) / splits;
  const int beg = meta[Q + q] + s * per, end = meta[Q + q] + min(cnt, (s + 1) * per);
  if (beg >= end) return;
  const int KT = R * C;
  const int m0 = blockIdx.x * 64, p0 = blockIdx.y * 64;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int tm = t & 63, tr = t >> 6;  // staging: column tm, instance rows tr + 4 j
  const int mg = m0 + tm, f = mg < KT ? mg / C : -2, c = mg - (mg / C) * C;
  const bool pok = p0 + tm < P;
  const int fr = lane & 15, fk = lane >> 4, wm = (w >> 1) * 32, wn = (w & 1) * 32;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float rx[8], rd[8];
  for (int sg = beg; sg < end; sg += kRaSeg) {
    const int sn = min(kRaSeg, end - sg);
    __syncthreads();
    if (t < sn) {
      const int i = perm[sg + t];
      int pf[R], px[R];
      ra_peers<R>(ro, ld, i, B, pf, px);
      sinst[t] = i;
      unsigned dup = 0;
#pragma unroll
      for (int k = 0; k < R; ++k) {
        spf[k][t] = pf[k];
        spx[k][t] = px[k];
      }
#pragma unroll
      for (int ff = 0; ff < R; ++ff) {
        int m = -1, cnt = 0;
#pragma unroll
        for (int k = 0; k < R; ++k)
          if (pf[k] == ff) {
            if (m < 0) m = px[k];
            ++cnt;
          }
        spm[ff][t] = m;
        if (cnt > 1) dup |= 1u << ff;
      }
      sdup[t] = dup;
    }
    __syncthreads();
    // every row's x / dout address first (one LDS read each, from the
    // per-rank match table: a compare chain over the peer table made every
    // row wait on R dependent LDS reads), then all 16 loads unconditionally
    // (clamped addresses, select after the load).  Further peers with the
    // same faster rank (never in page-view data) are added by `add_extra`.
    unsigned extra = 0;
    auto load = [&](int k0) {
      int64_t xa[8], da[8];
      extra = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int u = k0 + tr + 4 * j;
        const bool ok = u < sn;
        const int m = (ok && f >= 0) ? spm[f][u] : -1;
        xa[j] = m >= 0 ? (int64_t)m * C + c : -1;
        if (ok && f >= 0 && ((sdup[u] >> f) & 1u)) extra |= 1u << j;
        da[j] = (ok && pok) ? (int64_t)sinst[u] * P + p0 + tm : -1;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float a = x[xa[j] >= 0 ? xa[j] : 0], d = dout[da[j] >= 0 ? da[j] : 0];
        rx[j] = xa[j] >= 0 ? a : 0.f;
        rd[j] = da[j] >= 0 ? d : 0.f;
      }
    };
    auto add_extra = [&](int k0) {  // the further same-rank peers of flagged rows
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (!(extra & (1u << j))) continue;
        const int u = k0 + tr + 4 * j;
        int hits = 0;
        for (int k = 0; k < R; ++k)
          if (spf[k][u] == f && hits++ > 0) rx[j] += x[(int64_t)spx[k][u] * C + c];
      }
    };
    load(0);
    for (int k0 = 0; k0 < sn; k0 += KC) {
      if (extra) add_extra(k0);
      __syncthreads();
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        Xs[tr + 4 * j][tm] = rx[j];
        Ds[tr + 4 * j][tm] = rd[j];
      }
      __syncthreads();
      if (k0 + KC < sn) load(k0 + KC);
#pragma unroll
      for (int kk = 0; kk < KC; kk += 4) {
        const float a0 = Xs[kk + fk][wm + fr], a1 = Xs[kk + fk][wm + 16 + fr];
        const float b0 = Ds[kk + fk][wn + fr], b1 = Ds[kk + fk][wn + 16 + fr];
        acc[0][0] = mfma4(a0, b0, acc[0][0]);
        acc[0][1] = mfma4(a0, b1, acc[0][1]);
        acc[1][0] = mfma4(a1, b0, acc[1][0]);
        acc[1][1] = mfma4(a1, b1, acc[1][1]);
      }
    }
  }
  if (dbg & 1) {  // keep the GEMM live, skip the atomics
    const float z = acc[0][0][0] + acc[0][1][1] + acc[1][0][2] + acc[1][1][3];
    if (z == 1234.5f) dW[t] = z;
    return;
  }
  float* dWq = dW + (int64_t)q * KT * P;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int jn = 0; jn < 2; ++jn) {
      const int p = p0 + wn + jn * 16 + fr;
      if (p >= P) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm + i * 16 + 4 * fk + r;
        if (m < KT && acc[i][jn][r] != 0.f) atomicAdd(&dWq[(int64_t)m * P + p], acc[i][jn][r]);
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

__global__ void k_zero_mat(float* __restrict__ C, int batch, int M, int N, int64_t sC, int64_t ldc) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)batch * M * N) return;
  const int64_t b = t / ((int64_t)M * N), r = t % ((int64_t)M * N);
  C[b * sC + (r / N) * ldc + (r % N)] = 0.f;
}

void launch_sgemm(const SgemmArgs& g0, hipStream_t s) {
  if (g0.M == 0 || g0.N == 0 || g0.batch == 0) return;
  SgemmArgs g = g0;
  // fewer output tiles than ~2 waves of workgroups over 256 CUs and a long K:
  // split K (each slice >= 256 deep)
  const int64_t tiles = (int64_t)((g.N + 63) / 64) * ((g.M + 63) / 64) * g.batch;
  g.ksplit = 1;
  if (tiles < 512 && g.K >= 512) {
    const int64_t want = (1024 + tiles - 1) / tiles;
    g.ksplit = (int)std::max<int64_t>(1, std::min<int64_t>(want, g.K / 256));
  }
  if (g.ksplit > 1 && !g.accumulate)
    hipLaunchKernelGGL(k_zero_mat, dim3(nblk((int64_t)g.batch * g.M * g.N)), dim3(256), 0, s, g.C, g.batch, g.M,
                       g.N, g.sC, g.ldc);
  dim3 grid((g.N + 63) / 64, (g.M + 63) / 64, g.batch * g.ksplit);
  hipLaunchKernelGGL(k_mgemm, grid, dim3(256), 0, s, g);
}

namespace {
bool bfc_fits(const BfcArgs& a) {
  auto al = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  return a.I > 0 && a.O > 0 && a.I <= 64 && a.O <= 64 && a.I % 4 == 0 && a.O % 4 == 0 && a.rx % 4 == 0 &&
         a.sx % 4 == 0 && a.rw % 4 == 0 && a.sw % 4 == 0 && a.ry % 4 == 0 && a.sy % 4 == 0 && al(a.x) && al(a.W) &&
         al(a.y ? (const void*)a.y : (const void*)a.dy) && (a.dx == nullptr || al(a.dx));
}
}  // namespace

bool launch_batch_fc_fwd(const BfcArgs& a0, hipStream_t s) {
  if (!bfc_fits(a0)) return false;
  if (a0.N == 0 || a0.P == 0) return true;
  BfcArgs a = a0;
  a.tiles = batch_fc_tiles(a.P, a.N, 1024);  // 4 blocks / CU fit their 35 KB of LDS
  const int ntile = (a.N + 63) / 64;
  hipLaunchKernelGGL(k_bfc_fwd, dim3((ntile + a.tiles - 1) / a.tiles, a.P), dim3(256), 0, s, a);
  return true;
}

bool launch_batch_fc_bwd(const BfcArgs& a0, hipStream_t s) {
  if (!bfc_fits(a0)) return false;
  if (a0.N == 0 || a0.P == 0) return true;
  if (a0.ws == nullptr) return false;
  BfcArgs a = a0;
  a.tiles = batch_fc_tiles(a.P, a.N, 768);  // 3 blocks / CU fit their 52 KB of LDS
  const int G = batch_fc_bwd_groups(a.P, a.N);
  hipLaunchKernelGGL(k_bfc_bwd, dim3(G, a.P), dim3(256), 0, s, a);
  hipLaunchKernelGGL(k_bfc_reduce, dim3(nblk((int64_t)a.P * kBfcPart)), dim3(256), 0, s, a, G);
  return true;
}

void launch_hgemm(const HgemmArgs& g0, hipStream_t s) {
  if (g0.M == 0 || g0.N == 0) return;
  HgemmArgs g = g0;
  if (g.ksplit > 1) {
    (void)hipMemsetAsync(g.ws, 0, (size_t)g.M * g.N * sizeof(float), s);
  } else {
    g.ksplit = 1;
  }
  dim3 grid((g.N + 63) / 64, (g.M + 63) / 64, g.ksplit);
  hipLaunchKernelGGL(k_hgemm, grid, dim3(256), 0, s, g);
  if (g.ksplit > 1) hipLaunchKernelGGL(k_hgemm_epi, dim3(nblk((int64_t)g.M * g.N)), dim3(256), 0, s, g);
}

void launch_h16_epi(const float* acc, const float* bias, int M, int N, float alpha, float bias_scale, float out_scale,
                    float* out, hipStream_t s) {
  if ((int64_t)M * N == 0) return;
  const bool al = ((reinterpret_cast<uintptr_t>(acc) | reinterpret_cast<uintptr_t>(out) |
                    reinterpret_cast<uintptr_t>(bias)) & 15) == 0;
  if (N % 4 == 0 && (int64_t)M * N < (int64_t)INT32_MAX && al) {
    hipLaunchKernelGGL(k_h16_epi4, dim3((unsigned)((((int64_t)M * N) / 4 + 255) / 256)), dim3(256), 0, s, acc, bias, M,
                       N, alpha, bias_scale, out_scale, out);
    return;
  }
  hipLaunchKernelGGL(k_h16_epi, dim3(nblk((int64_t)M * N)), dim3(256), 0, s, acc, bias, M, N, alpha, bias_scale,
                     out_scale, out);
}

bool launch_sfc(const float* A, const void* Bk_, int M, int Nd, int Kd, float a_scale, const float* bias,
                float alpha, float bias_scale, float out_scale, float* out, hipStream_t s) {
  const _Float16* Bk = static_cast<const _Float16*>(Bk_);
  if ((Kd % 8) != 0 || ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(Bk)) & 15) != 0) return false;
  if ((int64_t)M * Nd == 0) return true;
  const int tiles = ((Nd + kSfcBN - 1) / kSfcBN) * ((M + kSfcBM - 1) / kSfcBM);
  hipLaunchKernelGGL(k_sfc, dim3(tiles), dim3(256), 0, s, A, Bk, M, Nd, Kd, a_scale, bias, alpha, bias_scale, out_scale,
                     out);
  return true;
}

bool launch_f3gemm_nt(const float* A, const void* Bh, const void* Bl, int M, int Nd, int Kd, float* out,
                      hipStream_t s) {
  if ((Kd % 8) != 0 || ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(Bh) |
                         reinterpret_cast<uintptr_t>(Bl)) & 15) != 0)
    return false;
  if ((int64_t)M * Nd == 0) return true;
  const int tiles = ((Nd + kSfcBN - 1) / kSfcBN) * ((M + kSfcBM - 1) / kSfcBM);
  hipLaunchKernelGGL(k_f3gemm_nt, dim3(tiles), dim3(256), 0, s, A, static_cast<const short*>(Bh),
                     static_cast<const short*>(Bl), M, Nd, Kd, out);
  return true;
}

bool launch_sfc_dw(const SfcDwArgs& a0, hipStream_t s) {
  const uintptr_t al = reinterpret_cast<uintptr_t>(a0.x) | reinterpret_cast<uintptr_t>(a0.d);
  if (a0.K % 4 || a0.O % 4 || a0.ldx % 4 || a0.ldd % 4 || (al & 15)) return false;
  if ((int64_t)a0.K * a0.O == 0) return true;
  SfcDwArgs a = a0;
  a.ntk = (a.K + kSdwT - 1) / kSdwT;
  a.nto = (a.O + kSdwT - 1) / kSdwT;
  if (a.N == 0) a.S = 1;
  if (a.S > 1 && (a.chunk % 64 || (int64_t)(a.S - 1) * a.chunk >= a.N || !a.slab || !a.cnt ||
                  (a.db && !a.db_slab)))
    return false;
  if (a.S == 1) a.chunk = a.N;
  if (a.mode == 1)
    hipLaunchKernelGGL(k_sfc_dw<1>, dim3(a.ntk * a.nto * a.S), dim3(kSdwNT), 0, s, a);
  else
    hipLaunchKernelGGL(k_sfc_dw<0>, dim3(a.ntk * a.nto * a.S), dim3(kSdwNT), 0, s, a);
  return true;
}

void launch_colsum_strided(const float* x, int batch, int M, int N, int64_t sb, int64_t ld, float* out, int64_t so,
                           bool accumulate, hipStream_t s) {
  if (batch * N == 0) return;
  if (!accumulate)
    hipLaunchKernelGGL(k_zero_strided, dim3(nblk((int64_t)batch * N)), dim3(256), 0, s, out, batch, N, so);
  if (M == 0) return;
  hipLaunchKernelGGL(k_colsum_strided, dim3((N + 63) / 64, (M + kColSlice - 1) / kColSlice, batch), dim3(256), 0, s,
                     x, batch, M, N, sb, ld, out, so);
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

#define PBX_RA_DISPATCH(KER, GRID, BLOCK, ...)                                       \
  switch (R) {                                                                       \
    case 1: hipLaunchKernelGGL(KER<1>, GRID, dim3(BLOCK), 0, s, __VA_ARGS__); break; \
    case 2: hipLaunchKernelGGL(KER<2>, GRID, dim3(BLOCK), 0, s, __VA_ARGS__); break; \
    case 3: hipLaunchKernelGGL(KER<3>, GRID, dim3(BLOCK), 0, s, __VA_ARGS__); break; \
    case 4: hipLaunchKernelGGL(KER<4>, GRID, dim3(BLOCK), 0, s, __VA_ARGS__); break; \
    case 5: hipLaunchKernelGGL(KER<5>, GRID, dim3(BLOCK), 0, s, __VA_ARGS__); break; \
    case 6: hipLaunchKernelGGL(KER<6>, GRID, dim3(BLOCK), 0, s, __VA_ARGS__); break; \
    case 7: hipLaunchKernelGGL(KER<7>, GRID, dim3(BLOCK), 0, s, __VA_ARGS__); break; \
    default: hipLaunchKernelGGL(KER<8>, GRID, dim3(BLOCK), 0, s, __VA_ARGS__); break; \
  }

template <int KC>
static void ra_fwd_launch(int R, dim3 g, hipStream_t s, const float* x, const int* ro, int ld, const float* W, int B,
                          int C, int P, const int* perm, const int* meta, float* out) {
  switch (R) {
    case 1: hipLaunchKernelGGL((k_ra_fwd<1, KC>), g, dim3(256), 0, s, x, ro, ld, W, B, C, P, perm, meta, out); break;
    case 2: hipLaunchKernelGGL((k_ra_fwd<2, KC>), g, dim3(256), 0, s, x, ro, ld, W, B, C, P, perm, meta, out); break;
    case 3: hipLaunchKernelGGL((k_ra_fwd<3, KC>), g, dim3(256), 0, s, x, ro, ld, W, B, C, P, perm, meta, out); break;
    case 4: hipLaunchKernelGGL((k_ra_fwd<4, KC>), g, dim3(256), 0, s, x, ro, ld, W, B, C, P, perm, meta, out); break;
    case 5: hipLaunchKernelGGL((k_ra_fwd<5, KC>), g, dim3(256), 0, s, x, ro, ld, W, B, C, P, perm, meta, out); break;
    case 6: hipLaunchKernelGGL((k_ra_fwd<6, KC>), g, dim3(256), 0, s, x, ro, ld, W, B, C, P, perm, meta, out); break;
    case 7: hipLaunchKernelGGL((k_ra_fwd<7, KC>), g, dim3(256), 0, s, x, ro, ld, W, B, C, P, perm, meta, out); break;
    default: hipLaunchKernelGGL((k_ra_fwd<8, KC>), g, dim3(256), 0, s, x, ro, ld, W, B, C, P, perm, meta, out); break;
  }
}

int rank_attention_bucket_ints(int B, int R) { return B + 3 * (R + 1) + 1; }

// upper bound on the tiles of the bucketed order: every bucket may end in a partial tile
static int ra_max_tiles(int B, int R) { return (B + kRaT - 1) / kRaT + R + 1; }

void launch_rank_attention_fwd(const float* x, const int* ro, int ld, const float* W, int B, int C, int P, int R,
                               int* bucket, float* out, hipStream_t s) {
  if (B == 0) return;
  int* perm = bucket;
  int* meta = bucket + B;
  PBX_RA_DISPATCH(k_ra_bucket, dim3(1), kRaBucketThreads, ro, ld, B, perm, meta);
  const dim3 gf(ra_max_tiles(B, R), (P + 63) / 64);
  const bool wide = C % 16 == 0 && P % 4 == 0 && ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(W)) & 15) == 0;
  if (wide && C % 32 == 0 && R * C >= 512)
    ra_fwd_launch<256>(R, gf, s, x, ro, ld, W, B, C, P, perm, meta, out);  // 2 chunk round trips at R*C = 512
  else if (wide)
    ra_fwd_launch<128>(R, gf, s, x, ro, ld, W, B, C, P, perm, meta, out);
  else
    ra_fwd_launch<64>(R, gf, s, x, ro, ld, W, B, C, P, perm, meta, out);
}

void launch_rank_attention_bwd(const float* x, const float* dout, const int* ro, int ld, const float* W, int B, int C,
                               int P, int R, const int* bucket, float* dexp, float* dx, float* dW, hipStream_t s) {
  if (B == 0) return;
  const int* perm = bucket;
  const int* meta = bucket + B;
  // timing experiments: PBX_RA_DEBUG 1 (dW without its atomics), 2 (G without its stores),
  // PBX_RA_DW_SPLITS, PBX_RA_G_BLOCKS (column blocks per k_ra_g workgroup)
  static const int dbg = getenv("PBX_RA_DEBUG") ? atoi(getenv("PBX_RA_DEBUG")) : 0;
  static const int dw_splits = getenv("PBX_RA_DW_SPLITS") ? atoi(getenv("PBX_RA_DW_SPLITS")) : 0;
  static const int g_blocks = getenv("PBX_RA_G_BLOCKS") ? atoi(getenv("PBX_RA_G_BLOCKS")) : 0;
  if (dx != nullptr) {  // G = dout W_r^T per instance, then the gather merge
    const int tiles = ra_max_tiles(B, R), ncb = (R * C + 63) / 64;
    int gy = std::min(ncb, std::max(1, (512 + tiles - 1) / tiles));
    if (g_blocks > 0) gy = (ncb + g_blocks - 1) / g_blocks;
    PBX_RA_DISPATCH(k_ra_g, dim3(tiles, gy), 256, dout, W, B, C, P, perm, meta, dexp, dbg);
    PBX_RA_DISPATCH(k_ra_dx, dim3(nblk((int64_t)B * C)), 256, dexp, ro, ld, B, C, dx);
  }
  if (dW == nullptr) return;
  // ~64 instances per split at an even rank mix (measured at B = 5k R = 8:
  // 128 per split 40 us, 64 25 us, 32 29 us -- the loop is latency bound, the
  // atomics grow with the splits); dW zeroed by the caller
  int splits = (B + R * 64 - 1) / (R * 64);
  splits = splits < 1 ? 1 : (splits > 64 ? 64 : splits);
  if (dw_splits > 0) splits = dw_splits;
  PBX_RA_DISPATCH(k_ra_dw, dim3((R * C + 63) / 64, (P + 63) / 64, R * splits), 256, x, dout, ro, ld, B, C, P, perm,
                  meta, splits, dW, dbg);
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

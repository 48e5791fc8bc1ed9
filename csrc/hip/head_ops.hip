// Fused CTR "head": data_norm + DeepFM first/second-order terms over the
// concatenated [pooled slots | dense] matrix, and its backward.
//
// Replaces a chain of ~10 kernels (data_norm fwd, bf16 cast for the MLP, FM
// fwd, first-order slice+sum; FM bwd, data_norm bwd + stats, 3 gradient adds)
// with one pass over x per direction.  A workgroup owns RB consecutive rows:
// rows are contiguous in memory, so the block's slab is staged into LDS with
// fully coalesced loads, then FM reductions read LDS; the data_norm summary
// statistics are reduced per block in LDS and added to a [2, C] accumulator
// with one atomic per column per block.
//
// Semantics: data_norm (reference paddle/fluid/operators/data_norm_op.cu:38-104)
// and the DeepFM FM term 0.5*sum_d[(sum_s v)^2 - sum_s v^2].
#include <hip/hip_bf16.h>
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "kernels.h"

namespace pbx {
namespace {

constexpr int kRB = 16;  // rows per workgroup

// width (elements) of the bf16 y slab; even, so the per-column arrays after
// it stay 4-byte aligned
__host__ __device__ inline int head_ys_width(int C, int Cp) {
  const int w = Cp > (C + 7) / 8 * 8 + 8 ? Cp : (C + 7) / 8 * 8 + 8;
  return (w + 1) / 2 * 2;
}

__device__ __forceinline__ unsigned short f2bf(float f) {
  // v_cvt_pk_bf16_f32 (gfx950): round-to-nearest-even in one instruction per
  // pair -- the same bits as the integer rounding (u + 0x7fff + lsb) >> 16
  // for every finite input, at a quarter of the VALU work
  return __builtin_bit_cast(unsigned short, static_cast<__bf16>(f));
}
__device__ __forceinline__ float bf2f(unsigned short h) { return __uint_as_float(((unsigned int)h) << 16); }

// dynamic LDS: xs[kRB][C] floats + s1[kRB][D].  512 threads per 16-row
// block: the row blocks are fixed at 16 (the tower's m-packed copy), so the
// extra waves come from wider blocks (the staging loop is latency-bound)
__global__ __launch_bounds__(512) void k_head_fwd(HeadArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* xs = lds;
  const int C = a.C, Cp = a.Cp;
  const int ldy = a.ldy ? a.ldy : Cp;
  const int row0 = blockIdx.x * kRB;
  const int rows = min(kRB, a.B - row0);
  if (rows <= 0) return;
  unsigned short* ys = reinterpret_cast<unsigned short*>(xs + kRB * (C + a.D));  // [kRB][Cp] bf16 (for y^T)
  // per-column data_norm mean / scale, once per block (not per element)
  float* cm = reinterpret_cast<float*>(ys + kRB * head_ys_width(C, Cp));
  float* cs = cm + C;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    if (a.bsize) {
      const float bs = a.bsize[c];
      cm[c] = a.bsum[c] / bs;
      cs[c] = sqrtf(bs / a.bsq[c]);
    } else {
      cm[c] = 0.f;
      cs[c] = 1.f;
    }
  }
  __syncthreads();
  // 1) stage + data_norm output (bf16, padded to Cp); r = i / Cp without an
  // integer division (exact: i < kRB * Cp << 2^23)
  const float inv_cp = 1.f / (float)Cp;
  for (int i = threadIdx.x; i < rows * Cp; i += blockDim.x) {
    const int r = (int)(((float)i + 0.5f) * inv_cp), c = i - r * Cp;
    float yv = 0.f;
    if (c < C) {
      const float v = a.x[(int64_t)(row0 + r) * C + c];
      xs[r * C + c] = v;
      yv = (v - cm[c]) * cs[c];
    }
    if (a.yf) {  // fp32 MLP input (fp32 tower)
      a.yf[(int64_t)(row0 + r) * ldy + c] = yv;
      continue;
    }
    const unsigned short yb = f2bf(yv);
    a.y[(int64_t)(row0 + r) * ldy + c] = yb;
    if (a.yT || a.ymp) ys[r * Cp + c] = yb;
  }
  if (a.ymp) {  // rows past B are zero in the m-packed copy
    for (int i = threadIdx.x; i < (kRB - rows) * Cp; i += blockDim.x) ys[rows * Cp + i] = 0;
  }
  if (blockIdx.x == 0 && a.means) {
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      a.means[c] = cm[c];
      a.scales[c] = cs[c];
    }
  }
  __syncthreads();
  if (a.ymp) {  // m-packed copy for the tower dW GEMM: chunk (row0/16, nb), 16 B per lane
    const int NB = Cp / 32;
    const int64_t mb = row0 / kRB;
    for (int i = threadIdx.x; i < NB * 64; i += blockDim.x) {
      const int nb = i >> 6, l = i & 63;
      unsigned int p[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        p[j] = (unsigned)ys[(8 * (l >> 5) + 2 * j) * Cp + 32 * nb + (l & 31)] |
               ((unsigned)ys[(8 * (l >> 5) + 2 * j + 1) * Cp + 32 * nb + (l & 31)] << 16);
      *reinterpret_cast<uint4*>(a.ymp + ((mb * NB + nb) * 64 + l) * 8) = make_uint4(p[0], p[1], p[2], p[3]);
    }
  }
  if (a.ympf) {  // MP32 copy for the fp32 tower: chunk (row0/16, nb), lane (c, g): rows 4g..4g+3, column 16nb + c
    const int NB = Cp / 16;
    const int64_t mb = row0 / kRB;
    for (int i = threadIdx.x; i < NB * 64; i += blockDim.x) {
      const int nb = i >> 6, l = i & 63;
      const int c = 16 * nb + (l & 15), g = l >> 4;
      float v[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int r = 4 * g + t;
        v[t] = (r < rows && c < C) ? (xs[r * C + c] - cm[c]) * cs[c] : 0.f;
      }
      *reinterpret_cast<float4*>(a.ympf + ((mb * NB + nb) * 64 + l) * 4) = make_float4(v[0], v[1], v[2], v[3]);
    }
  }
  if (a.stat_part && a.means) {  // data_norm batch statistics, per-block partial row
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      const float mean = cm[c];
      float sx = 0.f, sq = 0.f;
      for (int r = 0; r < rows; ++r) {
        const float v = xs[r * C + c];
        sx += v;
        sq += (v - mean) * (v - mean);
      }
      a.stat_part[(int64_t)blockIdx.x * 2 * C + c] = sx;
      a.stat_part[(int64_t)blockIdx.x * 2 * C + C + c] = sq;
    }
  }
  if (a.yT) {  // y^T[c][row0 .. row0+rows): one 32-byte run per column
    for (int c = threadIdx.x; c < Cp; c += blockDim.x) {
      unsigned short* dst = a.yT + (int64_t)c * a.ldyt + row0;
      if (rows == kRB && ((row0 & 7) == 0) && ((a.ldyt & 7) == 0)) {
        uint4 v0, v1;
        unsigned int p[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) p[j] = (unsigned)ys[(2 * j) * Cp + c] | ((unsigned)ys[(2 * j + 1) * Cp + c] << 16);
        v0 = make_uint4(p[0], p[1], p[2], p[3]);
        v1 = make_uint4(p[4], p[5], p[6], p[7]);
        reinterpret_cast<uint4*>(dst)[0] = v0;
        reinterpret_cast<uint4*>(dst)[1] = v1;
      } else {
        for (int r = 0; r < rows; ++r) dst[r] = ys[r * Cp + c];
      }
    }
  }
  // 2) first + FM per row: 16 threads per row (kRB=16 rows x 16 = 256)
  const int r = threadIdx.x >> 4, t = threadIdx.x & 15;
  float lin = 0.f;
  if (r < rows) {
    const float* xr = xs + r * C;
    // first order: sum over slots of embed_w column
    for (int s = t; s < a.S; s += 16) lin += xr[s * a.Eo + a.ew_col];
    // FM: lane t handles dims d = t, t+16, ... (D <= 16 typical)
    for (int d = t; d < a.D; d += 16) {
      float s1 = 0.f, s2 = 0.f;
      for (int s = 0; s < a.S; ++s) {
        const float v = xr[s * a.Eo + a.ew_col + 1 + d];
        s1 += v;
        s2 += v * v;
      }
      lin += 0.5f * (s1 * s1 - s2);
    }
  }
  for (int off = 8; off > 0; off >>= 1) lin += __shfl_xor(lin, off, 16);
  if (r < rows && t == 0) a.lin[row0 + r] = lin;
}

// RB rows per work-group: 16 when the data_norm statistics partials are
// produced (their [head_blocks][2C] layout), else 8 -- twice the
// work-groups, which the latency-bound gather/scale loop needs (2 -> 4 waves
// per SIMD at B = 8192).  The LDS layout is the kRB-row one either way.
template <int RB>
__global__ __launch_bounds__(256) void k_head_bwd(HeadArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int C = a.C, Cp = a.Cp, D = a.D;
  float* xs = lds;                 // [RB][C]
  float* s1s = lds + kRB * C;      // [RB][D]
  const int row0 = blockIdx.x * RB;
  const int rows = min(RB, a.B - row0);
  if (rows <= 0) return;
  for (int i = threadIdx.x; i < rows * C; i += blockDim.x) {
    xs[i] = a.x[(int64_t)row0 * C + i];  // rows are contiguous
  }
  __syncthreads();
  for (int i = threadIdx.x; i < rows * D; i += blockDim.x) {
    const int r = i / D, d = i - r * D;
    const float* xr = xs + r * C;
    float s1 = 0.f;
    for (int s = 0; s < a.S; ++s) s1 += xr[s * a.Eo + a.ew_col + 1 + d];
    s1s[r * D + d] = s1;
  }
  __syncthreads();
  // per-column scale and role (-1 plain, -2 first-order embed_w, d >= 0
  // embedx dim d of the FM) and per-row d lin, once per block
  float* cs = reinterpret_cast<float*>(reinterpret_cast<unsigned short*>(xs + kRB * (C + D)) +
                                       kRB * head_ys_width(C, Cp));
  int* jc = reinterpret_cast<int*>(cs + C);
  __shared__ float dls[RB];
  const int sparse_w = a.S * a.Eo;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    cs[c] = a.scales ? a.scales[c] : 1.f;
    int code = -1;
    if (c < sparse_w) {
      const int j = c % a.Eo;
      if (j == a.ew_col) code = -2;
      else if (j > a.ew_col && j <= a.ew_col + D) code = j - a.ew_col - 1;
    }
    jc[c] = code;
  }
  if (threadIdx.x < rows)
    dls[threadIdx.x] = a.dlin ? a.dlin[row0 + threadIdx.x] * (a.dlin_scale ? a.dlin_scale[0] : 1.f) : 0.f;
  __syncthreads();
  const int ldy = a.ldy ? a.ldy : Cp;
  const float inv_c = 1.f / (float)C;
  for (int i = threadIdx.x; i < rows * C; i += blockDim.x) {
    const int r = (int)(((float)i + 0.5f) * inv_c), c = i - r * C;
    float g = a.dyf  ? a.dyf[(int64_t)(row0 + r) * ldy + c] * cs[c]
              : a.dy ? bf2f(a.dy[(int64_t)(row0 + r) * ldy + c]) * cs[c]
                     : 0.f;
    const int code = jc[c];
    if (code != -1 && a.dlin) {
      const float dl = dls[r];
      g += code == -2 ? dl : dl * (s1s[r * D + code] - xs[i]);
    }
    a.dx[(int64_t)row0 * C + i] = g;
  }
  // data_norm summary partials: sum x and sum (x-mean)^2 per column
  if (a.stat_acc) {
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      const float mean = a.means[c];
      float sx = 0.f, sq = 0.f;
      for (int r = 0; r < rows; ++r) {
        const float v = xs[r * C + c];
        sx += v;
        sq += (v - mean) * (v - mean);
      }
      // per-block partial row (no same-address atomics across blocks)
      a.stat_acc[(int64_t)blockIdx.x * 2 * C + c] = sx;
      a.stat_acc[(int64_t)blockIdx.x * 2 * C + C + c] = sq;
    }
  }
}

// stats[3, C] from the column-reduced [2C] sums
__global__ void k_dn_stats(const float* __restrict__ acc, int C, int N, float eps, float* __restrict__ stats) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  stats[c] = 1.f;
  stats[C + c] = acc[c] / (float)N;
  stats[2 * C + c] = acc[C + c] / (float)N + eps;
}

}  // namespace

size_t head_lds_bytes(int C, int D, int Cp) {
  // fp32 row slab + FM sums, the bf16 y slab for the transposed / packed
  // write, then two per-column arrays (fwd: mean, scale; bwd: scale, role)
  return (size_t)kRB * (C + D) * sizeof(float) + (size_t)kRB * head_ys_width(C, Cp) * sizeof(unsigned short) +
         (size_t)2 * C * sizeof(float);
}

void launch_head_fwd(const HeadArgs& a, hipStream_t s) {
  if (a.B == 0) return;
  const unsigned g = (unsigned)((a.B + kRB - 1) / kRB);
  hipLaunchKernelGGL(k_head_fwd, dim3(g), dim3(512), head_lds_bytes(a.C, a.D, a.Cp), s, a);
}

void launch_head_bwd(const HeadArgs& a, hipStream_t s) {
  if (a.B == 0) return;
  if (a.stat_acc) {
    const unsigned g = (unsigned)((a.B + kRB - 1) / kRB);
    hipLaunchKernelGGL(k_head_bwd<kRB>, dim3(g), dim3(256), head_lds_bytes(a.C, a.D, a.Cp), s, a);
  } else {
    // rows per workgroup without the statistics (PBX_HEAD_BWD_RB 4 / 8)
    static const int rb = [] {
      const char* e = getenv("PBX_HEAD_BWD_RB");
      return (e && atoi(e) == 4) ? 4 : 8;
    }();
    const unsigned g = (unsigned)((a.B + rb - 1) / rb);
    if (rb == 4)
      hipLaunchKernelGGL(k_head_bwd<4>, dim3(g), dim3(256), head_lds_bytes(a.C, a.D, a.Cp), s, a);
    else
      hipLaunchKernelGGL(k_head_bwd<8>, dim3(g), dim3(256), head_lds_bytes(a.C, a.D, a.Cp), s, a);
  }
}

int head_blocks(int B) { return (B + kRB - 1) / kRB; }

void launch_dn_stats(const float* part, int nrows, int C, int N, float eps, float* stats, float* acc,
                     hipStream_t s) {
  if (C == 0) return;
  launch_fill32(acc, 0u, 2 * (int64_t)C, s);
  launch_colsum_acc(part, nrows, 2 * C, acc, -1, nullptr, s);
  hipLaunchKernelGGL(k_dn_stats, dim3((C + 255) / 256), dim3(256), 0, s, acc, C, N, eps, stats);
}

}  // namespace pbx

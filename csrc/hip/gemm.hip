// bf16 MFMA GEMM for the CTR MLP (gfx950, v_mfma_f32_32x32x16_bf16) with
// fused prologue/epilogues:
//   fwd   Y  = relu(X W^T + b)            (bf16 out)         EPI_BIAS_RELU / EPI_BIAS
//   bwd   dX = (dY . [Y>0]) W             (bf16 out)         relu mask fused in A staging
//   bwd   dW = (dY . [Y>0])^T [X | 1]     (fp32 split-K slabs; the virtual ones
//                                          column makes db fall out of the same GEMM)
// Tile 64x64x64, 4 waves (2x2), each wave a 32x32 accumulator (16 f32/lane);
// LDS double-buffered with the next tile's global loads issued before the MFMAs.
// LDS tiles are stored k-contiguous with a 16-B row pad (144-B stride) so the
// ds_read_b128 fragment reads are bank-conflict free; operands whose memory
// layout is m/n-contiguous are transposed on the LDS write.
// The hipBLASLt kernels picked for these skinny shapes (M=8192, N=400, K~300)
// ran at ~70 TFLOP/s with separate cast / bias / relu / reduce kernels around
// them; this removes all of those launches.
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace pbx {
namespace {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BK = 64, PAD = 8, LDK = BK + PAD;
constexpr int kGemvRows = 32;  // rows per workgroup in the output-layer backward

__device__ __forceinline__ unsigned short f2bf(float f) {
  // v_cvt_pk_bf16_f32 (gfx950): round-to-nearest-even in one instruction per
  // pair -- the same bits as the integer rounding (u + 0x7fff + lsb) >> 16
  // for every finite input, at a quarter of the VALU work
  return __builtin_bit_cast(unsigned short, static_cast<__bf16>(f));
}

// Register-staged, LDS double-buffered tile loader (software pipeline: the
// global loads of tile k+1 are in flight while the MFMAs of tile k run).
// A ROWS x BK tile is ROWS*BK/8 16-byte vectors, NV = ROWS/32 per thread.
template <int ROWS>
struct Stage {
  bf16x8 v[ROWS / 32];
};

// kcontig: vector vid -> tile row vid/8, k cols (vid%8)*8 .. +8 ;
// else     vector vid -> memory row (k) vid/(ROWS/8), r cols (vid%(ROWS/8))*8 .. +8
// (m/n-contiguous operand, transposed on the LDS write).
template <int ROWS>
__device__ __forceinline__ void load_tile(Stage<ROWS>& st, const unsigned short* __restrict__ base,
                                          const unsigned short* __restrict__ mask, int ld, bool kcontig, int r0,
                                          int k0, int R, int K, int ones_col) {
#pragma unroll
  for (int h = 0; h < ROWS / 32; ++h) {
    const int vid = threadIdx.x + 256 * h;
    bf16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
    int gr, gk;
    if (kcontig) { gr = r0 + vid / 8; gk = k0 + (vid % 8) * 8; }
    else { gk = k0 + vid / (ROWS / 8); gr = r0 + (vid % (ROWS / 8)) * 8; }
    if (kcontig) {
      if (gr < R && gk < K && gr != ones_col) {
        const int64_t off = (int64_t)gr * ld + gk;
        if (gk + 8 <= K) {
          v = *reinterpret_cast<const bf16x8*>(base + off);
          if (mask) {
            const bf16x8 mk = *reinterpret_cast<const bf16x8*>(mask + off);
#pragma unroll
            for (int j = 0; j < 8; ++j) if ((short)mk[j] <= 0) v[j] = 0;  // bf16 sign bit / zero => relu'=0
          }
        } else {
          for (int j = 0; j < 8 && gk + j < K; ++j) {
            unsigned short x = base[off + j];
            if (mask && (short)mask[off + j] <= 0) x = 0;
            v[j] = (short)x;
          }
        }
      }
      if (ones_col >= 0 && gr == ones_col) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (gk + j < K) ? (short)0x3F80 : 0;
      }
    } else {
      if (gk < K && gr < R) {
        const int64_t off = (int64_t)gk * ld + gr;
        if (gr + 8 <= R && ((off & 7) == 0)) {
          v = *reinterpret_cast<const bf16x8*>(base + off);
          if (mask) {
            const bf16x8 mk = *reinterpret_cast<const bf16x8*>(mask + off);
#pragma unroll
            for (int j = 0; j < 8; ++j) if ((short)mk[j] <= 0) v[j] = 0;
          }
        } else {
          for (int j = 0; j < 8 && gr + j < R; ++j) {
            unsigned short x = base[off + j];
            if (mask && (short)mask[off + j] <= 0) x = 0;
            v[j] = (short)x;
          }
        }
      }
      if (ones_col >= 0) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (gr + j == ones_col) v[j] = (gk < K) ? (short)0x3F80 : 0;
      }
    }
    st.v[h] = v;
  }
}

template <int ROWS>
__device__ __forceinline__ void store_tile(const Stage<ROWS>& st, unsigned short* __restrict__ lds, bool kcontig) {
#pragma unroll
  for (int h = 0; h < ROWS / 32; ++h) {
    const int vid = threadIdx.x + 256 * h;
    if (kcontig) {
      *reinterpret_cast<bf16x8*>(lds + (vid / 8) * LDK + (vid % 8) * 8) = st.v[h];
    } else {
      const int kk = vid / (ROWS / 8), rc = (vid % (ROWS / 8)) * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) lds[(rc + j) * LDK + kk] = (unsigned short)st.v[h][j];
    }
  }
}

// Block tile BM x BN, 4 waves laid out WM x WN; each wave owns a 32 x (32*NACC)
// sub-tile = NACC 32x32 MFMA accumulators.  XCD-aware remap: the blocks that
// share an A row-panel are dealt to the same XCD so the panel is served from
// that XCD's L2 for every column tile (MI355X: 8 XCDs with private L2s).
template <int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(256) void k_gemm(GemmArgs g) {
  constexpr int NACC = BN / WN / 32;
  static_assert(BM / WM == 32 && WM * WN == 4, "tile layout");
  __shared__ __attribute__((aligned(16))) unsigned short smem[2 * (BM + BN) * LDK];
  // bijective XCD remap of the (n, m) grid (z = split index untouched)
  const int nx = gridDim.x, ny = gridDim.y;
  const int nwg = nx * ny;
  const int lin = blockIdx.y * nx + blockIdx.x;
  const int q = nwg / 8, rr = nwg % 8, xcd = lin % 8;
  const int wgid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + lin / 8;
  const int bm = wgid / nx, bn = wgid % nx;
  const int m0 = bm * BM, n0 = bn * BN;
  const int kz = blockIdx.z;
  const int kbeg = kz * g.k_per_split;
  const int kend = min(g.K, kbeg + g.k_per_split);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = w / WN, wn = w % WN;
  const int r = lane & 31, hh = lane >> 5;
  f32x16 acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = (f32x16){0};
  const int NB = g.N + (g.ones_col_b >= 0 ? 1 : 0);
  // 1-tile-ahead register prefetch into a 2-deep LDS ring.  (Measured on
  // MI355X: a deeper all-tiles-in-registers variant was 2x slower -- the
  // per-tile guards made hipcc wait vmcnt(0) per load; see
  // profiles/r1_gemm_notes.md.)
  Stage<BM> sa;
  Stage<BN> sb;
  int buf = 0;
  if (kbeg < kend) {
    load_tile<BM>(sa, g.A, g.maskA, g.lda, g.a_kcontig, m0, kbeg, g.M, kend, -1);
    load_tile<BN>(sb, g.B, nullptr, g.ldb, g.b_kcontig, n0, kbeg, g.N, kend, g.ones_col_b);
    store_tile<BM>(sa, smem, g.a_kcontig);
    store_tile<BN>(sb, smem + BM * LDK, g.b_kcontig);
  }
  __syncthreads();
  for (int k0 = kbeg; k0 < kend; k0 += BK) {
    const unsigned short* As = smem + buf * (BM + BN) * LDK;
    const unsigned short* Bs = As + BM * LDK;
    const bool more = k0 + BK < kend;
    if (more) {  // issue the next tile's global loads before this tile's MFMAs
      load_tile<BM>(sa, g.A, g.maskA, g.lda, g.a_kcontig, m0, k0 + BK, g.M, kend, -1);
      load_tile<BN>(sb, g.B, nullptr, g.ldb, g.b_kcontig, n0, k0 + BK, g.N, kend, g.ones_col_b);
    }
#pragma unroll
    for (int ks = 0; ks < BK; ks += 16) {
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(As + (wm * 32 + r) * LDK + ks + 8 * hh);
#pragma unroll
      for (int i = 0; i < NACC; ++i) {
        const bf16x8 b = *reinterpret_cast<const bf16x8*>(Bs + (wn * 32 * NACC + i * 32 + r) * LDK + ks + 8 * hh);
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[i], 0, 0, 0);
      }
    }
    if (more) {
      unsigned short* An = smem + (buf ^ 1) * (BM + BN) * LDK;
      store_tile<BM>(sa, An, g.a_kcontig);
      store_tile<BN>(sb, An + BM * LDK, g.b_kcontig);
    }
    __syncthreads();
    buf ^= 1;
  }
  // epilogue (C/D map: col = lane&31, row = (reg&3) + 8*(reg>>2) + 4*(lane>>5))
#pragma unroll
  for (int i = 0; i < NACC; ++i) {
    const int n = n0 + wn * 32 * NACC + i * 32 + r;
    if (n >= NB) continue;
    const float bias = (g.bias && (g.epi == EPI_BIAS_RELU_BF16 || g.epi == EPI_BIAS_BF16)) ? g.bias[n] : 0.f;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int m = m0 + wm * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * hh;
      if (m >= g.M) continue;
      float v = acc[i][reg] + bias;
      if (g.epi == EPI_F32_SLAB) {
        reinterpret_cast<float*>(g.C)[(int64_t)kz * g.slab_stride + (int64_t)m * g.ldc + n] = v;
      } else {
        if (g.epi == EPI_BIAS_RELU_BF16) v = v > 0.f ? v : 0.f;
        reinterpret_cast<unsigned short*>(g.C)[(int64_t)m * g.ldc + n] = f2bf(v);
      }
    }
  }
}

// Reduce split-K slabs [S][M][ldc] -> dW [M][N] (+ db [M] from column N).
__global__ void k_slab_reduce(const float* __restrict__ slab, int splits, int64_t slab_stride, int M, int N, int ldc,
                              float* __restrict__ dW, float* __restrict__ db, float scale) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int W = N + (db ? 1 : 0);
  if (i >= (int64_t)M * W) return;
  const int m = (int)(i / W), n = (int)(i % W);
  float s = 0.f;
  for (int z = 0; z < splits; ++z) s += slab[z * slab_stride + (int64_t)m * ldc + n];
  s *= scale;
  // accumulate: the parameter grads live in the (per-step zeroed) dense arena
  if (n < N) dW[(int64_t)m * N + n] += s;
  else db[m] += s;
}

// last layer (N_out = 1): out[m] = sum_k h[m,k] w[k] + b
__global__ __launch_bounds__(256) void k_gemv_out(const unsigned short* __restrict__ h, int M, int K, int ldh,
                                                  const float* __restrict__ w, const float* __restrict__ b,
                                                  float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int m = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= M) return;
  float s = 0.f;
  for (int k = lane; k < K; k += 64) s += __uint_as_float(((unsigned)h[(int64_t)m * ldh + k]) << 16) * w[k];
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
  if (lane == 0) out[m] = s + (b ? b[0] : 0.f);
}

// last layer backward: dh[m,k] = dout[m]*w[k] (bf16; the relu' of h is applied
// by the next GEMM's A staging); dw[k] += sum_m dout[m]*h[m,k]; db += sum dout
__global__ __launch_bounds__(256) void k_gemv_out_bwd(const unsigned short* __restrict__ h, int M, int K, int ldh,
                                                      const float* __restrict__ w, const float* __restrict__ dout,
                                                      unsigned short* __restrict__ dh, float* __restrict__ dw_part) {
  // block handles kGemvRows rows x all K; thread -> k column
  const int m0 = blockIdx.x * kGemvRows;
  const int m1 = min(M, m0 + kGemvRows);
  for (int k = threadIdx.x; k < K; k += blockDim.x) {
    const float wk = w[k];
    float acc = 0.f;
    for (int m = m0; m < m1; ++m) {
      const float hv = __uint_as_float(((unsigned)h[(int64_t)m * ldh + k]) << 16);
      const float d = dout[m];
      acc += d * hv;
      dh[(int64_t)m * ldh + k] = f2bf(d * wk);
    }
    // per-block partial (slab row) -- no same-address atomics across blocks
    dw_part[(int64_t)blockIdx.x * (K + 1) + k] = acc;
  }
  if (threadIdx.x < 64) {
    float s = (threadIdx.x < kGemvRows && m0 + (int)threadIdx.x < m1) ? dout[m0 + threadIdx.x] : 0.f;
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
    if (threadIdx.x == 0) dw_part[(int64_t)blockIdx.x * (K + 1) + K] = s;
  }
}


__global__ void k_f32_to_bf16(const float* __restrict__ x, unsigned short* __restrict__ y, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = f2bf(x[i]);
}

inline unsigned int nblk(int64_t n, int per = 256) {
  int64_t b = (n + per - 1) / per;
  return (unsigned int)(b < 1 ? 1 : b);
}

}  // namespace

void launch_gemm(const GemmArgs& g, hipStream_t s) {
  const int NB = g.N + (g.ones_col_b >= 0 ? 1 : 0);
  const int splits = (g.K + g.k_per_split - 1) / g.k_per_split;
  dim3 grid((NB + 63) / 64, (g.M + 63) / 64, splits);
  hipLaunchKernelGGL((k_gemm<64, 64, 2, 2>), grid, dim3(256), 0, s, g);
}

void launch_slab_reduce(const float* slab, int splits, int64_t slab_stride, int M, int N, int ldc, float* dW,
                        float* db, float scale, hipStream_t s) {
  const int64_t n = (int64_t)M * (N + (db ? 1 : 0));
  hipLaunchKernelGGL(k_slab_reduce, dim3(nblk(n)), dim3(256), 0, s, slab, splits, slab_stride, M, N, ldc, dW, db, scale);
}

void launch_gemv_out(const unsigned short* h, int M, int K, int ldh, const float* w, const float* b, float* out,
                     hipStream_t s) {
  hipLaunchKernelGGL(k_gemv_out, dim3((M + 3) / 4), dim3(256), 0, s, h, M, K, ldh, w, b, out);
}

int gemv_out_bwd_blocks(int M) { return (M + kGemvRows - 1) / kGemvRows; }

void launch_gemv_out_bwd(const unsigned short* h, int M, int K, int ldh, const float* w, const float* dout,
                         unsigned short* dh, float* dw, float* db, float* part, hipStream_t s) {
  const int nb = gemv_out_bwd_blocks(M);
  hipLaunchKernelGGL(k_gemv_out_bwd, dim3(nb), dim3(256), 0, s, h, M, K, ldh, w, dout, dh, part);
  launch_colsum_acc(part, nb, K + 1, dw, K, db, s);
}

void launch_f32_to_bf16(const float* x, unsigned short* y, int64_t n, hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(k_f32_to_bf16, dim3(nblk(n)), dim3(256), 0, s, x, y, n);
}

}  // namespace pbx

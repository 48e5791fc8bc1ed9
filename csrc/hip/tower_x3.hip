// Fused CTR dense tower at fp32 precision on the bf16 matrix cores ("x3"):
// every fp32 operand v is carried as two bf16 halves, hi = bf16(v) and
// lo = bf16(v - hi) (16 significant bits together), and every product as three
// bf16 MFMAs -- hi*hi + hi*lo + lo*hi, fp32 accumulation.  The dropped lo*lo
// term and the split residue bound the error of a dot product by ~2^-15 of
// sum |a_k b_k|: finer than TF32 (2^-10 on its 11-bit inputs), which is what
// the reference's fp32 `fc` runs on by default (Blas<float>::GEMM ->
// CublasCall, paddle/phi/kernels/funcs/blas/blas_impl.cu.h:1059, picks the
// CUBLAS_TF32_TENSOR_OP_MATH handle whenever FLAGS_enable_cublas_tf32_op_math
// is set, default true: paddle/phi/backends/gpu/gpu_context.cc:65-67,400-410,580-588).
// gfx950 has no xf32 MFMA; its bf16 MFMA runs 16x the f32 MFMA rate, so three
// of them are ~5x cheaper than one exact-f32 product (tower32.hip).
//
// Same three-launch structure and layouts as the bf16 tower (tower.hip), with
// a lo twin of every bf16 buffer stored right after its hi half:
//   k_tx3_fwd  one 512-thread workgroup per 32-row tile; X0 arrives as fp32
//              rows (the data_norm head's fp32 output) and is split into hi /
//              lo LDS planes plus its m-packed hi / lo copies for the dW;
//              each layer: weight fragments (hi, lo) streamed from L2 into a
//              register ring, 3 MFMAs per k-step into separate accumulators
//              (no dependent MFMA back to back), bias + ReLU in fp32, split
//              again for the next layer; output GEMV on hi + lo, loss tail.
//   k_tx3_bwd  the dX chain the same way; dX0 leaves as fp32 rows.
//   k_tx3_dw   dW = dZ^T X over 64x64 tiles, the hi / lo panels of both
//              operands streamed by LDS-DMA; M split over dw_splits
//              workgroups per tile whose partials the last arriving split sums
//              in split order (bit-reproducible, no fp32 atomics); the bias /
//              data_norm reductions ride along.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "kernels.h"
#include "tower_common.h"

namespace pbx {
namespace {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned short u16;

constexpr int XBM = 32;   // rows per fwd / bwd workgroup
constexpr int XNT = 512;  // threads (8 waves, 2 per SIMD)
constexpr int XNW = XNT / 64;
// weight-ring depth (k-steps, 4 fragments each): forward 3 (0.2435 / 0.2472 vs
// 0.2488 / 0.2512 ms/step at 4, profiles/r6_x3_ring_depth_ab.txt), backward 3 (4
// spills registers there); PBX_X3_PF_F / PBX_X3_PF_B pick 3-5 / 2-3 for A/Bs
constexpr int kX3HeadMaxD = 16;  // fused head backward: embedx dims held per row in LDS
constexpr int kX3PfF = 3;
constexpr int kX3PfB = 3;

__device__ __forceinline__ u16 f2bf(float f) { return __builtin_bit_cast(unsigned short, static_cast<__bf16>(f)); }
__device__ __forceinline__ float bf2f(u16 h) { return __uint_as_float(((unsigned int)h) << 16); }
__device__ __forceinline__ void split2(float v, u16& hi, u16& lo) {
  hi = f2bf(v);
  lo = f2bf(v - bf2f(hi));
}
__device__ __forceinline__ int64_t mp_off(int mb, int NB, int nb, int lane_p) {
  return ((int64_t)(mb * NB + nb) * 64 + lane_p) * 8;
}
__device__ __forceinline__ f32x16 mf(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// h: hi x hi, c: A hi x W lo, d: A lo x W hi; suffix = column block 0 / 1
struct Acc3 {
  f32x16 h0, h1, c0, c1, d0, d1;
};
__device__ __forceinline__ void acc3_zero(Acc3& c) {
  c.h0 = c.h1 = c.c0 = c.c1 = c.d0 = c.d1 = (f32x16){0};
}

// acc += A (32 x 16 KS; hi plane Ah, lo plane Al, row stride ldl) x the
// packed weight fragments w0 / w1 (hi; the lo twin lo_off fragments later).
// Ring of XPF k-steps, each workgroup starting at its own k-step (rot) so the
// CUs of an XCD hit different L2 lines; branch-free steady state.
template <bool TWO, int XPF>
__device__ __forceinline__ void mma3(const u16* __restrict__ Ah, const u16* __restrict__ Al, int ldl,
                                     const bf16x8* __restrict__ w0, const bf16x8* __restrict__ w1, int64_t lo_off,
                                     int KS, int rot, Acc3& c, int lane) {
  const int aoff = (lane & 31) * ldl + 8 * (lane >> 5);
  const u16* ah = Ah + aoff;
  const u16* al = Al + aoff;
  rot = rot % KS;
  const int flast = rot == 0 ? KS - 1 : rot - 1;
  int fi = rot, fc = rot, issued = 0;
  auto adv = [&](int f) { return f + 1 == KS ? 0 : f + 1; };
  bf16x8 qh0[XPF], ql0[XPF], qh1[XPF], ql1[XPF];
#pragma unroll
  for (int p = 0; p < XPF; ++p) {
    const int f = issued < KS ? fi : flast;
    qh0[p] = w0[f * 64];
    ql0[p] = w0[lo_off + f * 64];
    if (TWO) {
      qh1[p] = w1[f * 64];
      ql1[p] = w1[lo_off + f * 64];
    }
    fi = adv(fi);
    ++issued;
  }
  bf16x8 avh = *reinterpret_cast<const bf16x8*>(ah + fc * 16);
  bf16x8 avl = *reinterpret_cast<const bf16x8*>(al + fc * 16);
  const int KM = KS - KS % XPF;
  for (int k0 = 0; k0 < KM; k0 += XPF) {
#pragma unroll
    for (int p = 0; p < XPF; ++p) {
      fc = adv(fc);
      const int fn = k0 + p + 1 < KS ? fc : flast;
      const bf16x8 anh = *reinterpret_cast<const bf16x8*>(ah + fn * 16);
      const bf16x8 anl = *reinterpret_cast<const bf16x8*>(al + fn * 16);
      c.h0 = mf(avh, qh0[p], c.h0);
      if (TWO) c.h1 = mf(avh, qh1[p], c.h1);
      c.c0 = mf(avh, ql0[p], c.c0);
      if (TWO) c.c1 = mf(avh, ql1[p], c.c1);
      c.d0 = mf(avl, qh0[p], c.d0);
      if (TWO) c.d1 = mf(avl, qh1[p], c.d1);
      const int f = issued < KS ? fi : flast;
      qh0[p] = w0[f * 64];
      ql0[p] = w0[lo_off + f * 64];
      if (TWO) {
        qh1[p] = w1[f * 64];
        ql1[p] = w1[lo_off + f * 64];
      }
      fi = adv(fi);
      ++issued;
      avh = anh;
      avl = anl;
    }
  }
#pragma unroll
  for (int p = 0; p < XPF; ++p) {  // tail: KS % XPF steps already in the ring
    if (KM + p < KS) {
      fc = adv(fc);
      const int fn = KM + p + 1 < KS ? fc : flast;
      const bf16x8 anh = *reinterpret_cast<const bf16x8*>(ah + fn * 16);
      const bf16x8 anl = *reinterpret_cast<const bf16x8*>(al + fn * 16);
      c.h0 = mf(avh, qh0[p], c.h0);
      if (TWO) c.h1 = mf(avh, qh1[p], c.h1);
      c.c0 = mf(avh, ql0[p], c.c0);
      if (TWO) c.c1 = mf(avh, ql1[p], c.c1);
      c.d0 = mf(avl, qh0[p], c.d0);
      if (TWO) c.d1 = mf(avl, qh1[p], c.d1);
      avh = anh;
      avl = anl;
    }
  }
}

__device__ __forceinline__ uint2 pk4(const u16 (&o)[4]) {
  return make_uint2((unsigned)o[0] | ((unsigned)o[1] << 16), (unsigned)o[2] | ((unsigned)o[3] << 16));
}

// C layout of a 32x32 accumulator: lane (c = l%32, h = l/32), register r ->
// row 8(r/4) + 4h + r%4, column c (tower.hip fwd_epilogue for the m-packing)
__device__ __forceinline__ void fwd_ep3(const f32x16& h, const f32x16& cc, const f32x16& dd, const TowerLayerDev& ly,
                                        int nb, int m0, u16* dst, int plane, int ldl, int Mp, int lane) {
  const int c = lane & 31, hh = lane >> 5;
  const int n = nb * 32 + c;
  const float bias = n < ly.N ? ly.bias[n] : 0.f;
  const int NB = ly.Np / 32;
  u16* mph = ly.xmp;
  u16* mpl = ly.xmp + (int64_t)Mp * ly.Np;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    u16 oh[4], ol[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      float v = h[q * 4 + t] + (cc[q * 4 + t] + dd[q * 4 + t]) + bias;
      v = v > 0.f ? v : 0.f;
      split2(v, oh[t], ol[t]);
      const int row = 8 * q + 4 * hh + t;
      dst[row * ldl + n] = oh[t];
      dst[plane + row * ldl + n] = ol[t];
    }
    const int64_t off = mp_off(m0 / 16 + (q >> 1), NB, nb, c + 32 * (q & 1)) + 4 * hh;
    *reinterpret_cast<uint2*>(mph + off) = pk4(oh);
    *reinterpret_cast<uint2*>(mpl + off) = pk4(ol);
  }
}

template <int XPF_F>
__global__ __launch_bounds__(XNT) void k_tx3_fwd(TowerArgs a) {
  extern __shared__ __attribute__((aligned(16))) u16 lds[];
  const int ldl = a.lds_ld, plane = XBM * ldl;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int m0 = blockIdx.x * XBM;
  u16* src = lds;              // [hi plane][lo plane]
  u16* dst = lds + 2 * plane;
  const int NL = a.ly[a.L - 1].N;
  TowerRowIn rin{0.f, 0.f, 0.f, 0.f};
  if (w < 2) rin = tower_row_in(a, m0, lane, XBM);
  constexpr int WO = 8;
  float wo[WO];
#pragma unroll
  for (int j = 0; j < WO; ++j) wo[j] = lane + 64 * j < NL ? a.w_out[lane + 64 * j] : 0.f;
  const int K0p = a.ly[0].Kp;
  {  // X0 tile: fp32 rows -> hi / lo planes (zero rows past M)
    const int c4n = K0p / 4;
    for (int i = tid; i < XBM * c4n; i += XNT) {
      const int r = i / c4n, cq = i - r * c4n;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (m0 + r < a.M) v = *reinterpret_cast<const float4*>(a.x0f + (int64_t)(m0 + r) * a.ld0 + cq * 4);
      u16 oh[4], ol[4];
      split2(v.x, oh[0], ol[0]);
      split2(v.y, oh[1], ol[1]);
      split2(v.z, oh[2], ol[2]);
      split2(v.w, oh[3], ol[3]);
      *reinterpret_cast<uint2*>(src + r * ldl + cq * 4) = pk4(oh);
      *reinterpret_cast<uint2*>(src + plane + r * ldl + cq * 4) = pk4(ol);
    }
  }
  __syncthreads();
  {  // X0's m-packed hi / lo copies (the layer-0 dW operand): piece (mb, nb, lp)
     // = rows 16 mb + 8 (lp / 32) + j, j < 8, of column 32 nb + lp % 32
    const int NB0 = K0p / 32;
    u16* mph = const_cast<u16*>(a.x0mp);
    u16* mpl = mph + (int64_t)a.Mp * K0p;
    for (int i = tid; i < 2 * NB0 * 64; i += XNT) {
      const int lp = i & 63, t = i >> 6;
      const int nb = t % NB0, mb = t / NB0;
      const int col = nb * 32 + (lp & 31), r0 = 16 * mb + 8 * (lp >> 5);
      unsigned hw[4], lw[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        hw[j] = (unsigned)src[(r0 + 2 * j) * ldl + col] | ((unsigned)src[(r0 + 2 * j + 1) * ldl + col] << 16);
        lw[j] = (unsigned)src[plane + (r0 + 2 * j) * ldl + col] |
                ((unsigned)src[plane + (r0 + 2 * j + 1) * ldl + col] << 16);
      }
      const int64_t off = mp_off(m0 / 16 + mb, NB0, nb, lp);
      *reinterpret_cast<uint4*>(mph + off) = make_uint4(hw[0], hw[1], hw[2], hw[3]);
      *reinterpret_cast<uint4*>(mpl + off) = make_uint4(lw[0], lw[1], lw[2], lw[3]);
    }
  }
  for (int l = 0; l < a.L; ++l) {
    const TowerLayerDev& ly = a.ly[l];
    const int NB = ly.Np / 32, KS = ly.Kp / 16;
    const bf16x8* wp = reinterpret_cast<const bf16x8*>(ly.wp);
    const int64_t lo_off = (int64_t)ly.Np * ly.Kp / 8;
    for (int nb0 = w; nb0 < NB; nb0 += 2 * XNW) {
      const int nb1 = nb0 + XNW;
      const bool two = nb1 < NB;
      Acc3 c;
      acc3_zero(c);
      const bf16x8* w0p = wp + (int64_t)nb0 * KS * 64 + lane;
      if (two)
        mma3<true, XPF_F>(src, src + plane, ldl, w0p, wp + (int64_t)nb1 * KS * 64 + lane, lo_off, KS, (int)blockIdx.x * a.x3_rot, c,
                   lane);
      else
        mma3<false, XPF_F>(src, src + plane, ldl, w0p, w0p, lo_off, KS, (int)blockIdx.x * a.x3_rot, c, lane);
      fwd_ep3(c.h0, c.c0, c.d0, ly, nb0, m0, dst, plane, ldl, a.Mp, lane);
      if (two) fwd_ep3(c.h1, c.c1, c.d1, ly, nb1, m0, dst, plane, ldl, a.Mp, lane);
    }
    __syncthreads();
    u16* t = src;
    src = dst;
    dst = t;
  }
  // output layer on hi + lo: 4 rows per wave, w_out from registers
  __shared__ float zrow[XBM];
  {
    constexpr int RPW = XBM / XNW;
    float s[RPW];
#pragma unroll
    for (int rr = 0; rr < RPW; ++rr) s[rr] = 0.f;
#pragma unroll
    for (int j = 0; j < WO; ++j) {
      const int k = lane + 64 * j;
      if (k < NL) {
#pragma unroll
        for (int rr = 0; rr < RPW; ++rr) {
          const int o = (w * RPW + rr) * ldl + k;
          s[rr] += (bf2f(src[o]) + bf2f(src[plane + o])) * wo[j];
        }
      }
    }
    for (int k = lane + 64 * WO; k < NL; k += 64) {
#pragma unroll
      for (int rr = 0; rr < RPW; ++rr) {
        const int o = (w * RPW + rr) * ldl + k;
        s[rr] += (bf2f(src[o]) + bf2f(src[plane + o])) * a.w_out[k];
      }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1)
#pragma unroll
      for (int rr = 0; rr < RPW; ++rr) s[rr] += __shfl_xor(s[rr], off);
    if (lane < RPW) {
      float mine = s[0];
#pragma unroll
      for (int rr = 1; rr < RPW; ++rr) mine = lane == rr ? s[rr] : mine;
      zrow[w * RPW + lane] = mine;
    }
  }
  __syncthreads();
  tower_loss_tail(a, zrow, rin, m0, w, lane, XBM);
}

// relu' masks of the previous layer's output at the accumulator positions
// (hi half: a positive fp32 value never rounds to a zero bf16)
struct Mask3 {
  uint2 v[4];
};
__device__ __forceinline__ Mask3 bwd_mask3(const TowerLayerDev& prev, int kb, int m0, int lane) {
  const int c = lane & 31, h = lane >> 5;
  const int NB = prev.Np / 32;
  Mask3 mk;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    mk.v[q] = *reinterpret_cast<const uint2*>(prev.xmp + mp_off(m0 / 16 + (q >> 1), NB, kb, c + 32 * (q & 1)) + 4 * h);
  return mk;
}

__device__ __forceinline__ void bwd_ep3(const f32x16& hacc, const f32x16& cc, const f32x16& dd,
                                        const TowerLayerDev& prev, const Mask3& mk, int kb, int m0, u16* dst,
                                        int plane, int ldl, int Mp, float* bp, int lane) {
  const int c = lane & 31, h = lane >> 5;
  const int NB = prev.Np / 32;
  u16* dzh = prev.dzmp;
  u16* dzl = prev.dzmp + (int64_t)Mp * prev.Np;
  float cs = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int64_t off = mp_off(m0 / 16 + (q >> 1), NB, kb, c + 32 * (q & 1)) + 4 * h;
    const uint2 xm = mk.v[q];
    const u16 xs[4] = {(u16)(xm.x & 0xffff), (u16)(xm.x >> 16), (u16)(xm.y & 0xffff), (u16)(xm.y >> 16)};
    u16 oh[4], ol[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      float v = hacc[q * 4 + t] + (cc[q * 4 + t] + dd[q * 4 + t]);
      if (!(bf2f(xs[t]) > 0.f)) v = 0.f;
      split2(v, oh[t], ol[t]);
      cs += v;
      const int row = 8 * q + 4 * h + t;
      dst[row * ldl + kb * 32 + c] = oh[t];
      dst[plane + row * ldl + kb * 32 + c] = ol[t];
    }
    *reinterpret_cast<uint2*>(dzh + off) = pk4(oh);
    *reinterpret_cast<uint2*>(dzl + off) = pk4(ol);
  }
  cs += __shfl_xor(cs, 32);
  if (h == 0) bp[prev.bias_off + kb * 32 + c] = cs;
}

template <int XPF_B>
__global__ __launch_bounds__(XNT) void k_tx3_bwd(TowerArgs a) {
  extern __shared__ __attribute__((aligned(16))) u16 lds[];
  __shared__ float gs[XBM];
  const int ldl = a.lds_ld, plane = XBM * ldl;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int m0 = blockIdx.x * XBM;
  u16* src = lds;
  u16* dst = lds + 2 * plane;
  __shared__ float s1s[XBM * kX3HeadMaxD];  // fused head: per-row FM sums over the slots
  float* bp = a.bias_part + (int64_t)blockIdx.x * a.bias_ld;
  const float gl = a.dloss ? a.dloss[0] : 1.f;
  if (tid < XBM) gs[tid] = (m0 + tid < a.M) ? a.dz[m0 + tid] * gl : 0.f;
  if (a.hdx && a.hlin) {
    for (int i = tid; i < XBM * a.hD; i += XNT) {
      const int r = i / a.hD, d = i - r * a.hD;
      float s1 = 0.f;
      if (m0 + r < a.M) {
        const float* xr = a.hx + (int64_t)(m0 + r) * a.hC + a.hew + 1 + d;
        for (int sl = 0; sl < a.hS; ++sl) s1 += xr[sl * a.hEo];
      }
      s1s[r * kX3HeadMaxD + d] = s1;
    }
  }
  __syncthreads();
  // dZ_L = (g w_out^T) . relu'(X_L), X_L = hi + lo from its m-packed halves
  const TowerLayerDev& lastl = a.ly[a.L - 1];
  {
    const int NpL = lastl.Np, NL = lastl.N, NBL = NpL / 32;
    const int64_t lo = (int64_t)a.Mp * NpL;
    for (int k = tid; k < NpL; k += XNT) {
      const float wk = k < NL ? a.w_out[k] : 0.f;
      const int nb = k / 32, c = k % 32;
      float dbs = 0.f, dws = 0.f;
#pragma unroll
      for (int mb = 0; mb < 2; ++mb) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int64_t off = mp_off(m0 / 16 + mb, NBL, nb, c + 32 * h);
          const uint4 xh = *reinterpret_cast<const uint4*>(lastl.xmp + off);
          const uint4 xl = *reinterpret_cast<const uint4*>(lastl.xmp + lo + off);
          const unsigned int hw[4] = {xh.x, xh.y, xh.z, xh.w}, lw[4] = {xl.x, xl.y, xl.z, xl.w};
          unsigned int oh[4], ol[4];
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            u16 h2[2], l2[2];
#pragma unroll
            for (int e = 0; e < 2; ++e) {
              const int r = 16 * mb + 8 * h + jj * 2 + e;
              const float x = bf2f((u16)((hw[jj] >> (16 * e)) & 0xffff)) + bf2f((u16)((lw[jj] >> (16 * e)) & 0xffff));
              const float g = gs[r];
              const float d = x > 0.f ? g * wk : 0.f;
              split2(d, h2[e], l2[e]);
              dbs += d;
              dws += g * x;
              src[r * ldl + k] = h2[e];
              src[plane + r * ldl + k] = l2[e];
            }
            oh[jj] = (unsigned)h2[0] | ((unsigned)h2[1] << 16);
            ol[jj] = (unsigned)l2[0] | ((unsigned)l2[1] << 16);
          }
          *reinterpret_cast<uint4*>(lastl.dzmp + off) = make_uint4(oh[0], oh[1], oh[2], oh[3]);
          *reinterpret_cast<uint4*>(lastl.dzmp + lo + off) = make_uint4(ol[0], ol[1], ol[2], ol[3]);
        }
      }
      bp[lastl.bias_off + k] = dbs;
      if (k < NL) bp[a.dwout_off + k] = dws;
    }
    if (tid == 0) {
      float s = 0.f;
      for (int r = 0; r < XBM; ++r) s += gs[r];
      bp[a.dbout_off] = s;
    }
  }
  __syncthreads();
  // dX_i = dZ_{i+1} W_i (i = L-1 .. 0); dZ_i = dX_i . relu'(X_i) for i >= 1;
  // dX_0 straight to the fp32 rows
  for (int i = a.L - 1; i >= 0; --i) {
    if (i == 0 && !a.need_dx0) break;
    const TowerLayerDev& ly = a.ly[i];
    const int KB = ly.Kp / 32, NS = ly.Np / 16;
    const bf16x8* wtp = reinterpret_cast<const bf16x8*>(ly.wtp);
    const int64_t lo_off = (int64_t)ly.Np * ly.Kp / 8;
    for (int kb0 = w; kb0 < KB; kb0 += 2 * XNW) {
      const int kb1 = kb0 + XNW;
      const bool two = kb1 < KB;
      Acc3 c;
      acc3_zero(c);
      const bf16x8* w0p = wtp + (int64_t)kb0 * NS * 64 + lane;
      if (two)
        mma3<true, XPF_B>(src, src + plane, ldl, w0p, wtp + (int64_t)kb1 * NS * 64 + lane, lo_off, NS, (int)blockIdx.x * a.x3_rot,
                   c, lane);
      else
        mma3<false, XPF_B>(src, src + plane, ldl, w0p, w0p, lo_off, NS, (int)blockIdx.x * a.x3_rot, c, lane);
      if (i > 0) {
        // relu' masks loaded after the MMAs (before them they cost the ring
        // registers a spill)
        Mask3 mk0, mk1;
        mk0 = bwd_mask3(a.ly[i - 1], kb0, m0, lane);
        if (two) mk1 = bwd_mask3(a.ly[i - 1], kb1, m0, lane);
        bwd_ep3(c.h0, c.c0, c.d0, a.ly[i - 1], mk0, kb0, m0, dst, plane, ldl, a.Mp, bp, lane);
        if (two) bwd_ep3(c.h1, c.c1, c.d1, a.ly[i - 1], mk1, kb1, m0, dst, plane, ldl, a.Mp, bp, lane);
      } else {  // dX0 as fp32 rows into the free tile (its 2 planes = 32 x ldl floats)
        float* t32 = reinterpret_cast<float*>(dst);
        const int cl = lane & 31, h = lane >> 5;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = 8 * (r >> 2) + 4 * h + (r & 3);
          t32[row * ldl + kb0 * 32 + cl] = c.h0[r] + (c.c0[r] + c.d0[r]);
          if (two) t32[row * ldl + kb1 * 32 + cl] = c.h1[r] + (c.c1[r] + c.d1[r]);
        }
      }
    }
    __syncthreads();
    u16* t = src;
    src = dst;
    dst = t;
  }
  if (a.need_dx0 && !a.hdx) {  // dX0 tile -> fp32 rows, 16-B stores
    const float* t32 = reinterpret_cast<const float*>(src);
    const int c4n = a.ly[0].Kp / 4;
    for (int i = tid; i < XBM * c4n; i += XNT) {
      const int r = i / c4n, cq = i - r * c4n;
      if (m0 + r < a.M)
        *reinterpret_cast<float4*>(a.dx0f + (int64_t)(m0 + r) * a.lddx0 + cq * 4) =
            *reinterpret_cast<const float4*>(t32 + r * ldl + cq * 4);
    }
  }
  if (a.hdx && a.need_dx0) {
    // the DeepFM head backward (head_ops.hip k_head_bwd semantics) on the
    // dX0 tile: dx = dX0 * scale (data_norm), plus on the sparse slots'
    // columns the d lin terms (d lin = dz * dloss = gs[row]): embed_w gets
    // d lin, embedx dim d gets d lin * (sum over slots of embedx d - x).
    // Saves the head launch and the dX0 round trip on the critical path.
    const float* t32 = reinterpret_cast<const float*>(src);
    const int C = a.hC;
    for (int i = tid; i < XBM * C; i += XNT) {
      const int r = i / C, col = i - r * C;
      const int m = m0 + r;
      if (m >= a.M) break;  // rows are walked in order
      float g = t32[r * ldl + col] * (a.hscales ? a.hscales[col] : 1.f);
      if (a.hlin && col < a.hS * a.hEo) {
        const int j = col % a.hEo;
        if (j == a.hew) g += gs[r];
        else if (j > a.hew && j <= a.hew + a.hD)
          g += gs[r] * (s1s[r * kX3HeadMaxD + (j - a.hew - 1)] - a.hx[(int64_t)m * C + col]);
      }
      a.hdx[(int64_t)m * C + col] = g;
    }
  }
}

// ---------------------------------------------------------------- dW
constexpr int X3_STEPS = 2;                     // m16 steps per ring stage
constexpr int X3_NST = 4;                       // ring stages
constexpr int X3_STAGE = X3_STEPS * 8 * 512;    // u16 per stage: 8 x 1 KB fragments per step

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__global__ __launch_bounds__(256) void k_tx3_dw(TowerArgs a, int ndw) {
  const int tid = threadIdx.x;
  if ((int)blockIdx.x >= ndw) {
    tower_col_reduce(a, (int)blockIdx.x - ndw, XBM);
    return;
  }
  __shared__ __attribute__((aligned(16))) u16 smem[X3_NST * X3_STAGE];
  // work id -> (tile, split): the splits of one tile are consecutive ids
  const int S = a.dw_splits;
  const int wid = xcd_work_id((int)blockIdx.x, ndw);
  const int split = wid % S;
  const int tile_g = wid / S;
  int t = tile_g;
  int l = 0;
  for (; l < a.L; ++l) {
    const int nt = ((a.ly[l].Np + 63) / 64) * ((a.ly[l].Kp + 63) / 64);
    if (t < nt) break;
    t -= nt;
  }
  const TowerLayerDev& ly = a.ly[l];
  const int NBn = ly.Np / 32, NBk = ly.Kp / 32;
  const int tk_n = (ly.Kp + 63) / 64;
  const int tn = t / tk_n, tk = t % tk_n;
  const u16* Amp = ly.dzmp;                             // dZ_{l+1}: [Mp/16][NBn] pieces, lo after Mp Np
  const u16* Bmp = l == 0 ? a.x0mp : a.ly[l - 1].xmp;   // X_l:      [Mp/16][NBk] pieces, lo after Mp Kp
  const int lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  // this wave's DMA: block w (0,1: dZ n-blocks; 2,3: X k-blocks), hi and lo
  const u16* gsrc;
  int64_t glo;
  int gstride;
  if (w < 2) {
    const int nb = min(tn * 2 + w, NBn - 1);
    gsrc = Amp + ((int64_t)nb * 64 + lane) * 8;
    glo = (int64_t)a.Mp * ly.Np;
    gstride = NBn * 512;
  } else {
    const int kb = min(tk * 2 + (w - 2), NBk - 1);
    gsrc = Bmp + ((int64_t)kb * 64 + lane) * 8;
    glo = (int64_t)a.Mp * ly.Kp;
    gstride = NBk * 512;
  }
  const int per = a.Mp / 16 / S;  // m16 steps of this split (a multiple of X3_STEPS: Mp % 128 == 0, S <= 4)
  const int mb0 = split * per;
  const int nstage = per / X3_STEPS;
  const unsigned lds0 = __builtin_amdgcn_readfirstlane(tower_lds_addr(smem));
  auto issue = [&](int slot, int stage) {
    const unsigned base = lds0 + (unsigned)(slot * X3_STAGE) * 2u;
#pragma unroll
    for (int st = 0; st < X3_STEPS; ++st) {
      const int64_t mb = (int64_t)(mb0 + stage * X3_STEPS + st) * gstride;
      tower_glds16(gsrc + mb, __builtin_amdgcn_readfirstlane(base + st * 8192u + (unsigned)w * 1024u));
      tower_glds16(gsrc + glo + mb, __builtin_amdgcn_readfirstlane(base + st * 8192u + (unsigned)(4 + w) * 1024u));
    }
  };
  const int wn = w & 1, wk = w >> 1;
  f32x16 acc = (f32x16){0}, accc = (f32x16){0}, accd = (f32x16){0};
  for (int p = 0; p < X3_NST - 1 && p < nstage; ++p) issue(p, p);
  for (int s = 0; s < nstage; ++s) {
    const int ahead = min(X3_NST - 2, nstage - 1 - s);
    if (ahead >= 2) wait_vm<4 * X3_STEPS>();
    else if (ahead == 1) wait_vm<2 * X3_STEPS>();
    else wait_vm<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (s + X3_NST - 1 < nstage) issue((s + X3_NST - 1) % X3_NST, s + X3_NST - 1);
    const u16* base = smem + (s % X3_NST) * X3_STAGE;
#pragma unroll
    for (int st = 0; st < X3_STEPS; ++st) {
      const u16* b = base + st * 4096 + lane * 8;
      const bf16x8 ah = *reinterpret_cast<const bf16x8*>(b + wn * 512);
      const bf16x8 al = *reinterpret_cast<const bf16x8*>(b + (4 + wn) * 512);
      const bf16x8 bh = *reinterpret_cast<const bf16x8*>(b + (2 + wk) * 512);
      const bf16x8 bl = *reinterpret_cast<const bf16x8*>(b + (6 + wk) * 512);
      acc = mf(ah, bh, acc);
      accc = mf(ah, bl, accc);
      accd = mf(al, bh, accd);
    }
  }
  const int nb = tn * 2 + wn, kb = tk * 2 + wk;
  const int c = lane & 31, h = lane >> 5;
  const int k = kb * 32 + c;
  const bool active = nb < NBn && kb < NBk && k < ly.K;
  f32x16 v;
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = acc[r] + (accc[r] + accd[r]);
  auto add_out = [&](const f32x16& x) {  // grads accumulate (+=); one writer per element
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int n = nb * 32 + 8 * (r >> 2) + 4 * h + (r & 3);
      if (n < ly.N) ly.dw[(int64_t)n * ly.K + k] += x[r];
    }
  };
  if (S == 1) {
    if (active) add_out(v);
    return;
  }
  // split-M partials: every split stores its 64x64 partial (a slab,
  // write-through sc1 stores), the tile's last arriving split sums the slabs
  // in split order -- bit-reproducible, no fp32 atomics (the tower32.hip
  // t32_dw_combine hand-off: counter after the drained stores, acquire in
  // the reducer)
  float* tile_slab = a.dw_slab + (int64_t)tile_g * S * 4096;
  {
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(tile_slab + (int64_t)split * 4096, 0, 4096 * 4, 0x00020000);
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 f = active ? make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3])
                              : make_float4(0.f, 0.f, 0.f, 0.f);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, f), rs, ((w * 4 + q) * 64 + lane) * 16, 0,
                                             16 /* sc1 */);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int* flag = reinterpret_cast<int*>(smem);  // the ring is drained: reuse its first word
  if (tid == 0) {
    const int old = __hip_atomic_fetch_add(&a.dw_cnt[tile_g], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == S - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(&a.dw_cnt[tile_g], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch from 0
    }
    *flag = last;
  }
  __syncthreads();
  if (!*flag || !active) return;
  f32x16 sum = (f32x16){0};
  const float4* base = reinterpret_cast<const float4*>(tile_slab) + w * 4 * 64 + lane;
  for (int sp = 0; sp < S; ++sp) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 f = base[(int64_t)sp * 1024 + q * 64];
      sum[4 * q] += f.x;
      sum[4 * q + 1] += f.y;
      sum[4 * q + 2] += f.z;
      sum[4 * q + 3] += f.w;
    }
  }
  add_out(sum);
}

// ---------------------------------------------------------------- packing
__device__ __forceinline__ int64_t wp_idx(int n, int k, int Kp) {
  return ((int64_t)((n >> 5) * (Kp >> 4) + (k >> 4)) * 64 + (n & 31) + 32 * ((k >> 3) & 1)) * 8 + (k & 7);
}
__device__ __forceinline__ int64_t wtp_idx(int n, int k, int Np) {
  return ((int64_t)((k >> 5) * (Np >> 4) + (n >> 4)) * 64 + (k & 31) + 32 * ((n >> 3) & 1)) * 8 + (n & 7);
}

struct X3PackJob {
  const float* w[kMaxTowerLayers];
  int64_t off[kMaxTowerLayers + 1];
};

__global__ void k_tx3_pack(TowerArgs a, X3PackJob j) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= j.off[a.L]) return;
  int l = 0;
  while (e >= j.off[l + 1]) ++l;
  const TowerLayerDev& ly = a.ly[l];
  const int64_t i = e - j.off[l];
  const int n = (int)(i / ly.K), k = (int)(i % ly.K);
  u16 hi, lo;
  split2(j.w[l][i], hi, lo);
  const int64_t lo_off = (int64_t)ly.Np * ly.Kp;
  u16* wp = const_cast<u16*>(ly.wp);
  u16* wtp = const_cast<u16*>(ly.wtp);
  const int64_t pi = wp_idx(n, k, ly.Kp), ti = wtp_idx(n, k, ly.Np);
  wp[pi] = hi;
  wp[lo_off + pi] = lo;
  wtp[ti] = hi;
  wtp[lo_off + ti] = lo;
}

template <typename K>
void x3_big_lds_one(K f) {
  if (hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024) != hipSuccess)
    (void)hipGetLastError();
}
void x3_big_lds() {
  static const bool once = [] {
    x3_big_lds_one(k_tx3_fwd<3>);
    x3_big_lds_one(k_tx3_fwd<4>);
    x3_big_lds_one(k_tx3_fwd<5>);
    x3_big_lds_one(k_tx3_bwd<2>);
    x3_big_lds_one(k_tx3_bwd<3>);
    return true;
  }();
  (void)once;
}
int x3_env(const char* n, int d) {
  const char* e = getenv(n);
  return e ? atoi(e) : d;
}

}  // namespace

size_t tower_x3_lds_bytes(int lds_ld) { return (size_t)4 * XBM * lds_ld * sizeof(u16); }

// PBX_X3_ROT: the per-workgroup k-step rotation multiplier (A/B knob)
static TowerArgs x3_args(const TowerArgs& a0) {
  static const int rot = x3_env("PBX_X3_ROT", 5);
  TowerArgs a = a0;
  a.x3_rot = rot > 0 ? rot : 5;
  return a;
}

void launch_tower_x3_fwd(const TowerArgs& a0, hipStream_t s) {
  if (a0.M == 0) return;
  const TowerArgs a = x3_args(a0);
  x3_big_lds();
  static const int pf = x3_env("PBX_X3_PF_F", kX3PfF);
  const dim3 g(a.Mp / XBM);
  const size_t lb = tower_x3_lds_bytes(a.lds_ld);
  if (pf == 3) hipLaunchKernelGGL(k_tx3_fwd<3>, g, dim3(XNT), lb, s, a);
  else if (pf == 5) hipLaunchKernelGGL(k_tx3_fwd<5>, g, dim3(XNT), lb, s, a);
  else hipLaunchKernelGGL(k_tx3_fwd<4>, g, dim3(XNT), lb, s, a);
}

void launch_tower_x3_bwd(const TowerArgs& a0, hipStream_t s) {
  if (a0.M == 0) return;
  const TowerArgs a = x3_args(a0);
  x3_big_lds();
  static const int pf = x3_env("PBX_X3_PF_B", kX3PfB);
  if (pf == 2) hipLaunchKernelGGL(k_tx3_bwd<2>, dim3(a.Mp / XBM), dim3(XNT), tower_x3_lds_bytes(a.lds_ld), s, a);
  else hipLaunchKernelGGL(k_tx3_bwd<3>, dim3(a.Mp / XBM), dim3(XNT), tower_x3_lds_bytes(a.lds_ld), s, a);
}

void launch_tower_x3_dw(const TowerArgs& a, hipStream_t s) {
  if (a.M == 0) return;
  int tiles = 0;
  for (int l = 0; l < a.L; ++l) tiles += ((a.ly[l].Np + 63) / 64) * ((a.ly[l].Kp + 63) / 64);
  const int nred = (a.bias_ld + 31) / 32 + (a.dn_part ? (a.dn_C + 31) / 32 : 0);
  hipLaunchKernelGGL(k_tx3_dw, dim3(tiles * a.dw_splits + nred), dim3(256), 0, s, a, tiles * a.dw_splits);
}

void launch_tower_x3_pack(const TowerArgs& a, const float* const* w, hipStream_t s) {
  X3PackJob j;
  j.off[0] = 0;
  for (int l = 0; l < a.L; ++l) {
    j.w[l] = w[l];
    j.off[l + 1] = j.off[l] + (int64_t)a.ly[l].N * a.ly[l].K;
  }
  const int64_t n = j.off[a.L];
  if (n == 0) return;
  hipLaunchKernelGGL(k_tx3_pack, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a, j);
}

}  // namespace pbx

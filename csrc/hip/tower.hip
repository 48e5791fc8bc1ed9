// Fused CTR dense tower on MI355X: the MLP of DeepFM / Wide&Deep / DCN heads
// (ReLU layers of a few hundred units, one logit), its loss and its backward
// as three launches instead of ~20.
//
//   k_tower_fwd  one 512-thread workgroup per 32-row tile.  The tile's
//                activations stay in LDS across all layers; each wave streams
//                pre-packed bf16 weight fragments (1 KB, fully coalesced)
//                from L2 into registers and runs v_mfma_f32_32x32x16_bf16.
//                Epilogue: bias + ReLU -> LDS (next layer's A operand) and the
//                m-packed copy for the dW GEMM.  The output GEMV, sigmoid,
//                log-loss, d loss/d logit and the AUC histogram are fused at
//                the end; the mean loss is reduced by the last workgroup.
//   k_tower_bwd  same tiling, backward chain dZ_L .. dZ_1 -> dX0 (ReLU masks
//                read from the m-packed activations), per-tile column sums
//                for the bias / output-layer gradients.
//   k_tower_dw   every layer's dW = dZ^T X as one grouped GEMM over 64x64
//                output tiles, both operands streamed HBM/L2 -> LDS by
//                global_load_lds (1 KB fragments), split over M in two with
//                fp32 atomics; extra workgroups reduce the bias partials and
//                the data_norm batch statistics.
//
// Replaces the per-layer GEMMs of mlp.hip (profiles/r2_v0_step_kernels.txt:
// 13 launches, ~160 us/step at M = 8192, 3 x 400 units).  Reference op
// semantics: fc/relu (paddle/phi/kernels/gpu/matmul_kernel.cu), log_loss +
// sigmoid (phi/kernels/gpu/log_loss_kernel.cu), auc (phi/kernels/gpu/auc_kernel.cu:25-80).
#include <hip/hip_runtime.h>

#include "kernels.h"
#include "tower_common.h"

namespace pbx {
namespace {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef const __attribute__((address_space(1))) void* gbl_ptr_t;
typedef unsigned short u16;

constexpr int TBM = 32;   // rows per workgroup (fwd / bwd)
constexpr int TNT = 512;  // threads per workgroup (8 waves, 2 per SIMD)
constexpr int TNW = TNT / 64;
constexpr int PF = 6;     // default weight-fragment prefetch depth (k-steps; PBX_TOWER_PF picks 4 / 6 / 8;
                          // same-box A/B 0.2515-0.2528 ms/step at 6 vs 0.2543-0.2660 at 8)
constexpr int kMpAlign = 128;

__device__ __forceinline__ u16 f2bf(float f) {
  // v_cvt_pk_bf16_f32 (gfx950): round-to-nearest-even in one instruction per
  // pair -- the same bits as the integer rounding (u + 0x7fff + lsb) >> 16
  // for every finite input, at a quarter of the VALU work
  return __builtin_bit_cast(unsigned short, static_cast<__bf16>(f));
}
__device__ __forceinline__ float bf2f(u16 h) { return __uint_as_float(((unsigned int)h) << 16); }

// acc{0,1} += A(32 x 16*KS, LDS rows of stride ldl starting at As) x
// B fragments w{0,1}[k*64] (k = 0..KS-1).  Weight fragments are prefetched PF
// k-steps ahead into registers; the A fragment is shared by both products.
// Every workgroup reads the same weight fragments, so each one walks the
// k-steps from its own starting point (rot): at any moment the 32 CUs of an
// XCD hit different L2 lines instead of queueing on one.
// The steady-state loop is branch-free (prefetch addresses are clamped, TWO
// is a template parameter) so hipcc keeps counted vmcnt waits across the
// ring instead of draining it every step.
template <bool TWO, int PF>
__device__ __forceinline__ void mma_pair(const u16* __restrict__ As, int ldl, const bf16x8* __restrict__ w0,
                                         const bf16x8* __restrict__ w1, int KS, int rot, f32x16& acc0,
                                         f32x16& acc1, int lane) {
  const u16* arow = As + (lane & 31) * ldl + 8 * (lane >> 5);
  rot = rot % KS;
  const int flast = rot == 0 ? KS - 1 : rot - 1;  // fragment of the last step
  // fi: fragment of the next load to issue; fc: fragment of the next step to compute
  int fi = rot, fc = rot, issued = 0;
  auto adv = [&](int f) { return f + 1 == KS ? 0 : f + 1; };
  bf16x8 q0[PF], q1[PF];
#pragma unroll
  for (int p = 0; p < PF; ++p) {
    const int f = issued < KS ? fi : flast;
    q0[p] = w0[f * 64];
    if (TWO) q1[p] = w1[f * 64];
    fi = adv(fi);
    ++issued;
  }
  bf16x8 av = *reinterpret_cast<const bf16x8*>(arow + fc * 16);
  const int KM = KS - KS % PF;
  for (int k0 = 0; k0 < KM; k0 += PF) {
#pragma unroll
    for (int p = 0; p < PF; ++p) {
      fc = adv(fc);
      // next step's A fragment (clamped on the last step) is read ahead of the MFMAs
      const bf16x8 an = *reinterpret_cast<const bf16x8*>(arow + (k0 + p + 1 < KS ? fc : flast) * 16);
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, q0[p], acc0, 0, 0, 0);
      if (TWO) acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, q1[p], acc1, 0, 0, 0);
      const int f = issued < KS ? fi : flast;
      q0[p] = w0[f * 64];
      if (TWO) q1[p] = w1[f * 64];
      fi = adv(fi);
      ++issued;
      av = an;
    }
  }
#pragma unroll
  for (int p = 0; p < PF; ++p) {  // tail: KS % PF steps already in the ring
    if (KM + p < KS) {
      fc = adv(fc);
      const bf16x8 an = *reinterpret_cast<const bf16x8*>(arow + (KM + p + 1 < KS ? fc : flast) * 16);
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, q0[p], acc0, 0, 0, 0);
      if (TWO) acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, q1[p], acc1, 0, 0, 0);
      av = an;
    }
  }
}

// C layout of a 32x32 accumulator: lane (c = l%32, h = l/32), register r ->
// row 8(r/4) + 4h + r%4, column c.  For the m-packed copy the 4 registers of
// group q form one 8-byte piece at chunk row q/2, lane' c + 32(q%2), j 4h..4h+3:
// the wave's 64 pieces of one q are 512 contiguous bytes.
__device__ __forceinline__ int64_t mp_off(int mb, int NB, int nb, int lane_p) {
  return ((int64_t)(mb * NB + nb) * 64 + lane_p) * 8;
}

__device__ __forceinline__ void fwd_epilogue(const f32x16& acc, const TowerLayerDev& ly, int nb, int m0, u16* dst,
                                             int ldl, int lane, bool mp = true) {
  const int c = lane & 31, h = lane >> 5;
  const int n = nb * 32 + c;
  const float bias = n < ly.N ? ly.bias[n] : 0.f;
  const int NB = ly.Np / 32;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    u16 o[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      float v = acc[q * 4 + t] + bias;
      v = v > 0.f ? v : 0.f;
      o[t] = f2bf(v);
      dst[(8 * q + 4 * h + t) * ldl + n] = o[t];
    }
    uint2 pk;
    pk.x = (unsigned)o[0] | ((unsigned)o[1] << 16);
    pk.y = (unsigned)o[2] | ((unsigned)o[3] << 16);
    if (mp) *reinterpret_cast<uint2*>(ly.xmp + mp_off(m0 / 16 + (q >> 1), NB, nb, c + 32 * (q & 1)) + 4 * h) = pk;
  }
}

template <int PFv>
__global__ __launch_bounds__(TNT) void k_tower_fwd(TowerArgs a) {
  extern __shared__ __attribute__((aligned(16))) u16 lds[];
  const int ldl = a.lds_ld;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int m0 = blockIdx.x * TBM;
  u16* src = lds;
  u16* dst = lds + TBM * ldl;
  // loss-tail inputs and the output-layer weights, loaded ahead of the layers
  const int NL = a.ly[a.L - 1].N;
  TowerRowIn rin{0.f, 0.f, 0.f, 0.f};
  if (w < 2) rin = tower_row_in(a, m0, lane, TBM);
  constexpr int WO = 8;
  float wo[WO];
#pragma unroll
  for (int j = 0; j < WO; ++j) wo[j] = lane + 64 * j < NL ? a.w_out[lane + 64 * j] : 0.f;
  {  // stage the X0 tile (row-major, zero rows past M)
    const int c8n = a.ly[0].Kp / 8;
    for (int i = tid; i < TBM * c8n; i += TNT) {
      const int r = i / c8n, c = i - r * c8n;
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (m0 + r < a.M) v = *reinterpret_cast<const uint4*>(a.x0 + (int64_t)(m0 + r) * a.ld0 + c * 8);
      *reinterpret_cast<uint4*>(src + r * ldl + c * 8) = v;
    }
  }
  __syncthreads();
  for (int l = 0; l < a.L; ++l) {
    const TowerLayerDev& ly = a.ly[l];
    const int NB = ly.Np / 32, KS = ly.Kp / 16;
    const bf16x8* wp = reinterpret_cast<const bf16x8*>(ly.wp);
    for (int nb0 = w; nb0 < NB; nb0 += 2 * TNW) {
      const int nb1 = nb0 + TNW;
      const bool two = nb1 < NB;
      f32x16 acc0 = (f32x16){0}, acc1 = (f32x16){0};
      const bf16x8* w0p = wp + (int64_t)nb0 * KS * 64 + lane;
      if (two) mma_pair<true, PFv>(src, ldl, w0p, wp + (int64_t)nb1 * KS * 64 + lane, KS, (int)blockIdx.x * 5, acc0, acc1, lane);
      else mma_pair<false, PFv>(src, ldl, w0p, w0p, KS, (int)blockIdx.x * 5, acc0, acc1, lane);
      const bool mp = !(a.debug & 8);
      fwd_epilogue(acc0, ly, nb0, m0, dst, ldl, lane, mp);
      if (two) fwd_epilogue(acc1, ly, nb1, m0, dst, ldl, lane, mp);
    }
    __syncthreads();
    u16* t = src;
    src = dst;
    dst = t;
  }
  if (a.debug & 16) return;
  // output layer: 4 rows per wave, independent accumulations, w_out from
  // registers; the logits meet in LDS for the loss tail
  __shared__ float zrow[TBM];
  {
    constexpr int RPW = TBM / TNW;
    float s[RPW];
#pragma unroll
    for (int rr = 0; rr < RPW; ++rr) s[rr] = 0.f;
#pragma unroll
    for (int j = 0; j < WO; ++j) {
      const int k = lane + 64 * j;
      if (k < NL) {
#pragma unroll
        for (int rr = 0; rr < RPW; ++rr) s[rr] += bf2f(src[(w * RPW + rr) * ldl + k]) * wo[j];
      }
    }
    for (int k = lane + 64 * WO; k < NL; k += 64) {  // widths past 512
#pragma unroll
      for (int rr = 0; rr < RPW; ++rr) s[rr] += bf2f(src[(w * RPW + rr) * ldl + k]) * a.w_out[k];
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
  tower_loss_tail(a, zrow, rin, m0, w, lane, TBM);
}

// dZ epilogue of the backward chain for output block kb of layer i: mask with
// relu'(X_i) (read from X_i's m-packed copy at exactly the accumulator's
// positions), write the LDS tile, the m-packed dZ_i and the column sums.
// The relu' masks are loaded before the block's MMA loop (bwd_mask) so their
// latency hides under it.
struct BwdMask {
  uint2 v[4];
};
__device__ __forceinline__ BwdMask bwd_mask(const TowerLayerDev& prev, int kb, int m0, int lane) {
  const int c = lane & 31, h = lane >> 5;
  const int NB = prev.Np / 32;
  BwdMask mk;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    mk.v[q] = *reinterpret_cast<const uint2*>(prev.xmp + mp_off(m0 / 16 + (q >> 1), NB, kb, c + 32 * (q & 1)) + 4 * h);
  return mk;
}

__device__ __forceinline__ void bwd_epilogue(const f32x16& acc, const TowerLayerDev& prev, const BwdMask& mk, int kb,
                                             int m0, u16* dst, int ldl, float* bp, int lane) {
  const int c = lane & 31, h = lane >> 5;
  const int NB = prev.Np / 32;
  float cs = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int64_t off = mp_off(m0 / 16 + (q >> 1), NB, kb, c + 32 * (q & 1)) + 4 * h;
    const uint2 xm = mk.v[q];
    const u16 xs[4] = {(u16)(xm.x & 0xffff), (u16)(xm.x >> 16), (u16)(xm.y & 0xffff), (u16)(xm.y >> 16)};
    u16 o[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      float v = acc[q * 4 + t];
      if (!(bf2f(xs[t]) > 0.f)) v = 0.f;
      o[t] = f2bf(v);
      cs += v;
      dst[(8 * q + 4 * h + t) * ldl + kb * 32 + c] = o[t];
    }
    uint2 pk;
    pk.x = (unsigned)o[0] | ((unsigned)o[1] << 16);
    pk.y = (unsigned)o[2] | ((unsigned)o[3] << 16);
    *reinterpret_cast<uint2*>(prev.dzmp + off) = pk;
  }
  cs += __shfl_xor(cs, 32);
  if (h == 0) bp[prev.bias_off + kb * 32 + c] = cs;
}

template <int PFv>
__global__ __launch_bounds__(TNT) void k_tower_bwd(TowerArgs a) {
  extern __shared__ __attribute__((aligned(16))) u16 lds[];
  __shared__ float gs[TBM];
  const int ldl = a.lds_ld;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int m0 = blockIdx.x * TBM;
  u16* src = lds;
  u16* dst = lds + TBM * ldl;
  float* bp = a.bias_part + (int64_t)blockIdx.x * a.bias_ld;
  const float gl = a.dloss ? a.dloss[0] : 1.f;
  if (tid < TBM) gs[tid] = (m0 + tid < a.M) ? a.dz[m0 + tid] * gl : 0.f;
  __syncthreads();
  // dZ_L = (g w_out^T) . relu'(X_L): one thread per column, 32 rows read as
  // four 16-B pieces of the m-packed X_L
  const TowerLayerDev& lastl = a.ly[a.L - 1];
  {
    const int NpL = lastl.Np, NL = lastl.N, NBL = NpL / 32;
    for (int k = tid; k < NpL; k += TNT) {
      const float wk = k < NL ? a.w_out[k] : 0.f;
      const int nb = k / 32, c = k % 32;
      float dbs = 0.f, dws = 0.f;
#pragma unroll
      for (int mb = 0; mb < 2; ++mb) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int64_t off = mp_off(m0 / 16 + mb, NBL, nb, c + 32 * h);
          const uint4 xv = *reinterpret_cast<const uint4*>(lastl.xmp + off);
          const unsigned int xw[4] = {xv.x, xv.y, xv.z, xv.w};
          unsigned int ow[4];
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            u16 o2[2];
#pragma unroll
            for (int e = 0; e < 2; ++e) {
              const int j = jj * 2 + e;
              const int r = 16 * mb + 8 * h + j;
              const float x = bf2f((u16)((xw[jj] >> (16 * e)) & 0xffff));
              const float g = gs[r];
              const float d = x > 0.f ? g * wk : 0.f;
              o2[e] = f2bf(d);
              dbs += d;
              dws += g * x;
              src[r * ldl + k] = o2[e];
            }
            ow[jj] = (unsigned)o2[0] | ((unsigned)o2[1] << 16);
          }
          *reinterpret_cast<uint4*>(lastl.dzmp + off) = make_uint4(ow[0], ow[1], ow[2], ow[3]);
        }
      }
      bp[lastl.bias_off + k] = dbs;
      if (k < NL) bp[a.dwout_off + k] = dws;
    }
    if (tid == 0) {
      float s = 0.f;
      for (int r = 0; r < TBM; ++r) s += gs[r];
      bp[a.dbout_off] = s;
    }
  }
  __syncthreads();
  // dX_i = dZ_{i+1} W_i  (i = L-1 .. 0); dZ_i = dX_i . relu'(X_i) for i >= 1
  for (int i = a.L - 1; i >= 0; --i) {
    if (i == 0 && !a.need_dx0) break;
    const TowerLayerDev& ly = a.ly[i];
    const int KB = ly.Kp / 32, NS = ly.Np / 16;
    const bf16x8* wtp = reinterpret_cast<const bf16x8*>(ly.wtp);
    for (int kb0 = w; kb0 < KB; kb0 += 2 * TNW) {
      const int kb1 = kb0 + TNW;
      const bool two = kb1 < KB;
      f32x16 acc0 = (f32x16){0}, acc1 = (f32x16){0};
      BwdMask mk0, mk1;
      if (i > 0) {
        mk0 = bwd_mask(a.ly[i - 1], kb0, m0, lane);
        if (two) mk1 = bwd_mask(a.ly[i - 1], kb1, m0, lane);
      }
      const bf16x8* w0p = wtp + (int64_t)kb0 * NS * 64 + lane;
      if (two) mma_pair<true, PFv>(src, ldl, w0p, wtp + (int64_t)kb1 * NS * 64 + lane, NS, (int)blockIdx.x * 5, acc0, acc1, lane);
      else mma_pair<false, PFv>(src, ldl, w0p, w0p, NS, (int)blockIdx.x * 5, acc0, acc1, lane);
      if (i > 0) {
        bwd_epilogue(acc0, a.ly[i - 1], mk0, kb0, m0, dst, ldl, bp, lane);
        if (two) bwd_epilogue(acc1, a.ly[i - 1], mk1, kb1, m0, dst, ldl, bp, lane);
      } else {
        const int c = lane & 31, h = lane >> 5;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = 8 * (r >> 2) + 4 * h + (r & 3);
          dst[row * ldl + kb0 * 32 + c] = f2bf(acc0[r]);
          if (two) dst[row * ldl + kb1 * 32 + c] = f2bf(acc1[r]);
        }
      }
    }
    __syncthreads();
    u16* t = src;
    src = dst;
    dst = t;
  }
  if (a.need_dx0) {  // dX0 tile -> global rows, 16-B stores
    const int c8n = a.ly[0].Kp / 8;
    const int wcols = a.lddx0 < a.ly[0].Kp ? a.lddx0 / 8 : c8n;
    for (int idx = tid; idx < TBM * c8n; idx += TNT) {
      const int r = idx / c8n, c = idx - r * c8n;
      if (m0 + r < a.M && c < wcols)
        *reinterpret_cast<uint4*>(a.dx0 + (int64_t)(m0 + r) * a.lddx0 + c * 8) =
            *reinterpret_cast<const uint4*>(src + r * ldl + c * 8);
    }
  }
}

// ---------------------------------------------------------------- grouped dW
constexpr int DW_STEPS = 4;  // m16 steps per ring stage
constexpr int DW_NST = 4;    // ring stages
constexpr int DW_STAGE = DW_STEPS * 4 * 512;  // elements per stage (4 x 1 KB fragments per step)

__device__ __forceinline__ int dw_tiles(const TowerLayerDev& ly) { return ((ly.Np + 63) / 64) * ((ly.Kp + 63) / 64); }

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// 16-B-per-lane LDS-DMA (lane l lands at lds_byte + 16 l).  Issued from inline
// asm so hipcc does not treat every later ds_read as aliasing it and drain the
// whole ring with vmcnt(0): completion is counted explicitly (wait_vm).
__device__ __forceinline__ void glds16(const void* gsrc, unsigned lds_byte) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_byte)
               : "memory");
}
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(uintptr_t)((const __attribute__((address_space(3))) char*)p);
}

__global__ __launch_bounds__(256) void k_tower_dw(TowerArgs a, int ndw) {
  const int tid = threadIdx.x;
  if ((int)blockIdx.x >= ndw && (a.debug & 2)) return;
  if ((int)blockIdx.x < ndw && (a.debug & 4)) return;
  if ((int)blockIdx.x >= ndw) {  // ---- column reductions (tower_common.h)
    tower_col_reduce(a, (int)blockIdx.x - ndw, TBM);
    return;
  }
  __shared__ __attribute__((aligned(16))) u16 smem[DW_NST * DW_STAGE];
  // ---- which layer / tile / split.  XCD-aware remap: blocks are dealt to
  // the 8 XCDs round-robin, so consecutive work ids (tiles sharing the dZ
  // panel of one n-range, then both M-halves) are placed on one XCD and
  // share its L2 instead of each XCD streaming the panel from HBM.
  const int S = a.dw_splits;
  const int q = ndw / 8, rr = ndw % 8, xcd = (int)blockIdx.x % 8;
  const int wid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (int)blockIdx.x / 8;
  int t = wid / S;
  const int split = wid % S;
  int l = 0;
  for (; l < a.L; ++l) {
    const int nt = dw_tiles(a.ly[l]);
    if (t < nt) break;
    t -= nt;
  }
  const TowerLayerDev& ly = a.ly[l];
  const int NBn = ly.Np / 32, NBk = ly.Kp / 32;
  const int tk_n = (ly.Kp + 63) / 64;
  const int tn = t / tk_n, tk = t % tk_n;
  const u16* Amp = ly.dzmp;                          // dZ_{l+1}: [Mp/16][NBn]
  const u16* Bmp = l == 0 ? a.x0mp : a.ly[l - 1].xmp;  // X_l:      [Mp/16][NBk]
  const int lane = tid & 63, w = tid >> 6;
  // this wave's DMA: fragment w (0,1: A n-blocks; 2,3: B k-blocks)
  const u16* gsrc;
  int gstride;  // elements between consecutive m16 chunks of the fragment column
  if (w < 2) {
    const int nb = min(tn * 2 + w, NBn - 1);
    gsrc = Amp + ((int64_t)nb * 64 + lane) * 8;
    gstride = NBn * 512;
  } else {
    const int kb = min(tk * 2 + (w - 2), NBk - 1);
    gsrc = Bmp + ((int64_t)kb * 64 + lane) * 8;
    gstride = NBk * 512;
  }
  const int nsteps_all = a.Mp / 16;
  const int per = nsteps_all / S;  // multiple of DW_STEPS (Mp is padded to 128)
  const int mb0 = split * per;
  const int nstage = per / DW_STEPS;
  const unsigned lds_w = __builtin_amdgcn_readfirstlane(lds_addr(smem) + (unsigned)w * 1024u);
  auto issue = [&](int slot, int stage) {
    const unsigned base = lds_w + (unsigned)(slot * DW_STAGE) * 2u;
#pragma unroll
    for (int st = 0; st < DW_STEPS; ++st) {
      const int mb = mb0 + stage * DW_STEPS + st;
      glds16(gsrc + (int64_t)mb * gstride, base + st * 4096u);
    }
  };
  const int wn = w & 1, wk = w >> 1;
  f32x16 acc = (f32x16){0};
  for (int p = 0; p < DW_NST - 1 && p < nstage; ++p) issue(p, p);
  for (int s = 0; s < nstage; ++s) {
    const int ahead = min(DW_NST - 2, nstage - 1 - s);
    if (ahead >= 2) wait_vm<2 * DW_STEPS>();
    else if (ahead == 1) wait_vm<DW_STEPS>();
    else wait_vm<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (s + DW_NST - 1 < nstage) issue((s + DW_NST - 1) % DW_NST, s + DW_NST - 1);
    const u16* base = smem + (s % DW_NST) * DW_STAGE;
#pragma unroll
    for (int st = 0; st < DW_STEPS; ++st) {
      const bf16x8 av = *reinterpret_cast<const bf16x8*>(base + st * 2048 + wn * 512 + lane * 8);
      const bf16x8 bv = *reinterpret_cast<const bf16x8*>(base + st * 2048 + (2 + wk) * 512 + lane * 8);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc, 0, 0, 0);
    }
  }
  // epilogue: rows n, cols k of dW; two 128-B row segments per atomic instruction
  const int nb = tn * 2 + wn, kb = tk * 2 + wk;
  if (nb >= NBn || kb >= NBk) return;
  const int c = lane & 31, h = lane >> 5;
  const int k = kb * 32 + c;
  if (k >= ly.K) return;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int n = nb * 32 + 8 * (r >> 2) + 4 * h + (r & 3);
    if (n < ly.N) atomicAdd(&ly.dw[(int64_t)n * ly.K + k], acc[r]);
  }
}

// ---------------------------------------------------------------- weight packing
__device__ __forceinline__ int64_t wp_index(int n, int k, int Kp) {
  return ((int64_t)((n >> 5) * (Kp >> 4) + (k >> 4)) * 64 + (n & 31) + 32 * ((k >> 3) & 1)) * 8 + (k & 7);
}
__device__ __forceinline__ int64_t wtp_index(int n, int k, int Np) {
  return ((int64_t)((k >> 5) * (Np >> 4) + (n >> 4)) * 64 + (k & 31) + 32 * ((n >> 3) & 1)) * 8 + (n & 7);
}

struct PackJob {
  const float* w[kMaxTowerLayers];
  int64_t off[kMaxTowerLayers + 1];
};

__global__ void k_tower_pack(TowerArgs a, PackJob j) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= j.off[a.L]) return;
  int l = 0;
  while (e >= j.off[l + 1]) ++l;
  const TowerLayerDev& ly = a.ly[l];
  const int64_t i = e - j.off[l];
  const int n = (int)(i / ly.K), k = (int)(i % ly.K);
  const u16 v = f2bf(j.w[l][i]);
  const_cast<u16*>(ly.wp)[wp_index(n, k, ly.Kp)] = v;
  const_cast<u16*>(ly.wtp)[wtp_index(n, k, ly.Np)] = v;
}

// ---------------------------------------------------------------- Adam (+ extras)
// Grid-stride over float4 groups with a capped grid: the beta-power ticket
// below is one same-address returning atomic per workgroup, and ~1700 of
// them (one group per thread) serialised at the memory side for several us.
__global__ __launch_bounds__(256) void k_adam_fused(float* __restrict__ p, float* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                    float lr, float b1, float b2, float eps, float* pows, float gs,
                                                    float wd, int clear_grad, AdamExtras x) {
  const float b1pow = pows[0] * b1, b2pow = pows[1] * b2;  // powers of this step
  const float lr_t = lr * sqrtf(1.f - b2pow) / (1.f - b1pow);
  const float epst = eps * sqrtf(1.f - b2pow);
  const int64_t stride4 = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i4 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i4 * 4 < n; i4 += stride4) {
    const int64_t e0 = i4 * 4;
    // fp32 tower re-pack destinations of this group, looked up BEFORE the
    // update (their position-table loads then overlap the p/g/m/v loads
    // instead of starting after the arithmetic); -1: not a packed weight
    int64_t dwp[4] = {-1, -1, -1, -1}, dwt[4] = {-1, -1, -1, -1};
    int rsel = -1;
    for (int r = 0; r < x.n_pack; ++r) {
      const int64_t off = x.pack_off[r];
      const int64_t cnt = (int64_t)x.pack_N[r] * x.pack_K[r];
      if (e0 + 3 < off || e0 >= off + cnt || !x.pack_wp32[r] || !x.pack_pos32[r]) continue;
      rsel = r;
      const int K = x.pack_K[r];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int64_t i = e0 + k - off;
        if (i < 0 || i >= cnt || e0 + k >= n) continue;
        const int nn = (int)((uint32_t)i / (uint32_t)K), kk = (int)((uint32_t)i - (uint32_t)nn * (uint32_t)K);
        dwp[k] = tower_wp32_index_pos(x.pack_pos32[r], nn, kk, x.pack_Kp[r]);
        dwt[k] = tower_wtp32_index_pos(x.pack_posT32[r], nn, kk, x.pack_Np[r]);
      }
    }
    float pa[4], ga[4], ma[4], va[4];
    const bool full = e0 + 4 <= n;
    if (full) {
      const float4 pp = reinterpret_cast<float4*>(p)[i4];
      const float4 gg = reinterpret_cast<const float4*>(g)[i4];
      const float4 mm = reinterpret_cast<float4*>(m)[i4];
      const float4 vv = reinterpret_cast<float4*>(v)[i4];
      pa[0] = pp.x; pa[1] = pp.y; pa[2] = pp.z; pa[3] = pp.w;
      ga[0] = gg.x; ga[1] = gg.y; ga[2] = gg.z; ga[3] = gg.w;
      ma[0] = mm.x; ma[1] = mm.y; ma[2] = mm.z; ma[3] = mm.w;
      va[0] = vv.x; va[1] = vv.y; va[2] = vv.z; va[3] = vv.w;
    } else {
      for (int k = 0; k < 4; ++k) {
        const bool ok = e0 + k < n;
        pa[k] = ok ? p[e0 + k] : 0.f;
        ga[k] = ok ? g[e0 + k] : 0.f;
        ma[k] = ok ? m[e0 + k] : 0.f;
        va[k] = ok ? v[e0 + k] : 0.f;
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float gk = ga[k] * gs + wd * pa[k];
      ma[k] = b1 * ma[k] + (1.f - b1) * gk;
      va[k] = b2 * va[k] + (1.f - b2) * gk * gk;
      pa[k] -= lr_t * ma[k] / (sqrtf(va[k]) + epst);
    }
    if (full) {
      reinterpret_cast<float4*>(p)[i4] = make_float4(pa[0], pa[1], pa[2], pa[3]);
      reinterpret_cast<float4*>(m)[i4] = make_float4(ma[0], ma[1], ma[2], ma[3]);
      reinterpret_cast<float4*>(v)[i4] = make_float4(va[0], va[1], va[2], va[3]);
      if (clear_grad) reinterpret_cast<float4*>(g)[i4] = make_float4(0.f, 0.f, 0.f, 0.f);
    } else {
      for (int k = 0; k < 4 && e0 + k < n; ++k) {
        p[e0 + k] = pa[k];
        m[e0 + k] = ma[k];
        v[e0 + k] = va[k];
        if (clear_grad) g[e0 + k] = 0.f;
      }
    }
    if (rsel >= 0) {  // fp32 tower copies (destinations resolved above)
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (dwp[k] >= 0) {
          x.pack_wp32[rsel][dwp[k]] = pa[k];
          x.pack_wtp32[rsel][dwt[k]] = pa[k];
        }
    }
    // bf16 tower copies of weight regions (and fp32 ones without position tables)
    for (int r = 0; r < x.n_pack; ++r) {
      if (r == rsel) continue;
      const int64_t off = x.pack_off[r];
      const int K = x.pack_K[r];
      const int64_t cnt = (int64_t)x.pack_N[r] * K;
      if (e0 + 3 < off || e0 >= off + cnt) continue;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int64_t i = e0 + k - off;
        if (i < 0 || i >= cnt || e0 + k >= n) continue;
        const int nn = (int)((uint32_t)i / (uint32_t)K), kk = (int)((uint32_t)i - (uint32_t)nn * (uint32_t)K);
        if (x.pack_wp32[r]) {  // fp32 tower
          if (x.pack_pos32[r]) {
            x.pack_wp32[r][tower_wp32_index_pos(x.pack_pos32[r], nn, kk, x.pack_Kp[r])] = pa[k];
            x.pack_wtp32[r][tower_wtp32_index_pos(x.pack_posT32[r], nn, kk, x.pack_Np[r])] = pa[k];
          } else {
            x.pack_wp32[r][tower_wp32_index(nn, kk, x.pack_Np[r], x.pack_Kp[r])] = pa[k];
            x.pack_wtp32[r][tower_wtp32_index(nn, kk, x.pack_Np[r], x.pack_Kp[r])] = pa[k];
          }
          continue;
        }
        const u16 bv = f2bf(pa[k]);
        const int64_t pi = wp_index(nn, kk, x.pack_Kp[r]), ti = wtp_index(nn, kk, x.pack_Np[r]);
        x.pack_wp[r][pi] = bv;
        x.pack_wtp[r][ti] = bv;
        if (x.pack_x3[r]) {  // x3 tower: lo half after the hi copy
          const int64_t lo = (int64_t)x.pack_Np[r] * x.pack_Kp[r];
          const u16 lv = f2bf(pa[k] - bf2f(bv));
          x.pack_wp[r][lo + pi] = lv;
          x.pack_wtp[r][lo + ti] = lv;
        }
      }
    }
  }
  // data_norm summaries: bsize = bsize*decay + stats0, ...
  for (int d = 0; d < x.n_dn; ++d) {
    const int C = x.dn_C[d];
    for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < C; c += gridDim.x * blockDim.x) {
      const float* st = x.dn_stats[d];
      const float dec = x.dn_decay[d];
      x.dn_bsize[d][c] = x.dn_bsize[d][c] * dec + st[c];
      x.dn_bsum[d][c] = x.dn_bsum[d][c] * dec + st[C + c];
      x.dn_bsq[d][c] = x.dn_bsq[d][c] * dec + st[2 * C + c];
    }
  }
  // the last workgroup to finish publishes the new beta powers
  __syncthreads();
  if (threadIdx.x == 0) {
    if (atomicAdd(x.ticket, 1u) == gridDim.x - 1) {
      pows[0] = b1pow;
      pows[1] = b2pow;
      *x.ticket = 0u;
    }
  }
}


// A per-layer pointer out of the kernel-argument arrays by a uniform layer
// index: a select chain (s_cselect) instead of dynamic indexing, which made
// hipcc copy the argument arrays to scratch and reload from it
template <typename T>
__device__ __forceinline__ T pick_layer(T const (&arr)[kMaxMlpLayers], int i) {
  T r = arr[0];
#pragma unroll
  for (int j = 1; j < kMaxMlpLayers; ++j) r = (i == j) ? arr[j] : r;
  return r;
}

// ---------------------------------------------------------------- DCN-V2 cross forward
// x_{l+1} = x_0 * (x_l W_l^T + b_l) + x_l for l < L, then s = x_L . w_c,
// one 512-thread workgroup per 32-row tile (kernels.h CrossFwdArgs).
__device__ __forceinline__ int cross_ldl(int P) { return P + 8; }
__device__ __forceinline__ int cross_ldf(int P) { return P + 4; }

template <int PFv>
__global__ __launch_bounds__(TNT) void k_cross_fwd(CrossFwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) u16 lds[];
  const int Np = a.Np, Kp = a.Kp;
  const int P = Np > Kp ? Np : Kp;
  const int ldl = cross_ldl(P), ldf = cross_ldf(P);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int m0 = blockIdx.x * TBM;
  u16* x0b = lds;
  u16* src = x0b + TBM * ldl;
  u16* dst = src + TBM * ldl;
  float* fsrc = reinterpret_cast<float*>(dst + TBM * ldl);
  float* fdst = fsrc + TBM * ldf;
  constexpr int WO = 8;
  float wo[WO];
#pragma unroll
  for (int j = 0; j < WO; ++j) wo[j] = lane + 64 * j < a.D ? a.wc[lane + 64 * j] : 0.f;
  {  // stage x_0: bf16 (epilogue operand + first A operand) and its fp32 residual
    const int c8n = Kp / 8;
    for (int i = tid; i < TBM * c8n; i += TNT) {
      const int r = i / c8n, c = i - r * c8n;
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (m0 + r < a.M) v = *reinterpret_cast<const uint4*>(a.x0 + (int64_t)(m0 + r) * a.ldx0 + c * 8);
      *reinterpret_cast<uint4*>(x0b + r * ldl + c * 8) = v;
      *reinterpret_cast<uint4*>(src + r * ldl + c * 8) = v;
      const unsigned int vw[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) fsrc[r * ldf + c * 8 + e] = bf2f((u16)((vw[e >> 1] >> (16 * (e & 1))) & 0xffff));
    }
  }
  __syncthreads();
  const int NB = Np / 32, KS = Kp / 16;
  // m-packed x_0 (the layer-0 dW operand): 8 rows of one column = 16 B
  for (int i = tid; i < Np * (TBM / 8); i += TNT) {
    const int n = i / (TBM / 8), g8 = i - n * (TBM / 8);
    unsigned int pk[4];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      pk[e] = (unsigned)x0b[(8 * g8 + 2 * e) * ldl + n] | ((unsigned)x0b[(8 * g8 + 2 * e + 1) * ldl + n] << 16);
    const int r0 = 8 * g8;
    *reinterpret_cast<uint4*>(pick_layer(a.xmp, 0) + mp_off(m0 / 16 + r0 / 16, NB, n >> 5, (n & 31) + 32 * ((r0 & 15) >> 3))) =
        make_uint4(pk[0], pk[1], pk[2], pk[3]);
  }
  for (int l = 0; l < a.L; ++l) {
    const bf16x8* wp = reinterpret_cast<const bf16x8*>(pick_layer(a.wp, l));
    const float* bias_l = pick_layer(a.bias, l);
    float* z_l = pick_layer(a.z, l);
    unsigned short* xmp_n = pick_layer(a.xmp, l + 1 < kMaxMlpLayers ? l + 1 : 0);
    const bool last = l + 1 == a.L;
    auto epi = [&](const f32x16& acc, int nb) {
      const int c = lane & 31, h = lane >> 5;
      const int n = nb * 32 + c;
      const bool nv = n < a.D;
      const float bn = nv ? bias_l[n] : 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        u16 o[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int r = 8 * q + 4 * h + t;
          const int m = m0 + r;
          const float z = acc[q * 4 + t] + bn;
          const float xn = nv ? bf2f(x0b[r * ldl + n]) * z + fsrc[r * ldf + n] : 0.f;
          fdst[r * ldf + n] = xn;
          o[t] = f2bf(xn);
          dst[r * ldl + n] = o[t];
          if (nv && m < a.M) {
            z_l[(int64_t)m * a.ldf + n] = z;
            if (last) a.xlast[(int64_t)m * a.ldf + n] = xn;
          }
          if (m >= a.M) o[t] = 0;
        }
        if (!last) {  // m-packed x_{l+1} (tower fwd_epilogue layout)
          uint2 pk;
          pk.x = (unsigned)o[0] | ((unsigned)o[1] << 16);
          pk.y = (unsigned)o[2] | ((unsigned)o[3] << 16);
          *reinterpret_cast<uint2*>(xmp_n + mp_off(m0 / 16 + (q >> 1), NB, nb, c + 32 * (q & 1)) + 4 * h) = pk;
        }
      }
    };
    for (int nb0 = w; nb0 < NB; nb0 += 2 * TNW) {
      const int nb1 = nb0 + TNW;
      const bool two = nb1 < NB;
      f32x16 acc0 = (f32x16){0}, acc1 = (f32x16){0};
      const bf16x8* w0p = wp + (int64_t)nb0 * KS * 64 + lane;
      if (two) mma_pair<true, PFv>(src, ldl, w0p, wp + (int64_t)nb1 * KS * 64 + lane, KS, (int)blockIdx.x * 5, acc0, acc1, lane);
      else mma_pair<false, PFv>(src, ldl, w0p, w0p, KS, (int)blockIdx.x * 5, acc0, acc1, lane);
      epi(acc0, nb0);
      if (two) epi(acc1, nb1);
    }
    __syncthreads();
    u16* t = src;
    src = dst;
    dst = t;
    float* tf = fsrc;
    fsrc = fdst;
    fdst = tf;
  }
  // s = x_L . w_c from the fp32 tile, 4 rows per wave
  constexpr int RPW = TBM / TNW;
  float sv[RPW];
#pragma unroll
  for (int rr = 0; rr < RPW; ++rr) sv[rr] = 0.f;
#pragma unroll
  for (int j = 0; j < WO; ++j) {
    const int k = lane + 64 * j;
    if (k < a.D) {
#pragma unroll
      for (int rr = 0; rr < RPW; ++rr) sv[rr] += fsrc[(w * RPW + rr) * ldf + k] * wo[j];
    }
  }
  for (int k = lane + 64 * WO; k < a.D; k += 64) {
#pragma unroll
    for (int rr = 0; rr < RPW; ++rr) sv[rr] += fsrc[(w * RPW + rr) * ldf + k] * a.wc[k];
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1)
#pragma unroll
    for (int rr = 0; rr < RPW; ++rr) sv[rr] += __shfl_xor(sv[rr], off);
  if (lane < RPW) {
    float mine = sv[0];
#pragma unroll
    for (int rr = 1; rr < RPW; ++rr) mine = lane == rr ? sv[rr] : mine;
    const int m = m0 + w * RPW + lane;
    if (m < a.M) a.s[m] = mine;
  }
}

struct CrossPackJob {
  const float* w[kMaxMlpLayers];
  u16* wp[kMaxMlpLayers];
  u16* wtp[kMaxMlpLayers];
};

__global__ void k_cross_pack(CrossPackJob j, int L, int D, int Kp, int Np) {
  const int64_t per = (int64_t)D * D;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= per * L) return;
  const int l = (int)(e / per);
  const int64_t i = e - (int64_t)l * per;
  const int n = (int)(i / D), k = (int)(i - (int64_t)n * D);
  const u16 v = f2bf(j.w[l][i]);
  j.wp[l][wp_index(n, k, Kp)] = v;
  if (j.wtp[l]) j.wtp[l][wtp_index(n, k, Np)] = v;
}

// ---------------------------------------------------------------- DCN-V2 cross backward chain
template <int PFv>
__global__ __launch_bounds__(TNT) void k_cross_bwd(CrossBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) u16 lds[];
  const int P = a.Np;
  const int ldl = cross_ldl(P), ldf = cross_ldf(P);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int m0 = blockIdx.x * TBM;
  u16* x0b = lds;
  u16* src = x0b + TBM * ldl;
  u16* dst = src + TBM * ldl;
  float* gs = reinterpret_cast<float*>(dst + TBM * ldl);  // g_{l+1}, updated in place
  float* as = gs + TBM * ldf;                             // sum_l z_l * g_{l+1}
  __shared__ float dss[TBM];
  if (tid < TBM) dss[tid] = m0 + tid < a.M ? a.ds[m0 + tid] * (a.ds_scale ? a.ds_scale[0] : 1.f) : 0.f;
  {
    const int c8n = P / 8;
    for (int i = tid; i < TBM * c8n; i += TNT) {
      const int r = i / c8n, c = i - r * c8n;
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (m0 + r < a.M) v = *reinterpret_cast<const uint4*>(a.x0 + (int64_t)(m0 + r) * a.ldx0 + c * 8);
      *reinterpret_cast<uint4*>(x0b + r * ldl + c * 8) = v;
    }
  }
  __syncthreads();
  const int L = a.L;
  // top, one column per thread (z_{L-1} and x_L rows read coalesced, 8 rows
  // of loads in flight): g_L = ds w_c, u_{L-1} = bf16(x_0 g_L),
  // acc = z_{L-1} g_L, and the tile's dw_c partial sum_m ds x_L
  const int NB = P / 32, NS = P / 16;
  const float* z_top = pick_layer(a.z, L - 1);
  unsigned short* ump_top = pick_layer(a.ump, L - 1);
  float* bpart = a.bias_part + (int64_t)blockIdx.x * a.bias_ld;
  for (int n = tid; n < P; n += TNT) {
    const bool nv = n < a.D;
    const float wcn = nv ? a.wc[n] : 0.f;
    float p = 0.f, du = 0.f;
    // 16 rows' z / x_L loads in flight at once (32 per thread, before any use;
    // all 32 rows at once pushed the kernel past 256 VGPRs into scratch)
    constexpr int TH = TBM / 2;
#pragma unroll 1
    for (int hr = 0; hr < TBM; hr += TH) {
    float zv[TH], xv[TH];
#pragma unroll
    for (int e = 0; e < TH; ++e) {
      const int m = m0 + hr + e;
      const bool ok = nv && m < a.M;
      zv[e] = ok ? z_top[(int64_t)m * a.ldf + n] : 0.f;
      xv[e] = ok ? a.xlast[(int64_t)m * a.ldf + n] : 0.f;
    }
#pragma unroll
    for (int rh = 0; rh < TH; rh += 8) {
      const int r0 = hr + rh;
      u16 uo[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int r = r0 + e;
        const float g = dss[r] * wcn;
        gs[r * ldf + n] = g;
        uo[e] = nv ? f2bf(bf2f(x0b[r * ldl + n]) * g) : (u16)0;
        src[r * ldl + n] = uo[e];
        du += bf2f(uo[e]);
        as[r * ldf + n] = zv[rh + e] * g;
        p += dss[r] * xv[rh + e];
      }
      // m-packed u_{L-1}: these 8 rows of column n are 16 contiguous bytes
      *reinterpret_cast<uint4*>(ump_top + mp_off(m0 / 16 + r0 / 16, NB, n >> 5, (n & 31) + 32 * ((r0 & 15) >> 3))) =
          make_uint4((unsigned)uo[0] | ((unsigned)uo[1] << 16), (unsigned)uo[2] | ((unsigned)uo[3] << 16),
                     (unsigned)uo[4] | ((unsigned)uo[5] << 16), (unsigned)uo[6] | ((unsigned)uo[7] << 16));
    }
    }
    bpart[(L - 1) * P + n] = du;
    if (nv) bpart[L * P + n] = p;
  }
  __syncthreads();
  for (int l = L - 1; l >= 0; --l) {
    const bf16x8* wtp = reinterpret_cast<const bf16x8*>(pick_layer(a.wtp, l));
    const float* z_prev = pick_layer(a.z, l > 0 ? l - 1 : 0);
    unsigned short* ump_prev = pick_layer(a.ump, l > 0 ? l - 1 : 0);
    auto epi = [&](const f32x16& acc, int kb, const float* zp) {
      const int c = lane & 31, h = lane >> 5;
      const int k = kb * 32 + c;
      const bool kv = k < a.D;
      float cs = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        u16 o[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int r = 8 * q + 4 * h + t;
          const int m = m0 + r;
          const float gl = acc[q * 4 + t] + gs[r * ldf + k];
          o[t] = 0;
          if (l > 0) {
            gs[r * ldf + k] = kv ? gl : 0.f;
            as[r * ldf + k] += kv ? zp[q * 4 + t] * gl : 0.f;
            o[t] = kv ? f2bf(bf2f(x0b[r * ldl + k]) * gl) : (u16)0;
            dst[r * ldl + k] = o[t];
            cs += bf2f(o[t]);
          } else if (kv && m < a.M) {
            float v0 = gl + as[r * ldf + k];
            u16* d = a.dy + (int64_t)m * a.ldy + k;
            if (a.add_dy) v0 += bf2f(*d);
            *d = f2bf(v0);
          }
        }
        if (l > 0) {  // m-packed u_{l-1}
          uint2 pk;
          pk.x = (unsigned)o[0] | ((unsigned)o[1] << 16);
          pk.y = (unsigned)o[2] | ((unsigned)o[3] << 16);
          *reinterpret_cast<uint2*>(ump_prev + mp_off(m0 / 16 + (q >> 1), NB, kb, c + 32 * (q & 1)) + 4 * h) = pk;
        }
      }
      if (l > 0) {  // db_{l-1} partial: column sum of the tile's u_{l-1}
        cs += __shfl_xor(cs, 32);
        if (h == 0) bpart[(l - 1) * P + k] = cs;
      }
    };
    for (int kb0 = w; kb0 < NB; kb0 += 2 * TNW) {
      const int kb1 = kb0 + TNW;
      const bool two = kb1 < NB;
      // z_{l-1} at the accumulator positions, loaded ahead of the MMA loop
      float z0[16], z1[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int r = 8 * (e >> 2) + 4 * (lane >> 5) + (e & 3);
        const int m = m0 + r;
        const int k0 = kb0 * 32 + (lane & 31), k1 = kb1 * 32 + (lane & 31);
        z0[e] = (l > 0 && m < a.M && k0 < a.D) ? z_prev[(int64_t)m * a.ldf + k0] : 0.f;
        z1[e] = (l > 0 && two && m < a.M && k1 < a.D) ? z_prev[(int64_t)m * a.ldf + k1] : 0.f;
      }
      f32x16 acc0 = (f32x16){0}, acc1 = (f32x16){0};
      const bf16x8* w0p = wtp + (int64_t)kb0 * NS * 64 + lane;
      if (two) mma_pair<true, PFv>(src, ldl, w0p, wtp + (int64_t)kb1 * NS * 64 + lane, NS, (int)blockIdx.x * 5, acc0, acc1, lane);
      else mma_pair<false, PFv>(src, ldl, w0p, w0p, NS, (int)blockIdx.x * 5, acc0, acc1, lane);
      epi(acc0, kb0, z0);
      if (two) epi(acc1, kb1, z1);
    }
    __syncthreads();
    u16* t = src;
    src = dst;
    dst = t;
  }
}
}  // namespace

int tower_nwg(int M) { return ((M + kMpAlign - 1) / kMpAlign * kMpAlign) / TBM; }

size_t tower_lds_bytes(const TowerArgs& a) { return (size_t)2 * TBM * a.lds_ld * sizeof(u16); }

static int tower_pf() {
  static const int v = [] {
    const char* e = getenv("PBX_TOWER_PF");
    const int x = e ? atoi(e) : PF;
    return (x == 4 || x == 8) ? x : 6;
  }();
  return v;
}

// dynamic LDS above 64 KB must be opted into per kernel instantiation (static
// LDS of the kernels is < 1 KB); clear the runtime's sticky last-error if the
// call is refused
static void big_lds(const void* f) {
  if (hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024) != hipSuccess)
    (void)hipGetLastError();
}
template <int P>
static void allow_big_lds_pf() {
  static const bool once = [] {
    big_lds((const void*)k_tower_fwd<P>);
    big_lds((const void*)k_tower_bwd<P>);
    big_lds((const void*)k_cross_fwd<P>);
    big_lds((const void*)k_cross_bwd<P>);
    return true;
  }();
  (void)once;
}
#define PBX_PF_DISPATCH(KERN, GRID, LDS, STREAM, ARG)                                                       \
  do {                                                                                                     \
    switch (tower_pf()) {                                                                                  \
      case 4: allow_big_lds_pf<4>(); hipLaunchKernelGGL(KERN<4>, GRID, dim3(TNT), LDS, STREAM, ARG); break; \
      case 6: allow_big_lds_pf<6>(); hipLaunchKernelGGL(KERN<6>, GRID, dim3(TNT), LDS, STREAM, ARG); break; \
      default: allow_big_lds_pf<8>(); hipLaunchKernelGGL(KERN<8>, GRID, dim3(TNT), LDS, STREAM, ARG); break; \
    }                                                                                                      \
  } while (0)


size_t cross_fwd_lds_bytes(int Np, int Kp) {
  const int P = Np > Kp ? Np : Kp;
  const size_t b = (size_t)3 * TBM * (P + 8) * sizeof(u16) + (size_t)2 * TBM * (P + 4) * sizeof(float);
  return b <= (size_t)150 * 1024 ? b : 0;
}

void launch_cross_fwd(const CrossFwdArgs& a, hipStream_t s) {
  if (a.M == 0) return;
  PBX_PF_DISPATCH(k_cross_fwd, dim3((unsigned)((a.M + TBM - 1) / TBM)), cross_fwd_lds_bytes(a.Np, a.Kp), s, a);
}

void launch_cross_pack(const float* const* w, unsigned short* const* wp, unsigned short* const* wtp, int L, int D,
                       int Kp, int Np, hipStream_t s) {
  CrossPackJob j;
  for (int l = 0; l < L; ++l) {
    j.w[l] = w[l];
    j.wp[l] = wp[l];
    j.wtp[l] = wtp ? wtp[l] : nullptr;
  }
  const int64_t n = (int64_t)D * D * L;
  if (n == 0) return;
  hipLaunchKernelGGL(k_cross_pack, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, j, L, D, Kp, Np);
}

int cross_bwd_blocks(int M) { return (M + TBM - 1) / TBM; }

void launch_cross_bwd(const CrossBwdArgs& a, hipStream_t s) {
  if (a.M == 0) return;
  PBX_PF_DISPATCH(k_cross_bwd, dim3((unsigned)cross_bwd_blocks(a.M)), cross_fwd_lds_bytes(a.Np, a.Np), s, a);
}

void launch_tower_fwd(const TowerArgs& a, hipStream_t s) {
  if (a.M == 0) return;
  PBX_PF_DISPATCH(k_tower_fwd, dim3(a.Mp / TBM), tower_lds_bytes(a), s, a);
}

void launch_tower_bwd(const TowerArgs& a, hipStream_t s) {
  if (a.M == 0) return;
  PBX_PF_DISPATCH(k_tower_bwd, dim3(a.Mp / TBM), tower_lds_bytes(a), s, a);
}

void launch_tower_dw(const TowerArgs& a, hipStream_t s) {
  if (a.M == 0) return;
  int tiles = 0;
  for (int l = 0; l < a.L; ++l)
    tiles += ((a.ly[l].Np + 63) / 64) * ((a.ly[l].Kp + 63) / 64);
  const int ndw = tiles * a.dw_splits;
  const int nred = (a.bias_ld + 31) / 32 + (a.dn_part ? (a.dn_C + 31) / 32 : 0);
  hipLaunchKernelGGL(k_tower_dw, dim3(ndw + nred), dim3(256), 0, s, a, ndw);
}

void launch_tower_pack(const TowerArgs& a, const float* const* w, hipStream_t s) {
  PackJob j;
  j.off[0] = 0;
  for (int l = 0; l < a.L; ++l) {
    j.w[l] = w[l];
    j.off[l + 1] = j.off[l] + (int64_t)a.ly[l].N * a.ly[l].K;
  }
  const int64_t n = j.off[a.L];
  if (n == 0) return;
  hipLaunchKernelGGL(k_tower_pack, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a, j);
}

// Grid cap of the fused Adam (PBX_ADAM_MAX_BLOCKS): it runs on the side
// stream beside the critical-path pooling, and a smaller grid leaves that
// kernel more CUs -- x3 step 0.2452-0.2462 ms at 256 vs 0.2470-0.2472 at 512,
// 0.2494-0.2504 at 128 (profiles/r6_x3_adam_blocks_ab.txt)
static int adam_max_blocks() {
  static const int v = [] {
    const char* e = getenv("PBX_ADAM_MAX_BLOCKS");
    return e ? atoi(e) : 256;
  }();
  return v > 0 ? v : 256;
}

void launch_adam_fused(float* p, float* g, float* m, float* v, int64_t n, float lr, float b1, float b2, float eps,
                       float* pows, float grad_scale, float weight_decay, bool clear_grad, const AdamExtras& x,
                       hipStream_t s) {
  int64_t n4 = (n + 3) / 4;
  for (int d = 0; d < x.n_dn; ++d) n4 = n4 > x.dn_C[d] ? n4 : x.dn_C[d];
  if (n4 == 0) return;
  // <= 1 workgroup per CU by default (grid-stride loop inside): few ticket atomics
  int64_t blocks = (n4 + 255) / 256;
  const int64_t cap = (int64_t)adam_max_blocks();
  blocks = blocks < cap ? blocks : cap;
  hipLaunchKernelGGL(k_adam_fused, dim3((unsigned)blocks), dim3(256), 0, s, p, g, m, v, n, lr, b1, b2,
                     eps, pows, grad_scale, weight_decay, clear_grad ? 1 : 0, x);
}

}  // namespace pbx

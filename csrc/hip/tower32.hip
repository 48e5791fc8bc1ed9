// Fused CTR dense tower in exact fp32 on MI355X: the reference's `fc`
// precision (paddle/phi/kernels/gpu/matmul_kernel.cu runs fp32 GEMMs) with the
// same three-launch structure as the bf16 tower (tower.hip):
//
//   k_t32_fwd  one 512-thread workgroup per 32-row tile; the tile's fp32
//              activations stay in LDS across all layers; every wave streams
//              packed fp32 weight fragments (1 KB per 16x16 block and 16-deep
//              k-group, one dwordx4 per lane) and runs v_mfma_f32_16x16x4_f32.
//              Epilogue: bias + ReLU -> LDS and the MP32 copy (one dwordx4 per
//              lane: the accumulator IS the dW operand fragment).  Output GEMV,
//              sigmoid, log-loss, d loss/d logit and the AUC histogram fused.
//   k_t32_bwd  same tiling for the dX chain with ReLU masks read from the MP32
//              activations, per-tile column sums for the bias gradients.
//   k_t32_dw   dW = dZ^T X as one grouped GEMM over 64x64 output tiles, both
//              operands streamed HBM/L2 -> LDS by global_load_lds (1 KB per
//              wave instruction), M split over workgroups with fp32 atomics;
//              extra workgroups reduce bias partials and data_norm statistics.
//
// Why 16x16x4 and not 32x32x2: the f32 MFMA rate is 64 FLOP/clk/SIMD either
// way; 16-wide blocks pad a 400-unit layer to 400 (not 416) and split a layer
// into 25 column blocks x 2 row blocks, which balances over the 4 SIMDs.
// The 16x16x4 dependent latency (40 cycles) is covered by two accumulators
// per wave (both 16-row halves of the tile share every weight fragment).
#include <hip/hip_runtime.h>

#include "kernels.h"
#include "tower_common.h"

namespace pbx {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int BM = 32;    // rows per fwd / bwd workgroup
constexpr int NT = 512;   // threads per fwd / bwd workgroup
constexpr int NW = NT / 64;
constexpr int PF = 4;     // weight-fragment prefetch depth (16-deep k-groups)

__device__ __forceinline__ int64_t mp32(int m16, int nb16, int n16) { return ((int64_t)m16 * nb16 + n16) * 256; }

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// acc{0,1} += A{0,1}(16 rows x 16 KG, LDS) x B (packed fragments bfr[g * 64]).
// A0/A1: this lane's row pointer (+4 * (lane / 16)); TWO = both 16-row halves.
// Software pipeline, unrolled by 4 k-groups with NAMED registers: the weight
// fragments b0..b3 are each re-loaded right after the MFMAs that consumed
// them (4 groups = 32 MFMAs ahead) and the A fragments alternate between two
// register sets, so nothing is copied between registers at the loop edge (a
// rotated ring made hipcc move registers and drain vmcnt(0) every 4 groups).
// Addressing is pointer increments only: the loads run up to 8 groups past
// the end (the packed weights carry 8 KB of slack, the LDS tile 64 floats),
// so the loop needs no clamping or index arithmetic -- the first version's
// per-group scalar index math (~20 SALU between MFMA clusters) cost ~40% of
// the MFMA rate (timing experiments, profiles/r3_tower32_notes.txt).
template <bool TWO>
__device__ __forceinline__ void mma32(const float* __restrict__ A0, const float* __restrict__ A1,
                                      const f32x4* __restrict__ bp, int KG, f32x4& acc0, f32x4& acc1) {
  auto step = [&](const f32x4& a0, const f32x4& a1, const f32x4& b) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      acc0 = mfma4(a0[t], b[t], acc0);
      if (TWO) acc1 = mfma4(a1[t], b[t], acc1);
    }
  };
  auto lda = [](const float* p, int g) { return *reinterpret_cast<const f32x4*>(p + 16 * g); };
  f32x4 b0 = bp[0], b1 = bp[64], b2 = bp[128], b3 = bp[192];
  f32x4 e0 = lda(A0, 0), e1 = TWO ? lda(A1, 0) : e0;  // A of even groups
  f32x4 o0, o1;                                       // A of odd groups
  const int KM = KG & ~3;
  for (int k = 0; k < KM; k += 4) {
    o0 = lda(A0, 1);
    if (TWO) o1 = lda(A1, 1);
    __builtin_amdgcn_sched_barrier(0);
    step(e0, e1, b0);
    __builtin_amdgcn_sched_barrier(0);
    b0 = bp[256];
    e0 = lda(A0, 2);
    if (TWO) e1 = lda(A1, 2);
    __builtin_amdgcn_sched_barrier(0);
    step(o0, o1, b1);
    __builtin_amdgcn_sched_barrier(0);
    b1 = bp[320];
    o0 = lda(A0, 3);
    if (TWO) o1 = lda(A1, 3);
    __builtin_amdgcn_sched_barrier(0);
    step(e0, e1, b2);
    __builtin_amdgcn_sched_barrier(0);
    b2 = bp[384];
    e0 = lda(A0, 4);
    if (TWO) e1 = lda(A1, 4);
    __builtin_amdgcn_sched_barrier(0);
    step(o0, o1, b3);
    __builtin_amdgcn_sched_barrier(0);
    b3 = bp[448];
    bp += 256;
    A0 += 64;
    if (TWO) A1 += 64;
  }
  // tail: KG % 4 groups, their fragments already loaded (b0.., e)
  const int rem = KG - KM;
  if (rem > 0) {
    o0 = lda(A0, 1);
    if (TWO) o1 = lda(A1, 1);
    step(e0, e1, b0);
  }
  if (rem > 1) {
    e0 = lda(A0, 2);
    if (TWO) e1 = lda(A1, 2);
    step(o0, o1, b1);
  }
  if (rem > 2) step(e0, e1, b2);
}

// Work split of one layer over the 8 waves: NB column blocks, each a "pair"
// unit (both 16-row halves, sharing every weight fragment).  Full rounds go
// pair-wise; the remainder is dealt as single (block, half) items so that the
// 4 SIMDs (waves w and w + 4 share one) end within one item of each other.
template <typename F>
__device__ __forceinline__ void for_units(int NB, int w, F&& f) {
  const int q = NB / NW, r = NB % NW;
  for (int i = 0; i < q; ++i) f(w + NW * i, -1);
  for (int j = w; j < 2 * r; j += NW) f(NW * q + (j >> 1), j & 1);
}

// One unit: the epilogue's own global operands (bias, ReLU mask) are fetched
// by pre(nb, half) BEFORE the MFMA chain, so their latency hides under it
// instead of stalling the epilogue of both waves of a SIMD at once.
template <typename Pre, typename Epi>
__device__ __forceinline__ void run_unit(const float* src, int ldl, const f32x4* wbase, int KG, int nb, int half,
                                         int lane, Pre&& pre, Epi&& epi) {
  const int c = lane & 15, g = lane >> 4;
  const f32x4* bfr = wbase + (int64_t)nb * KG * 64 + lane;
  f32x4 acc0 = (f32x4){0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
  if (half < 0) {
    const f32x4 p0 = pre(nb, 0), p1 = pre(nb, 1);
    mma32<true>(src + c * ldl + 4 * g, src + (16 + c) * ldl + 4 * g, bfr, KG, acc0, acc1);
    epi(acc0, nb, 0, p0);
    epi(acc1, nb, 1, p1);
  } else {
    const f32x4 p0 = pre(nb, half);
    const float* A = src + (16 * half + c) * ldl + 4 * g;
    mma32<false>(A, A, bfr, KG, acc0, acc1);
    epi(acc0, nb, half, p0);
  }
}

__global__ __launch_bounds__(NT) void k_t32_fwd(TowerArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds32[];
  const int ldl = a.lds_ld;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int m0 = blockIdx.x * BM;
  float* src = lds32;
  float* dst = lds32 + BM * ldl;
  // waves 4-7 share SIMDs with 0-3 and lose every arbitration at equal
  // priority (MI355X_MICROARCH.md, two waves per SIMD, item 4)
  if (w >= 4) __builtin_amdgcn_s_setprio(1);
  long long* stp = a.stamps ? a.stamps + ((int64_t)blockIdx.x * NW + w) * 8 : nullptr;
  if (stp && lane == 0) stp[0] = __builtin_amdgcn_s_memtime();
  // loss-tail inputs and the output-layer weights, loaded ahead of the layers
  const int NL = a.ly[a.L - 1].N;
  TowerRowIn rin{0.f, 0.f, 0.f, 0.f};
  if (w < 2) rin = tower_row_in(a, m0, lane, BM);
  constexpr int WO = 8;
  float wo[WO];
#pragma unroll
  for (int j = 0; j < WO; ++j) wo[j] = lane + 64 * j < NL ? a.w_out[lane + 64 * j] : 0.f;
  {  // stage the X0 tile (zero rows past M)
    const int c4n = a.ly[0].Kp / 4;
    for (int i = tid; i < BM * c4n; i += NT) {
      const int r = i / c4n, c = i - r * c4n;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (m0 + r < a.M) v = *reinterpret_cast<const float4*>(a.x0f + (int64_t)(m0 + r) * a.ld0 + c * 4);
      *reinterpret_cast<float4*>(src + r * ldl + c * 4) = v;
    }
  }
  __syncthreads();
  for (int l = 0; l < a.L; ++l) {
    const TowerLayerDev& ly = a.ly[l];
    const int NB = ly.Np / 16, KG = ly.Kp / 16;
    const f32x4* wp = reinterpret_cast<const f32x4*>(ly.wpf);
    const int c = lane & 15, g = lane >> 4;
    for_units(NB, w, [&](int nb, int half) {
      run_unit(src, ldl, wp, KG, nb, half, lane, [&](int nbb, int) {
        const int n = nbb * 16 + c;
        return (f32x4){n < ly.N ? ly.bias[n] : 0.f, 0.f, 0.f, 0.f};
      }, [&](const f32x4& acc, int nbb, int mb, const f32x4& pb) {
        const int n = nbb * 16 + c;
        const float bias = pb[0];
        f32x4 o;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const float v = acc[t] + bias;
          o[t] = v > 0.f ? v : 0.f;
          dst[(16 * mb + 4 * g + t) * ldl + n] = o[t];
        }
        *reinterpret_cast<f32x4*>(ly.xmpf + mp32(m0 / 16 + mb, NB, nbb) + lane * 4) = o;
      });
    });
    if (stp && lane == 0) stp[1 + 2 * l] = __builtin_amdgcn_s_memtime();
    __syncthreads();
    if (stp && lane == 0) stp[2 + 2 * l] = __builtin_amdgcn_s_memtime();
    float* t = src;
    src = dst;
    dst = t;
  }
  // output layer: 4 rows per wave, independent accumulations, w_out from
  // registers; the logits meet in LDS for the loss tail
  __shared__ float zrow[BM];
  {
    constexpr int RPW = BM / NW;
    float s[RPW];
#pragma unroll
    for (int rr = 0; rr < RPW; ++rr) s[rr] = 0.f;
#pragma unroll
    for (int j = 0; j < WO; ++j) {
      const int k = lane + 64 * j;
      if (k < NL) {
#pragma unroll
        for (int rr = 0; rr < RPW; ++rr) s[rr] += src[(w * RPW + rr) * ldl + k] * wo[j];
      }
    }
    for (int k = lane + 64 * WO; k < NL; k += 64) {  // widths past 512
#pragma unroll
      for (int rr = 0; rr < RPW; ++rr) s[rr] += src[(w * RPW + rr) * ldl + k] * a.w_out[k];
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
  if (stp && lane == 0) stp[7] = __builtin_amdgcn_s_memtime();
  __syncthreads();
  tower_loss_tail(a, zrow, rin, m0, w, lane, BM);
}

__global__ __launch_bounds__(NT) void k_t32_bwd(TowerArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds32[];
  __shared__ float gs[BM];
  // per-layer column sums of dZ, one row per 16-row half; double-buffered by
  // layer parity so layer i's readers never race layer i-1's writers
  __shared__ float csum[2][2][kTower32MaxWidth];
  const int ldl = a.lds_ld;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int m0 = blockIdx.x * BM;
  float* src = lds32;
  float* dst = lds32 + BM * ldl;
  float* bp = a.bias_part + (int64_t)blockIdx.x * a.bias_ld;
  if (w >= 4) __builtin_amdgcn_s_setprio(1);
  const float gl = a.dloss ? a.dloss[0] : 1.f;
  if (tid < BM) gs[tid] = (m0 + tid < a.M) ? a.dz[m0 + tid] * gl : 0.f;
  __syncthreads();
  // dZ_L = (g w_out^T) . relu'(X_L), read from MP32(X_L): one (half, block, lane) per item
  const TowerLayerDev& lastl = a.ly[a.L - 1];
  {
    const int NpL = lastl.Np, NL = lastl.N, NBL = NpL / 16;
    float* red = dst;  // scratch [2][8][NpL]: db and dw_out partials per (half, lane group)
    for (int it = tid; it < 2 * NBL * 64; it += NT) {
      const int mb = it / (NBL * 64);
      const int rem = it - mb * NBL * 64;
      const int nb = rem >> 6, l = rem & 63, cc = l & 15, gg = l >> 4;
      const int k = nb * 16 + cc;
      const float wk = k < NL ? a.w_out[k] : 0.f;
      const int64_t off = mp32(m0 / 16 + mb, NBL, nb) + l * 4;
      const f32x4 x4 = *reinterpret_cast<const f32x4*>(lastl.xmpf + off);
      f32x4 o;
      float dbs = 0.f, dws = 0.f;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int r = 16 * mb + 4 * gg + t;
        const float x = x4[t], gr = gs[r];
        const float d = x > 0.f ? gr * wk : 0.f;
        o[t] = d;
        src[r * ldl + k] = d;
        dbs += d;
        dws += gr * x;
      }
      *reinterpret_cast<f32x4*>(lastl.dzmpf + off) = o;
      red[(mb * 4 + gg) * NpL + k] = dbs;
      red[8 * NpL + (mb * 4 + gg) * NpL + k] = dws;
    }
    __syncthreads();
    for (int k = tid; k < NpL; k += NT) {
      float db = 0.f, dw = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        db += red[j * NpL + k];
        dw += red[8 * NpL + j * NpL + k];
      }
      bp[lastl.bias_off + k] = db;
      if (k < NL) bp[a.dwout_off + k] = dw;
    }
    if (tid == 0) {
      float s = 0.f;
      for (int r = 0; r < BM; ++r) s += gs[r];
      bp[a.dbout_off] = s;
    }
    __syncthreads();
  }
  // dX_i = dZ_{i+1} W_i  (i = L-1 .. 0); dZ_i = dX_i . relu'(X_i) for i >= 1
  for (int i = a.L - 1; i >= 0; --i) {
    if (i == 0 && !a.need_dx0) break;
    const TowerLayerDev& ly = a.ly[i];
    const int KB = ly.Kp / 16, NG = ly.Np / 16;
    const f32x4* wtp = reinterpret_cast<const f32x4*>(ly.wtpf);
    float(*cs)[kTower32MaxWidth] = csum[i & 1];
    if (i > 0) {
      const TowerLayerDev& prev = a.ly[i - 1];
      const int PNB = prev.Np / 16;
      for_units(KB, w, [&](int kb, int half) {
        run_unit(src, ldl, wtp, NG, kb, half, lane, [&](int kbb, int mb) {
          return *reinterpret_cast<const f32x4*>(prev.xmpf + mp32(m0 / 16 + mb, PNB, kbb) + lane * 4);
        }, [&](const f32x4& acc, int kbb, int mb, const f32x4& x4) {
          const int64_t off = mp32(m0 / 16 + mb, PNB, kbb) + lane * 4;
          f32x4 o;
          float s = 0.f;
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            o[t] = x4[t] > 0.f ? acc[t] : 0.f;
            s += o[t];
            dst[(16 * mb + 4 * g + t) * ldl + kbb * 16 + c] = o[t];
          }
          *reinterpret_cast<f32x4*>(prev.dzmpf + off) = o;
          s += __shfl_xor(s, 16);
          s += __shfl_xor(s, 32);
          if (g == 0) cs[mb][kbb * 16 + c] = s;
        });
      });
    } else {
      for_units(KB, w, [&](int kb, int half) {
        run_unit(src, ldl, wtp, NG, kb, half, lane, [&](int, int) { return (f32x4){0.f, 0.f, 0.f, 0.f}; },
                 [&](const f32x4& acc, int kbb, int mb, const f32x4&) {
#pragma unroll
          for (int t = 0; t < 4; ++t) dst[(16 * mb + 4 * g + t) * ldl + kbb * 16 + c] = acc[t];
        });
      });
    }
    __syncthreads();
    if (i > 0) {
      const TowerLayerDev& prev = a.ly[i - 1];
      for (int col = tid; col < prev.Np; col += NT) bp[prev.bias_off + col] = cs[0][col] + cs[1][col];
    }
    float* t = src;
    src = dst;
    dst = t;
  }
  if (a.need_dx0) {  // dX0 tile -> global rows, 16-B stores
    const int c4n = a.ly[0].Kp / 4;
    const int wcols = a.lddx0 < a.ly[0].Kp ? a.lddx0 / 4 : c4n;
    for (int idx = tid; idx < BM * c4n; idx += NT) {
      const int r = idx / c4n, cc = idx - r * c4n;
      if (m0 + r < a.M && cc < wcols)
        *reinterpret_cast<float4*>(a.dx0f + (int64_t)(m0 + r) * a.lddx0 + cc * 4) =
            *reinterpret_cast<const float4*>(src + r * ldl + cc * 4);
    }
  }
}

// ---------------------------------------------------------------- grouped dW
constexpr int DSTEPS = 2;               // m16 steps per ring stage
constexpr int DNST = 3;                 // ring stages (48 KB: two dW workgroups per CU leave room for the
                                        // head backward that runs beside them on the compute stream)
constexpr int DSTAGE = DSTEPS * 8 * 256;  // floats per stage: 8 chunks of 1 KB per step (4 dZ, 4 X)

__device__ __forceinline__ int dw32_tiles(const TowerLayerDev& ly) {
  return ((ly.Np / 16 + 3) / 4) * ((ly.Kp / 16 + 3) / 4);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__global__ __launch_bounds__(256) void k_t32_dw(TowerArgs a, int ndw) {
  const int tid = threadIdx.x;
  if ((int)blockIdx.x >= ndw) {
    tower_col_reduce(a, (int)blockIdx.x - ndw, BM);
    return;
  }
  __shared__ __attribute__((aligned(16))) float smem[DNST * DSTAGE];
  const int S = a.dw_splits;
  int t, split;
  if (S == 8) {
    // one M split per XCD (blocks are dealt to the 8 XCDs round-robin; speed
    // only): an XCD's workgroups read the dZ / X panels of ONE 1/8 row range,
    // ~3 MB per layer, which stays in its 4 MB L2 instead of streaming every
    // panel from the Infinity Cache
    split = (int)blockIdx.x & 7;
    t = (int)blockIdx.x >> 3;
  } else {
    const int wid = xcd_work_id((int)blockIdx.x, ndw);
    t = wid / S;
    split = wid % S;
  }
  int l = 0;
  for (; l < a.L; ++l) {
    const int nt = dw32_tiles(a.ly[l]);
    if (t < nt) break;
    t -= nt;
  }
  const TowerLayerDev& ly = a.ly[l];
  const int NBn = ly.Np / 16, NBk = ly.Kp / 16;
  const int tk_n = (NBk + 3) / 4;
  const int tn = t / tk_n, tk = t % tk_n;
  const float* Amp = ly.dzmpf;                           // dZ_{l+1}: [Mp/16][NBn]
  const float* Bmp = l == 0 ? a.x0mpf : a.ly[l - 1].xmpf;  // X_l:      [Mp/16][NBk]
  const int lane = tid & 63, w = tid >> 6;
  // this wave's DMAs per step: dZ chunk (n-block tn*4 + w) and X chunk (k-block tk*4 + w)
  const float* gA = Amp + ((int64_t)min(tn * 4 + w, NBn - 1) * 64 + lane) * 4;
  const float* gB = Bmp + ((int64_t)min(tk * 4 + w, NBk - 1) * 64 + lane) * 4;
  const int64_t sA = (int64_t)NBn * 256, sB = (int64_t)NBk * 256;
  const int per = a.Mp / 16 / S;  // m16 steps of this split (multiple of DSTEPS)
  const int mb0 = split * per;
  const int nstage = per / DSTEPS;
  // wave-uniform LDS destinations (SGPRs: m0 is loaded from them)
  const unsigned ldsA = __builtin_amdgcn_readfirstlane(tower_lds_addr(smem) + (unsigned)w * 1024u);
  const unsigned ldsB = __builtin_amdgcn_readfirstlane(tower_lds_addr(smem) + (unsigned)(4 + w) * 1024u);
  auto issue = [&](int slot, int stage) {
    const unsigned so = (unsigned)(slot * DSTAGE) * 4u;
#pragma unroll
    for (int st = 0; st < DSTEPS; ++st) {
      const int mb = mb0 + stage * DSTEPS + st;
      tower_glds16(gA + mb * sA, ldsA + so + st * 8192u);
      tower_glds16(gB + mb * sB, ldsB + so + st * 8192u);
    }
  };
  const int wn = w & 1, wk = w >> 1;
  const bool active = (tn * 4 + 2 * wn < NBn) && (tk * 4 + 2 * wk < NBk);
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  for (int p = 0; p < DNST - 1 && p < nstage; ++p) issue(p, p);
  for (int s = 0; s < nstage; ++s) {
    const int ahead = min(DNST - 2, nstage - 1 - s);
    if (ahead >= 2) wait_vm<4 * DSTEPS>();
    else if (ahead == 1) wait_vm<2 * DSTEPS>();
    else wait_vm<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (s + DNST - 1 < nstage) issue((s + DNST - 1) % DNST, s + DNST - 1);
    if (active) {
      const float* base = smem + (s % DNST) * DSTAGE;
#pragma unroll
      for (int st = 0; st < DSTEPS; ++st) {
        const float* sb = base + st * 2048 + lane * 4;
        const f32x4 a0 = *reinterpret_cast<const f32x4*>(sb + (2 * wn) * 256);
        const f32x4 a1 = *reinterpret_cast<const f32x4*>(sb + (2 * wn + 1) * 256);
        const f32x4 b0 = *reinterpret_cast<const f32x4*>(sb + (4 + 2 * wk) * 256);
        const f32x4 b1 = *reinterpret_cast<const f32x4*>(sb + (4 + 2 * wk + 1) * 256);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          acc[0][0] = mfma4(a0[q], b0[q], acc[0][0]);
          acc[0][1] = mfma4(a0[q], b1[q], acc[0][1]);
          acc[1][0] = mfma4(a1[q], b0[q], acc[1][0]);
          acc[1][1] = mfma4(a1[q], b1[q], acc[1][1]);
        }
      }
    }
  }
  if (!active) return;
  // epilogue: lane (c, g) register q -> dW[16 nb + 4g + q][16 kb + c]
  const int c = lane & 15, g = lane >> 4;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int nb = tn * 4 + 2 * wn + i;
    if (nb >= NBn) continue;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int kb = tk * 4 + 2 * wk + j;
      const int k = kb * 16 + c;
      if (kb >= NBk || k >= ly.K) continue;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n = nb * 16 + 4 * g + q;
        if (n < ly.N) atomicAdd(&ly.dw[(int64_t)n * ly.K + k], acc[i][j][q]);
      }
    }
  }
}

// ---------------------------------------------------------------- weight packing (index maps: tower_common.h)

struct Pack32Job {
  const float* w[kMaxTowerLayers];
  int64_t off[kMaxTowerLayers + 1];
};

__global__ void k_t32_pack(TowerArgs a, Pack32Job j) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= j.off[a.L]) return;
  int l = 0;
  while (e >= j.off[l + 1]) ++l;
  const TowerLayerDev& ly = a.ly[l];
  const int64_t i = e - j.off[l];
  const int n = (int)(i / ly.K), k = (int)(i % ly.K);
  const float v = j.w[l][i];
  const_cast<float*>(ly.wpf)[tower_wp32_index(n, k, ly.Kp)] = v;
  const_cast<float*>(ly.wtpf)[tower_wtp32_index(n, k, ly.Np)] = v;
}

}  // namespace

// LDS row stride (floats) for the fwd / bwd tiles: the smallest >= maxw,
// multiple of 4, whose A-operand reads (ds_read_b128: lane l reads row l%16,
// dword 4(l/16)) hit all 64 banks exactly once in each of the instruction's
// four 16-lane groups (MI355X_MICROARCH.md, LDS table).
int tower32_lds_ld(int maxw) {
  static const int grp[4][16] = {{0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27},
                                 {4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31},
                                 {32, 33, 34, 35, 44, 45, 46, 47, 52, 53, 54, 55, 56, 57, 58, 59},
                                 {36, 37, 38, 39, 40, 41, 42, 43, 48, 49, 50, 51, 60, 61, 62, 63}};
  for (int ld = (maxw + 3) / 4 * 4; ld < maxw + 256; ld += 4) {
    bool ok = true;
    for (int gi = 0; gi < 4 && ok; ++gi) {
      bool used[64] = {false};
      for (int j = 0; j < 16 && ok; ++j) {
        const int l = grp[gi][j];
        const int addr = (l & 15) * ld + 4 * (l >> 4);
        for (int d = 0; d < 4; ++d) {
          const int b = (addr + d) & 63;
          if (used[b]) {
            ok = false;
            break;
          }
          used[b] = true;
        }
      }
    }
    if (ok) return ld;
  }
  return (maxw + 3) / 4 * 4;
}

// + 64 floats: the A-operand loads run up to 4 k-groups past a row's end
size_t tower32_lds_bytes(const TowerArgs& a) { return ((size_t)2 * BM * a.lds_ld + 64) * sizeof(float); }

static void allow_big_lds32() {
  static const bool once = [] {
    if (hipFuncSetAttribute((const void*)k_t32_fwd, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024) !=
        hipSuccess)
      (void)hipGetLastError();
    if (hipFuncSetAttribute((const void*)k_t32_bwd, hipFuncAttributeMaxDynamicSharedMemorySize, 140 * 1024) !=
        hipSuccess)
      (void)hipGetLastError();
    return true;
  }();
  (void)once;
}

void launch_tower32_fwd(const TowerArgs& a, hipStream_t s) {
  if (a.M == 0) return;
  allow_big_lds32();
  hipLaunchKernelGGL(k_t32_fwd, dim3(a.Mp / BM), dim3(NT), tower32_lds_bytes(a), s, a);
}

void launch_tower32_bwd(const TowerArgs& a, hipStream_t s) {
  if (a.M == 0) return;
  allow_big_lds32();
  hipLaunchKernelGGL(k_t32_bwd, dim3(a.Mp / BM), dim3(NT), tower32_lds_bytes(a), s, a);
}

void launch_tower32_dw(const TowerArgs& a, hipStream_t s) {
  if (a.M == 0) return;
  int tiles = 0;
  for (int l = 0; l < a.L; ++l) tiles += ((a.ly[l].Np / 16 + 3) / 4) * ((a.ly[l].Kp / 16 + 3) / 4);
  const int ndw = tiles * a.dw_splits;
  const int nred = (a.bias_ld + 31) / 32 + (a.dn_part ? (a.dn_C + 31) / 32 : 0);
  hipLaunchKernelGGL(k_t32_dw, dim3(ndw + nred), dim3(256), 0, s, a, ndw);
}

void launch_tower32_pack(const TowerArgs& a, const float* const* w, hipStream_t s) {
  Pack32Job j;
  j.off[0] = 0;
  for (int l = 0; l < a.L; ++l) {
    j.w[l] = w[l];
    j.off[l + 1] = j.off[l] + (int64_t)a.ly[l].N * a.ly[l].K;
  }
  const int64_t n = j.off[a.L];
  if (n == 0) return;
  hipLaunchKernelGGL(k_t32_pack, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a, j);
}

}  // namespace pbx

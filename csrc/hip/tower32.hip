// Fused CTR dense tower in exact fp32 on MI355X: the reference's `fc`
// precision (paddle/phi/kernels/gpu/matmul_kernel.cu runs fp32 GEMMs) with the
// same three-launch structure as the bf16 tower (tower.hip):
//
//   k_t32_fwd  one 256-thread workgroup (ONE wave per SIMD) per 32-row tile;
//              the tile's fp32 activations stay in LDS across all layers;
//              every wave streams packed fp32 weight fragments (2 KB per
//              step: two 16-column blocks x one 16-deep k-group, one dwordx4
//              per lane each) through a register ring and runs
//              v_mfma_f32_16x16x4_f32 on four independent accumulators (2
//              column blocks x 2 row halves).  Epilogue: bias + ReLU -> LDS
//              and the MP32 copy (one dwordx4 per lane: the accumulator IS the
//              dW operand fragment).  Output GEMV, sigmoid, log-loss,
//              d loss/d logit and the AUC histogram fused.
//   k_t32_bwd  same tiling for the dX chain with ReLU masks read from the MP32
//              activations, per-tile column sums for the bias gradients.
//   k_t32_dw   dW = dZ^T X as one grouped GEMM over 64x64 output tiles, both
//              operands streamed HBM/L2 -> LDS by global_load_lds (1 KB per
//              wave instruction), M split over workgroups; each split stores
//              its partial tile (a slab), the last arriving split of a tile
//              sums the slabs in split order (deterministic, no fp32
//              atomics); extra workgroups reduce bias partials and data_norm
//              statistics.
//
// Why one wave per SIMD (tower32_sched.h): with two, the waves shared the
// matrix pipe fully until the first finished its share of a layer, and the
// second then ran its tail at ~1/4 of the MFMA rate (per-wave s_memtime
// stamps, profiles/r5_t32_schedule_ab.txt); rebalancing work between them
// did not move the end.  One wave per SIMD has no tail by construction; its
// latency cover is a deeper register ring (kT32Ring steps = 16 MFMAs each).
// Why 16x16x4 and not 32x32x2: the f32 MFMA rate is 64 FLOP/clk/SIMD either
// way; 16-wide blocks pad a 400-unit layer to 400 (not 416).
#include <hip/hip_runtime.h>

#include "kernels.h"
#include "tower_common.h"

namespace pbx {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int BM = 32;          // rows per fwd / bwd workgroup
constexpr int NW = kT32Waves;   // waves per fwd / bwd workgroup (one per SIMD)
constexpr int NT = NW * 64;     // threads per fwd / bwd workgroup

__device__ __forceinline__ int64_t mp32(int m16, int nb16, int n16) { return ((int64_t)m16 * nb16 + n16) * 256; }

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// The m-packed activation / dZ copies (MP32) are written once per step and
// read once by a later kernel: non-temporal stores and loads stream them past
// L2, which then keeps the layer weights every workgroup re-reads
// (TowerArgs.debug 256: plain accesses, for the A/B).
__device__ __forceinline__ void mp_store(float* p, const f32x4& v, int debug) {
  if (debug & 256)
    *reinterpret_cast<f32x4*>(p) = v;
  else
    __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(p));
}
__device__ __forceinline__ f32x4 mp_load(const float* p, int debug) {
  if (debug & 256) return *reinterpret_cast<const f32x4*>(p);
  return __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
}

// The weight ring: kT32Ring steps of B fragments in flight per wave (two
// dwordx4 per lane each), refilled in stream order right after each step's
// MFMAs with the step kT32Ring ahead -- across unit / segment boundaries
// (tower32_sched.h pads every unit and segment to whole rings), so a unit
// starts with its first fragments in flight instead of cold.
struct Ring {
  f32x4 b[kT32Ring][2];
};

// The wave's stream is read through a buffer resource: the step offset is
// one SGPR add per step (soffset) and the lane offset a constant VGPR, so a
// refill costs two buffer loads and no 64-bit address arithmetic -- with no
// partner wave on the SIMD, every instruction between two MFMA groups that
// does not fit the MFMA's issue shadow is exposed.
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f32x4 ld_frag(__amdgpu_buffer_rsrc_t rs, int voff, int soff) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, 0));
}
__device__ __forceinline__ void ring_fill(Ring& rg, __amdgpu_buffer_rsrc_t rs, int voff) {
#pragma unroll
  for (int r = 0; r < kT32Ring; ++r) {
    rg.b[r][0] = ld_frag(rs, voff, r * 2048);
    rg.b[r][1] = ld_frag(rs, voff + 1024, r * 2048);
  }
}

// steps [0, nsteps) of one unit (PAIR: 2 column blocks x k-group g = step)
// or leftover segment (!PAIR: one block, k-groups 2 step and 2 step + 1 from
// A0 / A1), nsteps a whole number of rings; the MFMAs of steps >= n_real are
// skipped (pads), bp advances past them.  acc[j][h]: column block (PAIR) or
// k-group parity (!PAIR) j, row half h.  The activation fragments (LDS) are
// read one step ahead in an even / odd register pair: with no partner wave on
// the SIMD nothing else would cover the ds_read latency.  Reads past a row's
// end (one step ahead of the last) land in the tile's LDS slack, never used.
// Timing experiment (TowerArgs.debug 64, its own instantiation XP = 64): no
// weight loads in the loop (stale ring).
template <int XP, bool PAIR>
__device__ __forceinline__ void t32_run(Ring& rg, __amdgpu_buffer_rsrc_t rs, int voff, int& sbase, const float* A0,
                                        const float* A1, int n_real, int nsteps, int len, f32x4 (&acc)[2][2]) {
  constexpr int R = kT32Ring;
  static_assert(R % 2 == 0, "the even / odd activation buffers need an even ring");
  constexpr bool noB = XP & 64;
  constexpr int SA = PAIR ? 16 : 32;  // floats of A per step
  struct AF {
    f32x4 a0, a1, c0, c1;
  };
  auto lda = [&](AF& f, int st) {
    f.a0 = *reinterpret_cast<const f32x4*>(A0 + SA * st);
    f.a1 = *reinterpret_cast<const f32x4*>(A1 + SA * st);
    if (!PAIR) {
      f.c0 = *reinterpret_cast<const f32x4*>(A0 + SA * st + 16);
      f.c1 = *reinterpret_cast<const f32x4*>(A1 + SA * st + 16);
    }
  };
  auto step = [&](const AF& f, int r, int st) {
    if (PAIR) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        acc[0][0] = mfma4(f.a0[t], rg.b[r][0][t], acc[0][0]);
        acc[0][1] = mfma4(f.a1[t], rg.b[r][0][t], acc[0][1]);
        acc[1][0] = mfma4(f.a0[t], rg.b[r][1][t], acc[1][0]);
        acc[1][1] = mfma4(f.a1[t], rg.b[r][1][t], acc[1][1]);
      }
    } else {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        acc[0][0] = mfma4(f.a0[t], rg.b[r][0][t], acc[0][0]);
        acc[0][1] = mfma4(f.a1[t], rg.b[r][0][t], acc[0][1]);
      }
      if (2 * st + 1 < len) {  // the step's second k-group (wave-uniform)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          acc[1][0] = mfma4(f.c0[t], rg.b[r][1][t], acc[1][0]);
          acc[1][1] = mfma4(f.c1[t], rg.b[r][1][t], acc[1][1]);
        }
      }
    }
  };
  AF fe, fo;
  lda(fe, 0);
  for (int s0 = 0; s0 < nsteps; s0 += R) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int st = s0 + r;
      AF& cur = (r & 1) ? fo : fe;
      AF& nxt = (r & 1) ? fe : fo;
      lda(nxt, st + 1);
      __builtin_amdgcn_sched_barrier(0);
      if (st < n_real) step(cur, r, st);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (!noB) {
        const int so = (sbase + st + R) * 2048;
        rg.b[r][0] = ld_frag(rs, voff, so);
        rg.b[r][1] = ld_frag(rs, voff + 1024, so);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  sbase += nsteps;
}

// LDS scratch of the leftover partial sums: [waves][kT32MaxSeg][2 halves][64 lanes][4]
constexpr int kPartFloats = kT32Waves * kT32MaxSeg * 2 * 256;

// Workgroup barrier for LDS only: the global stores / loads in flight (MP32
// copies, the next unit's weight fragments) are NOT drained (a
// __syncthreads() fence would wait vmcnt(0)).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// One layer of the wave-stream schedule (tower32_sched.h): this wave's full
// pair units (epi(acc, col, half, pre) after each; pre(col, half) is fetched
// before its MFMA chain so the load hides under it), then its leftover
// range, whose K-partial sums go to LDS.  t32_layer_rem (after an LDS
// barrier) reduces the leftover blocks in wave order -- deterministic -- and
// applies epi.
template <int XP, typename Pre, typename Epi>
__device__ __forceinline__ void t32_layer(const float* src, int ldl, const f32x4* wl, int ncol, int ng, int w,
                                          int lane, float* part, Pre&& pre, Epi&& epi) {
  const int c = lane & 15, g = lane >> 4;
  const T32Sched s = t32_sched(ncol, ng);
  // this wave's stream; the ring reads kT32Ring steps past its end (into the
  // next wave's stream, or the allocation's slack after the last)
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<f32x4*>(wl + t32_wave_off(s, ng, w) * 128), 0, 0x7ffffff0, 0x00020000);
  const int voff = lane * 16;
  int sbase = 0;
  Ring rg;
  ring_fill(rg, rs, voff);
  const float* A0 = src + c * ldl + 4 * g;
  const float* A1 = A0 + 16 * ldl;
  const int ngp = t32_ceil_ring(ng);
  for (int u = 0; u < s.q; ++u) {
    const int col = 2 * (u * NW + w);
    const f32x4 p00 = pre(col, 0), p01 = pre(col, 1), p10 = pre(col + 1, 0), p11 = pre(col + 1, 1);
    __builtin_amdgcn_sched_barrier(0);  // issue the epilogue operands before the chain
    f32x4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    t32_run<XP, true>(rg, rs, voff, sbase, A0, A1, ng, ngp, ng, acc);
    epi(acc[0][0], col, 0, p00);
    epi(acc[0][1], col, 1, p01);
    epi(acc[1][0], col + 1, 0, p10);
    epi(acc[1][1], col + 1, 1, p11);
  }
  if (s.Rb == 0) return;
  const int lo = t32_rem_lo(s, w), hi = t32_rem_lo(s, w + 1);
  int seg = 0;
  for (int f = lo; f < hi; ++seg) {
    const int j = f / ng, g0 = f - j * ng;
    const int len = min(ng - g0, hi - f);
    f32x4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) acc[i][jj] = (f32x4){0.f, 0.f, 0.f, 0.f};
    const int nst = (len + 1) / 2;
    t32_run<XP, false>(rg, rs, voff, sbase, A0 + 16 * g0, A1 + 16 * g0, nst, t32_seg_steps(len), len, acc);
    float* sl = part + ((w * kT32MaxSeg + seg) * 2) * 256 + lane * 4;
    *reinterpret_cast<f32x4*>(sl) = acc[0][0] + acc[1][0];
    *reinterpret_cast<f32x4*>(sl + 256) = acc[0][1] + acc[1][1];
    f += len;
  }
}

template <typename Pre, typename Epi>
__device__ __forceinline__ void t32_layer_rem(int ncol, int ng, int w, int lane, const float* part, Pre&& pre,
                                              Epi&& epi) {
  const T32Sched s = t32_sched(ncol, ng);
  for (int j = w; j < s.Rb; j += NW) {
    const int col = 8 * s.q + j;
    const f32x4 p0 = pre(col, 0), p1 = pre(col, 1);
    const int wa = t32_rem_wave(s, j * ng), wb = t32_rem_wave(s, (j + 1) * ng - 1);
    f32x4 s0 = (f32x4){0.f, 0.f, 0.f, 0.f}, s1 = s0;
    for (int ww = wa; ww <= wb; ++ww) {
      const int lo = t32_rem_lo(s, ww);
      if (lo == t32_rem_lo(s, ww + 1)) continue;  // empty range
      const int seg = j - lo / ng;
      const float* sl = part + ((ww * kT32MaxSeg + seg) * 2) * 256 + lane * 4;
      s0 += *reinterpret_cast<const f32x4*>(sl);
      s1 += *reinterpret_cast<const f32x4*>(sl + 256);
    }
    epi(s0, col, 0, p0);
    epi(s1, col, 1, p1);
  }
}

template <int XP>
__global__ __launch_bounds__(NT) void k_t32_fwd(TowerArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds32[];
  const int ldl = a.lds_ld;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (SGPR): the stream's buffer resource
  const int m0 = blockIdx.x * BM;
  float* src = lds32;
  float* dst = lds32 + BM * ldl;
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
  float* part = lds32 + 2 * BM * ldl + 64;  // leftover partial sums
  // every layer's bias in LDS (at its bias_off): the epilogues then depend
  // on no global load, so hipcc has no reason to drain the weight ring
  float* sbias = part + (a.t32_part ? kPartFloats : 0);
  for (int l = 0; l < a.L; ++l) {
    const TowerLayerDev& ly = a.ly[l];
    for (int n = tid; n < ly.Np; n += NT) sbias[ly.bias_off + n] = n < ly.N ? ly.bias[n] : 0.f;
  }
  __syncthreads();
  for (int l = 0; l < a.L; ++l) {
    const TowerLayerDev& ly = a.ly[l];
    const int NB = ly.Np / 16, KG = ly.Kp / 16;
    const f32x4* wp = reinterpret_cast<const f32x4*>(ly.wpf);
    const int c = lane & 15, g = lane >> 4;
    const float* lb = sbias + ly.bias_off;
    auto pre = [&](int nbb, int) { return (f32x4){lb[nbb * 16 + c], 0.f, 0.f, 0.f}; };
    auto epi = [&](const f32x4& acc, int nbb, int mb, const f32x4& pb) {
      const int n = nbb * 16 + c;
      const float bias = pb[0];
      f32x4 o;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float v = acc[t] + bias;
        o[t] = v > 0.f ? v : 0.f;
        dst[(16 * mb + 4 * g + t) * ldl + n] = o[t];
      }
      if (!(a.debug & 8)) mp_store(ly.xmpf + mp32(m0 / 16 + mb, NB, nbb) + lane * 4, o, a.debug);
    };
    t32_layer<XP>(src, ldl, wp, NB, KG, w, lane, part, pre, epi);
    if (stp && lane == 0) stp[1 + 2 * l] = __builtin_amdgcn_s_memtime();
    lds_barrier();
    if (t32_sched(NB, KG).Rb) {
      t32_layer_rem(NB, KG, w, lane, part, pre, epi);
      lds_barrier();
    }
    if (stp && lane == 0) stp[2 + 2 * l] = __builtin_amdgcn_s_memtime();
    float* t = src;
    src = dst;
    dst = t;
  }
  // output layer: 8 rows per wave, independent accumulations, w_out from
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

template <int XP>
__global__ __launch_bounds__(NT) void k_t32_bwd(TowerArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds32[];
  __shared__ float gs[BM];
  // per-layer column sums of dZ, one row per 16-row half; double-buffered by
  // layer parity so layer i's readers never race layer i-1's writers
  __shared__ float csum[2][2][kTower32MaxWidth];
  const int ldl = a.lds_ld;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (SGPR): the stream's buffer resource
  const int c = lane & 15, g = lane >> 4;
  const int m0 = blockIdx.x * BM;
  float* src = lds32;
  float* dst = lds32 + BM * ldl;
  float* bp = a.bias_part + (int64_t)blockIdx.x * a.bias_ld;
  float* part = lds32 + 2 * BM * ldl + 64;  // leftover partial sums
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
      const f32x4 x4 = mp_load(lastl.xmpf + off, a.debug);
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
      mp_store(lastl.dzmpf + off, o, a.debug);
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
      auto pre = [&](int kbb, int mb) {
        return mp_load(prev.xmpf + mp32(m0 / 16 + mb, PNB, kbb) + lane * 4, a.debug);
      };
      auto epi = [&](const f32x4& acc, int kbb, int mb, const f32x4& x4) {
        const int64_t off = mp32(m0 / 16 + mb, PNB, kbb) + lane * 4;
        f32x4 o;
        float s = 0.f;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          o[t] = x4[t] > 0.f ? acc[t] : 0.f;
          s += o[t];
          dst[(16 * mb + 4 * g + t) * ldl + kbb * 16 + c] = o[t];
        }
        if (!(a.debug & 8)) mp_store(prev.dzmpf + off, o, a.debug);
        s += __shfl_xor(s, 16);
        s += __shfl_xor(s, 32);
        if (g == 0) cs[mb][kbb * 16 + c] = s;
      };
      t32_layer<XP>(src, ldl, wtp, KB, NG, w, lane, part, pre, epi);
      lds_barrier();
      if (t32_sched(KB, NG).Rb) {
        t32_layer_rem(KB, NG, w, lane, part, pre, epi);
        lds_barrier();
      }
      for (int col = tid; col < prev.Np; col += NT) bp[prev.bias_off + col] = cs[0][col] + cs[1][col];
    } else {
      auto pre = [&](int, int) { return (f32x4){0.f, 0.f, 0.f, 0.f}; };
      auto epi = [&](const f32x4& acc, int kbb, int mb, const f32x4&) {
#pragma unroll
        for (int t = 0; t < 4; ++t) dst[(16 * mb + 4 * g + t) * ldl + kbb * 16 + c] = acc[t];
      };
      t32_layer<XP>(src, ldl, wtp, KB, NG, w, lane, part, pre, epi);
      lds_barrier();
      if (t32_sched(KB, NG).Rb) {
        t32_layer_rem(KB, NG, w, lane, part, pre, epi);
        lds_barrier();
      }
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
// Ring of NS stages of DS m16 steps each (8 KB of dZ + X chunks per step).
// Stage s+NS-1 is issued while stage s is consumed, so NS-1 stages (the
// latency budget) are in flight.  Variants (PBX_T32_DW_RING = DSxNS):
// 2x3 (48 KB, two workgroups per CU beside the head backward), 1x6 (48 KB,
// deeper in time), 2x4 (64 KB), 2x5 (80 KB).
constexpr int kDwStep = 8 * 256;  // floats per m16 step: 8 chunks of 1 KB (4 dZ, 4 X)

__device__ __forceinline__ int dw32_tiles(const TowerLayerDev& ly) {
  return ((ly.Np / 16 + 3) / 4) * ((ly.Kp / 16 + 3) / 4);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// wait until at most `ahead` stages of 2*DS loads are outstanding
template <int DS>
__device__ __forceinline__ void wait_stages(int ahead) {
  switch (ahead) {
    case 0: wait_vm<0>(); break;
    case 1: wait_vm<2 * DS>(); break;
    case 2: wait_vm<4 * DS>(); break;
    case 3: wait_vm<6 * DS>(); break;
    default: wait_vm<8 * DS>(); break;
  }
}

// Split-M combine of one 64x64 dW tile (256 threads, wave w owns the 16x16
// blocks part[w][i][j], i, j < 2, as 16x16x4 accumulators: lane (c, g),
// register q = element [16 i' + 4g + q][16 j' + c]).  S = 1: the tile is
// added to dW directly.  Otherwise every split writes its partial to its slab
// (plain 16-B stores, 1 KB per wave instruction), publishes it with one
// agent-scope release and an arrival on the tile's counter; the split that
// arrives last acquires, sums the S slabs in split order 0..S-1 (the result
// does not depend on which split finished last, or where it ran) and adds the
// sum to dW -- one writer per element, so dW keeps its accumulate (+=)
// contract and the update is bit-reproducible.  flag: one LDS int.
// (MI355X_MICROARCH.md / cdna_hip_programming.md: the counter form of the
// split-K hand-off, release before the ticket, acquire in the reducer.)
__device__ __forceinline__ void t32_dw_combine(const TowerArgs& a, const TowerLayerDev& ly, int tile_g, int split,
                                               int tn, int tk, int w, int lane, bool active, const f32x4 (&acc)[2][2],
                                               int* flag) {
  const int S = a.dw_splits;
  const int NBn = ly.Np / 16, NBk = ly.Kp / 16;
  const int wn = w & 1, wk = w >> 1;
  const int c = lane & 15, g = lane >> 4;
  auto add_out = [&](int i, int j, const f32x4& v) {
    const int nb = tn * 4 + 2 * wn + i, kb = tk * 4 + 2 * wk + j;
    const int k = kb * 16 + c;
    if (nb >= NBn || kb >= NBk || k >= ly.K) return;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int n = nb * 16 + 4 * g + q;
      if (n < ly.N) ly.dw[(int64_t)n * ly.K + k] += v[q];
    }
  };
  if (S == 1) {
    if (active) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) add_out(i, j, acc[i][j]);
    }
    return;
  }
  float* tile_slab = a.dw_slab + (int64_t)tile_g * S * 4096;
  // slab layout: [split][wave][i][j][lane][4] (inactive waves write zeros:
  // every slab is whole, the reducer reads them unconditionally).  Stored
  // write-through (sc1: the line leaves this XCD's L2 with the store), so the
  // publish needs no L2 write-back fence -- a release per workgroup
  // (buffer_wbl2, ~1.7-6.5 us each) cost the 1064-workgroup launch ~12 us.
  {
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(tile_slab + (int64_t)split * 4096, 0, 4096 * 4, 0x00020000);
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const f32x4 v = active ? acc[i][j] : (f32x4){0.f, 0.f, 0.f, 0.f};
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rs,
                                               ((w * 4 + i * 2 + j) * 64 + lane) * 16, 0, 16 /* sc1 */);
      }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const int old = __hip_atomic_fetch_add(&a.dw_cnt[tile_g], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == S - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      // the next launch starts from zero (a dispatch boundary orders it)
      __hip_atomic_store(&a.dw_cnt[tile_g], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    *flag = last;
  }
  __syncthreads();
  if (!*flag || !active) return;
  f32x4 sum[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) sum[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const f32x4* base = reinterpret_cast<const f32x4*>(tile_slab) + w * 4 * 64 + lane;
  for (int sp = 0; sp < S; ++sp) {
    const f32x4* src = base + (int64_t)sp * 1024;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) sum[i][j] += src[(i * 2 + j) * 64];
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) add_out(i, j, sum[i][j]);
}

template <int DS, int NS>
__global__ __launch_bounds__(256) void k_t32_dw(TowerArgs a, int ndw) {
  static_assert(NS >= 3 && NS - 2 <= 4, "wait_stages covers up to 4 stages ahead");
  constexpr int DSTEPS = DS, DNST = NS, DSTAGE = DS * kDwStep;
  const int tid = threadIdx.x;
  if ((int)blockIdx.x >= ndw) {
    tower_col_reduce(a, (int)blockIdx.x - ndw, BM);
    return;
  }
  extern __shared__ __attribute__((aligned(16))) float smem[];
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
  const int tile_g = t;  // tile index over all layers (slab / counter)
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
    // stages s .. s + ahead are outstanding; stage s must have landed
    wait_stages<DSTEPS>(min(DNST - 2, nstage - 1 - s));
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
  // the ring's LDS is free: its first word carries the reducer flag
  __syncthreads();
  t32_dw_combine(a, ly, tile_g, split, tn, tk, w, lane, active, acc, reinterpret_cast<int*>(smem));
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
  const_cast<float*>(ly.wpf)[tower_wp32_index(n, k, ly.Np, ly.Kp)] = v;
  const_cast<float*>(ly.wtpf)[tower_wtp32_index(n, k, ly.Np, ly.Kp)] = v;
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

// + 64 floats: the A-operand loads run one k-group past a row's end; then the
// remainder partial sums of the wave-stream schedule when a layer has column
// blocks past a multiple of 8 (fwd: Np / 16, bwd: Kp / 16)
bool tower32_needs_part(const TowerArgs& a) {
  for (int l = 0; l < a.L; ++l)
    if (t32_sched(a.ly[l].Np / 16, a.ly[l].Kp / 16).Rb || t32_sched(a.ly[l].Kp / 16, a.ly[l].Np / 16).Rb) return true;
  return false;
}
size_t tower32_lds_bytes_for(int lds_ld, bool part, int bias_floats) {
  return ((size_t)2 * BM * lds_ld + 64 + (part ? kPartFloats : 0) + bias_floats) * sizeof(float);
}
// forward: + the layers' biases
static size_t fwd_lds_bytes(const TowerArgs& a) {
  return tower32_lds_bytes_for(a.lds_ld, a.t32_part != 0, a.ly[a.L - 1].bias_off + a.ly[a.L - 1].Np);
}
size_t tower32_lds_bytes(const TowerArgs& a) { return tower32_lds_bytes_for(a.lds_ld, tower32_needs_part(a), 0); }

template <int XP>
static void allow_big_lds32_xp() {
  // 160 KB per CU minus each kernel's static LDS (zrow; gs + csum)
  if (hipFuncSetAttribute((const void*)k_t32_fwd<XP>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          kTower32LdsTotal - 512) != hipSuccess)
    (void)hipGetLastError();
  if (hipFuncSetAttribute((const void*)k_t32_bwd<XP>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          kTower32LdsTotal - kTower32BwdStatic) != hipSuccess)
    (void)hipGetLastError();
}
static void allow_big_lds32() {
  static const bool once = [] {
    allow_big_lds32_xp<0>();
    allow_big_lds32_xp<64>();
    return true;
  }();
  (void)once;
}

void launch_tower32_fwd(const TowerArgs& a, hipStream_t s) {
  if (a.M == 0) return;
  allow_big_lds32();
  TowerArgs b = a;
  b.t32_part = tower32_needs_part(a) ? 1 : 0;
  // timing experiments (TowerArgs.debug 64 / 128) run their own instantiations
  if (a.debug & 64) hipLaunchKernelGGL(k_t32_fwd<64>, dim3(a.Mp / BM), dim3(NT), fwd_lds_bytes(b), s, b);
  else hipLaunchKernelGGL(k_t32_fwd<0>, dim3(a.Mp / BM), dim3(NT), fwd_lds_bytes(b), s, b);
}

void launch_tower32_bwd(const TowerArgs& a, hipStream_t s) {
  if (a.M == 0) return;
  allow_big_lds32();
  TowerArgs b = a;
  b.t32_part = tower32_needs_part(a) ? 1 : 0;
  if (a.debug & 64) hipLaunchKernelGGL(k_t32_bwd<64>, dim3(a.Mp / BM), dim3(NT), tower32_lds_bytes(b), s, b);
  else hipLaunchKernelGGL(k_t32_bwd<0>, dim3(a.Mp / BM), dim3(NT), tower32_lds_bytes(b), s, b);
}

void launch_tower32_dw(const TowerArgs& a, hipStream_t s) {
  if (a.M == 0) return;
  int tiles = 0;
  for (int l = 0; l < a.L; ++l) tiles += ((a.ly[l].Np / 16 + 3) / 4) * ((a.ly[l].Kp / 16 + 3) / 4);
  const int ndw = tiles * a.dw_splits;
  const int nred = (a.bias_ld + 31) / 32 + (a.dn_part ? (a.dn_C + 31) / 32 : 0);
  static const int ring = [] {
    const char* e = getenv("PBX_T32_DW_RING");
    // DS * 10 + NS of the LDS ring (default 2x3).  Same box, tower dW alone:
    // 2x3 99.9 us, 1x6 106.9; a register-streamed variant (no LDS) measured
    // 110-117 and was removed (profiles/r4_dw_variants.txt)
    return e ? atoi(e) : 23;
  }();
  const dim3 g(ndw + nred), b(256);
  switch (ring) {
    case 16: {
      static const bool big = hipFuncSetAttribute((const void*)k_t32_dw<1, 6>,
                                                  hipFuncAttributeMaxDynamicSharedMemorySize, 6 * kDwStep * 4) ==
                              hipSuccess;
      (void)big;
      hipLaunchKernelGGL((k_t32_dw<1, 6>), g, b, 6 * kDwStep * 4, s, a, ndw);
      break;
    }
    case 24: {
      static const bool big = hipFuncSetAttribute((const void*)k_t32_dw<2, 4>,
                                                  hipFuncAttributeMaxDynamicSharedMemorySize, 8 * kDwStep * 4) ==
                              hipSuccess;
      (void)big;
      hipLaunchKernelGGL((k_t32_dw<2, 4>), g, b, 8 * kDwStep * 4, s, a, ndw);
      break;
    }
    case 25: {
      static const bool big = hipFuncSetAttribute((const void*)k_t32_dw<2, 5>,
                                                  hipFuncAttributeMaxDynamicSharedMemorySize, 10 * kDwStep * 4) ==
                              hipSuccess;
      (void)big;
      hipLaunchKernelGGL((k_t32_dw<2, 5>), g, b, 10 * kDwStep * 4, s, a, ndw);
      break;
    }
    default: {
      // PBX_T32_DW_LDS: LDS bytes a 2x3 workgroup reserves (>= its 48 KB ring).
      // More caps the dW workgroups per CU (160 KB / bytes) and leaves LDS for
      // the sparse kernels running beside it (the table dedup needs 12 KB).
      // Default 64 KB: two per CU -- the dW alone is slower (110 vs 100 us)
      // but the pipelined step beside it faster (0.383 vs 0.397 ms/step;
      // 80 KB 0.404), profiles/r4_dw_lds_ab.txt
      static const int lds = [] {
        const char* e = getenv("PBX_T32_DW_LDS");
        const int v = e ? atoi(e) : 64 * 1024;
        return v > 6 * kDwStep * 4 ? (v < 150 * 1024 ? v : 150 * 1024) : 6 * kDwStep * 4;
      }();
      if (lds > 64 * 1024) {
        static const bool big = hipFuncSetAttribute((const void*)k_t32_dw<2, 3>,
                                                    hipFuncAttributeMaxDynamicSharedMemorySize, lds) == hipSuccess;
        (void)big;
      }
      hipLaunchKernelGGL((k_t32_dw<2, 3>), g, b, lds, s, a, ndw);
    }
  }
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

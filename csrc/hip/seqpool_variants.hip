// fused_seqpool_cvm variant family and fused_seq_tensor, hand-written for gfx950.
//
// The reference ships one CUDA op per variant (fused_seqpool_cvm_with_conv /
// _with_pcoc / _tradew / _with_credit / _with_diff_thres, each with its own
// forward and grad kernels, fused_seqpool_cvm_*_op.cu).  Here the variants
// share two kernels: the pre-pool work (show/click filter, embedding-norm
// filter, quantisation, trade weighting, embedx_concate blocks) is a handful
// of flags, and the per-variant CVM epilogue / gradient are column tables
// built on the host (ops/ctr_ext.py _spv_tables), so a new variant is a new
// table, not a new kernel.
//
// One wave owns one (slot, instance) sequence: lanes stride the columns, the
// pooled row lives in LDS for the epilogue's cross-column reads.
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace pbx {
namespace {

constexpr int kSpvWaves = 4;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// value of record column c after the quantiser (trunc(v*q + 0.5) / q for
// columns >= mcol), rounding exactly like the fp32 torch expression
__device__ __forceinline__ float qval(const SpvArgs& a, const float* xr, int c) {
  const float v = xr[c];
  if (!a.quant || c < a.mcol) return v;
  const float q = (float)a.quant;
  return truncf(__fadd_rn(__fmul_rn(v, q), 0.5f)) / q;
}

__device__ __forceinline__ bool keep_record(const SpvArgs& a, const float* xr, int s, int lane) {
  bool keep = true;
  if (a.need_filter) {
    const float show = xr[0], clk = a.E > 1 ? xr[1] : xr[0];
    keep = __fadd_rn(__fmul_rn(show - clk, a.show_coeff), __fmul_rn(clk, a.clk_coeff)) >= a.thr[s];
  }
  if (a.embed_filter) {
    float sq = 0.f;
    for (int e = 1 + lane; e < a.ets; e += 64) {
      const float v = xr[a.co + e];
      sq += v * v;
    }
    sq = wave_sum(sq);
    keep = keep && (sqrtf(sq) + fabsf(xr[a.co]) >= a.embed_threshold);
  }
  return keep;
}

__global__ __launch_bounds__(256) void k_spv_fwd(SpvArgs a) {
  extern __shared__ float lds[];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int PW = a.ecs * a.Epool;
  float* pool = lds + w * PW;
  const int64_t item = (int64_t)blockIdx.x * kSpvWaves + w;
  const bool valid = item < (int64_t)a.S * a.B;
  const int s = valid ? (int)(item / a.B) : 0, b = valid ? (int)(item % a.B) : 0;
  for (int e = lane; e < PW; e += 64) pool[e] = 0.f;
  if (valid) {
    const int* off = a.off + (int64_t)s * (a.B + 1);
    const int beg = off[b], end = off[b + 1];
    const float* xs = a.x + (int64_t)a.row_base[s] * a.E;
    for (int r = beg; r < end; ++r) {
      const int k = r - beg;
      if (a.ecs > 1 && k >= a.ecs) break;
      const float* xr = xs + (int64_t)r * a.E;
      if (!keep_record(a, xr, s, lane)) continue;  // wave-uniform
      const float wgt = (a.tradew && a.tid >= 0) ? qval(a, xr, a.co + a.tid) : 1.f;
      float* pb = pool + (a.ecs > 1 ? k * a.Epool : 0);
      for (int e = lane; e < a.Epool; e += 64) {
        const bool emb = a.tradew && e >= a.co;
        pb[e] += emb ? qval(a, xr, e + a.tn) * wgt : qval(a, xr, e);  // same lane owns column e
      }
    }
  }
  __syncthreads();
  if (!valid) return;
  float* o = a.out + item * (int64_t)(a.ecs * a.Eo);
  for (int blk = 0; blk < a.ecs; ++blk) {
    const float* pb = pool + blk * a.Epool;
    for (int c = lane; c < a.Eo; c += 64) {
      const int code = a.ftab[c];
      const int op = code >> 24, s1 = (code >> 12) & 0xfff, s2 = code & 0xfff;
      const float p1 = pb[s1] + a.pad;
      float v;
      if (op == 0) v = p1;
      else if (op == 1) v = logf(p1 + 1.f);
      else v = logf(p1 + 1.f) - logf(pb[s2] + a.pad + 1.f);
      o[blk * a.Eo + c] = v;
    }
  }
}

// dx[r] = the pooled gradient of r's sequence (block min(pos, ecs-1) under
// embedx_concate), statistic columns from the CVM input; trade weighting
// routes the embedding gradient through the weight column.
__global__ __launch_bounds__(256) void k_spv_bwd(SpvArgs a) {
  extern __shared__ float lds[];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int PW = a.ecs * a.Epool;
  float* g = lds + w * PW;
  const int64_t item = (int64_t)blockIdx.x * kSpvWaves + w;
  const bool valid = item < (int64_t)a.S * a.B;
  const int s = valid ? (int)(item / a.B) : 0, b = valid ? (int)(item % a.B) : 0;
  if (valid) {
    const float* d = a.dout + item * (int64_t)(a.ecs * a.Eo);
    for (int blk = 0; blk < a.ecs; ++blk)
      for (int e = lane; e < a.Epool; e += 64) {
        const int code = a.btab[e];
        const int op = code >> 24, idx = code & 0xffffff;
        float v = 0.f;
        if (op == 1) v = a.cvm[(int64_t)b * a.ncv + idx];
        else if (op == 2) v = a.qv[(int64_t)b * a.nq + idx];
        else if (op == 3) v = d[blk * a.Eo + idx];
        g[blk * a.Epool + e] = v;
      }
  }
  __syncthreads();
  if (!valid) return;
  const int* off = a.off + (int64_t)s * (a.B + 1);
  const int beg = off[b], end = off[b + 1];
  const int64_t base = a.row_base[s];
  for (int r = beg; r < end; ++r) {
    const int k = a.ecs > 1 ? min(r - beg, a.ecs - 1) : 0;
    const float* gb = g + k * a.Epool;
    float* dr = a.dx + (base + r) * a.E;
    if (!a.tradew) {
      for (int e = lane; e < a.E; e += 64) dr[e] = gb[e];
      continue;
    }
    const float* xr = a.x + (base + r) * a.E;
    const int nemb = a.Epool - a.co;
    const float wv = a.tid >= 0 ? xr[a.co + a.tid] : 1.f;
    float dot = 0.f;
    for (int j = lane; j < nemb; j += 64) {
      const float ge = gb[a.co + j];
      dr[a.co + a.tn + j] = ge * wv;
      dot += ge * xr[a.co + a.tn + j];
    }
    dot = wave_sum(dot);
    for (int e = lane; e < a.co + a.tn; e += 64) {
      float v = 0.f;
      if (e < a.co) v = a.tid >= 0 ? 0.f : gb[e];
      else if (a.tid >= 0 && e == a.co + a.tid) v = dot;
      dr[e] = v;
    }
  }
}

// one wave per (batch block, instance, step t): lanes stride the S*E record
__global__ __launch_bounds__(256) void k_fused_seq_tensor(const float* __restrict__ x, const float* __restrict__ ad,
                                                          int ins, int bc, int T, int E, int S, int A, int ad_off,
                                                          float* __restrict__ din, float* __restrict__ mask,
                                                          float* __restrict__ side, float* __restrict__ sess) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t item = (int64_t)blockIdx.x * 4 + w;
  if (item >= (int64_t)bc * ins * T) return;
  const int t = (int)(item % T);
  const int i = (int)((item / T) % ins);
  const int p = (int)(item / ((int64_t)T * ins));
  const int side_off = ad_off == 0 ? A : 0;
  const int SA = S - A;
  float sum = 0.f;
  // x[i][p][slot][t][e]
  const float* xb = x + ((int64_t)i * bc + p) * S * T * E;
  const float* ab = ad + ((int64_t)i * bc + p) * A * E;
  float* dn = din + item * 4 * A * E;
  for (int u = lane; u < S * E; u += 64) {
    const int slot = u / E, e = u % E;
    const float v = xb[((int64_t)slot * T + t) * E + e];
    sum += v;
    const int as = slot - ad_off;
    if (as >= 0 && as < A) {
      const float av = ab[as * E + e];
      const int c = as * E + e;
      dn[c] = v;
      dn[A * E + c] = av;
      dn[2 * A * E + c] = v - av;
      dn[3 * A * E + c] = v * av;
      sess[item * A * E + c] = v;
    }
    const int ss = slot - side_off;
    if (ss >= 0 && ss < SA) side[item * SA * E + ss * E + e] = v;
  }
  sum = wave_sum(sum);
  if (lane == 0) mask[item] = fabsf(sum) > 1e-8f ? 1.f : 0.f;
}

}  // namespace

void launch_spv_fwd(const SpvArgs& a, hipStream_t s) {
  const int64_t items = (int64_t)a.S * a.B;
  if (items == 0) return;
  const size_t lds = (size_t)kSpvWaves * a.ecs * a.Epool * sizeof(float);
  hipLaunchKernelGGL(k_spv_fwd, dim3((unsigned)((items + kSpvWaves - 1) / kSpvWaves)), dim3(64 * kSpvWaves), lds, s,
                     a);
}

void launch_spv_bwd(const SpvArgs& a, hipStream_t s) {
  const int64_t items = (int64_t)a.S * a.B;
  if (items == 0) return;
  const size_t lds = (size_t)kSpvWaves * a.ecs * a.Epool * sizeof(float);
  hipLaunchKernelGGL(k_spv_bwd, dim3((unsigned)((items + kSpvWaves - 1) / kSpvWaves)), dim3(64 * kSpvWaves), lds, s,
                     a);
}

void launch_fused_seq_tensor(const float* x, const float* ad, int ins, int bc, int T, int E, int S, int A, int ad_off,
                             float* din, float* mask, float* side, float* sess, hipStream_t s) {
  const int64_t items = (int64_t)bc * ins * T;
  if (items == 0) return;
  hipLaunchKernelGGL(k_fused_seq_tensor, dim3((unsigned)((items + 3) / 4)), dim3(256), 0, s, x, ad, ins, bc, T, E, S,
                     A, ad_off, din, mask, side, sess);
}

}  // namespace pbx

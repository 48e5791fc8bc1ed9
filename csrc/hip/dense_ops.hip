// Dense CTR kernels: data_norm, DeepFM FM term, fused sigmoid+logloss, device
// AUC histogram, flat Adam.
//
// Reference behaviour:
//   data_norm      paddle/fluid/operators/data_norm_op.cu:38-104,193-253
//   auc            paddle/phi/kernels/gpu/auc_kernel.cu:25-80, fleet/metrics.cc:38-54
//   adam           paddle/phi/kernels/gpu/adam_kernel.cu
// data_norm's backward reduces every column over the batch: here one
// workgroup owns a 64-column strip and its 4 waves split the rows, reducing
// through LDS (the reference walks all N rows with one thread per column).
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace pbx {
namespace {

inline unsigned int nblk(int64_t n, int per = 256) {
  int64_t b = (n + per - 1) / per;
  return (unsigned int)(b < 1 ? 1 : b);
}

// ---------------------------------------------------------------- data_norm
__global__ void k_dn_fwd(const float* __restrict__ x, int N, int C, const float* __restrict__ bsize,
                         const float* __restrict__ bsum, const float* __restrict__ bsq, float* __restrict__ y,
                         float* __restrict__ means, float* __restrict__ scales, const float* scale_w,
                         const float* bias) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)N * C) return;
  const int c = (int)(i % C);
  const float mean = bsum[c] / bsize[c];
  const float scale = sqrtf(bsize[c] / bsq[c]);
  float v = (x[i] - mean) * scale;
  if (scale_w) v = v * scale_w[c] + bias[c];
  y[i] = v;
  if (i < C) {
    means[c] = mean;
    scales[c] = scale;
  }
}

// grid: (ceil(C/64), row chunks of 64); block 256 = 4 waves; lane -> column,
// wave -> row phase.  Partial column sums go to acc[2, C] with one atomic per
// column per block; k_dn_finish turns them into the summary stats.
constexpr int kDnRows = 64;
__global__ __launch_bounds__(256) void k_dn_bwd(const float* __restrict__ x, const float* __restrict__ dy, int N,
                                                int C, const float* __restrict__ means,
                                                const float* __restrict__ scales, float* __restrict__ dx,
                                                float* __restrict__ acc, const float* scale_w) {
  __shared__ float s_sum[4][64];
  __shared__ float s_sq[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const int r0 = blockIdx.y * kDnRows;
  const int r1 = min(N, r0 + kDnRows);
  float sum = 0.f, sq = 0.f;
  if (c < C) {
    const float mean = means[c];
    const float sc = scales[c] * (scale_w ? scale_w[c] : 1.f);
    for (int r = r0 + w; r < r1; r += 4) {
      const int64_t i = (int64_t)r * C + c;
      const float xv = x[i];
      sum += xv;
      const float d = xv - mean;
      sq += d * d;
      if (dx) dx[i] = dy[i] * sc;
    }
  }
  s_sum[w][lane] = sum;
  s_sq[w][lane] = sq;
  __syncthreads();
  if (w == 0 && c < C) {
    atomicAdd(&acc[c], s_sum[0][lane] + s_sum[1][lane] + s_sum[2][lane] + s_sum[3][lane]);
    atomicAdd(&acc[C + c], s_sq[0][lane] + s_sq[1][lane] + s_sq[2][lane] + s_sq[3][lane]);
  }
}

__global__ void k_dn_finish(const float* __restrict__ acc, int C, int N, float eps, float* __restrict__ stats) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  stats[c] = 1.f;
  stats[C + c] = acc[c] / (float)N;
  stats[2 * C + c] = acc[C + c] / (float)N + eps;
}

__global__ void k_dn_update(float* bsize, float* bsum, float* bsq, const float* __restrict__ st, int C,
                            float decay) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  bsize[c] = bsize[c] * decay + st[c];
  bsum[c] = bsum[c] * decay + st[C + c];
  bsq[c] = bsq[c] * decay + st[2 * C + c];
}

// ---------------------------------------------------------------- FM
__global__ void k_fm_fwd(const float* __restrict__ x, int B, int S, int D, int rs, int col0, int fstride,
                         float* __restrict__ out) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const float* r = x + (int64_t)b * rs + col0;
  float acc = 0.f;
  for (int d = 0; d < D; ++d) {
    float s1 = 0.f, s2 = 0.f;
    for (int s = 0; s < S; ++s) {
      const float v = r[s * fstride + d];
      s1 += v;
      s2 += v * v;
    }
    acc += s1 * s1 - s2;
  }
  out[b] = 0.5f * acc;
}

__global__ void k_fm_bwd(const float* __restrict__ x, const float* __restrict__ dout, int B, int S, int D,
                         int rs, int col0, int fstride, float* __restrict__ dx, int dxs, int accumulate) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const float* r = x + (int64_t)b * rs + col0;
  float* o = dx + (int64_t)b * dxs + col0;
  const float g = dout[b];
  for (int d = 0; d < D; ++d) {
    float s1 = 0.f;
    for (int s = 0; s < S; ++s) s1 += r[s * fstride + d];
    for (int s = 0; s < S; ++s) {
      const float v = g * (s1 - r[s * fstride + d]);
      if (accumulate) o[s * fstride + d] += v; else o[s * fstride + d] = v;
    }
  }
}

// ---------------------------------------------------------------- loss
__global__ void k_sigmoid_logloss(const float* __restrict__ z, const float* __restrict__ y, int B,
                                  float* __restrict__ pred, float* __restrict__ loss_sum,
                                  float* __restrict__ dz, float gs) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  float l = 0.f;
  if (i < B) {
    const float zi = z[i], yi = y[i];
    const float p = 1.f / (1.f + expf(-zi));
    pred[i] = p;
    // stable BCE-with-logits
    l = fmaxf(zi, 0.f) - zi * yi + log1pf(expf(-fabsf(zi)));
    dz[i] = (p - yi) * gs;
  }
  for (int off = 32; off > 0; off >>= 1) l += __shfl_down(l, off);
  if ((threadIdx.x & 63) == 0 && loss_sum) atomicAdd(loss_sum, l);
}

// logit = a + b (deep + wide/FM parts), sigmoid, log-loss mean and its
// gradient in ONE launch (replaces the add, loss zero-fill, loss kernel,
// scale and bias-grad reduction kernels).  One 1024-thread block: the loss
// mean is a plain store, no zero-initialised accumulator.
// One element per thread over many blocks (a single 1024-thread block left
// the chip idle for ~11 us at B=8192).  Each block writes its partial loss
// sum; the last block to arrive (ticket counter) adds the partials in block
// order, so the mean is deterministic, and re-arms the ticket for the next
// launch (graph-replay safe).  The ticket + partials live in a caller-owned
// workspace (one per stream at the call site), so launches on different
// streams cannot interleave on one counter.
constexpr int kLossBlock = 256;

__global__ __launch_bounds__(kLossBlock) void k_logit_loss(const float* __restrict__ a, const float* __restrict__ b,
                                                           const float* __restrict__ y, int B, int per_thread,
                                                           float* __restrict__ pred, float* __restrict__ dz,
                                                           float* __restrict__ loss_mean, unsigned int* ticket,
                                                           float* part) {
  __shared__ float red[kLossBlock / 64];
  __shared__ bool last;
  const float inv = 1.f / (float)B;
  float l = 0.f;
  const int base = blockIdx.x * kLossBlock * per_thread + threadIdx.x;
  for (int k = 0; k < per_thread; ++k) {
    const int i = base + k * kLossBlock;
    if (i < B) {
      const float zi = a[i] + (b ? b[i] : 0.f), yi = y[i];
      const float p = 1.f / (1.f + __expf(-zi));
      pred[i] = p;
      l += fmaxf(zi, 0.f) - zi * yi + log1pf(__expf(-fabsf(zi)));
      dz[i] = (p - yi) * inv;
    }
  }
  for (int off = 32; off > 0; off >>= 1) l += __shfl_down(l, off);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = l;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int w = 0; w < kLossBlock / 64; ++w) s += red[w];
    part[blockIdx.x] = s;
    __threadfence();
    last = atomicAdd(ticket, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (last && threadIdx.x == 0) {
    __threadfence();
    float s = 0.f;
    for (unsigned int k = 0; k < gridDim.x; ++k) s += __hip_atomic_load(&part[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    loss_mean[0] = s * inv;
    *ticket = 0u;
  }
}

// ---------------------------------------------------------------- AUC
// Predictions of a converged CTR model pile up in a few buckets, so each
// block first counts its kAucItems*256 samples per bucket in an LDS hash
// (integer LDS atomics) and then issues one fp64 global atomic per distinct
// bucket; the five error sums are block-reduced to one atomic each.
constexpr int kAucItems = 4;
constexpr int kAucLds = 2048;
__global__ __launch_bounds__(256) void k_auc(const float* __restrict__ pred, const float* __restrict__ label,
                                             const float* __restrict__ mask, int B, int T,
                                             double* __restrict__ table, double* __restrict__ stats) {
  __shared__ int32_t hk[kAucLds];
  __shared__ int32_t hc[kAucLds];
  __shared__ double red[5][4];
  for (int e = threadIdx.x; e < kAucLds; e += blockDim.x) {
    hk[e] = -1;
    hc[e] = 0;
  }
  __syncthreads();
  double ae = 0, se = 0, ps = 0, ls = 0, cnt = 0;
#pragma unroll
  for (int t = 0; t < kAucItems; ++t) {
    const int i = (blockIdx.x * kAucItems + t) * blockDim.x + threadIdx.x;
    if (i >= B || (mask && mask[i] == 0.f)) continue;
    const float p = pred[i];
    const int lab = label[i] > 0.5f ? 1 : 0;
    int pos = (int)(p * T);
    pos = pos < 0 ? 0 : (pos > T - 1 ? T - 1 : pos);
    const int key = lab * T + pos;
    unsigned e = ((unsigned)key * 2654435761u) >> 21;  // 11 bits
    for (;;) {
      const int old = atomicCAS(&hk[e], -1, key);
      if (old == -1 || old == key) break;
      e = (e + 1) & (kAucLds - 1);
    }
    atomicAdd(&hc[e], 1);
    const double d = (double)p - (double)lab;
    ae += fabs(d);
    se += d * d;
    ps += p;
    ls += lab;
    cnt += 1;
  }
  for (int off = 32; off > 0; off >>= 1) {
    ae += __shfl_down(ae, off);
    se += __shfl_down(se, off);
    ps += __shfl_down(ps, off);
    ls += __shfl_down(ls, off);
    cnt += __shfl_down(cnt, off);
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    red[0][w] = ae;
    red[1][w] = se;
    red[2][w] = ps;
    red[3][w] = ls;
    red[4][w] = cnt;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < kAucLds; e += blockDim.x)
    if (hk[e] >= 0) atomicAdd(&table[hk[e]], (double)hc[e]);
  if (threadIdx.x < 5 && red[4][0] + red[4][1] + red[4][2] + red[4][3] > 0)
    atomicAdd(&stats[threadIdx.x],
              red[threadIdx.x][0] + red[threadIdx.x][1] + red[threadIdx.x][2] + red[threadIdx.x][3]);
}

// ---------------------------------------------------------------- Adam (flat)
// beta powers live on the device (pows[0]=beta1^t, pows[1]=beta2^t) so the
// whole optimizer step can be replayed from a HIP graph.
__global__ void k_adam_pows(float* pows, float b1, float b2) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    pows[0] *= b1;
    pows[1] *= b2;
  }
}

// clear_grad: zero the gradient after consuming it, so the next backward can
// accumulate into it without a separate zero-fill launch
__global__ void k_adam(float* __restrict__ p, float* __restrict__ g, float* __restrict__ m,
                       float* __restrict__ v, int64_t n, float lr, float b1, float b2, float eps,
                       const float* __restrict__ pows, float gs, float wd, int clear_grad) {
  const int64_t i4 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const float b1pow = pows[0], b2pow = pows[1];
  const float lr_t = lr * sqrtf(1.f - b2pow) / (1.f - b1pow);
  if ((i4 + 1) * 4 <= n) {
    float4 pp = reinterpret_cast<float4*>(p)[i4];
    const float4 gg = reinterpret_cast<const float4*>(g)[i4];
    if (clear_grad) reinterpret_cast<float4*>(g)[i4] = make_float4(0.f, 0.f, 0.f, 0.f);
    float4 mm = reinterpret_cast<float4*>(m)[i4];
    float4 vv = reinterpret_cast<float4*>(v)[i4];
    float* pa = &pp.x; const float* ga = &gg.x; float* ma = &mm.x; float* va = &vv.x;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float gk = ga[k] * gs + wd * pa[k];
      ma[k] = b1 * ma[k] + (1.f - b1) * gk;
      va[k] = b2 * va[k] + (1.f - b2) * gk * gk;
      pa[k] -= lr_t * ma[k] / (sqrtf(va[k]) + eps * sqrtf(1.f - b2pow));
    }
    reinterpret_cast<float4*>(p)[i4] = pp;
    reinterpret_cast<float4*>(m)[i4] = mm;
    reinterpret_cast<float4*>(v)[i4] = vv;
  } else {
    for (int64_t i = i4 * 4; i < n; ++i) {
      const float gk = g[i] * gs + wd * p[i];
      if (clear_grad) g[i] = 0.f;
      m[i] = b1 * m[i] + (1.f - b1) * gk;
      v[i] = b2 * v[i] + (1.f - b2) * gk * gk;
      p[i] -= lr_t * m[i] / (sqrtf(v[i]) + eps * sqrtf(1.f - b2pow));
    }
  }
}

}  // namespace

void launch_data_norm_fwd(const float* x, int N, int C, const float* bsize, const float* bsum,
                          const float* bsq, float* y, float* means, float* scales,
                          const float* scale_w, const float* bias, hipStream_t s) {
  const int64_t n = (int64_t)N * C;
  if (n == 0) return;
  hipLaunchKernelGGL(k_dn_fwd, dim3(nblk(n)), dim3(256), 0, s, x, N, C, bsize, bsum, bsq, y, means, scales, scale_w, bias);
}

void launch_data_norm_bwd(const float* x, const float* dy, int N, int C, const float* means,
                          const float* scales, float eps, float* dx, float* stats, float* acc,
                          const float* scale_w, hipStream_t s) {
  if (C == 0) return;
  launch_fill32(acc, 0u, 2 * (int64_t)C, s);
  const dim3 g((C + 63) / 64, (N + kDnRows - 1) / kDnRows);
  hipLaunchKernelGGL(k_dn_bwd, g, dim3(256), 0, s, x, dy, N, C, means, scales, dx, acc, scale_w);
  hipLaunchKernelGGL(k_dn_finish, dim3(nblk(C)), dim3(256), 0, s, acc, C, N, eps, stats);
}

void launch_data_norm_update(float* bsize, float* bsum, float* bsq, const float* stats, int C,
                             float decay, hipStream_t s) {
  if (C == 0) return;
  hipLaunchKernelGGL(k_dn_update, dim3(nblk(C)), dim3(256), 0, s, bsize, bsum, bsq, stats, C, decay);
}

void launch_fm_fwd(const float* x, int B, int S, int D, int row_stride, int col0, int fstride,
                   float* out, hipStream_t s) {
  if (B == 0) return;
  hipLaunchKernelGGL(k_fm_fwd, dim3(nblk(B)), dim3(256), 0, s, x, B, S, D, row_stride, col0, fstride, out);
}

void launch_fm_bwd(const float* x, const float* dout, int B, int S, int D, int row_stride,
                   int col0, int fstride, float* dx, int dx_stride, int accumulate, hipStream_t s) {
  if (B == 0) return;
  hipLaunchKernelGGL(k_fm_bwd, dim3(nblk(B)), dim3(256), 0, s, x, dout, B, S, D, row_stride, col0, fstride, dx, dx_stride, accumulate);
}

void launch_logit_loss(const float* a, const float* b, const float* label, int B, float* pred, float* dz,
                       float* loss_mean, uint32_t* ws, hipStream_t s) {
  if (B <= 0) return;
  int per_thread = 1;
  while ((B + kLossBlock * per_thread - 1) / (kLossBlock * per_thread) > kLogitLossMaxBlocks) per_thread *= 2;
  const int grid = (B + kLossBlock * per_thread - 1) / (kLossBlock * per_thread);
  hipLaunchKernelGGL(k_logit_loss, dim3(grid), dim3(kLossBlock), 0, s, a, b, label, B, per_thread, pred, dz, loss_mean,
                     ws, reinterpret_cast<float*>(ws + 1));
}

void launch_sigmoid_logloss(const float* logit, const float* label, int B, float* pred,
                            float* loss_sum, float* dlogit, float grad_scale, hipStream_t s) {
  if (B == 0) return;
  hipLaunchKernelGGL(k_sigmoid_logloss, dim3(nblk(B)), dim3(256), 0, s, logit, label, B, pred, loss_sum, dlogit, grad_scale);
}

void launch_auc_accumulate(const float* pred, const float* label, const float* mask, int B,
                           int nbuckets, double* table, double* stats, hipStream_t s) {
  if (B == 0) return;
  hipLaunchKernelGGL(k_auc, dim3(nblk(B, 256 * kAucItems)), dim3(256), 0, s, pred, label, mask, B, nbuckets, table,
                     stats);
}

void launch_adam_flat(float* p, float* g, float* m, float* v, int64_t n, float lr, float b1,
                      float b2, float eps, float* pows, float grad_scale, float weight_decay,
                      bool clear_grad, hipStream_t s) {
  if (n == 0) return;
  const int64_t n4 = (n + 3) / 4;
  hipLaunchKernelGGL(k_adam_pows, dim3(1), dim3(64), 0, s, pows, b1, b2);
  hipLaunchKernelGGL(k_adam, dim3(nblk(n4)), dim3(256), 0, s, p, g, m, v, n, lr, b1, b2, eps, pows, grad_scale,
                     weight_decay, clear_grad ? 1 : 0);
}

}  // namespace pbx

// Sparse feature types of the GPU parameter server (BoxPS GetInsEx feature
// types, reference box_wrapper.cu:37-143 / 146-322 and the SparseAdam rule of
// heter_ps/optimizer.cuh.h:147-330), re-designed as a row codec:
//
//   kind 0  fp32 embedx, sparse Adagrad        (the default engine layout)
//   kind 1  int16 embedx (+expand), Adagrad     value = q * pull_embedx_scale
//   kind 2  fp32 embedx (+expand), SparseAdam   per-element moments, per-row
//                                               beta powers (w and x separately)
//   kind 3  variable: one fp32 block of max(D, De) columns of which the
//           row's stored size (0, D or De) is live; a feature is created
//           with De columns when its slot is pulled into an expand output
//           (codec bitmap), else D.  Pull zeroes columns past the size and
//           reports it; push updates only the live columns (reference
//           PullCopyVariable / PushMergeCopyVariable, box_wrapper.cu:
//           271-322,714-875: embedx_size per feature, total_dims flags)
//
// and an optional expand block (NNCross / extended pull: De extra columns
// pulled next to embedx, pull_box_extended_sparse).  Rows keep the standard
// tail fields at make_row_layout(Wx + We) (so probe / insert / shrink /
// export are codec-agnostic); codec state follows the tail.  The hot pull
// path decodes the unique rows once into fp32 pull records that the fused
// seqpool kernel then reads, and the push merges into push records exactly
// as for kind 0 -- only the two row-touching kernels below know the codec.
#include <hip/hip_runtime.h>

#include "kernels.h"
#include "table_probe.h"

namespace pbx {
namespace {

__device__ __forceinline__ float clampf(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }

// one embedding column j < D + De of row v (embedx then expand)
__device__ __forceinline__ float load_col(const CodecDev& c, const float* v, int j) {
  if (c.kind == 3) return v[kEmbedx + j];
  if (c.kind == 1) {
    const int16_t* q = reinterpret_cast<const int16_t*>(v + kEmbedx);
    const int w = j < c.D ? j : 2 * c.Wx + (j - c.D);
    return (float)q[w] * c.qscale;
  }
  return v[kEmbedx + (j < c.D ? j : c.Wx + (j - c.D))];
}

__device__ __forceinline__ void store_col(const CodecDev& c, float* v, int j, float x) {
  if (c.kind == 3) {
    v[kEmbedx + j] = x;
    return;
  }
  if (c.kind == 1) {
    int16_t* q = reinterpret_cast<int16_t*>(v + kEmbedx);
    const int w = j < c.D ? j : 2 * c.Wx + (j - c.D);
    q[w] = (int16_t)clampf(rintf(x / c.qscale), -32768.f, 32767.f);
    return;
  }
  v[kEmbedx + (j < c.D ? j : c.Wx + (j - c.D))] = x;
}

// out[i] = [show, click, embed_w, embedx[D], expand[De]] of row rows[idx(i)]
// (idx = uid[i] when uid is given: the owner side of a sharded pull)
__global__ __launch_bounds__(256) void k_codec_pull(TableDev t, CodecDev c, const int64_t* __restrict__ rows,
                                                    const int32_t* __restrict__ uid, const int32_t* n_dev, int64_t n,
                                                    float* __restrict__ out, int out_stride) {
  const int64_t nn = n_dev ? (int64_t)*n_dev : n;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nn) return;
  float* o = out + i * out_stride;
  const int DXv = c.kind == 3 ? c.Wx : c.D + c.De;
  const int W = 3 + DXv;
  int64_t r = -1;
  if (uid) {
    const int32_t u = uid[i];
    r = u >= 0 ? rows[u] : -1;
  } else {
    r = rows[i];
  }
  const bool size_col = c.kind == 3 && out_stride > W;  // variable: the size rides in column W
  if (r < 0) {
    for (int j = 0; j < W; ++j) o[j] = 0.f;
    if (size_col) o[W] = 0.f;
    return;
  }
  const float* v = t.values + r * (int64_t)t.stride;
  o[0] = v[kShow];
  o[1] = v[kClick];
  o[2] = v[kEmbedW];
  if (c.kind == 3) {
    const int xs = (int)v[c.xsz];
    for (int j = 0; j < DXv; ++j) o[3 + j] = j < xs ? v[kEmbedx + j] : 0.f;
    if (size_col) o[W] = (float)xs;
    return;
  }
  for (int j = 0; j < c.D + c.De; ++j) o[3 + j] = load_col(c, v, j);
}

__device__ __forceinline__ bool expand_slot(const CodecDev& c, float slot) {
  const int s = (int)slot;
  return c.vslots && s >= 0 && s < c.vslot_bits && ((c.vslots[s >> 5] >> (s & 31)) & 1u);
}

// SparseAdam step of n values w[j] (j through col()) with moments m/v and
// the row's beta powers at pw[0..1] (heter_ps/optimizer.cuh.h:157-197)
__device__ __forceinline__ float adam_ratio(const SparseSGDConfig& cfg, const float* pw) {
  return cfg.learning_rate * sqrtf(1.f - pw[1]) / (1.f - pw[0]);
}

__global__ __launch_bounds__(256) void k_codec_update(TableDev t, CodecDev c, const int64_t* __restrict__ rows,
                                                      const float* __restrict__ push, int push_stride,
                                                      const int32_t* n_dev, int64_t n, SparseSGDConfig cfg,
                                                      uint64_t seed) {
  const int64_t nn = n_dev ? (int64_t)*n_dev : n;
  const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= nn) return;
  const int64_t r = rows[u];
  if (r < 0) return;
  float* v = t.values + r * (int64_t)t.stride;
  const float* g = push + u * push_stride;
  const int DX = c.kind == 3 ? c.Wx : c.D + c.De;
  const float slot = g[kPushSlot], g_show = g[kPushShow], g_click = g[kPushClick];
  v[c.slot] = slot;
  const float show = v[kShow] + g_show;
  const float click = v[kClick] + g_click;
  v[kShow] = show;
  v[kClick] = click;
  v[c.delta] += cfg.nonclk_coeff * (g_show - g_click) + cfg.clk_coeff * g_click;
  v[c.unseen] = 0.f;
  const float scale = g_show > 0.f ? g_show : 1.f;
  const bool create = v[c.mf] == 0.f;
  if (c.kind == 2) {
    float* st = v + c.adam;  // [w_m, w_v, w_b1p, w_b2p, x_m[DX], x_v[DX], x_b1p, x_b2p]
    {
      const float ratio = adam_ratio(cfg, st + 2);
      const float sg = g[kPushEmbedG] / scale;
      const float m = c.beta1 * st[0] + (1.f - c.beta1) * sg;
      const float s2 = c.beta2 * st[1] + (1.f - c.beta2) * sg * sg;
      v[kEmbedW] = clampf(v[kEmbedW] + ratio * (m / (sqrtf(s2) + c.eps)), cfg.mf_min_bound, cfg.mf_max_bound);
      st[0] = m;
      st[1] = s2;
      st[2] *= c.beta1;
      st[3] *= c.beta2;
    }
    float* xm = st + 4;
    float* xv = xm + DX;
    float* xp = xv + DX;
    if (create) {
      if (cfg.nonclk_coeff * (show - click) + cfg.clk_coeff * click >= cfg.mf_create_thresholds) {
        v[c.mf] = 1.f;
        const uint64_t salt = mf_create_salt(table_row_key(t, r));
        for (int j = 0; j < DX; ++j) store_col(c, v, j, hash_uniform(salt, j) * cfg.mf_initial_range);
        xp[0] = c.beta1;
        xp[1] = c.beta2;
      }
    } else {
      const float ratio = adam_ratio(cfg, xp);
      for (int j = 0; j < DX; ++j) {
        const float sg = g[kPushEmbedxG + j] / scale;
        const float m = c.beta1 * xm[j] + (1.f - c.beta1) * sg;
        const float s2 = c.beta2 * xv[j] + (1.f - c.beta2) * sg * sg;
        store_col(c, v, j,
                  clampf(load_col(c, v, j) + ratio * (m / (sqrtf(s2) + c.eps)), cfg.mf_min_bound, cfg.mf_max_bound));
        xm[j] = m;
        xv[j] = s2;
      }
      xp[0] *= c.beta1;
      xp[1] *= c.beta2;
    }
    return;
  }
  float lr = cfg.learning_rate, mf_lr = cfg.mf_learning_rate;
  if (cfg.use_feature_lr && slot != cfg.nodeid_slot) {
    lr = cfg.feature_learning_rate;
    mf_lr = cfg.feature_learning_rate;
  }
  {
    const float g2 = v[c.g2];
    const float ratio = lr * sqrtf(cfg.initial_g2sum / (cfg.initial_g2sum + g2));
    const float sg = g[kPushEmbedG] / scale;
    v[kEmbedW] = clampf(v[kEmbedW] + sg * ratio, cfg.min_bound, cfg.max_bound);
    v[c.g2] = g2 + sg * sg;
  }
  if (create) {
    if (cfg.nonclk_coeff * (show - click) + cfg.clk_coeff * click >= cfg.mf_create_thresholds) {
      v[c.mf] = 1.f;
      const uint64_t salt = mf_create_salt(table_row_key(t, r));
      const int nc = c.kind == 3 ? (expand_slot(c, slot) ? c.De : c.D) : DX;
      if (c.kind == 3) v[c.xsz] = (float)nc;
      for (int j = 0; j < nc; ++j) store_col(c, v, j, hash_uniform(salt, j) * cfg.mf_initial_range);
    }
    return;
  }
  if (c.kind == 3) {  // variable: one Adagrad group over the live columns
    int xs = (int)v[c.xsz];
    if (xs <= 0) return;
    // a row's size follows its slot: rows pre-populated with init_embedx
    // (k_codec_init knows no slot and creates D columns) that turn out to
    // belong to an expand slot are re-created at their first push with De
    // columns (fresh draws, fresh g2sum), as a push-created row would be
    const int want = expand_slot(c, slot) ? c.De : c.D;
    if (xs != want) {
      const uint64_t salt = mf_create_salt(table_row_key(t, r));
      for (int j = 0; j < want; ++j) store_col(c, v, j, hash_uniform(salt, j) * cfg.mf_initial_range);
      for (int j = want; j < c.Wx; ++j) store_col(c, v, j, 0.f);
      v[c.xsz] = (float)want;
      v[c.xg2] = 0.f;
      return;
    }
    const float g2 = v[c.xg2];
    const float ratio = mf_lr * sqrtf(cfg.mf_initial_g2sum / (cfg.mf_initial_g2sum + g2));
    float add = 0.f;
    for (int j = 0; j < xs; ++j) {
      const float sg = g[kPushEmbedxG + j] / scale;
      v[kEmbedx + j] = clampf(v[kEmbedx + j] + sg * ratio, cfg.mf_min_bound, cfg.mf_max_bound);
      add += sg * sg;
    }
    v[c.xg2] = g2 + add / (float)xs;
    return;
  }
  // embedx and expand are two Adagrad groups with their own g2sum
  for (int grp = 0; grp < (c.De > 0 ? 2 : 1); ++grp) {
    const int j0 = grp == 0 ? 0 : c.D, nj = grp == 0 ? c.D : c.De;
    const int gi = grp == 0 ? c.xg2 : c.eg2;
    const float g2 = v[gi];
    const float ratio = mf_lr * sqrtf(cfg.mf_initial_g2sum / (cfg.mf_initial_g2sum + g2));
    float add = 0.f;
    for (int j = j0; j < j0 + nj; ++j) {
      const float sg = g[kPushEmbedxG + j] / scale;
      store_col(c, v, j, clampf(load_col(c, v, j) + sg * ratio, cfg.mf_min_bound, cfg.mf_max_bound));
      add += sg * sg;
    }
    v[gi] = g2 + add / (float)nj;
  }
}

// codec state of freshly inserted rows (the insert zeroed them): Adam beta
// powers, and with init_embedx the embedding block (as if created)
__global__ void k_codec_init(TableDev t, CodecDev c, const int64_t* __restrict__ rows,
                             const uint64_t* __restrict__ keys, int64_t n, SparseSGDConfig cfg, uint64_t seed,
                             int init_embedx) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t r = rows[i];
  if (r < 0) return;
  float* v = t.values + r * (int64_t)t.stride;
  const int DX = c.kind == 3 ? c.D : c.D + c.De;  // variable: created with D columns
  if (c.kind == 2) {
    float* st = v + c.adam;
    st[2] = c.beta1;
    st[3] = c.beta2;
    st[4 + 2 * DX] = c.beta1;
    st[5 + 2 * DX] = c.beta2;
  }
  if (init_embedx) {  // same draws as the table insert's init_row
    v[c.mf] = 1.f;
    if (c.kind == 3) v[c.xsz] = (float)c.D;
    for (int j = 0; j < DX; ++j) store_col(c, v, j, hash_uniform(keys[i], seed + 1 + j) * cfg.mf_initial_range);
  }
}

inline unsigned nblk(int64_t n) { return (unsigned)((n + 255) / 256 > 0 ? (n + 255) / 256 : 1); }

}  // namespace

void launch_codec_pull(const TableDev& t, const CodecDev& c, const int64_t* rows, const int32_t* uid,
                       const int32_t* n_dev, int64_t n, float* out, int out_stride, hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(k_codec_pull, dim3(nblk(n)), dim3(256), 0, s, t, c, rows, uid, n_dev, n, out, out_stride);
}

void launch_codec_update(const TableDev& t, const CodecDev& c, const int64_t* rows, const float* push,
                         int push_stride, const int32_t* n_dev, int64_t n, const SparseSGDConfig& cfg, uint64_t seed,
                         hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(k_codec_update, dim3(nblk(n)), dim3(256), 0, s, t, c, rows, push, push_stride, n_dev, n, cfg,
                     seed);
}

void launch_codec_init(const TableDev& t, const CodecDev& c, const int64_t* rows, const uint64_t* keys, int64_t n,
                       const SparseSGDConfig& cfg, uint64_t seed, int init_embedx, hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(k_codec_init, dim3(nblk(n)), dim3(256), 0, s, t, c, rows, keys, n, cfg, seed, init_embedx);
}

}  // namespace pbx

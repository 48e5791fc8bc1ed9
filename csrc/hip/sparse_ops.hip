// Pull / seqpool+CVM / push-merge / sparse-Adagrad kernels for CDNA4.
//
// Reference behaviour:
//   pull copy        paddle/fluid/framework/fleet/box_wrapper.cu:74-143  (PullCopy)
//   push merge       box_wrapper.cu:417-512 (PushMergeCopy / ...Atomic)
//   seqpool + CVM    paddle/fluid/operators/fused/fused_seqpool_cvm_op.cu:34-527 (fwd),
//                    :813-1015 (bwd: CVM input written into the show/click columns)
//   sparse Adagrad   heter_ps/optimizer.cuh.h:42-133, ctr_accessor.cc:245-279
//
// MI355X design: the forward reads value rows straight out of the table (or
// the exchanged pull buffer) and writes the pooled, CVM-transformed slot block
// directly into the concatenated dense input (no [L, 11] intermediate, no
// separate concat).  The backward never materialises per-occurrence gradients:
// one thread per *sorted occurrence* gathers its pooled-output gradient and a
// wave-level segmented scan merges duplicates (skew-proof for Zipf-hot keys),
// then the Adagrad update runs in place on the table rows.
#include <hip/hip_runtime.h>

#include "kernels.h"
#include "table_probe.h"

namespace pbx {
namespace {

constexpr int kMaxE = 132;  // max pull width handled (D <= 128)

template <int E>
struct Acc {
  float v[E];
};

// ---------------------------------------------------------------- occurrence map
__global__ void k_fill_occ(const int64_t* __restrict__ lod, int S, int B, int32_t* __restrict__ occ_slot,
                           int32_t* __restrict__ occ_ins) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)S * B) return;
  const int s = (int)(t / B), b = (int)(t % B);
  const int64_t st = lod[(int64_t)s * (B + 1) + b], en = lod[(int64_t)s * (B + 1) + b + 1];
  for (int64_t k = st; k < en; ++k) {
    occ_slot[k] = s;
    occ_ins[k] = b;
  }
}

// ---------------------------------------------------------------- gather pull
__global__ void k_gather_pull(TableDev t, const int64_t* __restrict__ rows, const int32_t* n_dev, int64_t n,
                              float* __restrict__ out, int out_stride) {
  const int64_t nn = n_dev ? (int64_t)*n_dev : n;
  const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= nn) return;
  const int P = kPullHead + t.dim;
  const int64_t r = rows[u];
  float* o = out + u * out_stride;
  if (r < 0) {
    for (int c = 0; c < out_stride; ++c) o[c] = 0.f;
    return;
  }
  const float4* src = reinterpret_cast<const float4*>(t.values + r * (int64_t)t.stride);
  const int n4 = out_stride / 4;
  if ((out_stride & 3) == 0 && n4 * 4 <= t.stride) {
    float4* o4 = reinterpret_cast<float4*>(o);
    for (int c4 = 0; c4 < n4; ++c4) {
      float4 v = src[c4];
      const int c = c4 * 4;
      if (c + 0 >= P) v.x = 0.f;
      if (c + 1 >= P) v.y = 0.f;
      if (c + 2 >= P) v.z = 0.f;
      if (c + 3 >= P) v.w = 0.f;
      o4[c4] = v;
    }
  } else {
    const float* s1 = t.values + r * (int64_t)t.stride;
    for (int c = 0; c < out_stride; ++c) o[c] = c < P ? s1[c] : 0.f;
  }
}

// ---------------------------------------------------------------- seqpool + cvm fwd
__device__ __forceinline__ float quant(float v, int q) {
  return (float)((int)(v * q + 0.5f)) / (float)q;
}

template <int E>
__device__ __forceinline__ void load_row(const float* __restrict__ p, float* v) {
  if constexpr ((E + 3) / 4 * 4 <= 16) {
    // rows are 16-B aligned with stride >= round4(E)
    const float4* p4 = reinterpret_cast<const float4*>(p);
#pragma unroll
    for (int c4 = 0; c4 < (E + 3) / 4; ++c4) {
      const float4 x = p4[c4];
      if (c4 * 4 + 0 < E) v[c4 * 4 + 0] = x.x;
      if (c4 * 4 + 1 < E) v[c4 * 4 + 1] = x.y;
      if (c4 * 4 + 2 < E) v[c4 * 4 + 2] = x.z;
      if (c4 * 4 + 3 < E) v[c4 * 4 + 3] = x.w;
    }
  } else {
#pragma unroll
    for (int c = 0; c < E; ++c) v[c] = p[c];
  }
}

// record index of occurrence k: probed from its feasign (fused probe of the
// split pull, also recorded in rows_out) or read through uid / src_index
__device__ __forceinline__ int64_t seqpool_record(const SeqpoolCvmArgs& a, int64_t k) {
  if (a.probe_keys) {
    const uint64_t kk = a.probe_keys[k];
    const int64_t r = table_probe_thread(a.probe_t, kk == kEmptyKey ? kEmptyKey : mix64(kk));
    a.rows_out[k] = r;
    return r;
  }
  const int32_t u = a.uid ? a.uid[k] : (int32_t)k;
  if (u < 0) return -1;
  if (a.n_index && a.src_index && u >= a.n_index) {
    if (a.err) atomicOr(a.err, kSeqpoolGuardUid);
    return -1;
  }
  const int64_t r = a.src_index ? a.src_index[u] : (int64_t)u;
  if (a.src_rows && r >= a.src_rows) {
    if (a.err) atomicOr(a.err, kSeqpoolGuardRow);
    return -1;
  }
  return r;
}

// occurrence k inside the buffers the lod may index
__device__ __forceinline__ bool seqpool_occ_ok(const SeqpoolCvmArgs& a, int64_t k) {
  if (a.n_occ && (k < 0 || k >= a.n_occ)) {
    if (a.err) atomicOr(a.err, kSeqpoolGuardOcc);
    return false;
  }
  return true;
}

template <int E>
__global__ __launch_bounds__(256) void k_seqpool_cvm(SeqpoolCvmArgs a) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (a.sc_perm && t < 4) {  // fused dedup scatter: publish the counters, leave acc zero
    a.sc_u_count[t] = a.sc_acc[t];
    a.sc_acc[t] = 0;
  }
  if (t >= (int64_t)a.S * a.B) return;
  // instance-major so a wave writes contiguous output rows
  const int b = (int)(t / a.S), s = (int)(t % a.S);
  if (s == 0 && a.dense) {
    const float* src = a.dense + (int64_t)b * (a.dense_stride ? a.dense_stride : a.dense_dim);
    float* dst = a.out + (int64_t)b * a.out_stride + a.dense_col;
    for (int c = 0; c < a.dense_dim; ++c) dst[c] = src[c];
  }
  const int64_t st = a.lod[(int64_t)s * (a.B + 1) + b], en = a.lod[(int64_t)s * (a.B + 1) + b + 1];
  float acc[E];
#pragma unroll
  for (int c = 0; c < E; ++c) acc[c] = a.pad_value;
  for (int64_t k = st; k < en; ++k) {
    if (!seqpool_occ_ok(a, k)) continue;
    if (a.occ_slot) {
      a.occ_slot[k] = s;
      a.occ_ins[k] = b;
    }
    const int64_t ri = seqpool_record(a, k);
    if (a.sc_perm) {  // fused table-dedup scatter (k_table_scatter's per-occurrence work)
      if (ri >= 0) {
        const int32_t u = a.sc_uid_row[ri];
        a.sc_uid[k] = u;
        a.sc_perm[a.sc_seg[u] + a.sc_rank[k]] = (int32_t)k;
      } else {
        a.sc_uid[k] = -1;
      }
    }
    if (ri < 0) continue;
    float v[E];
    load_row<E>(a.src + ri * (int64_t)a.src_stride, v);
    if (a.need_filter || a.embed_threshold_filter) {
      const float show = v[0], clk = v[1];
      if ((show - clk) * a.show_coeff + clk * a.clk_coeff < a.threshold) continue;
      if (a.embed_threshold_filter) {
        // 0 means the whole embedding (fused_seqpool_cvm_op.cu:596-599)
        const int ets = a.embed_thres_size > 0 ? a.embed_thres_size : E - a.cvm_offset;
        float sc = 0.f;
        for (int i = 1; i < ets; ++i) sc += v[a.cvm_offset + i] * v[a.cvm_offset + i];
        sc = sqrtf(sc) + fabsf(v[a.cvm_offset]);
        if (sc < a.embed_threshold) continue;
      }
    }
    if (a.quant_ratio > 0) {
#pragma unroll
      for (int c = 0; c < E; ++c) acc[c] += (c < a.cvm_offset) ? v[c] : quant(v[c], a.quant_ratio);
    } else {
#pragma unroll
      for (int c = 0; c < E; ++c) acc[c] += v[c];
    }
  }
  // CVM epilogue, written straight into the concatenated output row
  const int skip = a.use_cvm ? 0 : a.cvm_offset + a.embed_thres_size;
  const int Eo = a.use_cvm ? (a.clk_filter ? E - 1 : E) : E - skip;
  float* o = a.out + (int64_t)b * a.out_stride + a.col_offset + (int64_t)s * Eo;
  if (a.use_cvm) {
    const float ls = logf(acc[0] + 1.f);
    if (a.clk_filter) {
      o[0] = ls;
#pragma unroll
      for (int c = 2; c < E; ++c) o[c - 1] = acc[c];
    } else {
      // the E floats of the row are contiguous and 4-B aligned: dwordx4
      // stores (3 requests instead of 11 for E = 11)
      typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));
      acc[1] = logf(acc[1] + 1.f) - ls;
      acc[0] = ls;
#pragma unroll
      for (int c = 0; c + 4 <= E; c += 4)
        *reinterpret_cast<f4u*>(o + c) = f4u{acc[c], acc[c + 1], acc[c + 2], acc[c + 3]};
#pragma unroll
      for (int c = E / 4 * 4; c < E; ++c) o[c] = acc[c];
    }
  } else {
#pragma unroll
    for (int c = 0; c < E; ++c)
      if (c >= skip) o[c - skip] = acc[c];
  }
}

// generic width (slow path, runtime E)
__global__ void k_seqpool_cvm_generic(SeqpoolCvmArgs a) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)a.S * a.B) return;
  const int b = (int)(t / a.S), s = (int)(t % a.S);
  const int E = a.E;
  if (s == 0 && a.dense) {
    const float* src = a.dense + (int64_t)b * (a.dense_stride ? a.dense_stride : a.dense_dim);
    float* dst = a.out + (int64_t)b * a.out_stride + a.dense_col;
    for (int c = 0; c < a.dense_dim; ++c) dst[c] = src[c];
  }
  const int64_t st = a.lod[(int64_t)s * (a.B + 1) + b], en = a.lod[(int64_t)s * (a.B + 1) + b + 1];
  const int skip = a.use_cvm ? 0 : a.cvm_offset + a.embed_thres_size;
  const int Eo = a.use_cvm ? (a.clk_filter ? E - 1 : E) : E - skip;
  const int ets = a.embed_thres_size > 0 ? a.embed_thres_size : E - a.cvm_offset;
  float* o = a.out + (int64_t)b * a.out_stride + a.col_offset + (int64_t)s * Eo;
  if (a.occ_slot) {
    for (int64_t k = st; k < en; ++k) {
      if (!seqpool_occ_ok(a, k)) continue;
      a.occ_slot[k] = s;
      a.occ_ins[k] = b;
    }
  }
  float show_sum = a.pad_value, clk_sum = a.pad_value;
  for (int c = 0; c < E; ++c) {
    float acc = a.pad_value;
    for (int64_t k = st; k < en; ++k) {
      if (!seqpool_occ_ok(a, k)) continue;
      const int64_t ri = seqpool_record(a, k);
      if (ri < 0) continue;
      const float* v = a.src + ri * (int64_t)a.src_stride;
      if ((a.need_filter || a.embed_threshold_filter) &&
          (v[0] - v[1]) * a.show_coeff + v[1] * a.clk_coeff < a.threshold)
        continue;
      if (a.embed_threshold_filter) {
        float sc = 0.f;
        for (int i = 1; i < ets; ++i) sc += v[a.cvm_offset + i] * v[a.cvm_offset + i];
        if (sqrtf(sc) + fabsf(v[a.cvm_offset]) < a.embed_threshold) continue;
      }
      acc += (a.quant_ratio > 0 && c >= a.cvm_offset) ? quant(v[c], a.quant_ratio) : v[c];
    }
    if (c == 0) show_sum = acc;
    if (c == 1) clk_sum = acc;
    if (a.use_cvm) {
      if (c == 0) o[0] = logf(show_sum + 1.f);
      else if (c == 1) { if (!a.clk_filter) o[1] = logf(clk_sum + 1.f) - logf(show_sum + 1.f); }
      else o[a.clk_filter ? c - 1 : c] = acc;
    } else if (c >= skip) {
      o[c - skip] = acc;
    }
  }
}

// ---------------------------------------------------------------- push merge
// Q = 3 + D merged values per unique: [show, click, embed_g, embedx_g...]
struct DoutSource {
  PushMergeArgs a;
  __device__ __forceinline__ void load(int32_t k, float* g, int Q) const {
    const int b = a.occ_ins[k], s = a.occ_slot[k];
    const int co = a.cvm_offset;
    const int ets = a.use_cvm ? 0 : a.embed_thres_size;
    // dropped columns: zero grads, and the cvm ones too (op.cu:958-969)
    g[0] = ets ? 0.f : a.cvm[(int64_t)b * co + 0];
    g[1] = (co > 1 && !ets) ? a.cvm[(int64_t)b * co + 1] : 0.f;
    const int E = a.E;
    const int Eo = a.use_cvm ? (a.clk_filter ? E - 1 : E) : E - co - ets;
    const float* d = a.dout + (int64_t)b * a.out_stride + a.col_offset + (int64_t)s * Eo;
    for (int c = co; c < E; ++c) {
      const int oc = a.use_cvm ? (a.clk_filter ? c - 1 : c) : c - co - ets;
      g[2 + (c - co)] = oc >= 0 ? d[oc] : 0.f;
    }
    (void)Q;
  }
  __device__ __forceinline__ float slot(int32_t k) const { return a.slot_ids ? a.slot_ids[a.occ_slot[k]] : (float)a.occ_slot[k]; }
  // common layout (use_cvm, no click filter, cvm_offset 2, E = 3 + D): the
  // D + 1 embedding grads are contiguous and 4-B aligned, so they move as
  // dwordx4 loads -- 4 memory requests per occurrence instead of 11 (the
  // scalar gathers were ~80% of this kernel's L2 requests, PMC TCC_HIT+MISS)
  __device__ __forceinline__ bool fast(int D) const {
    return a.use_cvm && !a.clk_filter && a.cvm_offset == 2 && a.E == 3 + D;
  }
  template <int D>
  __device__ __forceinline__ void load_fast(int32_t k, float* g) const {
    typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));
    typedef float f2u __attribute__((ext_vector_type(2), aligned(4)));
    const int b = a.occ_ins[k], s = a.occ_slot[k];
    const f2u c = *reinterpret_cast<const f2u*>(a.cvm + (int64_t)b * 2);
    g[0] = c.x;
    g[1] = c.y;
    const float* d = a.dout + (int64_t)b * a.out_stride + a.col_offset + (int64_t)s * (3 + D) + 2;
    constexpr int N = 1 + D;
#pragma unroll
    for (int i = 0; i + 4 <= N; i += 4) {
      const f4u x = *reinterpret_cast<const f4u*>(d + i);
      g[2 + i] = x.x;
      g[3 + i] = x.y;
      g[4 + i] = x.z;
      g[5 + i] = x.w;
    }
#pragma unroll
    for (int i = N / 4 * 4; i < N; ++i) g[2 + i] = d[i];
  }
};

template <int Q, typename Src>
__global__ __launch_bounds__(256) void k_push_merge(Src src, const int32_t* __restrict__ perm,
                                                    const int32_t* __restrict__ uid, const int32_t* n_valid,
                                                    int64_t n, float* __restrict__ push, int push_stride,
                                                    const int64_t* __restrict__ push_index, float neg_bs,
                                                    int scale_from) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t pv = n_valid ? (int64_t)*n_valid : n;
  const int lane = threadIdx.x & 63;
  const int64_t wave_base = p - lane;
  if (wave_base >= pv) return;  // whole wave idle
  int32_t u = -1;
  int32_t k = -1;
  float g[Q];
#pragma unroll
  for (int c = 0; c < Q; ++c) g[c] = 0.f;
  if (p < pv) {
    k = perm[p];
    u = uid[k];
    src.load(k, g, Q);
  }
  // wave segmented inclusive scan keyed by u
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int32_t uo = __shfl_up(u, off);
#pragma unroll
    for (int c = 0; c < Q; ++c) {
      const float go = __shfl_up(g[c], off);
      if (lane >= off && uo == u) g[c] += go;
    }
  }
  const int32_t un = __shfl_down(u, 1);
  const int32_t u_lane0 = __shfl(u, 0);
  const bool tail = (lane == 63) || (un != u);
  if (p >= pv || u < 0 || !tail) return;
  const int64_t prow = push_index ? push_index[u] : (int64_t)u;
  if (prow < 0) return;
  float* dst = push + prow * push_stride;
  // The in-wave scan covers the whole segment unless it spills over a wave
  // boundary (occurrences are sorted by unique id, so a segment is contiguous).
  bool complete = true;
  if (lane == 63 && p + 1 < pv && uid[perm[p + 1]] == u) complete = false;
  if (u_lane0 == u && wave_base > 0 && uid[perm[wave_base - 1]] == u) complete = false;
  if (complete) {
    dst[kPushSlot] = src.slot(k);
    dst[kPushShow] = g[0];
    dst[kPushClick] = g[1];
#pragma unroll
    for (int c = 2; c < Q; ++c) dst[kPushEmbedG + (c - 2)] = c >= scale_from ? g[c] * neg_bs : g[c];
  } else {
    dst[kPushSlot] = src.slot(k);
    atomicAdd(&dst[kPushShow], g[0]);
    atomicAdd(&dst[kPushClick], g[1]);
#pragma unroll
    for (int c = 2; c < Q; ++c) atomicAdd(&dst[kPushEmbedG + (c - 2)], c >= scale_from ? g[c] * neg_bs : g[c]);
  }
}

// records source: rec[k] = [slot, show, click, embed_g, embedx_g...] (already scaled)
struct RecordSource {
  const float* rec;
  int stride;
  __device__ __forceinline__ void load(int32_t k, float* g, int Q) const {
    const float* r = rec + (int64_t)k * stride;
    for (int c = 0; c < Q; ++c) g[c] = r[1 + c];
  }
  __device__ __forceinline__ float slot(int32_t k) const { return rec[(int64_t)k * stride]; }
};

// ---------------------------------------------------------------- sparse adagrad
__device__ __forceinline__ float clampf(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }

__global__ __launch_bounds__(256) void k_push_adagrad(TableDev t, const int64_t* __restrict__ rows,
                                                      const float* __restrict__ push, int push_stride,
                                                      const int32_t* n_dev, int64_t n, SparseSGDConfig cfg,
                                                      uint64_t seed) {
  const int64_t nn = n_dev ? (int64_t)*n_dev : n;
  const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= nn) return;
  const int64_t r = rows[u];
  if (r < 0) return;
  const RowLayout l = make_row_layout(t.dim);
  float* v = t.values + r * (int64_t)t.stride;
  const float* g = push + u * push_stride;
  const float slot = g[kPushSlot], g_show = g[kPushShow], g_click = g[kPushClick];
  v[l.slot] = slot;
  const float show = v[kShow] + g_show;
  const float click = v[kClick] + g_click;
  v[kShow] = show;
  v[kClick] = click;
  v[l.delta_score] += cfg.nonclk_coeff * (g_show - g_click) + cfg.clk_coeff * g_click;
  v[l.unseen_days] = 0.f;
  const float scale = g_show > 0.f ? g_show : 1.f;
  float lr = cfg.learning_rate, mf_lr = cfg.mf_learning_rate;
  if (cfg.use_feature_lr && slot != cfg.nodeid_slot) { lr = cfg.feature_learning_rate; mf_lr = cfg.feature_learning_rate; }
  {  // embed_w (1-d Adagrad)
    const float g2 = v[l.embed_g2sum];
    const float ratio = lr * sqrtf(cfg.initial_g2sum / (cfg.initial_g2sum + g2));
    const float sg = g[kPushEmbedG] / scale;
    v[kEmbedW] = clampf(v[kEmbedW] + sg * ratio, cfg.min_bound, cfg.max_bound);
    v[l.embed_g2sum] = g2 + sg * sg;
  }
  if (v[l.mf_size] == 0.f) {
    if (cfg.nonclk_coeff * (show - click) + cfg.clk_coeff * click >= cfg.mf_create_thresholds) {
      v[l.mf_size] = 1.f;
      const uint64_t salt = mf_create_salt(table_row_key(t, r));
      for (int d = 0; d < t.dim; ++d) v[kEmbedx + d] = hash_uniform(salt, d) * cfg.mf_initial_range;
    }
  } else {
    const float g2 = v[l.embedx_g2sum];
    const float ratio = mf_lr * sqrtf(cfg.mf_initial_g2sum / (cfg.mf_initial_g2sum + g2));
    float add = 0.f;
    for (int d = 0; d < t.dim; ++d) {
      const float sg = g[kPushEmbedxG + d] / scale;
      v[kEmbedx + d] = clampf(v[kEmbedx + d] + sg * ratio, cfg.mf_min_bound, cfg.mf_max_bound);
      add += sg * sg;
    }
    v[l.embedx_g2sum] = g2 + add / (float)t.dim;
  }
}

// Vectorised variant for the common embedx dims: the row (stride 4k floats,
// 16-B aligned) and the push record move as float4s with compile-time field
// indices, so the whole update is a handful of wide loads/stores instead of
// ~20 dependent scalar accesses per row.
template <int D>
struct RowF {
  static constexpr int kG2 = 3 + D, kXG2 = 4 + D, kDelta = 5 + D, kSlot = 6 + D, kUnseen = 7 + D, kMf = 8 + D;
  static constexpr int kStride = ((9 + D) + 3) & ~3;
  static constexpr int kQ = 4 + D;                 // push record floats used
  static constexpr int kQ4 = (kQ + 3) / 4;         // float4s covering it
};

template <int D>
__device__ __forceinline__ void adagrad_row(float* __restrict__ row, const float* g, const SparseSGDConfig& cfg,
                                            uint64_t seed, uint64_t rkey) {
  using L = RowF<D>;
  float v[L::kStride];
  float4* r4 = reinterpret_cast<float4*>(row);
#pragma unroll
  for (int i = 0; i < L::kStride / 4; ++i) {
    const float4 x = r4[i];
    v[4 * i] = x.x;
    v[4 * i + 1] = x.y;
    v[4 * i + 2] = x.z;
    v[4 * i + 3] = x.w;
  }
  const float slot = g[kPushSlot], g_show = g[kPushShow], g_click = g[kPushClick];
  v[L::kSlot] = slot;
  const float show = v[kShow] + g_show;
  const float click = v[kClick] + g_click;
  v[kShow] = show;
  v[kClick] = click;
  v[L::kDelta] += cfg.nonclk_coeff * (g_show - g_click) + cfg.clk_coeff * g_click;
  v[L::kUnseen] = 0.f;
  const float scale = g_show > 0.f ? g_show : 1.f;
  float lr = cfg.learning_rate, mf_lr = cfg.mf_learning_rate;
  if (cfg.use_feature_lr && slot != cfg.nodeid_slot) { lr = cfg.feature_learning_rate; mf_lr = cfg.feature_learning_rate; }
  {
    const float g2 = v[L::kG2];
    const float ratio = lr * sqrtf(cfg.initial_g2sum / (cfg.initial_g2sum + g2));
    const float sg = g[kPushEmbedG] / scale;
    v[kEmbedW] = clampf(v[kEmbedW] + sg * ratio, cfg.min_bound, cfg.max_bound);
    v[L::kG2] = g2 + sg * sg;
  }
  if (v[L::kMf] == 0.f) {
    if (cfg.nonclk_coeff * (show - click) + cfg.clk_coeff * click >= cfg.mf_create_thresholds) {
      v[L::kMf] = 1.f;
      const uint64_t salt = mf_create_salt(rkey);
#pragma unroll
      for (int d = 0; d < D; ++d) v[kEmbedx + d] = hash_uniform(salt, d) * cfg.mf_initial_range;
    }
  } else {
    const float g2 = v[L::kXG2];
    const float ratio = mf_lr * sqrtf(cfg.mf_initial_g2sum / (cfg.mf_initial_g2sum + g2));
    float add = 0.f;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const float sg = g[kPushEmbedxG + d] / scale;
      v[kEmbedx + d] = clampf(v[kEmbedx + d] + sg * ratio, cfg.mf_min_bound, cfg.mf_max_bound);
      add += sg * sg;
    }
    v[L::kXG2] = g2 + add / (float)D;
  }
#pragma unroll
  for (int i = 0; i < L::kStride / 4; ++i) r4[i] = make_float4(v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]);
}

template <int D>
__device__ __forceinline__ void load_push(const float* __restrict__ p, float* g) {
  using L = RowF<D>;
  const float4* p4 = reinterpret_cast<const float4*>(p);
#pragma unroll
  for (int i = 0; i < L::kQ4; ++i) {
    const float4 x = p4[i];
    if (4 * i < L::kQ) g[4 * i] = x.x;
    if (4 * i + 1 < L::kQ) g[4 * i + 1] = x.y;
    if (4 * i + 2 < L::kQ) g[4 * i + 2] = x.z;
    if (4 * i + 3 < L::kQ) g[4 * i + 3] = x.w;
  }
}

// push_stride must be a multiple of 4 and >= 4*kQ4 (the engine's padded record)
template <int D>
__global__ __launch_bounds__(256) void k_push_adagrad_v(TableDev t, const int64_t* __restrict__ rows,
                                                        const float* __restrict__ push, int push_stride,
                                                        const int32_t* n_dev, int64_t n, SparseSGDConfig cfg,
                                                        uint64_t seed) {
  const int64_t nn = n_dev ? (int64_t)*n_dev : n;
  const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= nn) return;
  const int64_t r = rows[u];
  if (r < 0) return;
  float g[RowF<D>::kQ4 * 4];
  load_push<D>(push + u * push_stride, g);
  adagrad_row<D>(t.values + r * (int64_t)t.stride, g, cfg, seed, table_row_key(t, r));
}

// Owner side of the sharded push: the records of unique u (at most one per
// sender, so a short bounded run) are perm[seg[u] .. seg[u]+cnt[u]) of the
// received buffer; merge them in registers and apply Adagrad in place --
// no merged-record buffer, no memset, no separate merge launch.
template <int D>
__global__ __launch_bounds__(256) void k_push_adagrad_seg(TableDev t, const int64_t* __restrict__ rows,
                                                          const float* __restrict__ rec, int rec_stride,
                                                          const int32_t* __restrict__ perm,
                                                          const int32_t* __restrict__ seg,
                                                          const int32_t* __restrict__ cnt, const int32_t* n_dev,
                                                          int64_t n, SparseSGDConfig cfg, uint64_t seed) {
  const int64_t nn = n_dev ? (int64_t)*n_dev : n;
  const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= nn) return;
  const int64_t r = rows[u];
  if (r < 0) return;
  constexpr int QP = RowF<D>::kQ4 * 4;
  float g[QP];
#pragma unroll
  for (int c = 0; c < QP; ++c) g[c] = 0.f;
  const int s0 = seg[u], m = cnt[u];
  for (int j = 0; j < m; ++j) {
    float x[QP];
    load_push<D>(rec + (int64_t)perm[s0 + j] * rec_stride, x);
    g[kPushSlot] = x[kPushSlot];
#pragma unroll
    for (int c = 1; c < QP; ++c) g[c] += x[c];
  }
  adagrad_row<D>(t.values + r * (int64_t)t.stride, g, cfg, seed, table_row_key(t, r));
}

// Single-shard push, merge + Adagrad in one pass over the batch gradients.
// perm lists the occurrences grouped by unique id (unique u owns the run
// perm[seg[u] .. seg[u]+cnt[u])).  Each wave segmented-scans 64 consecutive
// occurrences; a run lying wholly inside the wave is applied to its table
// row straight from registers.  A run crossing a wave boundary is summed
// into acc[u] (all-zero between steps) and the wave holding its first
// occurrence files u in inc[] for k_push_finish, which applies it and
// re-zeroes acc[u]: no merged-record buffer, no memset, one read of dout.
// (Reference: PushMergeCopy + PushSparseGPU, box_wrapper.cu:417-512.)
// What a completed run (one unique key's summed push record) turns into:
// the single-shard step applies Adagrad to the key's table row; the sharded
// step writes the record into the key's slot of the send buffer (no memset of
// the send buffer, no atomics for the runs that fit in a wave).
struct ApplyEmit {
  TableDev t;
  const int64_t* rows;
  SparseSGDConfig cfg;
  uint64_t seed;
  template <int D>
  __device__ __forceinline__ void emit(int32_t u, const float* rec) const {
    const int64_t r = rows[u];
    if (r < 0) return;
    if (r >= table_rows(t)) {  // corrupted row: recorded, never written
      if (t.err) atomicOr(t.err, 1);
      return;
    }
    adagrad_row<D>(t.values + r * (int64_t)t.stride, rec, cfg, seed, table_row_key(t, r));
  }
};
struct SendEmit {
  float* send;
  int stride;
  const int64_t* index;  // send row per unique (-1: dropped on overflow)
  template <int D>
  __device__ __forceinline__ void emit(int32_t u, const float* rec) const {
    const int64_t j = index[u];
    if (j < 0) return;
    float4* d = reinterpret_cast<float4*>(send + j * (int64_t)stride);
#pragma unroll
    for (int i = 0; i < RowF<D>::kQ4; ++i) d[i] = make_float4(rec[4 * i], rec[4 * i + 1], rec[4 * i + 2], rec[4 * i + 3]);
  }
};

// FUSED (ctr != nullptr): no k_push_finish.  Every piece of a straddling run
// adds its partial record into acc[u], then arrives on ctr[u] with ONE 64-bit
// atomic carrying (1 arrival | last piece: its wave index + 1 << 20 | first
// piece: its wave index + 1 << 41); the arrival that completes the count
// (arrivals == last - first + 1 waves, both ends seen) applies the summed
// record and re-zeroes acc[u] and ctr[u].  Exactly one arrival sees the run
// complete, nobody waits for anybody (no cross-workgroup spinning).
constexpr int kPcArrBits = 20, kPcLastShift = 20, kPcFirstShift = 41;
template <int D, class Emit, bool FUSED = false>
__global__ __launch_bounds__(256) void k_push_merge_apply(DoutSource src, Emit em, float* __restrict__ acc,
                                                          int acc_stride, int32_t* __restrict__ inc, float neg_bs,
                                                          unsigned long long* __restrict__ ctr = nullptr) {
  constexpr int Q = 3 + D;
  const PushMergeArgs& a = src.a;
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t pv = (int64_t)*a.n_valid;
  const int lane = threadIdx.x & 63;
  const int64_t wave_base = p - lane;
  if (wave_base >= pv) return;  // whole wave idle
  int32_t u = -1, k = -1;
  float g[Q];
#pragma unroll
  for (int c = 0; c < Q; ++c) g[c] = 0.f;
  if (p < pv) {
    k = a.perm[p];
    u = (k >= 0 && k < a.n) ? a.uid[k] : -2;
    if (u < -1 || u >= a.n) {  // an occurrence / unique id outside the batch
      if (a.err) atomicOr(a.err, 8);
      u = -1;
      k = -1;
    }
  }
  if (k >= 0) {
    if (src.fast(D))
      src.template load_fast<D>(k, g);
    else
      src.load(k, g, Q);
  }
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int32_t uo = __shfl_up(u, off);
#pragma unroll
    for (int c = 0; c < Q; ++c) {
      const float go = __shfl_up(g[c], off);
      if (lane >= off && uo == u) g[c] += go;
    }
  }
  const int32_t u_first = __shfl(u, 0), u_last = __shfl(u, 63);
  int cn = 0, cp = 0;
  auto uid_at = [&](int64_t q) {
    const int32_t kq = a.perm[q];
    return (kq >= 0 && kq < a.n) ? a.uid[kq] : -1;
  };
  if (lane == 63 && p + 1 < pv) cn = uid_at(p + 1) == u && u >= 0;
  if (lane == 0 && wave_base > 0) cp = uid_at(wave_base - 1) == u && u >= 0;
  const int cont_next = __shfl(cn, 63), cont_prev = __shfl(cp, 0);
  if (!FUSED && lane == 63) inc[wave_base >> 6] = (cont_next && !(cont_prev && u_first == u_last)) ? u_last : -1;
  const int32_t un = __shfl_down(u, 1);
  const bool tail = lane == 63 || un != u;
  if (p >= pv || u < 0 || !tail) return;
  float rec[RowF<D>::kQ4 * 4];
#pragma unroll
  for (int c = 0; c < RowF<D>::kQ4 * 4; ++c) rec[c] = 0.f;
  rec[kPushSlot] = src.slot(k);
  rec[kPushShow] = g[0];
  rec[kPushClick] = g[1];
#pragma unroll
  for (int c = 2; c < Q; ++c) rec[kPushEmbedG + (c - 2)] = g[c] * neg_bs;
  const bool straddle = (u == u_last && cont_next) || (u == u_first && cont_prev);
  if (!straddle) {
    em.template emit<D>(u, rec);
    return;
  }
  float* dst = acc + (int64_t)u * acc_stride;
  if (!FUSED) {
    dst[kPushSlot] = rec[kPushSlot];
#pragma unroll
    for (int c = 1; c < RowF<D>::kQ; ++c) atomicAdd(&dst[c], rec[c]);
    return;
  }
#pragma unroll
  for (int c = 1; c < RowF<D>::kQ; ++c) atomicAdd(&dst[c], rec[c]);
  const bool first = !(u == u_first && cont_prev), last = !(u == u_last && cont_next);
  const unsigned long long wv = (unsigned long long)(wave_base >> 6) + 1ull;
  const unsigned long long add =
      1ull + (last ? wv << kPcLastShift : 0ull) + (first ? wv << kPcFirstShift : 0ull);
  // this piece's acc atomics are acknowledged before its arrival (vmcnt
  // counts atomics on CDNA); no cache-maintenance fence
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const unsigned long long now = atomicAdd(&ctr[u], add) + add;
  const unsigned long long arr = now & ((1ull << kPcArrBits) - 1ull);
  const unsigned long long lw = (now >> kPcLastShift) & ((1ull << (kPcFirstShift - kPcLastShift)) - 1ull);
  const unsigned long long fw = now >> kPcFirstShift;
  if (lw == 0 || fw == 0 || arr != lw - fw + 1) return;
  // the completing arrival takes the sum and re-zeroes with atomic
  // exchanges (read at the atomics' coherence point, not a cached line)
  float sum[RowF<D>::kQ4 * 4];
#pragma unroll
  for (int c = 0; c < RowF<D>::kQ4 * 4; ++c) sum[c] = c < RowF<D>::kQ && c != kPushSlot ? atomicExch(&dst[c], 0.f) : 0.f;
  sum[kPushSlot] = rec[kPushSlot];
  atomicExch(&ctr[u], 0ull);
  em.template emit<D>(u, sum);
}

template <int D, class Emit>
__global__ __launch_bounds__(256) void k_push_finish(Emit em, float* __restrict__ acc, int acc_stride,
                                                     const int32_t* __restrict__ inc, const int32_t* n_valid) {
  const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= ((int64_t)*n_valid + 63) / 64) return;
  const int32_t u = inc[w];
  if (u < 0) return;
  float* ap = acc + (int64_t)u * acc_stride;
  float g[RowF<D>::kQ4 * 4];
  load_push<D>(ap, g);
  float4* a4 = reinterpret_cast<float4*>(ap);
#pragma unroll
  for (int i = 0; i < RowF<D>::kQ4; ++i) a4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  em.template emit<D>(u, g);
}

// No-dedup push (FLAGS_enable_pullpush_dedup_keys=false, single shard): the
// pull probed every occurrence, rows[k] is occurrence k's table row.  No
// sort, hash or scan of the keys at all (reference: the atomic push merge of
// box_wrapper.cu:1040-1047 + the PS-side merge of duplicate keys).
// Pass 1 aggregates in LDS first: a workgroup's occurrences are slot-major
// neighbours, so a popular key shows up many times in one workgroup; its
// records are summed with LDS atomics in an open-addressing table keyed by
// row (2 slots per thread, so it never fills), and only each distinct row of
// the workgroup goes to global memory: one CAS on lock[row] elects the row's
// leader (first workgroup representative wins), then one set of fp32 atomics
// into the leader's accumulator.  The accumulator has kOccRep replicas,
// picked by workgroup, so the hottest keys of a power-law batch (present in
// every workgroup) spread their atomics over 8 lines instead of serialising
// on one.  Pass 2: each leader sums and re-zeroes its replicas, applies
// Adagrad and frees the lock.
template <int D>
struct OccCfg {
  static constexpr int kThreads = D <= 8 ? 1024 : (D <= 16 ? 512 : 256);  // LDS table <= ~112 KB
  static constexpr int kSlots = 2 * kThreads;
};
template <int D>
__global__ __launch_bounds__(OccCfg<D>::kThreads) void k_push_occ_elect(DoutSource src, const int64_t* __restrict__ rows,
                                                                int64_t n, float* __restrict__ acc, int acc_stride,
                                                                int32_t* __restrict__ lock,
                                                                int32_t* __restrict__ lead, float neg_bs) {
  constexpr int Q = 3 + D;
  constexpr int QP = RowF<D>::kQ4 * 4;
  constexpr int NS = OccCfg<D>::kSlots;
  constexpr int NT = OccCfg<D>::kThreads;
  __shared__ unsigned int skey[NS];
  __shared__ int srep[NS];
  __shared__ float sacc[NS * QP];
  for (int i = threadIdx.x; i < NS; i += NT) {
    skey[i] = 0xFFFFFFFFu;
    srep[i] = 0x7FFFFFFF;
  }
  for (int i = threadIdx.x; i < NS * QP; i += NT) sacc[i] = 0.f;
  __syncthreads();
  const int64_t k = (int64_t)blockIdx.x * NT + threadIdx.x;
  const int64_t r = k < n ? rows[k] : -1;
  if (k < n) lead[k] = -1;
  if (r >= 0) {
    float g[Q];
    if (src.fast(D))
      src.template load_fast<D>((int32_t)k, g);
    else
      src.load((int32_t)k, g, Q);
    const unsigned int key = (unsigned int)r;
    unsigned int h = (unsigned int)(((uint64_t)key * 0x9E3779B97F4A7C15ull) >> 40) & (NS - 1);
    for (;;) {
      const unsigned int prev = atomicCAS(&skey[h], 0xFFFFFFFFu, key);
      if (prev == 0xFFFFFFFFu || prev == key) break;
      h = (h + 1) & (NS - 1);
    }
    atomicMin(&srep[h], (int)k);
    float* a = sacc + h * QP;
    a[kPushSlot] = src.slot((int32_t)k);  // same slot for every occurrence of a row
    atomicAdd(&a[kPushShow], g[0]);
    atomicAdd(&a[kPushClick], g[1]);
#pragma unroll
    for (int c = 2; c < Q; ++c) atomicAdd(&a[kPushEmbedG + (c - 2)], g[c] * neg_bs);
  }
  __syncthreads();
  const int rep_i = (int)(blockIdx.x % kOccRep);
  for (int i = threadIdx.x; i < NS; i += NT) {
    const unsigned int key = skey[i];
    if (key == 0xFFFFFFFFu) continue;
    const int rep = srep[i];
    const int32_t old = atomicCAS(&lock[key], -1, rep);
    const int32_t l = old == -1 ? rep : old;
    if (l == rep) lead[rep] = rep;
    float* dst = acc + ((int64_t)l * kOccRep + rep_i) * acc_stride;
    const float* a = sacc + i * QP;
    if (l == rep) dst[kPushSlot] = a[kPushSlot];  // only the leader's replica carries the slot
#pragma unroll
    for (int c = 1; c < RowF<D>::kQ; ++c) atomicAdd(&dst[c], a[c]);
  }
}

template <int D>
__global__ __launch_bounds__(256) void k_push_occ_apply(TableDev t, const int64_t* __restrict__ rows, int64_t n,
                                                        float* __restrict__ acc, int acc_stride,
                                                        int32_t* __restrict__ lock, const int32_t* __restrict__ lead,
                                                        SparseSGDConfig cfg, uint64_t seed) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n || lead[k] != (int32_t)k) return;
  const int64_t r = rows[k];
  constexpr int QP = RowF<D>::kQ4 * 4;
  float g[QP];
#pragma unroll
  for (int c = 0; c < QP; ++c) g[c] = 0.f;
#pragma unroll
  for (int q = 0; q < kOccRep; ++q) {
    float* ap = acc + (k * kOccRep + q) * (int64_t)acc_stride;
    float x[QP];
    load_push<D>(ap, x);
#pragma unroll
    for (int c = 0; c < QP; ++c) g[c] += x[c];
    float4* a4 = reinterpret_cast<float4*>(ap);
#pragma unroll
    for (int i = 0; i < RowF<D>::kQ4; ++i) a4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  adagrad_row<D>(t.values + r * (int64_t)t.stride, g, cfg, seed, table_row_key(t, r));
  lock[r] = -1;
}

// Owner-side push of the sharded step, no dedup of the received keys.  Pass
// 1: every received entry with a row elects a leader among the entries of
// that row (first CAS on lock[row] wins) and adds its merged gradient record
// into the leader's (the slot field is kept from the leader); pass 2: each
// leader applies Adagrad to the row and frees the lock.  A key asked by k
// peers costs k-1 record atomics instead of a sort or hash dedup of W*C keys.
template <int D>
__global__ __launch_bounds__(256) void k_owner_push_elect(const int64_t* __restrict__ rows, float* __restrict__ rec,
                                                          int rec_stride, int64_t n, int32_t* __restrict__ lock,
                                                          int32_t* __restrict__ lead) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const int64_t r = rows[e];
  if (r < 0) {
    lead[e] = -1;
    return;
  }
  const int32_t old = atomicCAS(&lock[r], -1, (int32_t)e);
  const int32_t l = old == -1 ? (int32_t)e : old;
  lead[e] = l;
  if (l == (int32_t)e) return;
  constexpr int Q = RowF<D>::kQ;
  const float* src = rec + e * (int64_t)rec_stride;
  float* dst = rec + (int64_t)l * rec_stride;
#pragma unroll
  for (int c = 1; c < Q; ++c) atomicAdd(&dst[c], src[c]);
}

template <int D>
__global__ __launch_bounds__(256) void k_owner_push_apply(TableDev t, const int64_t* __restrict__ rows,
                                                          const float* __restrict__ rec, int rec_stride, int64_t n,
                                                          int32_t* __restrict__ lock, const int32_t* __restrict__ lead,
                                                          SparseSGDConfig cfg, uint64_t seed) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n || lead[e] != (int32_t)e) return;
  const int64_t r = rows[e];
  float g[RowF<D>::kQ4 * 4];
  load_push<D>(rec + e * (int64_t)rec_stride, g);
  adagrad_row<D>(t.values + r * (int64_t)t.stride, g, cfg, seed, table_row_key(t, r));
  lock[r] = -1;
}

// ---------------------------------------------------------------- sharding helpers
__device__ __forceinline__ int64_t owner_lower_bound(const uint64_t* h, int64_t U, uint32_t o, uint32_t N) {
  int64_t lo = 0, hi = U;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (owner_of(h[mid], N) < o) lo = mid + 1; else hi = mid;
  }
  return lo;
}

__global__ void k_shard_pack_send(const uint64_t* __restrict__ uniq_h, const int32_t* u_count, int nranks,
                                  int64_t cap, uint64_t* __restrict__ send, int32_t* overflow) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)nranks * cap) return;
  const uint32_t o = (uint32_t)(t / cap);
  const int64_t j = t % cap;
  const int64_t U = *u_count;
  const int64_t st = owner_lower_bound(uniq_h, U, o, nranks);
  const int64_t en = owner_lower_bound(uniq_h, U, o + 1, nranks);
  const int64_t cnt = en - st;
  send[t] = (j < cnt) ? uniq_h[st + j] : kEmptyKey;
  if (j == 0 && cnt > cap) atomicOr(overflow, 1);
}

__global__ void k_shard_index(const uint64_t* __restrict__ uniq_h, const int32_t* u_count, int64_t u_cap,
                              int nranks, int64_t cap, int64_t* __restrict__ send_index) {
  const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= u_cap) return;
  const int64_t U = *u_count;
  if (u >= U) { send_index[u] = -1; return; }
  const uint32_t o = owner_of(uniq_h[u], nranks);
  const int64_t st = owner_lower_bound(uniq_h, U, o, nranks);
  const int64_t j = u - st;
  send_index[u] = j < cap ? (int64_t)o * cap + j : -1;
}

__global__ void k_gather_by_uid(const float* __restrict__ src, int src_stride, const int32_t* __restrict__ uid,
                                int64_t n, float* __restrict__ out, int out_stride, int width) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const int32_t u = uid[j];
  float* o = out + j * out_stride;
  if (u < 0) {
    for (int c = 0; c < width; ++c) o[c] = 0.f;
    return;
  }
  const float* s = src + (int64_t)u * src_stride;
  if ((width & 3) == 0 && (src_stride & 3) == 0 && (out_stride & 3) == 0) {
    const float4* s4 = reinterpret_cast<const float4*>(s);
    float4* o4 = reinterpret_cast<float4*>(o);
    for (int c = 0; c < width / 4; ++c) o4[c] = s4[c];
  } else {
    for (int c = 0; c < width; ++c) o[c] = s[c];
  }
}

// Sender-side owner pack after the sort-free dedup (unique ids in arbitrary
// order): per block, unique keys are counted per owner in LDS, one global
// atomic per (block, owner) reserves their slots in the owner's fixed-capacity
// segment of the send buffer.  send must be pre-filled with kEmptyKey and
// ocnt zeroed; keys past the capacity are flagged (overflow) and dropped.
constexpr int kMaxRanks = 64;
__global__ __launch_bounds__(256) void k_shard_pack_hash(const uint64_t* __restrict__ uniq_h,
                                                         const int32_t* __restrict__ u_count, int nranks,
                                                         int64_t cap, uint64_t* __restrict__ send,
                                                         int64_t* __restrict__ send_index, int32_t* __restrict__ ocnt,
                                                         int32_t* __restrict__ overflow) {
  __shared__ int32_t lc[kMaxRanks];
  __shared__ int32_t lb[kMaxRanks];
  const int64_t U = *u_count;
  const int64_t b0 = (int64_t)blockIdx.x * blockDim.x;
  if (b0 >= U) return;  // block-uniform
  if (threadIdx.x < nranks) lc[threadIdx.x] = 0;
  __syncthreads();
  const int64_t u = b0 + threadIdx.x;
  uint32_t o = 0;
  int lp = -1;
  uint64_t h = 0;
  if (u < U) {
    h = uniq_h[u];
    o = owner_of(h, (uint32_t)nranks);
    lp = atomicAdd(&lc[o], 1);
  }
  __syncthreads();
  if (threadIdx.x < nranks) lb[threadIdx.x] = lc[threadIdx.x] ? atomicAdd(&ocnt[threadIdx.x], lc[threadIdx.x]) : 0;
  __syncthreads();
  if (u < U) {
    const int64_t p = (int64_t)lb[o] + lp;
    if (p < cap) {
      send[(int64_t)o * cap + p] = h;
      send_index[u] = (int64_t)o * cap + p;
    } else {
      send_index[u] = -1;
      atomicOr(overflow, 1);
    }
  }
}

// Owner-side pull answer straight from the table: out[j] = pull head of the
// row of received entry j (zeros for padding / missing keys).
__global__ __launch_bounds__(256) void k_gather_rows_by_uid(TableDev t, const int64_t* __restrict__ rows,
                                                            const int32_t* __restrict__ uid, int64_t n,
                                                            float* __restrict__ out, int out_stride) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const int32_t u = uid[j];
  const int64_t r = u >= 0 ? rows[u] : -1;
  const int P = kPullHead + t.dim;
  float4* o4 = reinterpret_cast<float4*>(out + j * out_stride);
  const int n4 = out_stride / 4;
  if (r < 0) {
    for (int c = 0; c < n4; ++c) o4[c] = make_float4(0.f, 0.f, 0.f, 0.f);
    return;
  }
  const float4* s4 = reinterpret_cast<const float4*>(t.values + r * (int64_t)t.stride);
  for (int c = 0; c < n4; ++c) {
    float4 v = s4[c];
    const int b = c * 4;
    if (b + 0 >= P) v.x = 0.f;
    if (b + 1 >= P) v.y = 0.f;
    if (b + 2 >= P) v.z = 0.f;
    if (b + 3 >= P) v.w = 0.f;
    o4[c] = v;
  }
}

inline unsigned int nblk(int64_t n, int per = 256) {
  int64_t b = (n + per - 1) / per;
  return (unsigned int)(b < 1 ? 1 : b);
}

}  // namespace

void launch_fill_occurrence(const int64_t* lod, int S, int B, int32_t* occ_slot, int32_t* occ_ins,
                            hipStream_t s) {
  if ((int64_t)S * B == 0) return;
  hipLaunchKernelGGL(k_fill_occ, dim3(nblk((int64_t)S * B)), dim3(256), 0, s, lod, S, B, occ_slot, occ_ins);
}

void launch_gather_pull(const TableDev& t, const int64_t* rows, const int32_t* n_dev, int64_t n,
                        float* out, int out_stride, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_gather_pull, dim3(nblk(n)), dim3(256), 0, s, t, rows, n_dev, n, out, out_stride);
}

int seqpool_cvm_out_width(const SeqpoolCvmArgs& a) {
  return a.use_cvm ? (a.clk_filter ? a.E - 1 : a.E) : a.E - a.cvm_offset - a.embed_thres_size;
}

void launch_seqpool_cvm_fwd(const SeqpoolCvmArgs& a, hipStream_t s) {
  const int64_t n = (int64_t)a.S * a.B;
  if (n == 0) return;
  const dim3 g(nblk(n)), b(256);
  const bool aligned = (a.src_stride % 4) == 0;
  switch (aligned ? a.E : -1) {
    case 11: hipLaunchKernelGGL(k_seqpool_cvm<11>, g, b, 0, s, a); break;
    case 12: hipLaunchKernelGGL(k_seqpool_cvm<12>, g, b, 0, s, a); break;
    case 19: hipLaunchKernelGGL(k_seqpool_cvm<19>, g, b, 0, s, a); break;
    case 35: hipLaunchKernelGGL(k_seqpool_cvm<35>, g, b, 0, s, a); break;
    default: hipLaunchKernelGGL(k_seqpool_cvm_generic, g, b, 0, s, a); break;
  }
}

void launch_push_merge(const PushMergeArgs& a, hipStream_t s) {
  if (a.n <= 0) return;
  const dim3 g(nblk(a.n)), b(256);
  DoutSource src{a};
  const float neg_bs = -a.bs_scale;
  // values [show, click, embed_g, embedx_g...] -> scale from index 2 on
  switch (a.dim) {
    case 8: hipLaunchKernelGGL((k_push_merge<11, DoutSource>), g, b, 0, s, src, a.perm, a.uid, a.n_valid, a.n, a.push, a.push_stride, a.push_index, neg_bs, 2); break;
    case 16: hipLaunchKernelGGL((k_push_merge<19, DoutSource>), g, b, 0, s, src, a.perm, a.uid, a.n_valid, a.n, a.push, a.push_stride, a.push_index, neg_bs, 2); break;
    case 32: hipLaunchKernelGGL((k_push_merge<35, DoutSource>), g, b, 0, s, src, a.perm, a.uid, a.n_valid, a.n, a.push, a.push_stride, a.push_index, neg_bs, 2); break;
    case 4: hipLaunchKernelGGL((k_push_merge<7, DoutSource>), g, b, 0, s, src, a.perm, a.uid, a.n_valid, a.n, a.push, a.push_stride, a.push_index, neg_bs, 2); break;
    default: break;  // unsupported dims rejected on the host side
  }
}

void launch_push_merge_records(const float* rec, int rec_stride, const int32_t* perm,
                               const int32_t* uid, const int32_t* n_valid, int64_t n, int dim,
                               float* out, int out_stride, hipStream_t s) {
  if (n <= 0) return;
  const dim3 g(nblk(n)), b(256);
  RecordSource src{rec, rec_stride};
  switch (dim) {
    case 8: hipLaunchKernelGGL((k_push_merge<11, RecordSource>), g, b, 0, s, src, perm, uid, n_valid, n, out, out_stride, (const int64_t*)nullptr, 1.f, 1 << 20); break;
    case 16: hipLaunchKernelGGL((k_push_merge<19, RecordSource>), g, b, 0, s, src, perm, uid, n_valid, n, out, out_stride, (const int64_t*)nullptr, 1.f, 1 << 20); break;
    case 32: hipLaunchKernelGGL((k_push_merge<35, RecordSource>), g, b, 0, s, src, perm, uid, n_valid, n, out, out_stride, (const int64_t*)nullptr, 1.f, 1 << 20); break;
    case 4: hipLaunchKernelGGL((k_push_merge<7, RecordSource>), g, b, 0, s, src, perm, uid, n_valid, n, out, out_stride, (const int64_t*)nullptr, 1.f, 1 << 20); break;
#define PBX_MERGE_REC(DIM)                                                                                  \
  case DIM:                                                                                                 \
    hipLaunchKernelGGL((k_push_merge<DIM + 3, RecordSource>), g, b, 0, s, src, perm, uid, n_valid, n, out, \
                       out_stride, (const int64_t*)nullptr, 1.f, 1 << 20);                                  \
    break;
    PBX_MERGE_REC(12)
    PBX_MERGE_REC(20)
    PBX_MERGE_REC(24)
    PBX_MERGE_REC(28)
    PBX_MERGE_REC(36)
    PBX_MERGE_REC(40)
    PBX_MERGE_REC(44)
    PBX_MERGE_REC(48)
    PBX_MERGE_REC(52)
    PBX_MERGE_REC(56)
    PBX_MERGE_REC(60)
#undef PBX_MERGE_REC
    default: break;
  }
}

template <int D>
static bool vec_push_ok(const TableDev& t, int push_stride) {
  return t.dim == D && t.stride == RowF<D>::kStride && push_stride % 4 == 0 && push_stride >= RowF<D>::kQ4 * 4;
}

void launch_push_adagrad(const TableDev& t, const int64_t* rows, const float* push,
                         int push_stride, const int32_t* n_dev, int64_t n,
                         const SparseSGDConfig& cfg, uint64_t seed, hipStream_t s) {
  if (n <= 0) return;
  const dim3 g(nblk(n)), b(256);
  if (vec_push_ok<8>(t, push_stride))
    hipLaunchKernelGGL(k_push_adagrad_v<8>, g, b, 0, s, t, rows, push, push_stride, n_dev, n, cfg, seed);
  else if (vec_push_ok<16>(t, push_stride))
    hipLaunchKernelGGL(k_push_adagrad_v<16>, g, b, 0, s, t, rows, push, push_stride, n_dev, n, cfg, seed);
  else if (vec_push_ok<4>(t, push_stride))
    hipLaunchKernelGGL(k_push_adagrad_v<4>, g, b, 0, s, t, rows, push, push_stride, n_dev, n, cfg, seed);
  else if (vec_push_ok<32>(t, push_stride))
    hipLaunchKernelGGL(k_push_adagrad_v<32>, g, b, 0, s, t, rows, push, push_stride, n_dev, n, cfg, seed);
  else
    hipLaunchKernelGGL(k_push_adagrad, g, b, 0, s, t, rows, push, push_stride, n_dev, n, cfg, seed);
}

bool launch_push_adagrad_seg(const TableDev& t, const int64_t* rows, const float* rec, int rec_stride,
                             const int32_t* perm, const int32_t* seg, const int32_t* cnt, const int32_t* n_dev,
                             int64_t n, const SparseSGDConfig& cfg, uint64_t seed, hipStream_t s) {
  if (n <= 0) return true;
  const dim3 g(nblk(n)), b(256);
  if (vec_push_ok<8>(t, rec_stride))
    hipLaunchKernelGGL(k_push_adagrad_seg<8>, g, b, 0, s, t, rows, rec, rec_stride, perm, seg, cnt, n_dev, n, cfg, seed);
  else if (vec_push_ok<16>(t, rec_stride))
    hipLaunchKernelGGL(k_push_adagrad_seg<16>, g, b, 0, s, t, rows, rec, rec_stride, perm, seg, cnt, n_dev, n, cfg, seed);
  else if (vec_push_ok<4>(t, rec_stride))
    hipLaunchKernelGGL(k_push_adagrad_seg<4>, g, b, 0, s, t, rows, rec, rec_stride, perm, seg, cnt, n_dev, n, cfg, seed);
  else if (vec_push_ok<32>(t, rec_stride))
    hipLaunchKernelGGL(k_push_adagrad_seg<32>, g, b, 0, s, t, rows, rec, rec_stride, perm, seg, cnt, n_dev, n, cfg, seed);
  else
    return false;
  return true;
}

bool launch_owner_push(const TableDev& t, const int64_t* rows, float* rec, int rec_stride, int64_t n, int32_t* lock,
                       int32_t* lead, const SparseSGDConfig& cfg, uint64_t seed, hipStream_t s) {
  if (n <= 0) return true;
  const dim3 g(nblk(n)), b(256);
#define PBX_OWNER_PUSH(D)                                                                                  \
  if (t.dim == D && vec_push_ok<D>(t, rec_stride)) {                                                       \
    hipLaunchKernelGGL(k_owner_push_elect<D>, g, b, 0, s, rows, rec, rec_stride, n, lock, lead);           \
    hipLaunchKernelGGL(k_owner_push_apply<D>, g, b, 0, s, t, rows, rec, rec_stride, n, lock, lead, cfg, seed); \
    return true;                                                                                           \
  }
  PBX_OWNER_PUSH(8)
  PBX_OWNER_PUSH(16)
  PBX_OWNER_PUSH(4)
  PBX_OWNER_PUSH(32)
#undef PBX_OWNER_PUSH
  return false;
}

bool launch_push_merge_apply(const PushMergeArgs& a, const TableDev& t, const int64_t* rows, int32_t* inc,
                             unsigned long long* ctr, const SparseSGDConfig& cfg, uint64_t seed, hipStream_t s) {
  if (a.cvm_offset != 2 || a.push_index != nullptr || a.n_valid == nullptr || a.E != 3 + t.dim) return false;
  if (a.n <= 0) return true;
  const dim3 g(nblk(a.n)), gf(nblk((a.n + 63) / 64)), b(256);
  DoutSource src{a};
  const float neg_bs = -a.bs_scale;
  const ApplyEmit em{t, rows, cfg, seed};
#define PBX_MERGE_APPLY(D)                                                                                    \
  if (vec_push_ok<D>(t, a.push_stride)) {                                                                     \
    if (ctr) {                                                                                                \
      hipLaunchKernelGGL((k_push_merge_apply<D, ApplyEmit, true>), g, b, 0, s, src, em, a.push, a.push_stride, \
                         nullptr, neg_bs, ctr);                                                               \
      return true;                                                                                            \
    }                                                                                                         \
    hipLaunchKernelGGL((k_push_merge_apply<D, ApplyEmit>), g, b, 0, s, src, em, a.push, a.push_stride, inc,   \
                       neg_bs, nullptr);                                                                      \
    hipLaunchKernelGGL((k_push_finish<D, ApplyEmit>), gf, b, 0, s, em, a.push, a.push_stride, inc, a.n_valid); \
    return true;                                                                                              \
  }
  PBX_MERGE_APPLY(8)
  PBX_MERGE_APPLY(16)
  PBX_MERGE_APPLY(4)
  PBX_MERGE_APPLY(32)
#undef PBX_MERGE_APPLY
  return false;
}

bool launch_push_occ(const PushMergeArgs& a, const TableDev& t, const int64_t* rows, int32_t* lock, int32_t* lead,
                     const SparseSGDConfig& cfg, uint64_t seed, hipStream_t s) {
  if (a.cvm_offset != 2 || a.E != 3 + t.dim) return false;
  if (a.n <= 0) return true;
  const dim3 g(nblk(a.n)), b(256);
  DoutSource src{a};
  const float neg_bs = -a.bs_scale;
#define PBX_PUSH_OCC(D)                                                                                          \
  if (vec_push_ok<D>(t, a.push_stride)) {                                                                        \
    constexpr int T = OccCfg<D>::kThreads;                                                                      \
    hipLaunchKernelGGL(k_push_occ_elect<D>, dim3((unsigned)((a.n + T - 1) / T)), dim3(T), 0, s, src, rows, a.n,  \
                       a.push, a.push_stride, lock, lead, neg_bs);                                               \
    hipLaunchKernelGGL(k_push_occ_apply<D>, g, b, 0, s, t, rows, a.n, a.push, a.push_stride, lock, lead, cfg, seed); \
    return true;                                                                                                 \
  }
  PBX_PUSH_OCC(8)
  PBX_PUSH_OCC(16)
  PBX_PUSH_OCC(4)
  PBX_PUSH_OCC(32)
#undef PBX_PUSH_OCC
  return false;
}

bool launch_push_merge_send(const PushMergeArgs& a, int dim, float* send, int send_stride, const int64_t* send_index,
                            int32_t* inc, unsigned long long* ctr, hipStream_t s) {
  if (a.cvm_offset != 2 || a.n_valid == nullptr || a.E != 3 + dim || send_stride % 4 != 0) return false;
  if (a.n <= 0) return true;
  const dim3 g(nblk(a.n)), gf(nblk((a.n + 63) / 64)), b(256);
  DoutSource src{a};
  const float neg_bs = -a.bs_scale;
  const SendEmit em{send, send_stride, send_index};
#define PBX_MERGE_SEND(D)                                                                                     \
  if (dim == D && send_stride >= RowF<D>::kQ4 * 4 && a.push_stride >= RowF<D>::kQ4 * 4 && a.push_stride % 4 == 0) { \
    if (ctr) {                                                                                                \
      hipLaunchKernelGGL((k_push_merge_apply<D, SendEmit, true>), g, b, 0, s, src, em, a.push, a.push_stride,  \
                         nullptr, neg_bs, ctr);                                                               \
      return true;                                                                                            \
    }                                                                                                         \
    hipLaunchKernelGGL((k_push_merge_apply<D, SendEmit>), g, b, 0, s, src, em, a.push, a.push_stride, inc,    \
                       neg_bs, nullptr);                                                                      \
    hipLaunchKernelGGL((k_push_finish<D, SendEmit>), gf, b, 0, s, em, a.push, a.push_stride, inc, a.n_valid);  \
    return true;                                                                                              \
  }
  PBX_MERGE_SEND(8)
  PBX_MERGE_SEND(16)
  PBX_MERGE_SEND(4)
  PBX_MERGE_SEND(32)
#undef PBX_MERGE_SEND
  return false;
}

void launch_shard_pack_hash(const uint64_t* uniq_h, const int32_t* u_count, int64_t u_cap, int nranks, int64_t cap,
                            uint64_t* send, int64_t* send_index, int32_t* ocnt, int32_t* overflow, bool prezeroed,
                            hipStream_t s) {
  if (!prezeroed) {
    launch_fill32(send, 0xFFFFFFFFu, 2 * (int64_t)nranks * cap, s);  // kEmptyKey
    launch_fill32(ocnt, 0u, nranks, s);
  }
  hipLaunchKernelGGL(k_shard_pack_hash, dim3(nblk(u_cap)), dim3(256), 0, s, uniq_h, u_count, nranks, cap, send,
                     send_index, ocnt, overflow);
}

void launch_gather_rows_by_uid(const TableDev& t, const int64_t* rows, const int32_t* uid, int64_t n, float* out,
                               int out_stride, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_gather_rows_by_uid, dim3(nblk(n)), dim3(256), 0, s, t, rows, uid, n, out, out_stride);
}

void launch_zero_rows(float* buf, int stride, const int32_t* n_dev, int64_t cap, hipStream_t s) {
  (void)n_dev;
  launch_fill32(buf, 0u, (int64_t)cap * stride, s);
}

void launch_shard_pack(const uint64_t* uniq_h, const int32_t* u_count, int64_t u_cap, int nranks,
                       int64_t cap, uint64_t* send, int64_t* send_index, int32_t* overflow,
                       hipStream_t s) {
  hipLaunchKernelGGL(k_shard_pack_send, dim3(nblk((int64_t)nranks * cap)), dim3(256), 0, s, uniq_h, u_count, nranks, cap, send, overflow);
  hipLaunchKernelGGL(k_shard_index, dim3(nblk(u_cap)), dim3(256), 0, s, uniq_h, u_count, u_cap, nranks, cap, send_index);
}

void launch_gather_by_uid(const float* src, int src_stride, const int32_t* uid, int64_t n,
                          float* out, int out_stride, int width, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_gather_by_uid, dim3(nblk(n)), dim3(256), 0, s, src, src_stride, uid, n, out, out_stride, width);
}

}  // namespace pbx

// On-device batch assembly from a device-resident pass.
//
// The reference builds every minibatch on the host (data_feed.cc
// PackBatchTask / MiniBatchGpuPack: per-slot offset scans and key copies by
// CPU threads, then an H2D per batch).  On MI355X the whole pass's record
// store fits in HBM next to the embedding table (a 100M-instance pass of ~30
// keys is ~50 GB of 288 GB), so the pass is uploaded once and each batch is
// assembled by two kernels straight into the captured step's input buffers:
//
//   k_batch_scan  one workgroup per sparse slot: gathers the B records'
//                 lengths of that slot through the shuffled order and turns
//                 them into slot-local offsets (1024-lane block scan);
//                 writes the slot's key total.
//   k_batch_fill  grid-stride over (slot, record): slot bases from the
//                 totals (LDS), absolute lod, key copy, -1 padding of the
//                 key buffer to its captured length, dense-slot gather.
//
// Outputs match SlotDataset::build_batch exactly (slot-major keys, lod
// [S][B+1], dense [B][Dw] with missing values zero).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "kernels.h"

namespace pbx {
namespace {

constexpr int kScanThreads = 1024;
constexpr int kMaxSlots = 1024;

__device__ inline int64_t wave_incl_scan(int64_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t u = __shfl_up(v, o, 64);
    if (lane >= o) v += u;
  }
  return v;
}

__global__ __launch_bounds__(kScanThreads) void k_batch_scan(BatchSrc src, int64_t begin, int B, int64_t* lod,
                                                              int64_t* tot) {
  __shared__ int64_t wsum[kScanThreads / 64];
  const int s = blockIdx.x;
  const int j = src.sparse_idx[s];
  int64_t* l = lod + (int64_t)s * (B + 1);
  const int per = (B + kScanThreads - 1) / kScanThreads;
  const int b0 = threadIdx.x * per, b1 = min(b0 + per, B);
  const int64_t* __restrict__ order = src.order + begin;
  const int64_t* __restrict__ uoff = src.uoff;
  int64_t sum = 0;
  // kScanUnroll records per round with every load of the round in flight
  // together (order -> offsets is a dependent pair per record; one record at
  // a time left the 26 workgroups latency-bound: 38 us per batch)
  constexpr int kScanUnroll = 8;
  if (per <= kScanUnroll) {
    // one round (B <= 8192): the lengths stay in registers for the offset
    // pass (re-reading the just-written lod entries was a serial chain of
    // global round trips per thread)
    int64_t iv[kScanUnroll], n[kScanUnroll];
#pragma unroll
    for (int u = 0; u < kScanUnroll; ++u) iv[u] = b0 + u < b1 ? order[b0 + u] : -1;
#pragma unroll
    for (int u = 0; u < kScanUnroll; ++u) {
      n[u] = 0;
      if (iv[u] >= 0) {
        const int64_t* o = uoff + iv[u] * src.nu + j;
        n[u] = o[1] - o[0];
      }
      sum += n[u];
    }
    const int64_t incl = wave_incl_scan(sum);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 63) wsum[w] = incl;
    __syncthreads();
    int64_t before = 0, all = 0;
    for (int k = 0; k < kScanThreads / 64; ++k) {
      if (k < w) before += wsum[k];
      all += wsum[k];
    }
    int64_t run = before + incl - sum;
#pragma unroll
    for (int u = 0; u < kScanUnroll; ++u)
      if (b0 + u < b1) {
        l[b0 + u] = run;
        run += n[u];
      }
    if (threadIdx.x == 0) tot[s] = all;
    return;
  }
  for (int bb = b0; bb < b1; bb += kScanUnroll) {
    int64_t iv[kScanUnroll], n[kScanUnroll];
#pragma unroll
    for (int u = 0; u < kScanUnroll; ++u) iv[u] = bb + u < b1 ? order[bb + u] : -1;
#pragma unroll
    for (int u = 0; u < kScanUnroll; ++u) {
      n[u] = 0;
      if (iv[u] >= 0) {
        const int64_t* o = uoff + iv[u] * src.nu + j;
        n[u] = o[1] - o[0];
      }
    }
#pragma unroll
    for (int u = 0; u < kScanUnroll; ++u)
      if (bb + u < b1) {
        l[bb + u] = n[u];
        sum += n[u];
      }
  }
  const int64_t incl = wave_incl_scan(sum);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 63) wsum[w] = incl;
  __syncthreads();
  int64_t before = 0, all = 0;
  for (int k = 0; k < kScanThreads / 64; ++k) {
    if (k < w) before += wsum[k];
    all += wsum[k];
  }
  int64_t run = before + incl - sum;
  for (int b = b0; b < b1; ++b) {
    const int64_t n = l[b];
    l[b] = run;
    run += n;
  }
  if (threadIdx.x == 0) tot[s] = all;
}

__global__ __launch_bounds__(256) void k_batch_fill(BatchSrc src, int64_t begin, int B, int64_t* lod,
                                                     const int64_t* tot, int64_t* keys, int64_t keys_cap,
                                                     float* dense, int32_t* overflow) {
  __shared__ int64_t base[kMaxSlots + 1];
  const int S = src.S;
  if (threadIdx.x == 0) {
    int64_t acc = 0;
    for (int s = 0; s < S; ++s) {
      base[s] = acc;
      acc += tot[s];
    }
    base[S] = acc;
  }
  __syncthreads();
  const int64_t L = base[S];
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t SB = (int64_t)S * B;
  for (int64_t q = t0; q < SB; q += stride) {
    const int s = (int)(q / B), b = (int)(q - (int64_t)s * B);
    int64_t* l = lod + (int64_t)s * (B + 1);
    const int64_t off = base[s] + l[b];
    l[b] = off;
    if (b == 0) l[B] = base[s + 1];
    const int64_t i = src.order[begin + b];
    const int64_t* o = src.uoff + i * src.nu + src.sparse_idx[s];
    const int64_t e0 = o[0], n = o[1] - e0;
    for (int64_t k = 0; k < n; ++k)
      if (off + k < keys_cap) keys[off + k] = src.u64[e0 + k];
  }
  for (int64_t k = L + t0; k < keys_cap; k += stride) keys[k] = -1;
  const int64_t BR = (int64_t)B * src.ndref;
  for (int64_t q = t0; q < BR; q += stride) {
    const int b = (int)(q / src.ndref), r = (int)(q - (int64_t)b * src.ndref);
    const int32_t* d = src.drefs + 4 * r;
    const int64_t i = src.order[begin + b];
    const bool is_u = d[0] == 0;
    const int64_t* o = is_u ? src.uoff + i * src.nu + d[1] : src.foff + i * src.nf + d[1];
    const int64_t e0 = o[0], e1 = o[1];
    float* row = dense + (int64_t)b * src.Dw + d[3];
    for (int c = 0; c < d[2]; ++c) {
      const int64_t e = e0 + c;
      float v = 0.f;
      if (e < e1) v = is_u ? (float)(uint64_t)src.u64[e] : src.f32[e];
      row[c] = v;
    }
  }
  if (t0 == 0) overflow[0] = L > keys_cap ? 1 : 0;
}

}  // namespace

void launch_batch_assemble(const BatchSrc& src, int64_t begin, int B, int64_t* lod, int64_t* tot, int64_t* keys,
                           int64_t keys_cap, float* dense, int32_t* overflow, hipStream_t st) {
  if (B <= 0 || src.S <= 0) return;
  hipLaunchKernelGGL(k_batch_scan, dim3(src.S), dim3(kScanThreads), 0, st, src, begin, B, lod, tot);
  const int64_t work = (int64_t)src.S * B;
  const int blocks = (int)std::min<int64_t>(std::max<int64_t>((work + 255) / 256, 1), 4096);
  hipLaunchKernelGGL(k_batch_fill, dim3(blocks), dim3(256), 0, st, src, begin, B, lod, tot, keys, keys_cap, dense,
                     overflow);
}

int batch_assemble_max_slots() { return kMaxSlots; }

}  // namespace pbx

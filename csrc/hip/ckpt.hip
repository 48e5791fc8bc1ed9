// Streaming sparse checkpoint, device side: compact one range of table rows
// that a save selects (batch model: every row; xbox base / delta: the
// ctr_accessor rules) into a bounded chunk buffer -- feasign (unmixed) +
// value row -- and reset delta_score of the saved rows in place.  The host
// side (ckpt_saver.cpp) walks the table range by range, double-buffered, so
// a save needs two chunk buffers of HBM instead of a copy of the table.
// Selection semantics: distributed/ps/table/ctr_accessor.cc:102-170 (Save /
// SaveCache / UpdateStatAfterSave), reference call sites
// box_wrapper.cc:1286-1318.
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace pbx {
namespace {

__global__ __launch_bounds__(256) void k_save_chunk(TableDev t, int64_t r0, int64_t r1, SaveSelect sel,
                                                    SaveDecode dec, uint64_t* __restrict__ okeys,
                                                    float* __restrict__ ovals, unsigned long long* __restrict__ count) {
  const RowLayout l = make_row_layout(t.dim);
  const int64_t total = (int64_t)t.nb * kBucketSlots;
  const uint32_t sn = t.stash_n ? (*t.stash_n < t.stash_cap ? *t.stash_n : t.stash_cap) : 0u;
  const int64_t end = r1 < total + (int64_t)sn ? r1 : total + (int64_t)sn;
  const int lane = threadIdx.x & 63;
  // the loop bound is wave-uniform (the ballot below needs every lane)
  for (int64_t wb = r0 + (int64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63); wb < end;
       wb += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = wb + lane;
    bool take = false;
    uint64_t key = kEmptyKey;
    if (row < end) {
      if (row < total) {
        const uint64_t b = (uint64_t)row / kBucketSlots;
        if ((uint32_t)(row % kBucketSlots) < t.fill[b]) key = t.keys[row];
      } else {
        key = t.stash_keys[row - total];
      }
      take = key != kEmptyKey && save_keep(sel, t.values + row * (int64_t)t.stride, l);
    }
    // wave compaction: one counter add per wave
    const uint64_t m = __ballot(take);
    if (!m) continue;
    unsigned long long wbase = 0;
    const int first = __ffsll((long long)m) - 1;
    if (lane == first) wbase = atomicAdd(count, (unsigned long long)__popcll(m));
    wbase = __shfl(wbase, first);
    if (!take) continue;
    const unsigned long long o = wbase + __popcll(m & ((1ull << lane) - 1ull));
    okeys[o] = unmix64(key);
    float* v = t.values + row * (int64_t)t.stride;
    if (dec.n == 0) {
      const float4* s4 = reinterpret_cast<const float4*>(v);
      float4* d4 = reinterpret_cast<float4*>(ovals + (int64_t)o * t.stride);
      for (int c = 0; c < t.stride / 4; ++c) d4[c] = s4[c];
    } else {  // codec table: decoded canonical row (reset applied below, on the stored row and the copy)
      float* d = ovals + (int64_t)o * dec.n;
      const int16_t* q = reinterpret_cast<const int16_t*>(v + kEmbedx);
      for (int c = 0; c < dec.n; ++c) {
        const int m = dec.map[c];
        d[c] = m >= 0 ? v[m] : (m == -1 ? 0.f : (float)q[-2 - m] * dec.scale);
      }
    }
    if (sel.reset_delta) v[l.delta_score] = 0.f;
  }
}

}  // namespace

void launch_save_chunk(const TableDev& t, int64_t r0, int64_t r1, const SaveSelect& sel, const SaveDecode& dec,
                       uint64_t* okeys, float* ovals, unsigned long long* count, hipStream_t s) {
  if (r1 <= r0) return;
  const int64_t n = r1 - r0;
  int blocks = (int)((n + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(k_save_chunk, dim3(blocks), dim3(256), 0, s, t, r0, r1, sel, dec, okeys, ovals, count);
}

}  // namespace pbx

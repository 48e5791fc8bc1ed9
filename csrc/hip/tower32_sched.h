// Wave-stream schedule of the fp32 tower (tower32.hip), shared by the device
// code (kernels, packing) and the host (buffer sizes and the fused Adam's
// re-pack position tables in bindings_tower.cpp).
#pragma once
#include <cstdint>

#if defined(__HIPCC__)
#define T32_HD __host__ __device__
#else
#define T32_HD
#endif

namespace pbx {

// ---------------------------------------------------------------- fp32 tower wave streams
// One layer of the fp32 tower is ncol column blocks of 16 outputs, each a
// K-reduction over ng k-groups of 16.  A workgroup is ONE wave per SIMD (4
// waves, 256 threads) on a 32-row tile, so no wave shares its SIMD's matrix
// pipe and none is left running alone at the end of a layer (with two waves
// per SIMD the second to finish ran its tail at ~1/4 of the MFMA rate:
// profiles/r5_t32_schedule_ab.txt).  The 4 waves split a layer evenly:
//   * full units: PAIRS of column blocks (2p, 2p + 1), pair p = 4u + w for
//     u < q = ncol / 8 -- both 16-row halves, all ng k-groups: four
//     independent accumulators, every weight fragment feeds 2 MFMAs and every
//     LDS activation fragment 2;
//   * the Rb = ncol - 8q leftover blocks (0..7), flattened block-major into T
//     = Rb ng (block, k-group) items, cut into 4 contiguous ranges
//     [lo(w), lo(w + 1)), lo(w) = w T / 4: each wave computes K-partial sums
//     of at most kT32MaxSeg leftover blocks (segments), reduced in wave order
//     (deterministic).
// Each wave's weight fragments (1 KB per (block, k-group): 64 lanes x f32x4)
// form ONE contiguous stream of 2 KB steps: a unit's step g holds the
// fragments of k-group g of its two blocks; a leftover segment's step i holds
// k-groups 2i and 2i + 1 of its block.  Every unit / segment is padded at its
// END to a multiple of kT32Ring steps (pad steps are loaded, never
// multiplied), so the kernel's register ring of kT32Ring steps is refilled in
// stream order across unit boundaries without register moves.
constexpr int kT32Waves = 4;
constexpr int kT32Ring = 4;    // steps (2 KB each) in flight per wave
constexpr int kT32MaxSeg = 3;  // leftover segments per wave (a range of <= 7 ng / 4 + 1 items spans <= 3 blocks)
struct T32Sched {
  int q, Rb, T;
};
T32_HD inline T32Sched t32_sched(int ncol, int ng) {
  T32Sched s;
  s.q = ncol / 8;
  s.Rb = ncol - 8 * s.q;
  s.T = s.Rb * ng;
  return s;
}
T32_HD inline int t32_ceil_ring(int x) { return (x + kT32Ring - 1) / kT32Ring * kT32Ring; }
// first leftover item of wave w (w = 4: T)
T32_HD inline int t32_rem_lo(const T32Sched& s, int w) { return (w * s.T) / kT32Waves; }
// the wave whose leftover range holds item f (< T)
T32_HD inline int t32_rem_wave(const T32Sched& s, int f) {
  int w = kT32Waves - 1;
  while (w > 0 && t32_rem_lo(s, w) > f) --w;
  return w;
}
// padded steps of a leftover segment of len items (2 k-groups per step)
T32_HD inline int t32_seg_steps(int len) { return t32_ceil_ring((len + 1) / 2); }
// padded steps of wave w's leftover segments
T32_HD inline int t32_rem_steps(const T32Sched& s, int ng, int w) {
  const int hi = t32_rem_lo(s, w + 1);
  int n = 0;
  for (int f = t32_rem_lo(s, w); f < hi;) {
    const int g0 = f % ng;
    const int len = (ng - g0) < (hi - f) ? (ng - g0) : (hi - f);
    n += t32_seg_steps(len);
    f += len;
  }
  return n;
}
// step offset of wave w's stream within the layer (w = 4: the layer's total)
T32_HD inline int64_t t32_wave_off(const T32Sched& s, int ng, int w) {
  int64_t off = 0;
  for (int v = 0; v < w; ++v) off += (int64_t)s.q * t32_ceil_ring(ng) + t32_rem_steps(s, ng, v);
  return off;
}
// fragments (1 KB) of a layer's streams
T32_HD inline int64_t t32_stream_groups(int ncol, int ng) { return 2 * t32_wave_off(t32_sched(ncol, ng), ng, kT32Waves); }
// fragment position of column block c, k-group g
T32_HD inline int64_t t32_group_pos(int ncol, int ng, int c, int g) {
  const T32Sched s = t32_sched(ncol, ng);
  if (c < 8 * s.q) {
    const int p = c >> 1, u = p / kT32Waves, w = p % kT32Waves;
    return 2 * (t32_wave_off(s, ng, w) + (int64_t)u * t32_ceil_ring(ng) + g) + (c & 1);
  }
  const int f = (c - 8 * s.q) * ng + g;
  const int w = t32_rem_wave(s, f);
  int64_t st = t32_wave_off(s, ng, w) + (int64_t)s.q * t32_ceil_ring(ng);
  const int hi = t32_rem_lo(s, w + 1);
  for (int f0 = t32_rem_lo(s, w); f0 < hi;) {
    const int g0 = f0 % ng;
    const int len = (ng - g0) < (hi - f0) ? (ng - g0) : (hi - f0);
    if (f < f0 + len) return 2 * (st + (f - f0) / 2) + ((f - f0) & 1);
    st += t32_seg_steps(len);
    f0 += len;
  }
  return 0;  // not reached
}
}  // namespace pbx

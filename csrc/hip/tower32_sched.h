// Wave-stream schedule of the fp32 tower (tower32.hip), shared by the device
// code (packing, kernels) and the host (buffer sizes in bindings_tower.cpp).
#pragma once
#include <cstdint>

#if defined(__HIPCC__)
#define T32_HD __host__ __device__
#else
#define T32_HD
#endif

namespace pbx {

// ---------------------------------------------------------------- fp32 tower wave streams
// One layer of the fp32 tower (tower32.hip) is ncol column blocks of 16
// outputs, each a K-reduction over ng k-groups of 16.  The 8 waves of a
// workgroup (waves w and w + 4 share a SIMD) split it evenly:
//   * full units: column blocks 8i + w (i < q = ncol / 8) -- both 16-row
//     halves of the tile, all ng k-groups;
//   * the R = ncol % 8 remainder blocks, flattened block-major into
//     T = R * ng (block, k-group) pairs, are cut into 8 contiguous ranges
//     [lo(w), lo(w + 1)), lo(w) = w T / 8: every wave computes K-partial sums
//     of at most two remainder blocks (segments), reduced in wave order.
// So every SIMD carries 2 q ng + T / 4 k-groups (+-1).  The packed weights
// follow that schedule: each wave's fragments (1 KB per k-group: 64 lanes x
// f32x4) are ONE contiguous stream -- its full units in order, then its
// remainder segments -- each segment led by pad groups up to a multiple of
// kT32Ring, so every segment fills whole blocks of the kernel's weight ring,
// whose slots are then always refilled in stream order; the ring runs
// from one unit into the next without a cold start (pad groups are loaded,
// never multiplied).
// Priority-aware split (x = 1): waves 4-7 run at s_setprio 1 and win their
// SIMD's issue arbitration (~58 / 42 of the MFMA pipe, per-wave s_memtime
// stamps, scripts/tower32_stamps.py); a wave left alone on its SIMD runs at
// ~1/4 of the MFMA rate (its weight stream's latency is no longer hidden by
// the partner wave).  So when 1 <= ncol % 8 <= 4 the four high-priority waves
// take one extra full unit each -- column blocks ncol - 4 .. ncol - 1 -- and
// the remainder (R = ncol % 8 + 4 <= 8 blocks, q one less) is split over all
// eight waves: at ncol = 25 waves 0-3 carry 2.625 units and waves 4-7 3.625,
// so both waves of a SIMD finish together.  (x = 0: the even split, q =
// ncol / 8 full units per wave.)
// Measured (profiles/r5_t32_schedule_ab.txt): the high-priority waves then
// finish first anyway and the low-priority ones still end ~53k cycles into
// the layer -- no gain (0.356-0.358 ms/step vs 0.355-0.357 even), so it
// is off by default.
#ifndef PBX_T32_PRIO_SPLIT
#define PBX_T32_PRIO_SPLIT 0
#endif
struct T32Sched {
  int q, R, T, x;
};
T32_HD inline T32Sched t32_sched(int ncol, int ng) {
  T32Sched s;
  s.q = ncol / 8;
  // (not when ncol % 8 == 0: the even split then needs no remainder, and
  // the partial-sum LDS a remainder costs does not fit beside 512-wide tiles)
  s.x = (PBX_T32_PRIO_SPLIT && s.q >= 1 && ncol % 8 >= 1 && ncol % 8 <= 4) ? 1 : 0;
  if (s.x) s.q -= 1;
  s.R = ncol - 8 * s.q - 4 * s.x;
  s.T = s.R * ng;
  return s;
}
// the extra full unit of wave w (x = 1, w >= 4): column block ncol - 8 + w
T32_HD inline bool t32_has_extra(const T32Sched& s, int w) { return s.x && w >= 4; }
// depth of the kernel's weight ring (k-groups in flight per wave) = the
// segment padding granularity
constexpr int kT32Ring = 4;
T32_HD inline int t32_ceil4(int x) { return (x + kT32Ring - 1) / kT32Ring * kT32Ring; }
// Which waves take the remainder K-ranges: all eight (default), or with
// R <= 4 blocks and no extra units the four waves 4-7 / 0-3 only (a range
// of at most ng k-groups still spans at most two blocks).  Waves 4-7 only
// measured 0.352-0.354 ms/step vs 0.355-0.357 (profiles/
// r5_t32_schedule_ab.txt) but made the pipelined-vs-plain equality tests
// (tests/test_gpu_pipeline.py, 1e-6) fail intermittently -- a
// timing-dependent difference not yet explained -- so it stays off.
// PBX_T32_REM: 0 all eight waves, 1 waves 4-7, 2 waves 0-3.
#ifndef PBX_T32_REM
#define PBX_T32_REM 0
#endif
// first flattened remainder pair of wave w (w = 8: T)
T32_HD inline int t32_rem_lo(const T32Sched& s, int w) {
  if (PBX_T32_REM == 0 || s.x || s.R > 4) return (w * s.T) / 8;
  const int v = w - (PBX_T32_REM == 1 ? 4 : 0);
  return v <= 0 ? 0 : v >= 4 ? s.T : (v * s.T) / 4;
}
// the wave whose remainder range holds flattened pair f (< T)
T32_HD inline int t32_rem_wave(const T32Sched& s, int f) {
  int w = 7;
  while (w > 0 && t32_rem_lo(s, w) > f) --w;
  return w;
}
// padded stream length (k-groups) of wave w's remainder segments
T32_HD inline int t32_rem_len(const T32Sched& s, int ng, int w) {
  const int hi = t32_rem_lo(s, w + 1);
  int L = 0;
  for (int f = t32_rem_lo(s, w); f < hi;) {
    const int g0 = f % ng;
    const int len = (ng - g0) < (hi - f) ? (ng - g0) : (hi - f);
    L += t32_ceil4(len);
    f += len;
  }
  return L;
}
// k-group offset of wave w's stream within the layer (w = 8: the layer's total)
T32_HD inline int64_t t32_wave_off(const T32Sched& s, int ng, int w) {
  int64_t off = 0;
  for (int v = 0; v < w; ++v)
    off += (int64_t)(s.q + (t32_has_extra(s, v) ? 1 : 0)) * t32_ceil4(ng) + t32_rem_len(s, ng, v);
  return off;
}
T32_HD inline int64_t t32_stream_groups(int ncol, int ng) {
  return t32_wave_off(t32_sched(ncol, ng), ng, 8);
}
// stream position (in k-groups) of column block c, k-group g
T32_HD inline int64_t t32_group_pos(int ncol, int ng, int c, int g) {
  const T32Sched s = t32_sched(ncol, ng);
  if (c < 8 * s.q)
    return t32_wave_off(s, ng, c & 7) + (int64_t)(c >> 3) * t32_ceil4(ng) + (t32_ceil4(ng) - ng) + g;
  if (s.x && c >= ncol - 4)  // the extra unit of wave ncol - c ... : w = c - (ncol - 8)
    return t32_wave_off(s, ng, c - (ncol - 8)) + (int64_t)s.q * t32_ceil4(ng) + (t32_ceil4(ng) - ng) + g;
  const int f = (c - 8 * s.q) * ng + g;
  const int w = t32_rem_wave(s, f);
  int64_t pos = t32_wave_off(s, ng, w) + (int64_t)(s.q + (t32_has_extra(s, w) ? 1 : 0)) * t32_ceil4(ng);
  const int hi = t32_rem_lo(s, w + 1);
  for (int f0 = t32_rem_lo(s, w); f0 < hi;) {
    const int g0 = f0 % ng;
    const int len = (ng - g0) < (hi - f0) ? (ng - g0) : (hi - f0);
    if (f < f0 + len) return pos + (t32_ceil4(len) - len) + (f - f0);
    pos += t32_ceil4(len);
    f0 += len;
  }
  return pos;  // not reached
}
}  // namespace pbx

// Shared definitions for the host (CPU) and device (HIP/gfx950) sides of the
// PaddleBox-capability engine.
//
// Feature value layout (fp32 words, one row per feature).  The first
// kPullHead+D words are exactly the *pull record* ([show, click, embed_w,
// embedx[D]]), so a pull is a contiguous (3+D)*4-byte read of the row.
// Mirrors the fields BoxPS exposes through FeaturePullOffset/FeaturePushOffset
// (reference: paddle/fluid/framework/fleet/box_wrapper.cc:1140-1181) and the
// HeterPS/PSCore value layouts (heter_ps/feature_value.h:42-160,
// distributed/ps/table/ctr_accessor.h:32-66) -- re-laid out so that the pull
// head is contiguous and 16-B aligned for vector loads on CDNA4.
#pragma once
#include <cstdint>

#if defined(__HIPCC__)
#define PBX_HD __host__ __device__ __forceinline__
#else
#define PBX_HD inline
#endif

namespace pbx {

// ---- value row layout -------------------------------------------------------
enum : int {
  kShow = 0,
  kClick = 1,
  kEmbedW = 2,
  kEmbedx = 3,  // embedx_w[0..D)
  kPullHead = 3,
};
// Tail fields follow the embedx block: [embed_g2sum, embedx_g2sum, delta_score,
// slot, unseen_days, mf_size(=embedx created flag)] then optional Adam state.
struct RowLayout {
  int dim;          // embedx dim D
  int embed_g2sum;  // index
  int embedx_g2sum;
  int delta_score;
  int slot;
  int unseen_days;
  int mf_size;
  int stride;  // row stride in floats (multiple of 4 -> 16-B rows)
};

PBX_HD RowLayout make_row_layout(int dim) {
  RowLayout l;
  l.dim = dim;
  l.embed_g2sum = kEmbedx + dim;
  l.embedx_g2sum = l.embed_g2sum + 1;
  l.delta_score = l.embed_g2sum + 2;
  l.slot = l.embed_g2sum + 3;
  l.unseen_days = l.embed_g2sum + 4;
  l.mf_size = l.embed_g2sum + 5;
  int used = l.mf_size + 1;
  l.stride = (used + 3) & ~3;
  return l;
}

// Push record (per unique key): [slot, show, click, embed_g, embedx_g[D]]
enum : int { kPushSlot = 0, kPushShow = 1, kPushClick = 2, kPushEmbedG = 3, kPushEmbedxG = 4 };
PBX_HD int push_width(int dim) { return kPushEmbedxG + dim; }
PBX_HD int pull_width(int dim) { return kPullHead + dim; }

// ---- sparse optimizer config (Adagrad family) ------------------------------
// Defaults from heter_ps/optimizer_conf.h:20-45; semantic per
// heter_ps/optimizer.cuh.h:42-133 and ctr_accessor.cc:245-279.
struct SparseSGDConfig {
  float nonclk_coeff = 0.1f;
  float clk_coeff = 1.0f;
  float min_bound = -10.f;
  float max_bound = 10.f;
  float learning_rate = 0.05f;
  float initial_g2sum = 3.0f;
  float initial_range = 0.0f;
  float mf_create_thresholds = 10.f;
  float mf_learning_rate = 0.05f;
  float mf_initial_g2sum = 3.0f;
  float mf_initial_range = 1e-4f;
  float mf_min_bound = -10.f;
  float mf_max_bound = 10.f;
  float nodeid_slot = 9008.f;
  float feature_learning_rate = 0.05f;
  int use_feature_lr = 0;  // per-slot lr override (optimizer.cuh.h:52-55)
};

// ---- 64-bit mixing -----------------------------------------------------------
// Keys are stored in the tables as h = mix64(key).  mix64 is a bijection
// (splitmix64 finalizer), so dedup on h == dedup on key, the owner shard is a
// monotone function of h (so sorting by h groups keys by owner), and the key is
// recovered for checkpoints with unmix64.
PBX_HD uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
PBX_HD uint64_t unxorshift(uint64_t x, int s) {
  uint64_t r = x;
  for (int i = 0; i < 64 / s + 1; ++i) r = x ^ (r >> s);
  return r;
}
PBX_HD uint64_t unmix64(uint64_t z) {
  z = unxorshift(z, 31);
  z *= 0x319642b2d24d8ec3ULL;  // inverse of 0x94d049bb133111eb
  z = unxorshift(z, 27);
  z *= 0x96de1b173f119089ULL;  // inverse of 0xbf58476d1ce4e5b9
  z = unxorshift(z, 30);
  return z;
}
// secondary hash for cuckoo bucket 2
PBX_HD uint64_t rehash64(uint64_t h) {
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdULL;
  h ^= h >> 33;
  h *= 0xc4ceb9fe1a85ec53ULL;
  h ^= h >> 33;
  return h;
}
// Owner shard of a mixed key: floor(h * n / 2^64) -- monotone in h.
PBX_HD uint32_t owner_of(uint64_t h, uint32_t n) {
#if defined(__HIP_DEVICE_COMPILE__)
  return (uint32_t)__umul64hi(h, (uint64_t)n);
#else
  return (uint32_t)(((unsigned __int128)h * n) >> 64);
#endif
}
PBX_HD uint64_t fast_range64(uint64_t h, uint64_t n) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __umul64hi(h, n);
#else
  return (uint64_t)(((unsigned __int128)h * n) >> 64);
#endif
}
// counter-based uniform in [0,1)
PBX_HD float hash_uniform(uint64_t a, uint64_t b) {
  uint64_t z = mix64(a * 0x9E3779B97F4A7C15ULL + b + 0x632BE59BD9B4E019ULL);
  return (float)(z >> 40) * (1.0f / 16777216.0f);
}

// Salt of a row's lazily created embedx (hash_uniform(salt, d) * mf_initial_range):
// a function of the row's mixed key only -- not of the push counter -- so the
// same feature gets the same initial vector in eager steps, captured-graph
// replays (which would repeat a captured counter) and under any sharding.
PBX_HD uint64_t mf_create_salt(uint64_t rkey) { return 0x6D665F637265ULL ^ rkey * 0x9E3779B97F4A7C15ULL; }

constexpr uint64_t kEmptyKey = 0xFFFFFFFFFFFFFFFFULL;  // sentinel in tables / padding
constexpr int kBucketSlots = 16;                       // 16 x 8 B = one 128-B line

}  // namespace pbx

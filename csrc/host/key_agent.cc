#include "key_agent.h"

#include <algorithm>

namespace pbx {

namespace {
inline uint64_t mix(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ULL;
  k ^= k >> 33;
  return k;
}
}  // namespace

KeyAgent::KeyAgent(int shards) {
  int b = 0;
  while ((1 << b) < std::max(1, shards)) ++b;
  bits_ = b;
  for (int i = 0; i < (1 << b); ++i) {
    shards_.emplace_back(new Shard());
    shards_.back()->slot.assign(1024, 0);
  }
}

void KeyAgent::Shard::grow() {
  std::vector<uint64_t> old;
  old.swap(slot);
  slot.assign(old.size() * 2, 0);
  n = 0;
  for (uint64_t k : old)
    if (k) insert(k);
}

void KeyAgent::Shard::insert(uint64_t k) {
  if ((n + 1) * 10 > slot.size() * 7) grow();
  const size_t mask = slot.size() - 1;
  size_t i = (size_t)(mix(k) * 0x9E3779B97F4A7C15ULL >> 7) & mask;
  for (;;) {
    const uint64_t cur = slot[i];
    if (cur == k) return;
    if (cur == 0) {
      slot[i] = k;
      ++n;
      return;
    }
    i = (i + 1) & mask;
  }
}

void KeyAgent::add(const uint64_t* keys, size_t n) {
  const int S = (int)shards_.size();
  if (S == 1) {
    std::lock_guard<std::mutex> lk(shards_[0]->mu);
    for (size_t i = 0; i < n; ++i)
      if (keys[i] != 0 && keys[i] != ~0ULL) shards_[0]->insert(keys[i]);
    return;
  }
  // bucket by shard first so each shard lock is taken once per batch
  std::vector<uint32_t> cnt(S + 1, 0);
  std::vector<uint64_t> tmp(n);
  std::vector<uint16_t> sid(n);
  for (size_t i = 0; i < n; ++i) {
    sid[i] = (uint16_t)(mix(keys[i]) >> (64 - bits_));
    ++cnt[sid[i] + 1];
  }
  for (int s = 0; s < S; ++s) cnt[s + 1] += cnt[s];
  std::vector<uint32_t> pos(cnt.begin(), cnt.end() - 1);
  for (size_t i = 0; i < n; ++i) tmp[pos[sid[i]]++] = keys[i];
  for (int s = 0; s < S; ++s) {
    if (cnt[s] == cnt[s + 1]) continue;
    Shard& sh = *shards_[s];
    std::lock_guard<std::mutex> lk(sh.mu);
    for (uint32_t i = cnt[s]; i < cnt[s + 1]; ++i) {
      const uint64_t k = tmp[i];
      if (k != 0 && k != ~0ULL) sh.insert(k);
    }
  }
}

std::vector<uint64_t> KeyAgent::keys() const {
  std::vector<size_t> off(shards_.size() + 1, 0);
  for (size_t s = 0; s < shards_.size(); ++s) off[s + 1] = off[s] + shards_[s]->n;
  std::vector<uint64_t> out(off.back());
  for (size_t s = 0; s < shards_.size(); ++s) {
    Shard& sh = *shards_[s];
    std::lock_guard<std::mutex> lk(sh.mu);
    size_t j = off[s];
    for (uint64_t k : sh.slot)
      if (k) out[j++] = k;
  }
  return out;
}

size_t KeyAgent::size() const {
  size_t n = 0;
  for (auto& s : shards_) {
    std::lock_guard<std::mutex> lk(s->mu);
    n += s->n;
  }
  return n;
}

void KeyAgent::clear() {
  for (auto& s : shards_) {
    std::lock_guard<std::mutex> lk(s->mu);
    s->slot.assign(1024, 0);
    s->n = 0;
  }
}

}  // namespace pbx

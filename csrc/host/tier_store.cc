#include "tier_store.h"

#include <dirent.h>
#include <fcntl.h>
#include <omp.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <thread>

namespace pbx {

// ====================================================================== HostTier
static std::vector<int> parse_cpulist(const std::string& s) {
  std::vector<int> out;
  std::stringstream ss(s);
  std::string tok;
  while (std::getline(ss, tok, ',')) {
    if (tok.empty()) continue;
    const auto dash = tok.find('-');
    if (dash == std::string::npos) {
      out.push_back(std::atoi(tok.c_str()));
    } else {
      const int a = std::atoi(tok.substr(0, dash).c_str()), b = std::atoi(tok.substr(dash + 1).c_str());
      for (int c = a; c <= b; ++c) out.push_back(c);
    }
  }
  return out;
}

static std::vector<std::vector<int>> numa_topology() {
  std::vector<std::vector<int>> nodes;
  for (int n = 0; n < 64; ++n) {
    std::ifstream f("/sys/devices/system/node/node" + std::to_string(n) + "/cpulist");
    if (!f) break;
    std::string s;
    std::getline(f, s);
    auto cpus = parse_cpulist(s);
    if (!cpus.empty()) nodes.push_back(cpus);
  }
  return nodes;
}

HostTier::HostTier(int stride, int threads, int64_t chunk_rows)
    : stride_(stride), chunk_rows_(chunk_rows < 1024 ? 1024 : chunk_rows), shards_(kShards) {
  if (stride < 1) throw std::runtime_error("HostTier: stride");
  node_cpus_ = numa_topology();
  // chunk pointers never move: readers index chunks_ while a writer appends
  chunks_.reserve(kMaxChunks);
  epochs_.reserve(kMaxChunks);
  pool_ = std::make_unique<ThreadPool>(threads < 1 ? 1 : threads);
  for (auto& s : shards_) {
    s.keys.assign(1024, kEmptyKey);
    s.rows.assign(1024, -1);
  }
}

HostTier::~HostTier() {
  for (float* c : chunks_) munmap(c, (size_t)chunk_rows_ * stride_ * sizeof(float));
}

void HostTier::add_chunk() { add_chunks(1); }

// map `count` chunks and first-touch them in parallel, each from a thread
// bound to its NUMA node (round-robin over nodes)
void HostTier::add_chunks(int count) {
  if (chunks_.size() + (size_t)count > (size_t)kMaxChunks) throw std::runtime_error("HostTier: arena full");
  const size_t bytes = (size_t)chunk_rows_ * stride_ * sizeof(float);
  std::vector<std::thread> th;
  for (int c = 0; c < count; ++c) {
    void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
    if (p == MAP_FAILED) throw std::runtime_error("HostTier: mmap failed");
    madvise(p, bytes, MADV_HUGEPAGE);
    const int node = node_cpus_.empty() ? -1 : (int)(chunks_.size() % node_cpus_.size());
    th.emplace_back([this, p, bytes, node] {
      if (node >= 0) {
        cpu_set_t set;
        CPU_ZERO(&set);
        for (int cpu : node_cpus_[node]) CPU_SET(cpu, &set);
        pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
      }
      std::memset(p, 0, bytes);
    });
    chunks_.push_back(static_cast<float*>(p));
    epochs_.emplace_back(new uint32_t[chunk_rows_]());
  }
  for (auto& t : th) t.join();
}

int64_t HostTier::alloc_row() {
  std::lock_guard<std::mutex> lk(alloc_mu_);
  if (!free_rows_.empty()) {
    const int64_t r = free_rows_.back();
    free_rows_.pop_back();
    return r;
  }
  if (next_row_ >= (int64_t)chunks_.size() * chunk_rows_) add_chunk();
  return next_row_++;
}

namespace {
using KeyIdx = std::pair<uint64_t, int64_t>;  // (key, batch index)
constexpr size_t kAhead = 12;                  // prefetch distance of the shard lookups (miss-bound)
template <class S>
inline void prefetch_slot(const S& s, uint64_t j) {
  __builtin_prefetch(&s.keys[j]);
  __builtin_prefetch(&s.rows[j]);
}
}  // namespace

int64_t HostTier::find(const Shard& s, uint64_t h) const {
  const uint64_t mask = s.keys.size() - 1;
  for (uint64_t i = mix64(h) & mask;; i = (i + 1) & mask) {
    const uint64_t k = s.keys[i];
    if (k == h) return (int64_t)i;
    if (k == kEmptyKey) return -1;
  }
}

void HostTier::grow(Shard* s) {
  std::vector<uint64_t> ok;
  std::vector<int64_t> orow;
  ok.swap(s->keys);
  orow.swap(s->rows);
  size_t cap = ok.size();
  while ((double)s->live / cap > 0.35) cap *= 2;
  s->keys.assign(cap, kEmptyKey);
  s->rows.assign(cap, -1);
  const uint64_t mask = cap - 1;
  s->used = 0;
  for (size_t j = 0; j < ok.size(); ++j) {
    if (ok[j] == kEmptyKey || ok[j] == kTomb) continue;
    uint64_t i = mix64(ok[j]) & mask;
    while (s->keys[i] != kEmptyKey) i = (i + 1) & mask;
    s->keys[i] = ok[j];
    s->rows[i] = orow[j];
    ++s->used;
  }
}

int64_t HostTier::size() const {
  int64_t n = 0;
  for (auto& s : shards_) {
    std::lock_guard<std::mutex> lk(s.mu);
    n += s.live;
  }
  return n;
}

int64_t HostTier::memory_bytes() const {
  int64_t b = (int64_t)chunks_.size() * chunk_rows_ * stride_ * 4;
  for (auto& s : shards_) b += (int64_t)s.keys.size() * 16;
  return b;
}

void HostTier::probe(const uint64_t* h, int64_t n, int64_t* rows) const {
  const int T = pool_->size();
  if (n < 65536 || T <= 1) {
    pool_->parallel_range(n, [&](int, int64_t b, int64_t e) {
      for (int64_t i = b; i < e; ++i) {
        const Shard& s = shards_[shard_of(h[i])];
        std::lock_guard<std::mutex> lk(s.mu);
        const int64_t p = find(s, h[i]);
        rows[i] = p < 0 ? -1 : s.rows[p];
      }
    });
    return;
  }
  // Large batches: one shard lock per shard and call, not per key (a lock per
  // key across the pool's threads made a 14M-key probe take 3.6 s on 8 cores,
  // 4x an insert of the same keys).  Each worker buckets its contiguous range
  // by shard, then each shard resolves all of its keys under one lock.
  // (key, batch index) pairs: the per-shard pass then never re-reads h[] at
  // random, and the prefetch of a later key's home slot does not stall on it
  std::vector<std::vector<std::vector<KeyIdx>>> loc(T, std::vector<std::vector<KeyIdx>>(kShards));
  pool_->parallel_range(n, [&](int tid, int64_t b, int64_t e) {
    auto& L = loc[tid];
    for (auto& v : L) v.reserve((size_t)((e - b) / kShards + 16));
    for (int64_t i = b; i < e; ++i) L[shard_of(h[i])].emplace_back(h[i], i);
  });
  pool_->parallel_range(kShards, [&](int, int64_t sb, int64_t se) {
    for (int64_t si = sb; si < se; ++si) {
      const Shard& s = shards_[si];
      std::lock_guard<std::mutex> lk(s.mu);
      const uint64_t pmask = s.keys.size() - 1;
      for (int t = 0; t < T; ++t) {
        const auto& L = loc[t][si];
        for (size_t q = 0; q < L.size(); ++q) {
          if (q + kAhead < L.size()) prefetch_slot(s, mix64(L[q + kAhead].first) & pmask);
          const int64_t p = find(s, L[q].first);
          rows[L[q].second] = p < 0 ? -1 : s.rows[p];
        }
      }
    }
  });
}

void HostTier::insert(const uint64_t* h, int64_t n, int64_t* rows, int64_t* n_new, uint8_t* fresh_out) {
  // 1) bucket the batch by shard: each worker its contiguous range (the
  //    per-shard lists of all workers, in worker order, keep batch order)
  const int T = std::max(1, pool_->size());
  std::vector<std::vector<std::vector<KeyIdx>>> loc(T, std::vector<std::vector<KeyIdx>>(kShards));
  pool_->parallel_range(n, [&](int tid, int64_t b, int64_t e) {
    auto& L = loc[tid];
    for (auto& v : L) v.reserve((size_t)((e - b) / kShards + 16));
    for (int64_t i = b; i < e; ++i) L[shard_of(h[i])].emplace_back(h[i], i);
  });
  // 2) per shard (parallel): resolve present keys, collect the distinct
  //    absent ones, size the shard's table for them once
  std::vector<std::vector<KeyIdx>> fresh(kShards);  // (key, batch index of first occurrence)
  pool_->parallel_range(kShards, [&](int, int64_t b, int64_t e) {
    for (int64_t si = b; si < e; ++si) {
      Shard& s = shards_[si];
      std::lock_guard<std::mutex> lk(s.mu);
      auto& f = fresh[si];
      const uint64_t pmask = s.keys.size() - 1;
      for (int t = 0; t < T; ++t) {
        const auto& L = loc[t][si];
        for (size_t q = 0; q < L.size(); ++q) {
          if (q + kAhead < L.size()) prefetch_slot(s, mix64(L[q + kAhead].first) & pmask);
          const uint64_t k = L[q].first;
          const int64_t i = L[q].second;
          if (k == kEmptyKey || k == kTomb) {
            rows[i] = -1;
            continue;
          }
          const int64_t p = find(s, k);
          rows[i] = p < 0 ? -2 : s.rows[p];
          if (p < 0) f.emplace_back(k, i);
        }
      }
      // dedup absent keys within the batch: sort the (key, first index)
      // pairs (an index sort comparing through h[] missed the cache on
      // every comparison: most of a 14M-new-key insert)
      std::sort(f.begin(), f.end());
      size_t w = 0;
      for (size_t q = 0; q < f.size(); ++q)
        if (q == 0 || f[q].first != f[q - 1].first) f[w++] = f[q];
      f.resize(w);
      if ((double)(s.used + (int64_t)f.size()) / s.keys.size() > 0.7) {
        s.live += (int64_t)f.size();  // grow() sizes for live
        grow(&s);
        s.live -= (int64_t)f.size();
      }
    }
  });
  // 3) one allocation for all new rows: recycled rows first (zeroed), then
  //    fresh arena rows (already zero), adding first-touched chunks as needed
  std::vector<int64_t> base(kShards + 1, 0);
  for (int si = 0; si < kShards; ++si) base[si + 1] = base[si] + (int64_t)fresh[si].size();
  const int64_t total = base[kShards];
  std::vector<int64_t> alloc(total);
  {
    std::lock_guard<std::mutex> lk(alloc_mu_);
    int64_t k = 0;
    std::vector<int64_t> recycled;
    while (k < total && !free_rows_.empty()) {
      alloc[k++] = free_rows_.back();
      recycled.push_back(free_rows_.back());
      free_rows_.pop_back();
    }
    const int64_t need = next_row_ + (total - k);
    const int64_t have = (int64_t)chunks_.size() * chunk_rows_;
    if (need > have) add_chunks((int)((need - have + chunk_rows_ - 1) / chunk_rows_));
    while (k < total) alloc[k++] = next_row_++;
    for (int64_t r : recycled) std::memset(row_ptr(r), 0, (size_t)stride_ * sizeof(float));
    const uint32_t ep = cur_epoch_.load(std::memory_order_relaxed);
    for (int64_t r : alloc) epochs_[r / chunk_rows_][r % chunk_rows_] = ep;
  }
  // 4) per shard (parallel): place the new keys
  pool_->parallel_range(kShards, [&](int, int64_t b, int64_t e) {
    for (int64_t si = b; si < e; ++si) {
      Shard& s = shards_[si];
      std::lock_guard<std::mutex> lk(s.mu);
      const uint64_t mask = s.keys.size() - 1;
      for (size_t q = 0; q < fresh[si].size(); ++q) {
        const uint64_t k = fresh[si][q].first;
        uint64_t j = mix64(k) & mask;
        while (s.keys[j] != kEmptyKey && s.keys[j] != kTomb) j = (j + 1) & mask;
        if (s.keys[j] == kEmptyKey) ++s.used;
        s.keys[j] = k;
        s.rows[j] = alloc[base[si] + (int64_t)q];
        ++s.live;
      }
      for (int t = 0; t < T; ++t)
        for (const auto& ki : loc[t][si]) {
          const bool was_absent = rows[ki.second] == -2;
          if (fresh_out) fresh_out[ki.second] = was_absent ? 1 : 0;
          if (was_absent) rows[ki.second] = s.rows[find(s, ki.first)];
        }
    }
  });
  if (n_new) *n_new = total;
}

void HostTier::gather(const int64_t* rows, int64_t n, float* out, int out_stride) const {
  const int w = std::min(out_stride, stride_);
  pool_->parallel_range(n, [&](int, int64_t b, int64_t e) {
    for (int64_t i = b; i < e; ++i) {
      float* o = out + i * out_stride;
      if (rows[i] < 0) {
        std::memset(o, 0, (size_t)out_stride * sizeof(float));
        continue;
      }
      std::memcpy(o, row_ptr(rows[i]), (size_t)w * sizeof(float));
      if (out_stride > w) std::memset(o + w, 0, (size_t)(out_stride - w) * sizeof(float));
    }
  });
}

void HostTier::scatter(const int64_t* rows, int64_t n, const float* vals, int vstride) {
  const int w = std::min(vstride, stride_);
  pool_->parallel_range(n, [&](int, int64_t b, int64_t e) {
    for (int64_t i = b; i < e; ++i)
      if (rows[i] >= 0) std::memcpy(row_ptr(rows[i]), vals + i * vstride, (size_t)w * sizeof(float));
  });
}

int64_t HostTier::erase(const uint64_t* h, int64_t n) {
  int64_t gone = 0;
  for (int64_t i = 0; i < n; ++i) {
    Shard& s = shards_[shard_of(h[i])];
    std::lock_guard<std::mutex> lk(s.mu);
    const int64_t p = find(s, h[i]);
    if (p < 0) continue;
    {
      std::lock_guard<std::mutex> lk2(alloc_mu_);
      free_rows_.push_back(s.rows[p]);
    }
    s.keys[p] = kTomb;
    s.rows[p] = -1;
    --s.live;
    ++gone;
  }
  return gone;
}

void HostTier::export_all(std::vector<uint64_t>* keys, std::vector<float>* vals) const {
  keys->clear();
  vals->clear();
  for (auto& s : shards_) {
    std::lock_guard<std::mutex> lk(s.mu);
    for (size_t j = 0; j < s.keys.size(); ++j) {
      if (s.keys[j] == kEmptyKey || s.keys[j] == kTomb) continue;
      keys->push_back(s.keys[j]);
      const float* v = row_ptr(s.rows[j]);
      vals->insert(vals->end(), v, v + stride_);
    }
  }
}

void HostTier::extract(const std::function<bool(int64_t, const float*)>& pred, bool erase,
                       std::vector<uint64_t>* keys, std::vector<float>* vals) {
  extract_to(pred, erase, [&](size_t n) {
    keys->resize(n);
    vals->resize(n * (size_t)stride_);
    return std::make_pair(keys->data(), vals->data());
  });
}

void HostTier::extract_to(const std::function<bool(int64_t, const float*)>& pred, bool erase,
                          const OutAlloc& alloc) {
  // pass 1 (parallel over shards, each under its lock): select, tombstone,
  // remember the selected rows; pass 2: every shard copies its rows straight
  // into its slice of the output (one allocation, no per-row vector growth
  // and no concatenation copy)
  std::vector<std::vector<uint64_t>> lk(kShards);
  std::vector<std::vector<int64_t>> lr(kShards);
  pool_->parallel_range(kShards, [&](int, int64_t b, int64_t e) {
    for (int64_t si = b; si < e; ++si) {
      Shard& s = shards_[si];
      std::lock_guard<std::mutex> g(s.mu);
      for (size_t j = 0; j < s.keys.size(); ++j) {
        if (s.keys[j] == kEmptyKey || s.keys[j] == kTomb) continue;
        const int64_t r = s.rows[j];
        if (!pred(r, row_ptr(r))) continue;
        lk[si].push_back(s.keys[j]);
        lr[si].push_back(r);
        if (erase) {
          s.keys[j] = kTomb;
          s.rows[j] = -1;
          --s.live;
        }
      }
    }
  });
  std::vector<size_t> off(kShards + 1, 0);
  for (int si = 0; si < kShards; ++si) off[si + 1] = off[si] + lk[si].size();
  const size_t n = off[kShards];
  const auto out = alloc(n);
  pool_->parallel_range(kShards, [&](int, int64_t b, int64_t e) {
    for (int64_t si = b; si < e; ++si) {
      std::copy(lk[si].begin(), lk[si].end(), out.first + off[si]);
      float* dst = out.second + off[si] * (size_t)stride_;
      for (size_t q = 0; q < lr[si].size(); ++q)
        std::memcpy(dst + q * (size_t)stride_, row_ptr(lr[si][q]), (size_t)stride_ * sizeof(float));
    }
  });
  if (erase) {
    std::lock_guard<std::mutex> g(alloc_mu_);
    for (auto& f : lr) free_rows_.insert(free_rows_.end(), f.begin(), f.end());
  }
}

void HostTier::select_ge(int col, float thr, std::vector<uint64_t>* keys, std::vector<float>* vals) const {
  keys->clear();
  vals->clear();
  if (col < 0 || col >= stride_) return;
  const_cast<HostTier*>(this)->extract([&](int64_t, const float* v) { return v[col] >= thr; }, false, keys, vals);
}

void HostTier::select_ge_to(int col, float thr, const OutAlloc& alloc) const {
  if (col < 0 || col >= stride_) {
    alloc(0);
    return;
  }
  const_cast<HostTier*>(this)->extract_to([&](int64_t, const float* v) { return v[col] >= thr; }, false, alloc);
}

void HostTier::stamp(const int64_t* rows, int64_t n, uint32_t epoch) {
  uint32_t cur = cur_epoch_.load(std::memory_order_relaxed);
  while (epoch > cur && !cur_epoch_.compare_exchange_weak(cur, epoch)) {
  }
  pool_->parallel_range(n, [&](int, int64_t b, int64_t e) {
    for (int64_t i = b; i < e; ++i)
      if (rows[i] >= 0) epochs_[rows[i] / chunk_rows_][rows[i] % chunk_rows_] = epoch;
  });
}

int64_t HostTier::spill_oldest(int64_t keep_rows, std::vector<uint64_t>* keys, std::vector<float>* vals) {
  keys->clear();
  vals->clear();
  return spill_oldest_to(keep_rows, [&](size_t n) {
    keys->resize(n);
    vals->resize(n * (size_t)stride_);
    return std::make_pair(keys->data(), vals->data());
  });
}

int64_t HostTier::spill_oldest_to(int64_t keep_rows, const OutAlloc& alloc) {
  const int64_t need = size() - (keep_rows < 0 ? 0 : keep_rows);
  if (need <= 0) {
    alloc(0);
    return 0;
  }
  // pass histogram over the live rows: small pass ids in a flat array per
  // shard (the common case), larger ones in a map
  constexpr uint32_t kFlat = 4096;
  std::vector<std::vector<int64_t>> hf(kShards, std::vector<int64_t>(kFlat, 0));
  std::vector<std::map<uint32_t, int64_t>> hs(kShards);
  pool_->parallel_range(kShards, [&](int, int64_t b, int64_t e) {
    for (int64_t si = b; si < e; ++si) {
      const Shard& s = shards_[si];
      std::lock_guard<std::mutex> g(s.mu);
      for (size_t j = 0; j < s.keys.size(); ++j)
        if (s.keys[j] != kEmptyKey && s.keys[j] != kTomb) {
          const uint32_t ep = epoch_of_row(s.rows[j]);
          if (ep < kFlat)
            hf[si][ep]++;
          else
            hs[si][ep]++;
        }
    }
  });
  std::map<uint32_t, int64_t> h;
  for (int si = 0; si < kShards; ++si) {
    for (uint32_t ep = 0; ep < kFlat; ++ep)
      if (hf[si][ep]) h[ep] += hf[si][ep];
    for (auto& kv : hs[si]) h[kv.first] += kv.second;
  }
  // boundary pass T: every row of an older pass goes, then `quota` rows of T
  uint32_t T = 0;
  int64_t below = 0;
  for (auto& kv : h) {
    T = kv.first;
    if (below + kv.second >= need) break;
    below += kv.second;
  }
  std::atomic<int64_t> quota{need - below};
  // the boundary pass taken whole: no per-row quota atomic (8M contended
  // fetch_subs were a large part of a spill)
  const bool whole = need - below >= h[T];
  size_t got = 0;
  extract_to(
      [&](int64_t r, const float*) {
        const uint32_t e = epoch_of_row(r);
        return e < T || (e == T && (whole || quota.fetch_sub(1, std::memory_order_relaxed) > 0));
      },
      true, [&](size_t n) {
        got = n;
        return alloc(n);
      });
  return (int64_t)got;
}

int64_t HostTier::shrink(float decay, int unseen_col, float nonclk_coeff, float clk_coeff, float delete_threshold,
                         float max_unseen) {
  if (unseen_col < 2 || unseen_col >= stride_) throw std::runtime_error("HostTier::shrink: unseen column");
  std::vector<std::vector<int64_t>> freed(kShards);
  std::atomic<int64_t> gone{0};
  pool_->parallel_range(kShards, [&](int, int64_t b, int64_t e) {
    for (int64_t si = b; si < e; ++si) {
      Shard& s = shards_[si];
      std::lock_guard<std::mutex> lk(s.mu);
      int64_t g = 0;
      for (size_t j = 0; j < s.keys.size(); ++j) {
        if (s.keys[j] == kEmptyKey || s.keys[j] == kTomb) continue;
        float* v = row_ptr(s.rows[j]);
        v[0] *= decay;
        v[1] *= decay;
        v[unseen_col] += 1.f;
        const float score = (v[0] - v[1]) * nonclk_coeff + v[1] * clk_coeff;
        if (score < delete_threshold || v[unseen_col] > max_unseen) {
          freed[si].push_back(s.rows[j]);
          s.keys[j] = kTomb;
          s.rows[j] = -1;
          --s.live;
          ++g;
        }
      }
      gone += g;
    }
  });
  std::lock_guard<std::mutex> lk(alloc_mu_);
  for (auto& f : freed) free_rows_.insert(free_rows_.end(), f.begin(), f.end());
  return gone.load();
}

void HostTier::visit(int s0, int s1, const std::function<void(int, uint64_t, float*)>& fn) {
  s0 = std::max(0, s0);
  s1 = std::min(kShards, s1);
  if (s1 <= s0) return;
  pool_->parallel_range(s1 - s0, [&](int, int64_t b, int64_t e) {
    for (int64_t q = b; q < e; ++q) {
      const int si = s0 + (int)q;
      Shard& s = shards_[si];
      std::lock_guard<std::mutex> lk(s.mu);
      for (size_t j = 0; j < s.keys.size(); ++j)
        if (s.keys[j] != kEmptyKey && s.keys[j] != kTomb) fn(si, s.keys[j], row_ptr(s.rows[j]));
    }
  });
}

void HostTier::clear() {
  for (auto& s : shards_) {
    std::lock_guard<std::mutex> lk(s.mu);
    s.keys.assign(1024, kEmptyKey);
    s.rows.assign(1024, -1);
    s.used = s.live = 0;
  }
  std::lock_guard<std::mutex> lk(alloc_mu_);
  free_rows_.clear();
  next_row_ = 0;
  cur_epoch_ = 0;
  // insert() relies on never-used arena rows being zero: release the arena
  for (float* c : chunks_) munmap(c, (size_t)chunk_rows_ * stride_ * sizeof(float));
  chunks_.clear();
  epochs_.clear();
}

// ====================================================================== SsdLog
// record: [u64 key][u32 flags][f32 x stride]; flags bit0 = tombstone
static constexpr int64_t kPage = 4096;

SsdLog::SsdLog(const std::string& dir, int stride, int64_t segment_bytes)
    : dir_(dir), stride_(stride), rec_bytes_(12 + 4 * stride) {
  if (stride < 1 || rec_bytes_ > kPage) throw std::runtime_error("SsdLog: record must fit a 4 KiB page");
  per_page_ = (int)(kPage / rec_bytes_);
  seg_pages_ = std::max<int64_t>(1, segment_bytes / kPage);
  mkdir(dir.c_str(), 0755);
  if (posix_memalign(reinterpret_cast<void**>(&active_buf_), kPage, (size_t)(seg_pages_ * kPage)) != 0)
    throw std::runtime_error("SsdLog: buffer allocation failed");
  // replay existing segments (seg-NNNNNN.log) in id order
  std::vector<int> ids;
  if (DIR* d = opendir(dir.c_str())) {
    while (dirent* e = readdir(d)) {
      int id;
      if (std::sscanf(e->d_name, "seg-%06d.log", &id) == 1) ids.push_back(id);
    }
    closedir(d);
  }
  std::sort(ids.begin(), ids.end());
  for (size_t i = 0; i < ids.size(); ++i) {
    char name[64];
    std::snprintf(name, sizeof(name), "/seg-%06d.log", ids[i]);
    auto s = std::make_unique<Seg>();
    s->id = (int)segs_.size();
    s->path = dir_ + name;
    if (ids[i] != s->id) {  // renumber densely
      char nn[64];
      std::snprintf(nn, sizeof(nn), "/seg-%06d.log", s->id);
      std::rename(s->path.c_str(), (dir_ + nn).c_str());
      s->path = dir_ + nn;
    }
    s->fd = open(s->path.c_str(), O_RDWR);
    if (s->fd < 0) throw std::runtime_error("SsdLog: cannot open " + s->path);
    segs_.push_back(std::move(s));
    replay(segs_.back().get());
  }
  open_segment();
}

SsdLog::~SsdLog() {
  for (auto& s : segs_)
    if (s->fd >= 0) close(s->fd);
  std::free(active_buf_);
}

void SsdLog::replay(Seg* s) {
  struct stat st;
  fstat(s->fd, &st);
  const int64_t pages = st.st_size / kPage;
  std::vector<char> page(kPage);
  for (int64_t p = 0; p < pages; ++p) {
    if (pread(s->fd, page.data(), kPage, p * kPage) != kPage) break;
    for (int r = 0; r < per_page_; ++r) {
      const char* rec = page.data() + (int64_t)r * rec_bytes_;
      uint64_t key;
      uint32_t flags;
      std::memcpy(&key, rec, 8);
      std::memcpy(&flags, rec + 8, 4);
      if (key == kEmptyKey) continue;  // unused slot (pages are 0xFF-filled)
      const int64_t slot = p * per_page_ + r;
      s->slots = std::max(s->slots, slot + 1);
      if (flags & 1u) {
        const int32_t old = index_.erase(key);
        if (old >= 0) segs_[old]->live--;
      } else {
        const int32_t old = index_.set(key, Loc{s->id, slot});
        if (old >= 0) segs_[old]->live--;
        s->live++;
      }
    }
  }
}

void SsdLog::open_segment() {
  auto s = std::make_unique<Seg>();
  s->id = (int)segs_.size();
  char name[64];
  std::snprintf(name, sizeof(name), "/seg-%06d.log", s->id);
  s->path = dir_ + name;
  int fd = -1;
  if (direct_) {
    fd = open(s->path.c_str(), O_RDWR | O_CREAT | O_TRUNC | O_DIRECT, 0644);
    if (fd < 0 && errno == EINVAL) direct_ = false;  // e.g. tmpfs
  }
  if (fd < 0) fd = open(s->path.c_str(), O_RDWR | O_CREAT | O_TRUNC, 0644);
  if (fd < 0) throw std::runtime_error("SsdLog: cannot create " + s->path);
  s->fd = fd;
  segs_.push_back(std::move(s));
  // no clearing of the whole mirror (a 0xFF memset of every segment's
  // buffer on one thread): write_batch packs pages from slot 0 and fills the
  // unused slots of a partly written last page with 0xFF before its flush,
  // and nothing reads past the written slots (replay stops at empty keys)
}

void SsdLog::flush_pages(Seg* s, int64_t first_page, int64_t npages) {
  if (npages <= 0) return;
  // large flushes as up to 8 concurrent pwrites of >= 4 MiB page ranges (an
  // NVMe drive serves several writes in flight; one synchronous pwrite of a
  // whole spill leaves it mostly idle)
  constexpr int64_t kMinPages = 1024;
  const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(8, npages / kMinPages));
  std::atomic<bool> failed{false};
  auto write_range = [&](int64_t p0, int64_t np) {
    const char* src = active_buf_ + p0 * kPage;
    const int64_t bytes = np * kPage;
    int64_t done = 0;
    while (done < bytes) {
      const ssize_t w = pwrite(s->fd, src + done, (size_t)(bytes - done), p0 * kPage + done);
      if (w <= 0) {
        failed = true;
        return;
      }
      done += w;
    }
  };
  if (nt > 1) {
#pragma omp parallel for num_threads(nt) schedule(static, 1)
    for (int t = 0; t < nt; ++t) {
      const int64_t b = npages * t / nt, e = npages * (t + 1) / nt;
      write_range(first_page + b, e - b);
    }
  } else {
    write_range(first_page, npages);
  }
  if (failed && direct_) {
    // O_DIRECT refused a write (e.g. tmpfs): buffered IO on this fd, once more
    int fl = fcntl(s->fd, F_GETFL);
    fcntl(s->fd, F_SETFL, fl & ~O_DIRECT);
    direct_ = false;
    failed = false;
    write_range(first_page, npages);
  }
  if (failed) throw std::runtime_error("SsdLog: write failed");
}

// append records (tomb: deletions) in page-aligned batches, one pwrite per
// touched page range of each segment
void SsdLog::write_batch(const uint64_t* h, const float* vals, int64_t n, int vstride, bool tomb,
                         std::vector<std::pair<uint64_t, Loc>>* placed) {
  const int w = std::min(vstride, stride_);
  int64_t i = 0;
  while (i < n) {
    if (segs_.back()->slots >= seg_pages_ * per_page_) open_segment();
    Seg* s = segs_.back().get();
    const int64_t slot0 = s->slots;
    const int64_t first_page = page_of(slot0);
    const int64_t take = std::min<int64_t>(seg_pages_ * per_page_ - slot0, n - i);
    const size_t pbase = placed->size();
    placed->resize(pbase + (size_t)take);
    // records land in consecutive slots: pack them (and their index
    // entries) in parallel
#pragma omp parallel for schedule(static) if (take > 65536)
    for (int64_t j = 0; j < take; ++j) {
      const int64_t slot = slot0 + j;
      char* rec = active_buf_ + page_of(slot) * kPage + (slot % per_page_) * rec_bytes_;
      const uint32_t flags = tomb ? 1u : 0u;
      std::memcpy(rec, h + i + j, 8);
      std::memcpy(rec + 8, &flags, 4);
      if (tomb) {
        std::memset(rec + 12, 0, (size_t)stride_ * 4);
      } else {
        std::memcpy(rec + 12, vals + (i + j) * vstride, (size_t)w * 4);
        if (w < stride_) std::memset(rec + 12 + (size_t)w * 4, 0, (size_t)(stride_ - w) * 4);
      }
      (*placed)[pbase + (size_t)j] = std::make_pair(h[i + j], Loc{tomb ? -1 : s->id, slot});
    }
    s->slots += take;
    i += take;
    {  // unused slots of the last, partly written page read as empty (0xFF keys)
      const int64_t end_slot = s->slots, page_end = (page_of(end_slot - 1) + 1) * per_page_;
      if (end_slot < page_end)
        std::memset(active_buf_ + page_of(end_slot - 1) * kPage + (end_slot % per_page_) * rec_bytes_, 0xFF,
                    (size_t)((page_end - end_slot) * rec_bytes_));
    }
    flush_pages(s, first_page, page_of(s->slots - 1) - first_page + 1);
  }
}

void SsdLog::put(const uint64_t* h, const float* vals, int64_t n, int vstride) {
  std::lock_guard<std::mutex> lk(mu_);
  std::vector<std::pair<uint64_t, Loc>> placed;
  placed.reserve(n);
  const auto t0 = std::chrono::steady_clock::now();
  write_batch(h, vals, n, vstride, false, &placed);
  const auto t1 = std::chrono::steady_clock::now();
  // index updates shard-parallel; live counts from the returned previous
  // segments (sequential over a few segments' counters)
  std::vector<int32_t> old;
  index_.set_many(placed, &old);
  const auto t2 = std::chrono::steady_clock::now();
  for (size_t i = 0; i < placed.size(); ++i) {
    if (old[i] >= 0) segs_[old[i]]->live--;
    segs_[placed[i].second.seg]->live++;
  }
  if (getenv("PBX_SSD_TIMING"))
    std::fprintf(stderr, "[ssd] put %lld: write %.3f s, index %.3f s, live %.3f s\n", (long long)n,
                 std::chrono::duration<double>(t1 - t0).count(), std::chrono::duration<double>(t2 - t1).count(),
                 std::chrono::duration<double>(std::chrono::steady_clock::now() - t2).count());
}

int64_t SsdLog::erase(const uint64_t* h, int64_t n) {
  std::lock_guard<std::mutex> lk(mu_);
  std::vector<uint64_t> dead;
  std::vector<int32_t> old;
  index_.erase_many(h, n, &old);  // shard-parallel
  for (int64_t i = 0; i < n; ++i) {
    if (old[(size_t)i] < 0) continue;
    segs_[old[(size_t)i]]->live--;
    dead.push_back(h[i]);
  }
  std::vector<std::pair<uint64_t, Loc>> placed;
  write_batch(dead.data(), nullptr, (int64_t)dead.size(), 0, true, &placed);
  return (int64_t)dead.size();
}

// Records of the closed segments are read page-wise: the distinct (segment,
// page) pairs of the request are sorted, consecutive pages of a segment are
// merged into one pread, and the reads of a batch run on up to 16 threads
// (an NVMe drive serves many requests in flight; one synchronous 4 KiB read
// at a time leaves it mostly idle).  Batches bound the read buffer (32 MiB).
void SsdLog::get(const uint64_t* h, int64_t n, uint8_t* found, float* out, int out_stride) const {
  std::lock_guard<std::mutex> lk(mu_);
  const int w = std::min(out_stride, stride_);
  const int active = segs_.back()->id;
  struct Want {
    int32_t seg;
    int64_t page;
    int64_t i;
    int64_t slot;
  };
  // index lookups in parallel (read-only probes; most requested keys of a
  // staging are brand new and miss): per-thread want lists, concatenated in
  // thread order
  const int nt = n > 65536 ? std::max(1, std::min(16, omp_get_max_threads())) : 1;
  std::vector<std::vector<Want>> parts(nt);
#pragma omp parallel num_threads(nt)
  {
    std::vector<Want>& mine = parts[omp_get_thread_num()];
#pragma omp for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
      float* o = out + i * out_stride;
      const Loc* it = index_.find(h[i]);
      if (it == nullptr) {
        found[i] = 0;
        std::memset(o, 0, (size_t)out_stride * 4);
        continue;
      }
      const Loc l = *it;
      found[i] = 1;
      if (l.seg == active) {
        const char* rec = active_buf_ + page_of(l.slot) * kPage + (l.slot % per_page_) * rec_bytes_;
        std::memcpy(o, rec + 12, (size_t)w * 4);
        if (out_stride > w) std::memset(o + w, 0, (size_t)(out_stride - w) * 4);
      } else {
        mine.push_back(Want{l.seg, page_of(l.slot), i, l.slot});
      }
    }
  }
  std::vector<Want> want;
  if (nt == 1) {
    want.swap(parts[0]);
  } else {
    size_t tot = 0;
    for (auto& q : parts) tot += q.size();
    want.reserve(tot);
    for (auto& q : parts) want.insert(want.end(), q.begin(), q.end());
  }
  if (want.empty()) return;
  std::sort(want.begin(), want.end(), [](const Want& a, const Want& b) {
    return a.seg != b.seg ? a.seg < b.seg : a.page < b.page;
  });
  constexpr int64_t kBatchPages = 8192;
  // wanted pages at most this far apart are read as one run (the gap read
  // along); reads are cut to kReadPages pages for the thread pool
  constexpr int64_t kGapPages = 8, kReadPages = 256;
  char* buf = nullptr;
  if (posix_memalign(reinterpret_cast<void**>(&buf), kPage, (size_t)(kBatchPages * kPage)) != 0)
    throw std::runtime_error("SsdLog: alloc");
  std::unique_ptr<char, decltype(&std::free)> guard(buf, &std::free);
  size_t wi = 0;
  while (wi < want.size()) {
    // distinct pages of this batch, merged into runs of consecutive pages
    struct Run {
      int32_t seg;
      int64_t page, npages, buf_page;
    };
    std::vector<Run> runs;
    std::vector<std::pair<size_t, int64_t>> where;  // want index -> buffer page
    int64_t used = 0;
    size_t wj = wi;
    for (; wj < want.size(); ++wj) {
      const Want& q = want[wj];
      const bool same = !runs.empty() && runs.back().seg == q.seg;
      const int64_t end = same ? runs.back().page + runs.back().npages : 0;  // first page past the run
      if (same && end - 1 == q.page) {  // page already in the run
      } else if (same && q.page >= end && q.page - end <= kGapPages) {
        // the next wanted page is close: read through the gap -- one
        // sequential read instead of one 4 KiB read per page once a reload
        // touches a dense part of a spilled segment (a pass's spill is one
        // contiguous run of pages, so a reload of 1 in 5 of its rows hits
        // nearly every page)
        const int64_t add = q.page - end + 1;
        if (used + add > kBatchPages) break;
        runs.back().npages += add;
        used += add;
      } else {
        if (used == kBatchPages) break;
        runs.push_back(Run{q.seg, q.page, 1, used});
        used++;
      }
      const Run& r = runs.back();
      where.emplace_back(wj, r.buf_page + (q.page - r.page));
    }
    // reads of at most kReadPages pages, spread over up to 16 threads (the
    // device sees a queue of them instead of one long read at a time)
    std::vector<Run> reads;
    for (const Run& r : runs)
      for (int64_t o = 0; o < r.npages; o += kReadPages)
        reads.push_back(Run{r.seg, r.page + o, std::min<int64_t>(kReadPages, r.npages - o), r.buf_page + o});
    const int T = (int)std::min<int64_t>(16, std::max<int64_t>(1, (int64_t)reads.size() / 4));
    std::atomic<bool> bad{false};
    auto read_runs = [&](size_t r0, size_t r1) {
      for (size_t k = r0; k < r1; ++k) {
        const Run& r = reads[k];
        const ssize_t bytes = (ssize_t)(r.npages * kPage);
        if (pread(segs_[r.seg]->fd, buf + r.buf_page * kPage, (size_t)bytes, r.page * kPage) != bytes) bad = true;
      }
    };
    if (T == 1) {
      read_runs(0, reads.size());
    } else {
      std::vector<std::thread> th;
      for (int t = 0; t < T; ++t)
        th.emplace_back(read_runs, reads.size() * t / T, reads.size() * (t + 1) / T);
      for (auto& x : th) x.join();
    }
    if (bad) throw std::runtime_error("SsdLog: read failed");
    for (auto& wp : where) {
      const Want& q = want[wp.first];
      const char* rec = buf + wp.second * kPage + (q.slot % per_page_) * rec_bytes_;
      float* o = out + q.i * out_stride;
      std::memcpy(o, rec + 12, (size_t)w * 4);
      if (out_stride > w) std::memset(o + w, 0, (size_t)(out_stride - w) * 4);
    }
    wi = wj;
  }
}

std::vector<uint64_t> SsdLog::keys() const {
  std::lock_guard<std::mutex> lk(mu_);
  std::vector<uint64_t> out;
  out.reserve(index_.size());
  index_.for_each([&](uint64_t k, const Loc&) { out.push_back(k); });
  return out;
}

int64_t SsdLog::disk_bytes() const {
  int64_t b = 0;
  for (auto& s : segs_) b += ((s->slots + per_page_ - 1) / per_page_) * kPage;
  return b;
}

int64_t SsdLog::compact(double min_live) {
  std::vector<uint64_t> keys;
  std::vector<int> victims;
  {
    std::lock_guard<std::mutex> lk(mu_);
    const int active = segs_.back()->id;
    for (auto& s : segs_)
      if (s->id != active && s->fd >= 0 && s->slots > 0 && (double)s->live / (double)s->slots < min_live)
        victims.push_back(s->id);
    if (victims.empty()) return 0;
    index_.for_each([&](uint64_t k, const Loc& l) {
      if (std::find(victims.begin(), victims.end(), l.seg) != victims.end()) keys.push_back(k);
    });
  }
  // re-append the victims' live records (newest copy wins through the index)
  std::vector<uint8_t> f(keys.size());
  std::vector<float> v(keys.size() * stride_);
  get(keys.data(), (int64_t)keys.size(), f.data(), v.data(), stride_);
  put(keys.data(), v.data(), (int64_t)keys.size(), stride_);
  std::lock_guard<std::mutex> lk(mu_);
  // Tombstones in a victim may still shadow an older put of the same key in
  // a segment that survives (replay would resurrect it): carry forward every
  // victim tombstone whose key is still absent when some older segment
  // survives the compaction.
  {
    std::vector<uint64_t> carry;
    char* page = nullptr;
    if (posix_memalign(reinterpret_cast<void**>(&page), kPage, kPage) != 0) throw std::runtime_error("SsdLog: alloc");
    for (int id : victims) {
      bool older = false;
      for (auto& s : segs_)
        if (s->id < id && s->fd >= 0 && std::find(victims.begin(), victims.end(), s->id) == victims.end()) {
          older = true;
          break;
        }
      if (!older) continue;
      Seg* s = segs_[id].get();
      const int64_t pages = s->slots > 0 ? page_of(s->slots - 1) + 1 : 0;
      for (int64_t p = 0; p < pages; ++p) {
        if (pread(s->fd, page, kPage, p * kPage) != kPage) break;
        for (int r = 0; r < per_page_; ++r) {
          const char* rec = page + (int64_t)r * rec_bytes_;
          uint64_t key;
          uint32_t flags;
          std::memcpy(&key, rec, 8);
          std::memcpy(&flags, rec + 8, 4);
          if (key != kEmptyKey && (flags & 1u) && index_.find(key) == nullptr) carry.push_back(key);
        }
      }
    }
    free(page);
    std::sort(carry.begin(), carry.end());
    carry.erase(std::unique(carry.begin(), carry.end()), carry.end());
    if (!carry.empty()) {
      std::vector<std::pair<uint64_t, Loc>> placed;
      write_batch(carry.data(), nullptr, (int64_t)carry.size(), 0, true, &placed);
    }
  }
  for (int id : victims) {  // now record-free: drop the file, keep the id slot
    Seg* s = segs_[id].get();
    close(s->fd);
    s->fd = -1;
    std::remove(s->path.c_str());
    s->slots = 0;
    s->live = 0;
  }
  return (int64_t)keys.size();
}

int64_t SsdLog::rewrite(const std::function<int(uint64_t, float*)>& fn, const std::function<void()>& after_run) {
  std::lock_guard<std::mutex> lk(mu_);
  constexpr int64_t kRunPages = 8192;  // 32 MiB per read
  char* buf = nullptr;
  if (posix_memalign(reinterpret_cast<void**>(&buf), kPage, (size_t)(kRunPages * kPage)) != 0)
    throw std::runtime_error("SsdLog: alloc");
  std::unique_ptr<char, decltype(&std::free)> guard(buf, &std::free);
  const int active = segs_.back()->id;
  int64_t deleted = 0;
  std::vector<uint8_t> dirty;
  for (auto& sp : segs_) {
    Seg* s = sp.get();
    if (s->slots == 0 || (s->fd < 0 && s->id != active)) continue;
    const int64_t pages = page_of(s->slots - 1) + 1;
    for (int64_t p0 = 0; p0 < pages; p0 += kRunPages) {
      const int64_t np = std::min(kRunPages, pages - p0);
      // the active segment is edited in its write-through mirror
      char* base = s->id == active ? active_buf_ + p0 * kPage : buf;
      if (s->id != active) {
        const ssize_t want = (ssize_t)(np * kPage);
        if (pread(s->fd, buf, (size_t)want, p0 * kPage) != want) throw std::runtime_error("SsdLog: read failed");
      }
      dirty.assign((size_t)np, 0);
      for (int64_t p = 0; p < np; ++p) {
        for (int r = 0; r < per_page_; ++r) {
          const int64_t slot = (p0 + p) * per_page_ + r;
          if (slot >= s->slots) break;
          char* rec = base + p * kPage + (int64_t)r * rec_bytes_;
          uint64_t key;
          uint32_t flags;
          std::memcpy(&key, rec, 8);
          std::memcpy(&flags, rec + 8, 4);
          if (key == kEmptyKey || (flags & 1u)) continue;
          const Loc* l = index_.find(key);
          if (l == nullptr || l->seg != s->id || l->slot != slot) continue;  // superseded record
          const int act = fn(key, reinterpret_cast<float*>(rec + 12));
          if (act == kModified) {
            dirty[p] = 1;
          } else if (act == kDelete) {
            flags = 1u;
            std::memcpy(rec + 8, &flags, 4);
            std::memset(rec + 12, 0, (size_t)stride_ * 4);
            index_.erase(key);
            s->live--;
            ++deleted;
            dirty[p] = 1;
          }
        }
      }
      // write the dirty pages back, one pwrite per consecutive range
      for (int64_t p = 0; p < np;) {
        if (!dirty[p]) {
          ++p;
          continue;
        }
        int64_t q = p;
        while (q < np && dirty[q]) ++q;
        if (s->id == active) {
          flush_pages(s, p0 + p, q - p);
        } else {
          const int64_t bytes = (q - p) * kPage;
          int64_t done = 0;
          while (done < bytes) {
            const ssize_t w = pwrite(s->fd, buf + p * kPage + done, (size_t)(bytes - done), (p0 + p) * kPage + done);
            if (w <= 0) throw std::runtime_error("SsdLog: write failed");
            done += w;
          }
        }
        p = q;
      }
      if (after_run) after_run();
    }
  }
  return deleted;
}

int64_t SsdLog::shrink(float decay, int unseen_col, float nonclk_coeff, float clk_coeff, float delete_threshold,
                       float max_unseen) {
  if (unseen_col < 2 || unseen_col >= stride_) throw std::runtime_error("SsdLog::shrink: unseen column");
  return rewrite([&](uint64_t, float* v) {
    v[0] *= decay;
    v[1] *= decay;
    v[unseen_col] += 1.f;
    const float score = (v[0] - v[1]) * nonclk_coeff + v[1] * clk_coeff;
    return (score < delete_threshold || v[unseen_col] > max_unseen) ? (int)kDelete : (int)kModified;
  });
}

int64_t SsdLog::live_fraction_permille() const {
  std::lock_guard<std::mutex> lk(mu_);
  int64_t slots = 0, live = 0;
  for (auto& s : segs_) {
    slots += s->slots;
    live += s->live;
  }
  return slots ? live * 1000 / slots : 1000;
}

}  // namespace pbx

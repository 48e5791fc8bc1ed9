#include "side_tables.h"

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

namespace pbx {

int64_t ReplicaStore::add(const float* v, int n) {
  std::lock_guard<std::mutex> lk(mu_);
  const int64_t off = (int64_t)(rows_.size() / dim_);
  const size_t base = rows_.size();
  rows_.resize(base + dim_, 0.f);
  std::copy(v, v + std::min(n, dim_), rows_.begin() + base);
  return off;
}

int64_t ReplicaStore::size() const {
  std::lock_guard<std::mutex> lk(mu_);
  return (int64_t)(rows_.size() / dim_);
}

std::vector<float> ReplicaStore::data() const {
  std::lock_guard<std::mutex> lk(mu_);
  return rows_;
}

void ReplicaStore::clear() {
  std::lock_guard<std::mutex> lk(mu_);
  rows_.clear();
}

uint64_t InputIndex::add(const std::string& key, const float* v, int n) {
  std::unique_lock<std::shared_mutex> lk(mu_);
  if (dim_ == 0) dim_ = n;
  auto it = index_.find(key);
  if (it != index_.end()) return it->second;
  const uint64_t off = (uint64_t)(rows_.size() / dim_);
  const size_t base = rows_.size();
  rows_.resize(base + dim_, 0.f);
  std::copy(v, v + std::min(n, dim_), rows_.begin() + base);
  index_.emplace(key, off);
  return off;
}

uint64_t InputIndex::offset(const char* key, size_t len) const {
  std::shared_lock<std::shared_mutex> lk(mu_);
  auto it = index_.find(std::string(key, len));
  return it == index_.end() ? kMissing : it->second;
}

int64_t InputIndex::size() const {
  std::shared_lock<std::shared_mutex> lk(mu_);
  return (int64_t)index_.size();
}

std::vector<float> InputIndex::data() const {
  std::shared_lock<std::shared_mutex> lk(mu_);
  return rows_;
}

int64_t InputIndex::load_text(const std::vector<std::string>& files, int threads) {
  std::atomic<size_t> next{0};
  std::atomic<int64_t> n{0};
  std::vector<std::thread> th;
  const int T = std::max(1, std::min<int>(threads, (int)files.size()));
  for (int t = 0; t < T; ++t)
    th.emplace_back([&] {
      std::vector<float> vec;
      for (;;) {
        const size_t fi = next++;
        if (fi >= files.size()) break;
        FILE* fp = fopen(files[fi].c_str(), "r");
        if (!fp) continue;
        char* line = nullptr;
        size_t cap = 0;
        ssize_t len;
        while ((len = getline(&line, &cap, fp)) > 0) {
          char* p = line;
          while (*p == ' ' || *p == '\t') ++p;
          char* k = p;
          while (*p && *p != ' ' && *p != '\t' && *p != '\n') ++p;
          if (p == k) continue;
          const std::string key(k, p - k);
          vec.clear();
          for (;;) {
            char* e = nullptr;
            const float f = strtof(p, &e);
            if (e == p) break;
            vec.push_back(f);
            p = e;
          }
          add(key, vec.data(), (int)vec.size());
          ++n;
        }
        free(line);
        fclose(fp);
      }
    });
  for (auto& x : th) x.join();
  return n.load();
}

}  // namespace pbx

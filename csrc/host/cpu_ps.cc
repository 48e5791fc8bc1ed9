#include "cpu_ps.h"

#include <cmath>

namespace pbx {

CpuTable::CpuTable(int dim, int nshards) : dim_(dim), nshards_(nshards < 1 ? 1 : nshards) {
  layout_ = make_row_layout(dim);
  maps_.resize(nshards_);
}

int64_t CpuTable::size() const {
  int64_t s = 0;
  for (auto& m : maps_) s += (int64_t)m.size();
  return s;
}

void CpuTable::probe(const uint64_t* h, int64_t n, int64_t* rows) const {
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) {
    const auto& m = maps_[shard_of(h[i])];
    auto it = m.find(h[i]);
    rows[i] = it == m.end() ? -1 : it->second;
  }
}

int64_t CpuTable::alloc_row() {
  if (!free_rows_.empty()) {
    int64_t r = free_rows_.back();
    free_rows_.pop_back();
    return r;
  }
  const int64_t r = (int64_t)row_key_.size();
  row_key_.push_back(kEmptyKey);
  arena_.resize(arena_.size() + layout_.stride, 0.f);
  return r;
}

void CpuTable::insert(const uint64_t* h, int64_t n, float initial_range, float mf_initial_range, bool init_embedx,
                      uint64_t seed) {
  // phase 1 (serial): allocate rows for absent keys (dedup inside the batch)
  std::vector<std::pair<uint64_t, int64_t>> fresh;
  fresh.reserve(n);
  {
    std::unordered_map<uint64_t, int64_t> seen;
    for (int64_t i = 0; i < n; ++i) {
      const uint64_t k = h[i];
      if (k == kEmptyKey) continue;
      auto& m = maps_[shard_of(k)];
      if (m.count(k) || seen.count(k)) continue;
      const int64_t r = alloc_row();
      seen[k] = r;
      fresh.emplace_back(k, r);
    }
  }
  // phase 2: init rows + insert into shard maps (parallel over shards)
  std::vector<std::vector<std::pair<uint64_t, int64_t>>> by_shard(nshards_);
  for (auto& kr : fresh) by_shard[shard_of(kr.first)].push_back(kr);
#pragma omp parallel for schedule(dynamic)
  for (int s = 0; s < nshards_; ++s) {
    for (auto& kr : by_shard[s]) {
      float* v = &arena_[kr.second * layout_.stride];
      for (int c = 0; c < layout_.stride; ++c) v[c] = 0.f;
      if (initial_range > 0.f) v[kEmbedW] = (hash_uniform(kr.first, seed) * 2.f - 1.f) * initial_range;
      if (init_embedx) {
        for (int d = 0; d < dim_; ++d) v[kEmbedx + d] = hash_uniform(kr.first, seed + 1 + d) * mf_initial_range;
        v[layout_.mf_size] = 1.f;
      }
      row_key_[kr.second] = kr.first;
      maps_[s][kr.first] = kr.second;
    }
  }
}

void CpuTable::gather(const int64_t* rows, int64_t n, float* out) const {
  const int st = layout_.stride;
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) {
    float* o = out + i * st;
    if (rows[i] < 0) {
      for (int c = 0; c < st; ++c) o[c] = 0.f;
    } else {
      const float* v = &arena_[rows[i] * st];
      for (int c = 0; c < st; ++c) o[c] = v[c];
    }
  }
}

void CpuTable::assign(const int64_t* rows, int64_t n, const float* vals, int vstride) {
  const int st = layout_.stride;
  const int w = vstride < st ? vstride : st;
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) {
    if (rows[i] < 0) continue;
    float* v = &arena_[rows[i] * st];
    for (int c = 0; c < w; ++c) v[c] = vals[i * vstride + c];
  }
}

static inline float clampf(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }

void CpuTable::push_adagrad(const int64_t* rows, int64_t n, const float* push, int pstride,
                            const SparseSGDConfig& cfg, uint64_t seed) {
  const RowLayout l = layout_;
#pragma omp parallel for schedule(static)
  for (int64_t u = 0; u < n; ++u) {
    const int64_t r = rows[u];
    if (r < 0) continue;
    float* v = &arena_[r * l.stride];
    const float* g = push + u * pstride;
    const float slot = g[kPushSlot], g_show = g[kPushShow], g_click = g[kPushClick];
    v[l.slot] = slot;
    const float show = v[kShow] + g_show, click = v[kClick] + g_click;
    v[kShow] = show;
    v[kClick] = click;
    v[l.delta_score] += cfg.nonclk_coeff * (g_show - g_click) + cfg.clk_coeff * g_click;
    v[l.unseen_days] = 0.f;
    const float scale = g_show > 0.f ? g_show : 1.f;
    float lr = cfg.learning_rate, mf_lr = cfg.mf_learning_rate;
    if (cfg.use_feature_lr && slot != cfg.nodeid_slot) lr = mf_lr = cfg.feature_learning_rate;
    {
      const float g2 = v[l.embed_g2sum];
      const float ratio = lr * std::sqrt(cfg.initial_g2sum / (cfg.initial_g2sum + g2));
      const float sg = g[kPushEmbedG] / scale;
      v[kEmbedW] = clampf(v[kEmbedW] + sg * ratio, cfg.min_bound, cfg.max_bound);
      v[l.embed_g2sum] = g2 + sg * sg;
    }
    if (v[l.mf_size] == 0.f) {
      if (cfg.nonclk_coeff * (show - click) + cfg.clk_coeff * click >= cfg.mf_create_thresholds) {
        v[l.mf_size] = 1.f;
        const uint64_t salt = seed ^ (uint64_t)r * 0x9E3779B97F4A7C15ULL;
        for (int d = 0; d < dim_; ++d) v[kEmbedx + d] = hash_uniform(salt, d) * cfg.mf_initial_range;
      }
    } else {
      const float g2 = v[l.embedx_g2sum];
      const float ratio = mf_lr * std::sqrt(cfg.mf_initial_g2sum / (cfg.mf_initial_g2sum + g2));
      float add = 0.f;
      for (int d = 0; d < dim_; ++d) {
        const float sg = g[kPushEmbedxG + d] / scale;
        v[kEmbedx + d] = clampf(v[kEmbedx + d] + sg * ratio, cfg.mf_min_bound, cfg.mf_max_bound);
        add += sg * sg;
      }
      v[l.embedx_g2sum] = g2 + add / (float)dim_;
    }
  }
}

int64_t CpuTable::shrink(float decay, float delete_threshold, float delete_after_unseen_days, float nonclk,
                         float clk) {
  const RowLayout l = layout_;
  std::vector<int64_t> deleted_count(nshards_, 0);
  std::vector<std::vector<int64_t>> freed(nshards_);
#pragma omp parallel for schedule(dynamic)
  for (int s = 0; s < nshards_; ++s) {
    auto& m = maps_[s];
    for (auto it = m.begin(); it != m.end();) {
      float* v = &arena_[it->second * l.stride];
      v[kShow] *= decay;
      v[kClick] *= decay;
      v[l.unseen_days] += 1.f;
      const float score = (v[kShow] - v[kClick]) * nonclk + v[kClick] * clk;
      if (score < delete_threshold || v[l.unseen_days] > delete_after_unseen_days) {
        freed[s].push_back(it->second);
        it = m.erase(it);
        ++deleted_count[s];
      } else {
        ++it;
      }
    }
  }
  int64_t total = 0;
  for (int s = 0; s < nshards_; ++s) {
    total += deleted_count[s];
    for (int64_t r : freed[s]) {
      row_key_[r] = kEmptyKey;
      free_rows_.push_back(r);
    }
  }
  return total;
}

void CpuTable::export_all(std::vector<uint64_t>* keys, std::vector<float>* vals) const {
  keys->clear();
  vals->clear();
  keys->reserve(size());
  vals->reserve(size() * layout_.stride);
  for (auto& m : maps_)
    for (auto& kv : m) {
      keys->push_back(kv.first);
      const float* v = &arena_[kv.second * layout_.stride];
      vals->insert(vals->end(), v, v + layout_.stride);
    }
}

void CpuTable::select_for_save(int mode, const SaveFilter& f, std::vector<uint64_t>* keys,
                               std::vector<float>* vals) {
  const RowLayout l = layout_;
  keys->clear();
  vals->clear();
  for (auto& m : maps_)
    for (auto& kv : m) {
      float* v = &arena_[kv.second * l.stride];
      bool keep = true;
      if (mode != 2) {
        const float score = (v[kShow] - v[kClick]) * f.nonclk_coeff + v[kClick] * f.clk_coeff;
        keep = score >= f.base_threshold && v[l.unseen_days] <= f.delta_keep_days;
        if (mode == 1) keep = keep && v[l.delta_score] >= f.delta_threshold;
      }
      if (!keep) continue;
      keys->push_back(kv.first);
      vals->insert(vals->end(), v, v + l.stride);
      if (mode == 0 || mode == 1) v[l.delta_score] = 0.f;  // saving resets delta score
    }
}

void CpuTable::clear() {
  for (auto& m : maps_) m.clear();
  arena_.clear();
  row_key_.clear();
  free_rows_.clear();
}

int64_t CpuTable::erase(const uint64_t* h, int64_t n) {
  int64_t c = 0;
  for (int64_t i = 0; i < n; ++i) {
    auto& m = maps_[shard_of(h[i])];
    auto it = m.find(h[i]);
    if (it == m.end()) continue;
    row_key_[it->second] = kEmptyKey;
    free_rows_.push_back(it->second);
    m.erase(it);
    ++c;
  }
  return c;
}

}  // namespace pbx

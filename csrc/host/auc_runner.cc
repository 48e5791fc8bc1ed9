#include "auc_runner.h"

#include <algorithm>
#include <stdexcept>
#include <thread>

namespace pbx {

AucRunner::AucRunner(int pool_size, int threads, uint64_t seed)
    : pool_size_(pool_size < 1 ? 1 : pool_size), threads_(threads < 1 ? 1 : threads), pools_(threads_) {
  for (int t = 0; t < threads_; ++t) pools_[t].rng.seed(seed * 0x9E3779B97F4A7C15ULL + (uint64_t)t + 1);
}

void AucRunner::set_eval_slots(const std::vector<int>& u64_idx) {
  eval_ = u64_idx;
  std::sort(eval_.begin(), eval_.end());
  eval_.erase(std::unique(eval_.begin(), eval_.end()), eval_.end());
  int mx = eval_.empty() ? 0 : eval_.back() + 1;
  eval_pos_.assign(mx, -1);
  for (size_t k = 0; k < eval_.size(); ++k) eval_pos_[eval_[k]] = (int)k;
  for (auto& p : pools_) {  // candidate layout changed: start over
    p.off.assign(1, 0);
    p.vals.clear();
    p.slot_entry.clear();
    p.seen = 0;
  }
}

int64_t AucRunner::add_entry(Pool* p, const RecordStore& st, int64_t rec) const {
  const int nu = st.nu;
  for (int u : eval_) {
    const int64_t b = st.u64_off[rec * nu + u], e = st.u64_off[rec * nu + u + 1];
    p->vals.insert(p->vals.end(), st.u64.begin() + b, st.u64.begin() + e);
    p->off.push_back((int64_t)p->vals.size());
  }
  return (int64_t)(p->off.size() - 1) / (int64_t)std::max<size_t>(eval_.size(), 1) - 1;
}

// keep only the entries the reservoir still references (entries written by
// earlier passes and since evicted are dropped), renumbered
void AucRunner::compact(Pool* p) const {
  const int64_t K = (int64_t)eval_.size();
  if (K == 0) return;
  std::vector<int64_t> off{0};
  std::vector<uint64_t> vals;
  for (auto& e : p->slot_entry) {
    for (int64_t k = 0; k < K; ++k) {
      const int64_t b = p->off[e * K + k], f = p->off[e * K + k + 1];
      vals.insert(vals.end(), p->vals.begin() + b, p->vals.begin() + f);
      off.push_back((int64_t)vals.size());
    }
    e = (int64_t)(off.size() - 1) / K - 1;
  }
  p->off.swap(off);
  p->vals.swap(vals);
}

void AucRunner::sample(const RecordStore& st) {
  if (replaced_) throw std::runtime_error("AucRunner.sample: restore the replaced slots first");
  if (eval_.empty()) throw std::runtime_error("AucRunner.sample: no evaluated slots");
  if (eval_.back() >= st.nu) throw std::runtime_error("AucRunner.sample: eval slot out of range");
  const int64_t n = st.nrec();
  cand_pool_.assign(n, 0);
  cand_entry_.assign(n, 0);
  std::vector<std::thread> th;
  for (int t = 0; t < threads_; ++t) {
    th.emplace_back([this, &st, n, t] {
      Pool& p = pools_[t];
      compact(&p);
      const int64_t b = n * t / threads_, e = n * (t + 1) / threads_;
      for (int64_t i = b; i < e; ++i) {
        ++p.seen;
        if ((int64_t)p.slot_entry.size() < pool_size_) {
          p.slot_entry.push_back(add_entry(&p, st, i));
        } else {
          // reservoir: record i replaces a random slot with prob pool/seen
          const uint64_t r = p.rng() % (uint64_t)p.seen;
          if (r < (uint64_t)pool_size_) p.slot_entry[r] = add_entry(&p, st, i);
        }
        // the record's candidate: a random reservoir slot as of now (entries
        // are immutable, so later evictions do not change it)
        const uint64_t pick = p.rng() % (uint64_t)p.slot_entry.size();
        cand_pool_[i] = t;
        cand_entry_[i] = p.slot_entry[pick];
      }
    });
  }
  for (auto& x : th) x.join();
}

std::vector<uint64_t> AucRunner::candidate_keys() const {
  std::vector<uint64_t> out;
  for (const auto& p : pools_) out.insert(out.end(), p.vals.begin(), p.vals.end());
  std::sort(out.begin(), out.end());
  out.erase(std::unique(out.begin(), out.end()), out.end());
  return out;
}

int64_t AucRunner::pool_entries() const {
  int64_t s = 0;
  for (const auto& p : pools_) s += (int64_t)p.slot_entry.size();
  return s;
}

int64_t AucRunner::shuffle(RecordStore* st, const std::vector<int>& u64_idx) {
  if (replaced_) {  // RecordReplaceBack
    st->u64.swap(orig_u64_);
    st->u64_off.swap(orig_off_);
    std::vector<uint64_t>().swap(orig_u64_);
    std::vector<int64_t>().swap(orig_off_);
    replaced_ = false;
  }
  if (u64_idx.empty()) return 0;
  const int64_t n = st->nrec();
  if ((int64_t)cand_entry_.size() != n) throw std::runtime_error("AucRunner.shuffle: store changed since sample()");
  const int nu = st->nu;
  const int64_t K = (int64_t)eval_.size();
  // per used slot: candidate slot position k, or -1 = keep
  std::vector<int> rep(nu, -1);
  for (int u : u64_idx) {
    if (u < 0 || u >= nu || u >= (int)eval_pos_.size() || eval_pos_[u] < 0)
      throw std::runtime_error("AucRunner.shuffle: slot was not registered for evaluation");
    rep[u] = eval_pos_[u];
  }
  const auto& src_off = st->u64_off;
  const auto& src = st->u64;
  auto span = [&](int64_t i, int u, const uint64_t** ptr) -> int64_t {
    if (rep[u] < 0) {
      *ptr = src.data() + src_off[i * nu + u];
      return src_off[i * nu + u + 1] - src_off[i * nu + u];
    }
    const Pool& p = pools_[cand_pool_[i]];
    const int64_t c = cand_entry_[i] * K + rep[u];
    *ptr = p.vals.data() + p.off[c];
    return p.off[c + 1] - p.off[c];
  };
  // pass 1: lengths; pass 2: fill (partitioned by record range)
  std::vector<int64_t> off(n * nu + 1, 0);
  std::vector<int64_t> part_total(threads_, 0), part_rep(threads_, 0);
  std::vector<std::thread> th;
  for (int t = 0; t < threads_; ++t)
    th.emplace_back([&, t] {
      const int64_t b = n * t / threads_, e = n * (t + 1) / threads_;
      int64_t s = 0;
      for (int64_t i = b; i < e; ++i)
        for (int u = 0; u < nu; ++u) {
          const uint64_t* q;
          const int64_t len = span(i, u, &q);
          off[i * nu + u + 1] = len;
          s += len;
          if (rep[u] >= 0) part_rep[t] += len;
        }
      part_total[t] = s;
    });
  for (auto& x : th) x.join();
  th.clear();
  std::vector<int64_t> base(threads_ + 1, 0);
  for (int t = 0; t < threads_; ++t) base[t + 1] = base[t] + part_total[t];
  std::vector<uint64_t> vals(base[threads_]);
  for (int t = 0; t < threads_; ++t)
    th.emplace_back([&, t] {
      const int64_t b = n * t / threads_, e = n * (t + 1) / threads_;
      int64_t pos = base[t];
      for (int64_t i = b; i < e; ++i)
        for (int u = 0; u < nu; ++u) {
          const uint64_t* q;
          const int64_t len = span(i, u, &q);
          std::copy(q, q + len, vals.begin() + pos);
          pos += len;
          off[i * nu + u + 1] = pos;
        }
    });
  for (auto& x : th) x.join();
  orig_u64_.swap(st->u64);
  orig_off_.swap(st->u64_off);
  st->u64.swap(vals);
  st->u64_off.swap(off);
  replaced_ = true;
  int64_t r = 0;
  for (auto v : part_rep) r += v;
  return r;
}

}  // namespace pbx

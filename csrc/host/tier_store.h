// Host and SSD tiers of the HBM -> host -> SSD embedding store.
//
// BoxPS keeps these inside the closed libbox_ps.so (LoadSSD2Mem /
// FeedPass staging / EndPass write-back, box_wrapper.h:1142-1183,
// box_wrapper.cc:120-210); the open reference analogue is the PSCore SSD
// sparse table (distributed/ps/table/ssd_sparse_table.cc).  Designed here
// for the MI355X node: the GPU tier holds a pass's working set (up to
// hundreds of GB of HBM per GPU), so the host tier is a staging-friendly
// row arena and the SSD tier a log-structured segment store.
//
//   HostTier  64 shards of open-addressing key -> row maps (per-shard locks,
//             so feed-pass loader threads can insert concurrently) over one
//             chunked row arena; chunks are mmap'ed with huge-page advice and
//             first-touched by a thread bound to the chunk's NUMA node
//             (round-robin), so gathers into the pinned H2D staging buffer
//             stream from local memory.  gather / scatter are multi-threaded.
//   SsdLog    append-only segment files of fixed-size records packed into
//             4 KiB pages, written with O_DIRECT (page-aligned batches; falls
//             back to buffered IO where the filesystem refuses O_DIRECT);
//             in-memory key -> (segment, slot) index, tombstone records for
//             deletes so the index is rebuilt exactly by replaying segments;
//             compaction rewrites segments whose live fraction is low.
#pragma once

#include <atomic>
#include <cstdint>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include <omp.h>

#include "../common/pbx_common.h"
#include "runtime.h"

namespace pbx {

class HostTier {
 public:
  HostTier(int stride, int threads = 16, int64_t chunk_rows = 1 << 20);
  ~HostTier();
  int stride() const { return stride_; }
  int64_t size() const;
  int64_t memory_bytes() const;
  int numa_nodes() const { return (int)node_cpus_.size(); }

  void probe(const uint64_t* h, int64_t n, int64_t* rows) const;
  // insert absent keys with zeroed rows (duplicates allowed); rows[i] = row of h[i]
  // fresh (optional, [n]): 1 where h[i] was absent before this call
  void insert(const uint64_t* h, int64_t n, int64_t* rows, int64_t* n_new, uint8_t* fresh = nullptr);
  void gather(const int64_t* rows, int64_t n, float* out, int out_stride) const;
  void scatter(const int64_t* rows, int64_t n, const float* vals, int vstride);
  int64_t erase(const uint64_t* h, int64_t n);
  void export_all(std::vector<uint64_t>* keys, std::vector<float>* vals) const;
  // keys/rows whose column `col` >= thr (cold rows for the SSD spill)
  void select_ge(int col, float thr, std::vector<uint64_t>* keys, std::vector<float>* vals) const;
  // pass stamps: every arena row carries the id of the pass that last wrote
  // it (write-back / SSD reload); spill_oldest removes the rows of the oldest
  // passes (whole passes, then part of the boundary pass) until at most
  // keep_rows remain, returning them for the SSD tier.  Parallel over shards.
  void stamp(const int64_t* rows, int64_t n, uint32_t epoch);
  int64_t spill_oldest(int64_t keep_rows, std::vector<uint64_t>* keys, std::vector<float>* vals);
  // output buffers for n selected rows (keys [n], vals [n * stride]), filled in parallel
  using OutAlloc = std::function<std::pair<uint64_t*, float*>(size_t)>;
  int64_t spill_oldest_to(int64_t keep_rows, const OutAlloc& alloc);
  void select_ge_to(int col, float thr, const OutAlloc& alloc) const;
  uint32_t epoch_of_row(int64_t r) const { return epochs_[r / chunk_rows_][r % chunk_rows_]; }
  // end-of-day shrink over every row, in parallel over the shards
  // (ctr_accessor.cc:63-80): show/click *= decay, unseen_days += 1, delete
  // rows with score < delete_threshold or unseen_days > max_unseen.
  // Column indices: show 0, click 1, unseen_col.  Returns rows deleted.
  int64_t shrink(float decay, int unseen_col, float nonclk_coeff, float clk_coeff, float delete_threshold,
                 float max_unseen);
  void clear();
  // every live row of shards [s0, s1), shards in parallel on the pool, each
  // under its lock and visited by one thread: fn(shard, key, row) may modify
  // the row in place (saves, delta reset)
  static constexpr int kNumShards = 64;
  void visit(int s0, int s1, const std::function<void(int, uint64_t, float*)>& fn);
  int threads() const { return pool_->size(); }

 private:
  struct Shard {
    std::vector<uint64_t> keys;  // open addressing, kEmptyKey = free, kTomb = deleted
    std::vector<int64_t> rows;
    int64_t used = 0, live = 0;
    mutable std::mutex mu;
  };
  static constexpr int kShards = kNumShards;
  static constexpr int kMaxChunks = 1 << 16;
  static constexpr uint64_t kTomb = 0xFFFFFFFFFFFFFFFEULL;
  int shard_of(uint64_t h) const { return (int)(h >> 58); }  // top 6 bits
  int64_t find(const Shard& s, uint64_t h) const;
  void grow(Shard* s);
  int64_t alloc_row();
  float* row_ptr(int64_t r) const { return chunks_[r / chunk_rows_] + (r % chunk_rows_) * stride_; }
  void add_chunk();
  void add_chunks(int count);
  // rows matching pred(row, values), in shard order; erased from the tier when `erase`
  void extract(const std::function<bool(int64_t, const float*)>& pred, bool erase, std::vector<uint64_t>* keys,
               std::vector<float>* vals);
  void extract_to(const std::function<bool(int64_t, const float*)>& pred, bool erase, const OutAlloc& alloc);

  int stride_;
  int64_t chunk_rows_;
  std::vector<Shard> shards_;
  std::vector<float*> chunks_;
  std::vector<std::unique_ptr<uint32_t[]>> epochs_;  // one stamp per arena row, chunked like chunks_
  std::vector<int64_t> free_rows_;
  int64_t next_row_ = 0;
  // newest pass stamp seen: rows entering by insert() carry it, so a row
  // loaded / assigned outside a write-back does not look like the oldest
  // pass to spill_oldest (nor inherit a recycled row's stamp)
  std::atomic<uint32_t> cur_epoch_{0};
  std::mutex alloc_mu_;
  std::vector<std::vector<int>> node_cpus_;
  std::unique_ptr<ThreadPool> pool_;
};

// key -> record location of the SSD log: open addressing over flat arrays
// (linear probing, backward-shift deletion, load <= 1/2).  A node-based map
// costs an allocation per record, which dominated a multi-million-row spill.
class LocIndex {
 public:
  struct Loc {
    int32_t seg;
    int64_t slot;
  };
  LocIndex() { rehash(1024); }
  int64_t size() const { return n_; }
  const Loc* find(uint64_t k) const {
    for (uint64_t i = home(k);; i = (i + 1) & mask_) {
      if (keys_[i] == k) return &locs_[i];
      if (keys_[i] == kEmptyKey) return nullptr;
    }
  }
  // insert or overwrite; returns the previous location's segment (-1: new key)
  int32_t set(uint64_t k, Loc l) {
    if ((n_ + 1) * 2 > (int64_t)keys_.size()) rehash(keys_.size() * 2);
    for (uint64_t i = home(k);; i = (i + 1) & mask_) {
      if (keys_[i] == k) {
        const int32_t old = locs_[i].seg;
        locs_[i] = l;
        return old;
      }
      if (keys_[i] == kEmptyKey) {
        keys_[i] = k;
        locs_[i] = l;
        ++n_;
        return -1;
      }
    }
  }
  // returns the erased location's segment (-1: absent)
  int32_t erase(uint64_t k) {
    uint64_t i = home(k);
    for (;; i = (i + 1) & mask_) {
      if (keys_[i] == k) break;
      if (keys_[i] == kEmptyKey) return -1;
    }
    const int32_t old = locs_[i].seg;
    // backward shift: pull later members of the probe chain into the hole
    uint64_t j = i;
    for (;;) {
      j = (j + 1) & mask_;
      if (keys_[j] == kEmptyKey) break;
      const uint64_t h = home(keys_[j]);
      const bool movable = (i <= j) ? (h <= i || h > j) : (h <= i && h > j);
      if (movable) {
        keys_[i] = keys_[j];
        locs_[i] = locs_[j];
        i = j;
      }
    }
    keys_[i] = kEmptyKey;
    --n_;
    return old;
  }
  template <class F>
  void for_each(F f) const {
    for (size_t i = 0; i < keys_.size(); ++i)
      if (keys_[i] != kEmptyKey) f(keys_[i], locs_[i]);
  }
  // grow once for n more keys instead of doubling inside a long insert run
  void reserve_more(int64_t n) {
    size_t cap = keys_.size();
    while ((n_ + n + 1) * 2 > (int64_t)cap) cap *= 2;
    if (cap != keys_.size()) rehash(cap);
  }
  // hide the two cache misses of a later set()/find() of k
  void prefetch(uint64_t k) const {
    const uint64_t i = home(k);
    __builtin_prefetch(&keys_[i], 1);
    __builtin_prefetch(&locs_[i], 1);
  }

 private:
  uint64_t home(uint64_t k) const { return (k ^ (k >> 29) ^ (k >> 47)) * 0x9E3779B97F4A7C15ULL >> 7 & mask_; }
  void rehash(size_t cap) {
    std::vector<uint64_t> ok;
    std::vector<Loc> ol;
    ok.swap(keys_);
    ol.swap(locs_);
    keys_.assign(cap, kEmptyKey);
    locs_.resize(cap);
    mask_ = cap - 1;
    n_ = 0;
    for (size_t i = 0; i < ok.size(); ++i)
      if (ok[i] != kEmptyKey) set(ok[i], ol[i]);
  }
  std::vector<uint64_t> keys_;
  std::vector<Loc> locs_;
  uint64_t mask_ = 0;
  int64_t n_ = 0;
};

// The SSD record index split into 64 independent LocIndex shards by the
// key's top bits: bulk insert / erase of a spill (millions of keys per
// write-back) run one shard per thread -- the single open-addressing table
// took most of an 8.6M-row SsdLog::put in one thread.  Single-key calls keep
// the LocIndex interface.
class ShardedLocIndex {
 public:
  using Loc = LocIndex::Loc;
  static constexpr int kShards = 64;
  int64_t size() const {
    int64_t n = 0;
    for (const auto& s : sh_) n += s.size();
    return n;
  }
  const Loc* find(uint64_t k) const { return sh_[shard(k)].find(k); }
  int32_t set(uint64_t k, Loc l) { return sh_[shard(k)].set(k, l); }
  int32_t erase(uint64_t k) { return sh_[shard(k)].erase(k); }
  void prefetch(uint64_t k) const { sh_[shard(k)].prefetch(k); }
  template <class F>
  void for_each(F f) const {
    for (const auto& s : sh_) s.for_each(f);
  }
  // old[i] = set(keys[i], locs[i]) for every i, shards in parallel
  void set_many(const std::vector<std::pair<uint64_t, Loc>>& kl, std::vector<int32_t>* old) {
    const int64_t n = (int64_t)kl.size();
    old->assign((size_t)n, -1);
    std::vector<std::vector<int64_t>> by(kShards);
    bucket(n, [&](int64_t i) { return kl[(size_t)i].first; }, &by);
#pragma omp parallel for schedule(dynamic, 1)
    for (int q = 0; q < kShards; ++q) {
      LocIndex& s = sh_[q];
      s.reserve_more((int64_t)by[q].size());
      const auto& ids = by[q];
      for (size_t j = 0; j < ids.size(); ++j) {
        if (j + 16 < ids.size()) s.prefetch(kl[(size_t)ids[j + 16]].first);
        (*old)[(size_t)ids[j]] = s.set(kl[(size_t)ids[j]].first, kl[(size_t)ids[j]].second);
      }
    }
  }
  // old[i] = erase(keys[i]), shards in parallel
  void erase_many(const uint64_t* keys, int64_t n, std::vector<int32_t>* old) {
    old->assign((size_t)n, -1);
    std::vector<std::vector<int64_t>> by(kShards);
    bucket(n, [&](int64_t i) { return keys[i]; }, &by);
#pragma omp parallel for schedule(dynamic, 1)
    for (int q = 0; q < kShards; ++q)
      for (int64_t i : by[q]) (*old)[(size_t)i] = sh_[q].erase(keys[i]);
  }

 private:
  static int shard(uint64_t k) { return (int)((k * 0x9E3779B97F4A7C15ULL) >> 58); }
  template <class K>
  static void bucket(int64_t n, K key, std::vector<std::vector<int64_t>>* by) {
    // per-thread buckets, concatenated in thread order: each shard's keys
    // stay in input order (a repeated key keeps its last placement)
    const int nt = n > 65536 ? std::max(1, std::min(16, omp_get_max_threads())) : 1;
    std::vector<std::vector<std::vector<int64_t>>> part(nt, std::vector<std::vector<int64_t>>(kShards));
#pragma omp parallel num_threads(nt)
    {
      const int t = omp_get_thread_num();
      const int64_t b = n * t / nt, e = n * (t + 1) / nt;
      for (int64_t i = b; i < e; ++i) part[t][shard(key(i))].push_back(i);
    }
#pragma omp parallel for schedule(dynamic, 1)
    for (int q = 0; q < kShards; ++q) {
      size_t tot = 0;
      for (int t = 0; t < nt; ++t) tot += part[t][q].size();
      (*by)[q].reserve(tot);
      for (int t = 0; t < nt; ++t) (*by)[q].insert((*by)[q].end(), part[t][q].begin(), part[t][q].end());
    }
  }
  LocIndex sh_[kShards];
};

class SsdLog {
 public:
  SsdLog(const std::string& dir, int stride, int64_t segment_bytes = 64ll << 20);
  ~SsdLog();
  int stride() const { return stride_; }
  int64_t size() const { return index_.size(); }
  int64_t disk_bytes() const;
  bool direct_io() const { return direct_; }
  int64_t segments() const { return (int64_t)segs_.size(); }

  void put(const uint64_t* h, const float* vals, int64_t n, int vstride);
  // found[i] = 1 and out[i] = record when present
  void get(const uint64_t* h, int64_t n, uint8_t* found, float* out, int out_stride) const;
  int64_t erase(const uint64_t* h, int64_t n);
  // rewrite segments whose live fraction < min_live; returns records moved
  int64_t compact(double min_live = 0.5);
  // In-place pass over every live record, segment by segment (sequential
  // reads of up to 32 MiB): fn(key, values) returns kKeep, kModified (its
  // page is written back in place) or kDelete (the record becomes a
  // tombstone in place and leaves the index -- replay stays exact: no later
  // segment holds the key).  after_run() runs after each read run, so a
  // consumer can flush what fn collected.  Returns the records deleted.
  enum : int { kKeep = 0, kModified = 1, kDelete = 2 };
  int64_t rewrite(const std::function<int(uint64_t, float*)>& fn, const std::function<void()>& after_run = {});
  // end-of-day shrink of every SSD record (HostTier::shrink's rule, applied
  // eagerly through rewrite); returns rows deleted
  int64_t shrink(float decay, int unseen_col, float nonclk_coeff, float clk_coeff, float delete_threshold,
                 float max_unseen);
  int64_t live_fraction_permille() const;
  std::vector<uint64_t> keys() const;

 private:
  struct Seg {
    int id;
    int fd;
    int64_t slots = 0;  // records written
    int64_t live = 0;
    std::string path;
  };
  using Loc = LocIndex::Loc;
  void open_segment();
  void replay(Seg* s);
  void write_batch(const uint64_t* h, const float* vals, int64_t n, int vstride, bool tomb,
                   std::vector<std::pair<uint64_t, Loc>>* placed);
  void flush_pages(Seg* s, int64_t first_page, int64_t npages);
  int64_t page_of(int64_t slot) const { return slot / per_page_; }

  std::string dir_;
  int stride_;
  int rec_bytes_;
  int per_page_;
  int64_t seg_pages_;
  bool direct_ = true;
  std::vector<std::unique_ptr<Seg>> segs_;  // segs_[i]->id == i (closed segments keep their fd)
  ShardedLocIndex index_;
  // the active segment is mirrored in memory (page-aligned, written through)
  char* active_buf_ = nullptr;
  mutable std::mutex mu_;
};

}  // namespace pbx

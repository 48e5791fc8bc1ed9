// Side tables the data feed fills while loading (reference: BoxWrapper's
// gpu_replica_cache / input_table_deque_, box_wrapper.h:63-197, fed by
// SlotPaddleBoxDataFeedWithGpuReplicaCache / InputTableDataFeed /
// InputIndexDataFeed, data_feed.cc:4155-4635).
//
//   ReplicaStore  fixed-width float rows appended by the loader threads (one
//                 per instance that carries a cache vector); the instance
//                 stores the row offset as a feasign and pull_cache_value
//                 gathers the rows from the HBM copy.
//   InputIndex    string key -> dense vector table (lookup_input): filled
//                 from index files ("key v1 v2 ... vD" lines or a plugin's
//                 parse_index), queried by the loader to turn an instance's
//                 string key into a row offset.
#pragma once

#include <cstdint>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <unordered_map>
#include <vector>

namespace pbx {

class ReplicaStore {
 public:
  explicit ReplicaStore(int dim) : dim_(dim) {}
  int dim() const { return dim_; }
  // appends one row (n values, zero padded / truncated to dim); returns its offset
  int64_t add(const float* v, int n);
  int64_t size() const;
  std::vector<float> data() const;
  void clear();

 private:
  int dim_;
  mutable std::mutex mu_;
  std::vector<float> rows_;
};

class InputIndex {
 public:
  explicit InputIndex(int dim = 0) : dim_(dim) {}
  int dim() const { return dim_; }
  // first insert of a key wins; returns the key's offset
  uint64_t add(const std::string& key, const float* v, int n);
  // offset of key, or kMissing
  uint64_t offset(const char* key, size_t len) const;
  int64_t size() const;
  std::vector<float> data() const;
  // "key v1 ... vD" text lines (whitespace separated), files split over threads
  int64_t load_text(const std::vector<std::string>& files, int threads);
  static constexpr uint64_t kMissing = ~0ULL;

 private:
  int dim_;
  mutable std::shared_mutex mu_;
  std::unordered_map<std::string, uint64_t> index_;
  std::vector<float> rows_;
};

}  // namespace pbx

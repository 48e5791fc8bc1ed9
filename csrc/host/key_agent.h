// Feed-pass key registration (reference: boxps::PSAgentBase AddKey/AddKeys
// fed by the dataset's loader / merge threads, box_wrapper.cc:1185-1232,
// data_set.cc:2293-2349).  Loader threads stage the feasigns of the records
// they parse in thread-local buffers and flush them in batches into a set
// sharded by key hash (one lock per shard, 64 shards), so the pass's unique
// key set is complete when the load returns -- no separate walk over the
// store, no global sort.
#pragma once

#include <cstdint>
#include <memory>
#include <mutex>
#include <vector>

namespace pbx {

class KeyAgent {
 public:
  explicit KeyAgent(int shards = 64);
  // thread-safe; key 0 and ~0 (padding / empty) are ignored
  void add(const uint64_t* keys, size_t n);
  // unique keys in unspecified order
  std::vector<uint64_t> keys() const;
  size_t size() const;
  void clear();

  // per-thread staging buffer: add() on flush (and on destruction)
  class Stage {
   public:
    explicit Stage(KeyAgent* a, size_t cap = 1 << 16) : a_(a), cap_(cap) { buf_.reserve(cap); }
    ~Stage() { flush(); }
    void push(uint64_t k) {
      buf_.push_back(k);
      if (buf_.size() >= cap_) flush();
    }
    void flush() {
      if (a_ && !buf_.empty()) a_->add(buf_.data(), buf_.size());
      buf_.clear();
    }

   private:
    KeyAgent* a_;
    size_t cap_;
    std::vector<uint64_t> buf_;
  };

 private:
  struct Shard {
    std::mutex mu;
    std::vector<uint64_t> slot;  // open addressing, 0 = empty
    size_t n = 0;
    void insert(uint64_t k);
    void grow();
  };
  std::vector<std::unique_ptr<Shard>> shards_;
  int bits_;
};

}  // namespace pbx

// AucRunner: slot-importance evaluation by feature replacement
// (reference BoxWrapper::InitializeAucRunner / GetRandomReplace /
// RecordReplace / RecordReplaceBack / AddReplaceFeasign,
// box_wrapper.h:906-1011, box_wrapper.cc:212-368, and the reservoir
// candidate pool FeasignValuesCandidateList, data_feed.h:1774-1962).
//
// Re-designed for the columnar pass store (RecordStore, one CSR of uint64
// feasigns per (record, slot)): each partition of the pass keeps a reservoir
// of sampled records' evaluated-slot values; every record is assigned one
// candidate.  Replacing a slot set rebuilds the CSR in two parallel passes
// (count, fill) with the evaluated slots taken from the candidates, and the
// original arrays are kept for the restore -- no per-record objects.
#pragma once

#include <cstdint>
#include <random>
#include <vector>

#include "slot_dataset.h"

namespace pbx {

class AucRunner {
 public:
  // pool_size: reservoir capacity per partition; threads: partitions
  AucRunner(int pool_size, int threads, uint64_t seed);

  // used-uint64 slot indexes whose values candidates carry (the union of all
  // evaluated slot groups)
  void set_eval_slots(const std::vector<int>& u64_idx);

  // GetRandomReplace: feed this pass's records through the reservoirs and
  // assign every record a candidate.  Must run on the unreplaced store.
  void sample(const RecordStore& st);

  // AddReplaceFeasign: every feasign a replacement can introduce
  std::vector<uint64_t> candidate_keys() const;

  // BoxHelper::SlotsShuffle: restore the previously replaced slots, then
  // replace `u64_idx` (empty = restore only).  Returns #feasigns written
  // from candidates.
  int64_t shuffle(RecordStore* st, const std::vector<int>& u64_idx);
  bool replaced() const { return replaced_; }

  int64_t pool_entries() const;

 private:
  struct Pool {
    // candidate store: entry e holds, per eval slot k, vals[off[e*K+k] .. off[e*K+k+1])
    std::vector<int64_t> off{0};
    std::vector<uint64_t> vals;
    std::vector<int64_t> slot_entry;  // reservoir slot -> entry
    int64_t seen = 0;                 // records offered so far (all passes)
    std::mt19937_64 rng;
  };
  int64_t add_entry(Pool* p, const RecordStore& st, int64_t rec) const;
  void compact(Pool* p) const;

  int pool_size_;
  int threads_;
  std::vector<int> eval_;      // eval slot k -> used u64 idx
  std::vector<int> eval_pos_;  // used u64 idx -> k (or -1)
  std::vector<Pool> pools_;
  // per record of the sampled pass: (pool, entry)
  std::vector<int32_t> cand_pool_;
  std::vector<int64_t> cand_entry_;
  bool replaced_ = false;
  std::vector<uint64_t> orig_u64_;
  std::vector<int64_t> orig_off_;
};

}  // namespace pbx

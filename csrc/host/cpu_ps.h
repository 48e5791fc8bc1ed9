// In-process CPU sparse parameter server (BASELINE config 1; also the host tier
// of the HBM -> host -> SSD embedding cache and the oracle for the GPU table).
//
// Same value-row layout and Adagrad rule as the GPU table
// (csrc/common/pbx_common.h).  Sharded open hash maps (key -> row) over one
// row arena; shards are processed in parallel with OpenMP.  Semantics:
// heter_ps/optimizer.cuh.h:42-133, distributed/ps/table/ctr_accessor.cc:63-341.
#pragma once
#include <cstdint>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../common/pbx_common.h"

namespace pbx {

struct SaveFilter {
  float base_threshold = 1.5f;
  float delta_threshold = 0.25f;
  float delta_keep_days = 16.f;
  float embedx_threshold = 10.f;
  float nonclk_coeff = 0.1f;
  float clk_coeff = 1.f;
};

class CpuTable {
 public:
  CpuTable(int dim, int nshards);
  int dim() const { return dim_; }
  int stride() const { return layout_.stride; }
  int64_t size() const;

  // rows[i] = row of mixed key h[i] or -1
  void probe(const uint64_t* h, int64_t n, int64_t* rows) const;
  // insert keys that are absent; new rows initialised
  void insert(const uint64_t* h, int64_t n, float initial_range, float mf_initial_range, bool init_embedx,
              uint64_t seed);
  void gather(const int64_t* rows, int64_t n, float* out /*[n, stride]*/) const;
  void assign(const int64_t* rows, int64_t n, const float* vals, int vstride);
  void push_adagrad(const int64_t* rows, int64_t n, const float* push, int pstride, const SparseSGDConfig& cfg,
                    uint64_t seed);
  int64_t shrink(float decay, float delete_threshold, float delete_after_unseen_days, float nonclk, float clk);
  // all live (h, row)
  void export_all(std::vector<uint64_t>* keys, std::vector<float>* vals) const;
  // keys whose rows satisfy the xbox base/delta filter (ctr_accessor.cc:102-144);
  // mode 0 = base (resets delta_score), 1 = delta, 2 = everything (batch model)
  void select_for_save(int mode, const SaveFilter& f, std::vector<uint64_t>* keys, std::vector<float>* vals);
  void clear();
  int64_t erase(const uint64_t* h, int64_t n);

 private:
  int shard_of(uint64_t h) const { return (int)((h >> 7) % (uint64_t)nshards_); }
  int64_t alloc_row();
  int dim_;
  int nshards_;
  RowLayout layout_;
  std::vector<std::unordered_map<uint64_t, int64_t>> maps_;
  std::vector<float> arena_;
  std::vector<uint64_t> row_key_;  // row -> key (kEmptyKey if free)
  std::vector<int64_t> free_rows_;
  mutable std::mutex alloc_mu_;
};

}  // namespace pbx

// Streaming CTR metrics (BasicAucCalculator semantics: reference
// paddle/fluid/framework/fleet/metrics.{h,cc}: bucketed AUC :284-372,
// bucket_error :374-409, uAUC/wuAUC :421-588, continue-value :600-645,
// nan/inf :647-652).
#pragma once
#include <cstdint>
#include <mutex>
#include <vector>

namespace pbx {

class AucCalculator {
 public:
  explicit AucCalculator(int table_size = 1000000);
  void reset();
  int table_size() const { return table_size_; }
  // label in {0,1}; sample_scale weights the instance
  void add(const float* pred, const float* label, const float* mask, int64_t n, float sample_scale = 1.f);
  void add_float_label(const float* pred, const float* label, const float* mask, int64_t n);
  void add_continue(const float* pred, const float* label, const float* mask, int64_t n);
  void add_uid(const float* pred, const float* label, const uint64_t* uid, int64_t n);
  void add_nan_inf(const float* pred, int64_t n);
  // merge a device-accumulated histogram [2, T] + stats[5]
  void merge_tables(const double* table, const double* stats);

  // compute() from (possibly externally all-reduced) tables/error sums
  void compute(const double* neg, const double* pos, const double* err5);
  void compute_local() { compute(table_[0].data(), table_[1].data(), nullptr); }
  void compute_continue(const double* err5);
  void compute_wuauc();
  void compute_nan_inf();

  std::vector<double>& neg() { return table_[0]; }
  std::vector<double>& pos() { return table_[1]; }
  std::vector<double> local_err() const {
    return {local_abserr_, local_sqrerr_, local_pred_, local_label_, local_total_};
  }

  double auc = 0, bucket_error = 0, mae = 0, rmse = 0, actual_ctr = 0, predicted_ctr = 0, size = 0;
  double actual_value = 0, predicted_value = 0;
  double uauc = 0, wuauc = 0, user_cnt = 0;
  double nan_cnt = 0, inf_cnt = 0, nan_rate = 0, inf_rate = 0, nan_inf_rate = 0, nan_inf_size = 0;

 private:
  void bucket_err(const double* neg, const double* pos);
  struct Rec {
    uint64_t uid;
    int label;
    float pred;
  };
  int table_size_;
  std::vector<double> table_[2];
  double local_abserr_ = 0, local_sqrerr_ = 0, local_pred_ = 0, local_label_ = 0, local_total_ = 0;
  std::vector<Rec> recs_;
  std::mutex mu_;
};

}  // namespace pbx

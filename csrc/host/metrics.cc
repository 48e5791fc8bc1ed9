#include "metrics.h"

#include <algorithm>
#include <cmath>
#include <stdexcept>

namespace pbx {

static constexpr double kMaxSpan = 0.01;
static constexpr double kRelativeErrorBound = 0.05;

AucCalculator::AucCalculator(int table_size) : table_size_(table_size) { reset(); }

void AucCalculator::reset() {
  std::lock_guard<std::mutex> lk(mu_);
  table_[0].assign(table_size_, 0.0);
  table_[1].assign(table_size_, 0.0);
  local_abserr_ = local_sqrerr_ = local_pred_ = local_label_ = local_total_ = 0;
  recs_.clear();
  nan_cnt = inf_cnt = nan_rate = inf_rate = nan_inf_rate = nan_inf_size = 0;
  uauc = wuauc = user_cnt = 0;
}

void AucCalculator::add(const float* pred, const float* label, const float* mask, int64_t n, float sample_scale) {
  std::lock_guard<std::mutex> lk(mu_);
  for (int64_t i = 0; i < n; ++i) {
    if (mask && mask[i] == 0.f) continue;
    const double p = pred[i];
    if (!(p >= 0.0 && p <= 1.0)) throw std::runtime_error("pred must be in [0,1]");
    const int lab = label[i] > 0.5f ? 1 : 0;
    int pos = (int)(p * table_size_);
    if (pos > table_size_ - 1) pos = table_size_ - 1;
    local_abserr_ += std::fabs(p - lab);
    local_sqrerr_ += (p - lab) * (p - lab);
    local_pred_ += p * sample_scale;
    local_label_ += lab;
    table_[lab][pos] += sample_scale;
    local_total_ += sample_scale;
  }
}

void AucCalculator::add_float_label(const float* pred, const float* label, const float* mask, int64_t n) {
  std::lock_guard<std::mutex> lk(mu_);
  for (int64_t i = 0; i < n; ++i) {
    if (mask && mask[i] == 0.f) continue;
    const double p = pred[i], l = label[i];
    int pos = (int)(p * table_size_);
    pos = pos < 0 ? 0 : (pos > table_size_ - 1 ? table_size_ - 1 : pos);
    local_abserr_ += std::fabs(p - l);
    local_sqrerr_ += (p - l) * (p - l);
    local_pred_ += p;
    local_label_ += l;
    table_[0][pos] += 1 - l;
    table_[1][pos] += l;
    local_total_ += 1.0;
  }
}

void AucCalculator::add_continue(const float* pred, const float* label, const float* mask, int64_t n) {
  std::lock_guard<std::mutex> lk(mu_);
  for (int64_t i = 0; i < n; ++i) {
    if (mask && mask[i] == 0.f) continue;
    const double p = pred[i], l = label[i];
    local_abserr_ += std::fabs(p - l);
    local_sqrerr_ += (p - l) * (p - l);
    local_pred_ += p;
    local_label_ += l;
    local_total_ += 1.0;
  }
}

void AucCalculator::add_uid(const float* pred, const float* label, const uint64_t* uid, int64_t n) {
  std::lock_guard<std::mutex> lk(mu_);
  for (int64_t i = 0; i < n; ++i) recs_.push_back({uid[i], label[i] > 0.5f ? 1 : 0, pred[i]});
}

void AucCalculator::add_nan_inf(const float* pred, int64_t n) {
  std::lock_guard<std::mutex> lk(mu_);
  for (int64_t i = 0; i < n; ++i) {
    nan_inf_size += 1;
    if (std::isnan(pred[i])) nan_cnt += 1;
    else if (std::isinf(pred[i])) inf_cnt += 1;
  }
}

void AucCalculator::merge_tables(const double* table, const double* stats) {
  std::lock_guard<std::mutex> lk(mu_);
  for (int i = 0; i < table_size_; ++i) {
    table_[0][i] += table[i];
    table_[1][i] += table[table_size_ + i];
  }
  local_abserr_ += stats[0];
  local_sqrerr_ += stats[1];
  local_pred_ += stats[2];
  local_label_ += stats[3];
  local_total_ += stats[4];
}

void AucCalculator::compute(const double* neg, const double* pos, const double* err5) {
  double area = 0, fp = 0, tp = 0;
  for (int i = table_size_ - 1; i >= 0; --i) {
    const double nfp = fp + neg[i], ntp = tp + pos[i];
    area += (nfp - fp) * (tp + ntp) / 2;
    fp = nfp;
    tp = ntp;
  }
  auc = (fp < 1e-3 || tp < 1e-3) ? -0.5 : area / (fp * tp);
  const double ae = err5 ? err5[0] : local_abserr_;
  const double se = err5 ? err5[1] : local_sqrerr_;
  const double ps = err5 ? err5[2] : local_pred_;
  const double tot = fp + tp;
  mae = tot > 0 ? ae / tot : 0;
  rmse = tot > 0 ? std::sqrt(se / tot) : 0;
  predicted_ctr = tot > 0 ? ps / tot : 0;
  actual_ctr = tot > 0 ? tp / tot : 0;
  size = tot;
  bucket_err(neg, pos);
}

void AucCalculator::bucket_err(const double* neg, const double* pos) {
  double last_ctr = -1, impression_sum = 0, ctr_sum = 0, click_sum = 0, error_sum = 0, error_count = 0;
  for (int i = 0; i < table_size_; ++i) {
    const double click = pos[i];
    const double show = neg[i] + pos[i];
    const double ctr = (double)i / table_size_;
    if (std::fabs(ctr - last_ctr) > kMaxSpan) {
      last_ctr = ctr;
      impression_sum = ctr_sum = click_sum = 0;
    }
    impression_sum += show;
    ctr_sum += ctr * show;
    click_sum += click;
    const double adjust_ctr = ctr_sum / impression_sum;
    const double relative_error = std::sqrt((1 - adjust_ctr) / (adjust_ctr * impression_sum));
    if (relative_error < kRelativeErrorBound) {
      const double actual = click_sum / impression_sum;
      error_sum += std::fabs(actual / adjust_ctr - 1) * impression_sum;
      error_count += impression_sum;
      last_ctr = -1;
    }
  }
  bucket_error = error_count > 0 ? error_sum / error_count : 0.0;
}

void AucCalculator::compute_continue(const double* err5) {
  const double ae = err5 ? err5[0] : local_abserr_;
  const double se = err5 ? err5[1] : local_sqrerr_;
  const double ps = err5 ? err5[2] : local_pred_;
  const double ls = err5 ? err5[3] : local_label_;
  const double tot = err5 ? err5[4] : local_total_;
  mae = tot > 0 ? ae / tot : 0;
  rmse = tot > 0 ? std::sqrt(se / tot) : 0;
  predicted_value = tot > 0 ? ps / tot : 0;
  actual_value = tot > 0 ? ls / tot : 0;
  size = tot;
}

void AucCalculator::compute_wuauc() {
  std::sort(recs_.begin(), recs_.end(), [](const Rec& a, const Rec& b) {
    if (a.uid == b.uid) {
      if (a.pred == b.pred) return a.label < b.label;
      return a.pred > b.pred;
    }
    return a.uid > b.uid;
  });
  uauc = wuauc = user_cnt = 0;
  double sz = 0;
  size_t begin = 0;
  auto one_user = [&](size_t b, size_t e) {
    double tp = 0, fp = 0, area = 0;
    size_t i = b;
    while (i < e) {
      double ntp = tp, nfp = fp;
      if (recs_[i].label == 1) ntp += 1; else nfp += 1;
      while (i + 1 < e && recs_[i].pred == recs_[i + 1].pred) {
        if (recs_[i + 1].label == 1) ntp += 1; else nfp += 1;
        ++i;
      }
      area += (nfp - fp) * (tp + ntp) / 2.0;
      tp = ntp;
      fp = nfp;
      ++i;
    }
    if (tp > 0 && fp > 0) {
      const double a = area / (fp * tp + 1e-9);
      user_cnt += 1;
      sz += tp + fp;
      uauc += a;
      wuauc += a * (tp + fp);
    }
  };
  for (size_t i = 0; i <= recs_.size(); ++i) {
    if (i == recs_.size() || (i > begin && recs_[i].uid != recs_[begin].uid)) {
      if (i > begin) one_user(begin, i);
      begin = i;
    }
  }
  // reference reports uauc/wuauc normalised by users / instances
  if (user_cnt > 0) uauc /= user_cnt;
  if (sz > 0) wuauc /= sz;
  size = sz;
}

void AucCalculator::compute_nan_inf() {
  const double s = nan_inf_size > 0 ? nan_inf_size : 1;
  nan_rate = nan_cnt / s;
  inf_rate = inf_cnt / s;
  nan_inf_rate = (nan_cnt + inf_cnt) / s;
}

}  // namespace pbx

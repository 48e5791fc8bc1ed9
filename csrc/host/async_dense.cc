#include "async_dense.h"

#include <cmath>
#include <cstring>

namespace pbx {

AsyncDenseTable::AsyncDenseTable(const float* params, int64_t total_len, int64_t adam_len, const float* lr,
                                 int device_num, int n_threads, float beta1, float beta2, float eps,
                                 float summary_decay)
    : T_(total_len), A_(adam_len), b1_(beta1), b2_(beta2), eps_(eps), decay_(summary_decay) {
  p_.assign(params, params + total_len);
  m_.assign(adam_len, 0.f);
  v_.assign(adam_len, 0.f);
  lr_.assign(lr, lr + adam_len);
  const int nb = std::max(1, device_num) * 4;
  bufs_.resize(nb);
  for (auto& b : bufs_) {
    b.resize(total_len);
    free_.push_back(b.data());
  }
  pool_.reset(new ThreadPool(std::max(1, n_threads)));
  th_ = std::thread([this] { loop(); });
}

AsyncDenseTable::~AsyncDenseTable() { finalize(); }

void AsyncDenseTable::pull(float* out) {
  std::shared_lock<std::shared_mutex> lk(plock_);
  std::memcpy(out, p_.data(), sizeof(float) * T_);
}

void AsyncDenseTable::push(const float* grad) {
  float* buf;
  {
    std::unique_lock<std::mutex> lk(qmu_);
    fcv_.wait(lk, [this] { return !free_.empty() || closed_; });
    if (closed_) return;
    buf = free_.front();
    free_.pop_front();
    ++inflight_;
  }
  std::memcpy(buf, grad, sizeof(float) * T_);
  {
    std::lock_guard<std::mutex> lk(qmu_);
    ready_.push_back(buf);
  }
  qcv_.notify_one();
}

void AsyncDenseTable::apply(const std::vector<float*>& gs) {
  const int n = (int)gs.size();
  std::unique_lock<std::shared_mutex> lk(plock_);
  pool_->parallel_range(T_, [&](int, int64_t b, int64_t e) {
    float* g0 = gs[0];
    for (int64_t j = b; j < e; ++j) {
      float g = g0[j];
      for (int k = 1; k < n; ++k) g += gs[k][j];
      g /= (float)n;
      if (j < A_) {
        m_[j] = b1_ * m_[j] + (1.f - b1_) * g;
        v_[j] = b2_ * v_[j] + (1.f - b2_) * g * g;
        p_[j] -= lr_[j] * (m_[j] / (std::sqrt(v_[j]) + eps_));
      } else {
        p_[j] = p_[j] * decay_ + g;
      }
    }
  });
}

void AsyncDenseTable::loop() {
  for (;;) {
    std::vector<float*> gs;
    {
      std::unique_lock<std::mutex> lk(qmu_);
      qcv_.wait(lk, [this] { return !ready_.empty() || closed_; });
      if (ready_.empty() && closed_) return;
      while (!ready_.empty() && gs.size() < 4) {
        gs.push_back(ready_.front());
        ready_.pop_front();
      }
    }
    apply(gs);
    updates_ += 1;
    {
      std::lock_guard<std::mutex> lk(qmu_);
      for (float* b : gs) free_.push_back(b);
      inflight_ -= (int)gs.size();
    }
    fcv_.notify_all();
    idle_cv_.notify_all();
  }
}

void AsyncDenseTable::wait_idle() {
  std::unique_lock<std::mutex> lk(qmu_);
  idle_cv_.wait(lk, [this] { return inflight_ == 0 || closed_; });
}

void AsyncDenseTable::finalize() {
  {
    std::lock_guard<std::mutex> lk(qmu_);
    if (closed_) return;
  }
  wait_idle();
  {
    std::lock_guard<std::mutex> lk(qmu_);
    closed_ = true;
  }
  qcv_.notify_all();
  fcv_.notify_all();
  idle_cv_.notify_all();
  if (th_.joinable()) th_.join();
}

void AsyncDenseTable::snapshot(float* params, float* m, float* v) {
  std::shared_lock<std::shared_mutex> lk(plock_);
  std::memcpy(params, p_.data(), sizeof(float) * T_);
  if (m) std::memcpy(m, m_.data(), sizeof(float) * A_);
  if (v) std::memcpy(v, v_.data(), sizeof(float) * A_);
}

}  // namespace pbx

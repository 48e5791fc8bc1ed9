// Asynchronous host-side dense parameter table.
//
// Behaviour of BoxPSAsynDenseTable (reference fw/boxps_worker.cc:61-370):
// the dense parameters live in one host buffer: an Adam region [0, A) and a
// data-norm summary region [A, T).  GPU workers pull a consistent snapshot
// (read lock) before a batch and push their gradient vector after it; one
// update thread merges up to 4 queued gradients (mean) and applies, split
// over a thread pool:
//   Adam region:    m = .99 m + .01 g;  v = .9999 v + 1e-4 g^2;
//                   p -= lr[j] * m / (sqrt(v) + 1e-8)
//   summary region: p = p * 0.9999999 + g
// Gradient buffers are recycled through a fixed pool (4 per device), so a
// worker blocks in push() when the updater falls behind.
#pragma once
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <thread>
#include <vector>

#include "runtime.h"

namespace pbx {

class AsyncDenseTable {
 public:
  // params: initial values [T]; adam_len: A; lr: per-element learning rates [A]
  AsyncDenseTable(const float* params, int64_t total_len, int64_t adam_len, const float* lr, int device_num,
                  int n_threads, float beta1 = 0.99f, float beta2 = 0.9999f, float eps = 1e-8f,
                  float summary_decay = 0.9999999f);
  ~AsyncDenseTable();
  void pull(float* out);
  void push(const float* grad);
  void finalize();           // drain the queue and stop the update thread
  void wait_idle();          // block until every pushed gradient is applied
  int64_t updates() const { return updates_.load(); }
  int64_t total_len() const { return T_; }
  void snapshot(float* params, float* m, float* v);

 private:
  void loop();
  void apply(const std::vector<float*>& gs);
  int64_t T_, A_;
  float b1_, b2_, eps_, decay_;
  std::vector<float> p_, m_, v_, lr_;
  std::vector<std::vector<float>> bufs_;
  std::deque<float*> free_, ready_;
  std::mutex qmu_;
  std::condition_variable qcv_, fcv_, idle_cv_;
  std::shared_mutex plock_;
  bool closed_ = false;
  int inflight_ = 0;
  std::atomic<int64_t> updates_{0};
  std::unique_ptr<ThreadPool> pool_;
  std::thread th_;
};

}  // namespace pbx

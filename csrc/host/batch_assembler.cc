#include "batch_assembler.h"

#include <chrono>
#include <stdexcept>

namespace pbx {

BatchAssembler::BatchAssembler(const SlotDataset* ds, std::vector<Job> jobs, int n_slots)
    : ds_(ds), jobs_(std::move(jobs)), slot_free_(n_slots > 0 ? n_slots : 0, 1) {}

BatchAssembler::~BatchAssembler() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_slot_.notify_all();
  cv_ready_.notify_all();
  if (th_.joinable()) th_.join();
}

void BatchAssembler::start() { th_ = std::thread([this] { run(); }); }

void BatchAssembler::run() {
  using clk = std::chrono::steady_clock;
  for (size_t i = 0; i < jobs_.size(); ++i) {
    const Job& j = jobs_[i];
    if (j.slot >= 0) {
      auto t0 = clk::now();
      std::unique_lock<std::mutex> lk(mu_);
      cv_slot_.wait(lk, [&] { return stop_ || slot_free_[j.slot]; });
      if (stop_) return;
      slot_free_[j.slot] = 0;
      wait_s_ += std::chrono::duration<double>(clk::now() - t0).count();
    }
    auto t1 = clk::now();
    try {
      // the buffer was sized for the pass's largest batch (batch_len at plan time)
      ds_->build_batch_staged(j.begin, j.count, j.keys, j.keys_cap, j.lod, j.dense);
    } catch (const std::exception& e) {
      std::lock_guard<std::mutex> lk(mu_);
      error_ = e.what();
      stop_ = true;
      cv_ready_.notify_all();
      return;
    }
    build_s_ += std::chrono::duration<double>(clk::now() - t1).count();
    {
      std::lock_guard<std::mutex> lk(mu_);
      ready_.push_back((int64_t)i);
    }
    cv_ready_.notify_one();
  }
}

int64_t BatchAssembler::next() {
  std::unique_lock<std::mutex> lk(mu_);
  if (handed_ >= (int64_t)jobs_.size()) return -1;
  cv_ready_.wait(lk, [&] { return !ready_.empty() || !error_.empty() || (stop_ && ready_.empty()); });
  if (!error_.empty()) throw std::runtime_error(error_);
  if (ready_.empty()) return -1;
  const int64_t i = ready_.front();
  ready_.pop_front();
  ++handed_;
  return i;
}

void BatchAssembler::release(int slot) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (slot >= 0 && slot < (int)slot_free_.size()) slot_free_[slot] = 1;
  }
  cv_slot_.notify_all();
}

}  // namespace pbx

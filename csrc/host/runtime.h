// Native host runtime primitives: thread pool with CPU affinity, blocking MPMC
// channel, flag registry, span timers.
//
// Reference analogues (behaviour, not code): fw/threadpool.h:53-253 (pool with
// SetCPUAffinity), fw/channel.h:39-200 (block channel), platform/flags.cc:926-1013
// (PaddleBox FLAGS_*), platform/timer.h (stage span timers).
#pragma once
#include <pthread.h>
#include <sched.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <deque>
#include <functional>
#include <future>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace pbx {

// ---------------------------------------------------------------- thread pool
class ThreadPool {
 public:
  explicit ThreadPool(int n, const std::vector<int>& cores = {}) : stop_(false) {
    if (n <= 0) n = 1;
    for (int i = 0; i < n; ++i) {
      workers_.emplace_back([this, i, cores] {
        if (!cores.empty()) {
          cpu_set_t set;
          CPU_ZERO(&set);
          CPU_SET(cores[i % cores.size()], &set);
          pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
        }
        for (;;) {
          std::function<void()> job;
          {
            std::unique_lock<std::mutex> lk(mu_);
            cv_.wait(lk, [this] { return stop_ || !jobs_.empty(); });
            if (stop_ && jobs_.empty()) return;
            job = std::move(jobs_.front());
            jobs_.pop_front();
          }
          job();
        }
      });
    }
  }
  ~ThreadPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& w : workers_) w.join();
  }
  template <typename F>
  std::future<void> run(F&& f) {
    auto task = std::make_shared<std::packaged_task<void()>>(std::forward<F>(f));
    auto fut = task->get_future();
    {
      std::lock_guard<std::mutex> lk(mu_);
      jobs_.emplace_back([task] { (*task)(); });
    }
    cv_.notify_one();
    return fut;
  }
  // Split [0, n) into size() contiguous ranges and run f(tid, begin, end).
  void parallel_range(int64_t n, const std::function<void(int, int64_t, int64_t)>& f) {
    const int t = (int)workers_.size();
    std::vector<std::future<void>> fs;
    for (int i = 0; i < t; ++i) {
      const int64_t b = n * i / t, e = n * (i + 1) / t;
      fs.push_back(run([=, &f] { f(i, b, e); }));
    }
    for (auto& x : fs) x.get();
  }
  int size() const { return (int)workers_.size(); }

 private:
  std::vector<std::thread> workers_;
  std::deque<std::function<void()>> jobs_;
  std::mutex mu_;
  std::condition_variable cv_;
  bool stop_;
};

// ---------------------------------------------------------------- channel
template <typename T>
class Channel {
 public:
  explicit Channel(size_t capacity = 0) : cap_(capacity) {}
  bool put(T&& v) {
    std::unique_lock<std::mutex> lk(mu_);
    not_full_.wait(lk, [this] { return closed_ || cap_ == 0 || q_.size() < cap_; });
    if (closed_) return false;
    q_.emplace_back(std::move(v));
    not_empty_.notify_one();
    return true;
  }
  // Blocks until an item or close; returns false when closed and drained.
  bool get(T* out) {
    std::unique_lock<std::mutex> lk(mu_);
    not_empty_.wait(lk, [this] { return closed_ || !q_.empty(); });
    if (q_.empty()) return false;
    *out = std::move(q_.front());
    q_.pop_front();
    not_full_.notify_one();
    return true;
  }
  void close() {
    std::lock_guard<std::mutex> lk(mu_);
    closed_ = true;
    not_empty_.notify_all();
    not_full_.notify_all();
  }
  size_t size() {
    std::lock_guard<std::mutex> lk(mu_);
    return q_.size();
  }

 private:
  size_t cap_;
  std::deque<T> q_;
  std::mutex mu_;
  std::condition_variable not_empty_, not_full_;
  bool closed_ = false;
};

// ---------------------------------------------------------------- flags
// Typed registry; FLAGS_<name> environment variables override defaults.
class Flags {
 public:
  static Flags& ins() {
    static Flags f;
    return f;
  }
  void define(const std::string& name, const std::string& def, const std::string& help) {
    std::lock_guard<std::mutex> lk(mu_);
    if (vals_.count(name)) return;
    const char* env = std::getenv(("FLAGS_" + name).c_str());
    vals_[name] = env ? std::string(env) : def;
    help_[name] = help;
  }
  std::string get(const std::string& name) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = vals_.find(name);
    if (it == vals_.end()) throw std::runtime_error("unknown flag " + name);
    return it->second;
  }
  void set(const std::string& name, const std::string& v) {
    std::lock_guard<std::mutex> lk(mu_);
    if (!vals_.count(name)) throw std::runtime_error("unknown flag " + name);
    vals_[name] = v;
  }
  bool get_bool(const std::string& name) {
    auto v = get(name);
    return v == "1" || v == "true" || v == "True";
  }
  // non-throwing reads for code that also runs without the registered
  // defaults (the standalone host self-test)
  std::string get_or(const std::string& name, const std::string& def) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = vals_.find(name);
    return it == vals_.end() ? def : it->second;
  }
  bool get_bool_or(const std::string& name, bool def) {
    const auto v = get_or(name, def ? "true" : "false");
    return v == "1" || v == "true" || v == "True";
  }
  int64_t get_int(const std::string& name) { return std::stoll(get(name)); }
  double get_double(const std::string& name) { return std::stod(get(name)); }
  std::map<std::string, std::string> all() {
    std::lock_guard<std::mutex> lk(mu_);
    return vals_;
  }
  std::map<std::string, std::string> help() {
    std::lock_guard<std::mutex> lk(mu_);
    return help_;
  }

 private:
  std::mutex mu_;
  std::map<std::string, std::string> vals_, help_;
};

void register_default_flags();

// ---------------------------------------------------------------- timer
class SpanTimer {
 public:
  void start() { t0_ = clock::now(); running_ = true; }
  void pause() {
    if (running_) total_ += std::chrono::duration<double>(clock::now() - t0_).count();
    running_ = false;
    ++count_;
  }
  void reset() { total_ = 0; count_ = 0; running_ = false; }
  double seconds() const { return total_; }
  int64_t count() const { return count_; }

 private:
  using clock = std::chrono::steady_clock;
  clock::time_point t0_;
  double total_ = 0;
  int64_t count_ = 0;
  bool running_ = false;
};

}  // namespace pbx

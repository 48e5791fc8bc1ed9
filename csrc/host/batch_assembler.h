// Native batch prefetcher for the graph-captured trainer.
//
// The reference's BoxPSWorker reads batches through the data feed's own
// threads (data_feed.cc PackBatchTask / MiniBatchGpuPack); a Python producer
// thread here would hand the GIL back and forth with the training loop every
// batch (measured: a 0.25 ms assembly became 1-5 ms under contention).  The
// assembler runs the whole pass's batch assembly on one native thread: jobs
// (record range -> pinned target buffers) are filled in order; a job that
// targets a ring slot waits until the consumer released that slot (its H2D
// finished).  The consumer blocks in next() with the GIL released.
#pragma once

#include <condition_variable>
#include <cstdint>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

#include "slot_dataset.h"

namespace pbx {

class BatchAssembler {
 public:
  struct Job {
    int64_t begin, count;
    int64_t* keys;
    int64_t keys_cap;
    int64_t* lod;
    float* dense;
    int slot;  // ring slot (>= 0) or -1 = dedicated buffer
  };
  BatchAssembler(const SlotDataset* ds, std::vector<Job> jobs, int n_slots);
  ~BatchAssembler();
  void start();
  // index of the next assembled job (in order), or -1 when all were handed out
  int64_t next();
  void release(int slot);
  double build_seconds() const { return build_s_; }
  double wait_seconds() const { return wait_s_; }

 private:
  void run();
  const SlotDataset* ds_;
  std::vector<Job> jobs_;
  std::vector<char> slot_free_;
  std::deque<int64_t> ready_;
  int64_t handed_ = 0;
  bool stop_ = false;
  std::string error_;
  std::mutex mu_;
  std::condition_variable cv_ready_, cv_slot_;
  std::thread th_;
  double build_s_ = 0, wait_s_ = 0;
};

}  // namespace pbx

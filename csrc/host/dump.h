// Instance-field / parameter dump writer (training "dump" subsystem).
//
// Behaviour follows BoxPSWorker::DumpField / DumpParam / OpenDump
// (reference fw/boxps_worker.cc:1593-1855): per-instance lines
//   <lineid>\t<name>:<len>:v1:v2...\t<name2>:<len>:...
// sampled by xxh64(lineid) % interval (mode 1), random (mode 2) or all
// (mode 0); floats "%.9f" with |v| < 1e-6 printed as "0"; each writer
// thread appends to its own rolling part file
//   <dir>/part-<device:02>-<tid:05>-<fileid:05>
// rotated at 2 GiB.  Formatting runs on a thread pool over instance ranges.
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "runtime.h"

namespace pbx {

uint64_t xxh64(const void* data, size_t len, uint64_t seed);

class DumpWriter {
 public:
  DumpWriter(const std::string& dir, int device_id, int n_threads, size_t max_file_len = (size_t)1 << 31);
  ~DumpWriter();
  // fields: data[k] is a row-major [B, widths[k]] float matrix
  int64_t dump_fields(const std::vector<std::string>& lineids, const std::vector<std::string>& names,
                      const std::vector<const float*>& data, const std::vector<int64_t>& widths, int64_t B,
                      int dump_mode, int dump_interval, bool lineid_have_extend_info);
  // "(batch_id,name,len):v1:v2..." one line per parameter
  void dump_params(int batch_id, const std::vector<std::string>& names, const std::vector<const float*>& data,
                   const std::vector<int64_t>& lens);
  void flush();
  std::vector<std::string> files() const;

 private:
  struct Fd {
    int fd = -1;
    size_t len = 0;
    int fileid = 0;
  };
  void open_if_needed(int tid);
  void write(int tid, const std::string& s);
  // open + write under the slot's own lock: a slot is touched by whichever pool
  // thread runs its task, by dump_params on the caller thread and by flush()
  void emit(int tid, const std::string& s);
  std::string dir_;
  int device_id_;
  size_t max_len_;
  std::vector<Fd> fds_;
  std::unique_ptr<std::mutex[]> fd_mu_;  // one per Fd slot (uncontended)
  std::vector<std::string> opened_;
  mutable std::mutex mu_;
  std::unique_ptr<ThreadPool> pool_;
};

void append_float(std::string* s, float v);

}  // namespace pbx

#include "dump.h"
#include "runtime.h"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <random>

namespace pbx {

// ---------------------------------------------------------------- xxh64
namespace {
constexpr uint64_t P1 = 11400714785074694791ULL, P2 = 14029467366897019727ULL, P3 = 1609587929392839161ULL,
                   P4 = 9650029242287828579ULL, P5 = 2870177450012600261ULL;
inline uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
inline uint64_t rd64(const uint8_t* p) {
  uint64_t v;
  std::memcpy(&v, p, 8);
  return v;
}
inline uint32_t rd32(const uint8_t* p) {
  uint32_t v;
  std::memcpy(&v, p, 4);
  return v;
}
inline uint64_t round1(uint64_t acc, uint64_t in) {
  acc += in * P2;
  acc = rotl(acc, 31);
  return acc * P1;
}
inline uint64_t merge(uint64_t acc, uint64_t v) {
  acc ^= round1(0, v);
  return acc * P1 + P4;
}
}  // namespace

uint64_t xxh64(const void* data, size_t len, uint64_t seed) {
  const uint8_t* p = static_cast<const uint8_t*>(data);
  const uint8_t* end = p + len;
  uint64_t h;
  if (len >= 32) {
    uint64_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
    const uint8_t* lim = end - 32;
    do {
      v1 = round1(v1, rd64(p));
      v2 = round1(v2, rd64(p + 8));
      v3 = round1(v3, rd64(p + 16));
      v4 = round1(v4, rd64(p + 24));
      p += 32;
    } while (p <= lim);
    h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
    h = merge(h, v1);
    h = merge(h, v2);
    h = merge(h, v3);
    h = merge(h, v4);
  } else {
    h = seed + P5;
  }
  h += (uint64_t)len;
  while (p + 8 <= end) {
    h ^= round1(0, rd64(p));
    h = rotl(h, 27) * P1 + P4;
    p += 8;
  }
  if (p + 4 <= end) {
    h ^= (uint64_t)rd32(p) * P1;
    h = rotl(h, 23) * P2 + P3;
    p += 4;
  }
  while (p < end) {
    h ^= (*p) * P5;
    h = rotl(h, 11) * P1;
    ++p;
  }
  h ^= h >> 33;
  h *= P2;
  h ^= h >> 29;
  h *= P3;
  h ^= h >> 32;
  return h;
}

void append_float(std::string* s, float v) {
  if (v > -1e-6f && v < 1e-6f) {
    s->push_back('0');
    return;
  }
  char buf[64];
  int n = std::snprintf(buf, sizeof(buf), "%.9f", v);
  s->append(buf, n);
}

// ---------------------------------------------------------------- writer
DumpWriter::DumpWriter(const std::string& dir, int device_id, int n_threads, size_t max_file_len)
    : dir_(dir), device_id_(device_id), max_len_(max_file_len) {
  if (n_threads <= 0) n_threads = 1;
  ::mkdir(dir.c_str(), 0777);
  fds_.resize(n_threads);
  fd_mu_.reset(new std::mutex[n_threads]);
  pool_.reset(new ThreadPool(n_threads));
}

DumpWriter::~DumpWriter() { flush(); }

void DumpWriter::open_if_needed(int tid) {
  Fd& f = fds_[tid];
  if (f.fd >= 0 && f.len < max_len_) return;
  if (f.fd >= 0) ::close(f.fd);
  char name[4096];
  std::snprintf(name, sizeof(name), "%s/part-%02d-%05d-%05d", dir_.c_str(), device_id_, tid, f.fileid);
  ++f.fileid;
  f.fd = ::open(name, O_CREAT | O_WRONLY | O_TRUNC | O_APPEND, 0666);
  if (f.fd < 0) throw std::runtime_error(std::string("dump: cannot open ") + name);
  f.len = 0;
  std::lock_guard<std::mutex> lk(mu_);
  opened_.emplace_back(name);
}

void DumpWriter::emit(int tid, const std::string& s) {
  std::lock_guard<std::mutex> lk(fd_mu_[tid]);
  open_if_needed(tid);
  write(tid, s);
}

void DumpWriter::write(int tid, const std::string& s) {
  Fd& f = fds_[tid];
  const char* p = s.data();
  size_t left = s.size();
  while (left) {
    ssize_t r = ::write(f.fd, p, left);
    if (r <= 0) throw std::runtime_error("dump: write failed");
    p += r;
    left -= (size_t)r;
    f.len += (size_t)r;
  }
}

int64_t DumpWriter::dump_fields(const std::vector<std::string>& lineids, const std::vector<std::string>& names,
                                const std::vector<const float*>& data, const std::vector<int64_t>& widths,
                                int64_t B, int dump_mode, int dump_interval, bool lineid_have_extend_info) {
  if (dump_interval <= 0) dump_interval = 1;
  // FLAGS_padbox_dump_debug_lineid: dump only the line whose id starts with
  // it (32 chars compared); FLAGS_dump_filed_same_as_aibox: field headers are
  // the name up to its first '.' without the ":<len>" count;
  // FLAGS_enable_print_dump_field_debug: log every dumped field
  // (boxps_worker.cc:1777-1815)
  const auto t_start = std::chrono::steady_clock::now();
  const std::string debug_lid = Flags::ins().get_or("padbox_dump_debug_lineid", "");
  const bool aibox = Flags::ins().get_bool_or("dump_filed_same_as_aibox", false);
  const bool field_debug = Flags::ins().get_bool_or("enable_print_dump_field_debug", false);
  std::atomic<int64_t> lines{0};
  const int T = (int)fds_.size();
  std::vector<std::future<void>> fs;
  for (int tid = 0; tid < T; ++tid) {
    const int64_t b0 = B * tid / T, b1 = B * (tid + 1) / T;
    fs.push_back(pool_->run([&, tid, b0, b1] {
      std::mt19937_64 rng(0x5eed + tid);
      std::string s;
      s.reserve(1 << 16);
      for (int64_t i = b0; i < b1; ++i) {
        const std::string& lid = i < (int64_t)lineids.size() ? lineids[i] : std::string();
        uint64_t r = 0;
        if (dump_mode == 1) r = xxh64(lid.data(), lid.size(), 0);
        else if (dump_mode == 2) r = rng() & 0x7fffffff;
        if (r % (uint64_t)dump_interval != 0) continue;
        if (!debug_lid.empty() && strncmp(lid.c_str(), debug_lid.c_str(), 32) != 0) continue;
        size_t pos = std::string::npos;
        if (lineid_have_extend_info) pos = lid.find(' ');
        s.append(lid, 0, pos == std::string::npos ? lid.size() : pos);
        for (size_t k = 0; k < names.size(); ++k) {
          const int64_t w = widths[k];
          s.push_back('\t');
          if (aibox) {
            const size_t dot = names[k].find('.');
            s.append(names[k], 0, dot == std::string::npos ? names[k].size() : dot);
          } else {
            s.append(names[k]);
            s.push_back(':');
            s.append(std::to_string(w));
          }
          if (field_debug)
            fprintf(stderr, "[pbx dump] tid=%d lineid:[%s] name=%s len=%lld\n", tid, lid.c_str(), names[k].c_str(),
                    (long long)w);
          const float* row = data[k] + i * w;
          for (int64_t j = 0; j < w; ++j) {
            s.push_back(':');
            append_float(&s, row[j]);
          }
        }
        if (pos != std::string::npos) {
          s.push_back('\t');
          s.append(lid, pos + 1, std::string::npos);
        }
        s.push_back('\n');
        ++lines;
        if (s.size() > (4u << 20)) {
          emit(tid, s);
          s.clear();
        }
      }
      if (!s.empty()) emit(tid, s);
    }));
  }
  for (auto& f : fs) f.get();
  if (Flags::ins().get_bool_or("enable_print_dump_info_debug", false))  // boxps_worker.cc:1849-1853
    fprintf(stderr, "[pbx dump] ins count=%lld field=%zu span=%.3f ms\n", (long long)lines.load(), names.size(),
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count());
  return lines.load();
}

void DumpWriter::dump_params(int batch_id, const std::vector<std::string>& names,
                             const std::vector<const float*>& data, const std::vector<int64_t>& lens) {
  std::string s;
  for (size_t k = 0; k < names.size(); ++k) {
    char head[512];
    std::snprintf(head, sizeof(head), "(%d,%s,%ld)", batch_id, names[k].c_str(), (long)lens[k]);
    s.append(head);
    for (int64_t j = 0; j < lens[k]; ++j) {
      s.push_back(':');
      append_float(&s, data[k][j]);
    }
    s.push_back('\n');
  }
  emit(0, s);
}

void DumpWriter::flush() {
  for (size_t t = 0; t < fds_.size(); ++t) {
    std::lock_guard<std::mutex> lk(fd_mu_[t]);
    Fd& f = fds_[t];
    if (f.fd < 0) continue;
    if (f.len > 0) ::fsync(f.fd);
    ::close(f.fd);
    f.fd = -1;
    f.len = 0;
  }
}

std::vector<std::string> DumpWriter::files() const {
  std::lock_guard<std::mutex> lk(mu_);
  return opened_;
}

}  // namespace pbx

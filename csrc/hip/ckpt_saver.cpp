// Streaming sparse checkpoint, host side.  The GPU table is walked in fixed
// ranges of row slots; each range is compacted on the device (ckpt.hip) into
// one of two chunk buffers, its live rows are copied into a pinned host
// buffer, and a writer thread turns the buffer into file bytes while the GPU
// compacts the next range:
//
//   range i:  k_save_chunk -> count (D2H) -> rows (D2H, pinned) -> queue
//   writer:   batch model: append raw keys / rows to two .npy files
//             xbox text:   T formatter threads print disjoint slices of the
//                          chunk (std::to_chars, = printf %.6g), appended
//                          to the part file under a lock
//
// Extra device memory is two chunk buffers (chunk_rows x (8 + 4*stride) B);
// host memory is three pinned buffers of the same size.  The .npy headers are
// written with a fixed 128-byte length and patched with the final shape.
// Reference contract: BoxPS SaveBase / SaveDelta (box_wrapper.cc:1286-1318);
// text layout of the xbox model: ctr_accessor.cc:310-341.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <charconv>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "kernels.h"

namespace pbx {
namespace {

#define CK(x)                                                                                \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) throw std::runtime_error(std::string("stream_save: ") + #x + ": " + \
                                                   hipGetErrorString(e_));                   \
  } while (0)

constexpr size_t kNpyHeader = 128;

std::string npy_header(const char* descr, int64_t n, int64_t cols) {
  char dict[128];
  if (cols > 0)
    snprintf(dict, sizeof(dict), "{'descr': '%s', 'fortran_order': False, 'shape': (%lld, %lld), }", descr,
             (long long)n, (long long)cols);
  else
    snprintf(dict, sizeof(dict), "{'descr': '%s', 'fortran_order': False, 'shape': (%lld,), }", descr,
             (long long)n);
  std::string d(dict);
  const size_t body = kNpyHeader - 10;  // magic(6) + version(2) + length(2)
  if (d.size() + 1 > body) throw std::runtime_error("stream_save: npy header too long");
  d.append(body - 1 - d.size(), ' ');
  d.push_back('\n');
  std::string h("\x93NUMPY\x01\x00", 8);
  h.push_back((char)(body & 0xff));
  h.push_back((char)(body >> 8));
  return h + d;
}

struct File {
  FILE* f = nullptr;
  explicit File(const std::string& p) {
    f = fopen(p.c_str(), "wb");
    if (!f) throw std::runtime_error("stream_save: cannot open " + p);
    setvbuf(f, nullptr, _IOFBF, 1 << 22);
  }
  ~File() {
    if (f) fclose(f);
  }
  void write(const void* p, size_t n) {
    if (n && fwrite(p, 1, n, f) != n) throw std::runtime_error("stream_save: write failed");
  }
  void close() {
    if (f && fclose(f) != 0) {
      f = nullptr;
      throw std::runtime_error("stream_save: close failed");
    }
    f = nullptr;
  }
};

struct HostBuf {
  uint64_t* keys = nullptr;
  float* vals = nullptr;
  int64_t n = 0;
};

// one xbox text line per row (same bytes as the Python writer's
// f"{key}\t" + " ".join(f"{x:.6g}") + "\n")
void format_rows(const HostBuf& b, int64_t i0, int64_t i1, int dim, int stride, const RowLayout& l,
                 const SaveSelect& sel, float embedx_threshold, std::string& out) {
  char tmp[48];
  auto put = [&](float x) {
    auto r = std::to_chars(tmp, tmp + sizeof(tmp), (double)x, std::chars_format::general, 6);
    out.append(tmp, r.ptr);
  };
  for (int64_t i = i0; i < i1; ++i) {
    const float* v = b.vals + i * (int64_t)stride;
    auto r = std::to_chars(tmp, tmp + sizeof(tmp), (unsigned long long)b.keys[i]);
    out.append(tmp, r.ptr);
    out.push_back('\t');
    const float head[7] = {v[l.slot], v[l.unseen_days], v[l.delta_score], v[kShow], v[kClick], v[kEmbedW],
                           v[l.embed_g2sum]};
    for (int c = 0; c < 7; ++c) {
      if (c) out.push_back(' ');
      put(head[c]);
    }
    const float score = (v[kShow] - v[kClick]) * sel.nonclk_coeff + v[kClick] * sel.clk_coeff;
    if (score >= embedx_threshold && v[l.mf_size] != 0.f) {
      for (int d = 0; d < dim; ++d) {
        out.push_back(' ');
        put(v[kEmbedx + d]);
      }
      out.push_back(' ');
      put(v[l.embedx_g2sum]);
    }
    out.push_back('\n');
  }
}

}  // namespace

SaveStats stream_save_table(const TableDev& t, int64_t total_rows, int kind, const SaveSelect& sel,
                            const SaveDecode& dec, int out_dim, float embedx_threshold, const std::string& keys_path,
                            const std::string& vals_path, int64_t chunk_rows, int threads,
                            std::vector<uint64_t>* saved_mixed, int device, hipStream_t s) {
  using clk = std::chrono::steady_clock;
  const auto t_start = clk::now();
  SaveStats st;
  if (chunk_rows < 1024) chunk_rows = 1024;
  if (threads < 1) threads = 1;
  // output rows: stored (plain layout) or decoded canonical (codec tables)
  const int stride = dec.n > 0 ? dec.n : t.stride;
  const int odim = dec.n > 0 ? out_dim : t.dim;
  const RowLayout l = make_row_layout(odim);
  CK(hipSetDevice(device));
  // ---- buffers
  struct Dev {
    uint64_t* keys = nullptr;
    float* vals = nullptr;
    unsigned long long* count = nullptr;
  } dev[2];
  const int NH = 3;
  HostBuf host[NH];
  auto release = [&]() {
    for (auto& d : dev) {
      if (d.keys) (void)hipFree(d.keys);
      if (d.vals) (void)hipFree(d.vals);
      if (d.count) (void)hipFree(d.count);
      d = Dev{};
    }
    for (auto& h : host) {
      if (h.keys) (void)hipHostFree(h.keys);
      if (h.vals) (void)hipHostFree(h.vals);
      h = HostBuf{};
    }
  };
  struct Guard {
    std::function<void()> f;
    ~Guard() { f(); }
  } guard{release};
  for (auto& d : dev) {
    CK(hipMalloc(&d.keys, chunk_rows * sizeof(uint64_t)));
    CK(hipMalloc(&d.vals, chunk_rows * (size_t)stride * sizeof(float)));
    CK(hipMalloc(&d.count, sizeof(unsigned long long)));
  }
  for (auto& h : host) {
    CK(hipHostMalloc(&h.keys, chunk_rows * sizeof(uint64_t), hipHostMallocDefault));
    CK(hipHostMalloc(&h.vals, chunk_rows * (size_t)stride * sizeof(float), hipHostMallocDefault));
  }
  // ---- files
  std::unique_ptr<File> fk(new File(keys_path)), fv;
  if (kind == 0) {
    fv.reset(new File(vals_path));
    fk->write(npy_header("<u8", 0, 0).data(), kNpyHeader);
    fv->write(npy_header("<f4", 0, stride).data(), kNpyHeader);
  }
  // ---- writer thread: consumes filled host buffers in order
  std::mutex mu;
  std::condition_variable cv;
  std::deque<int> ready, free_bufs{0, 1, 2};
  bool done = false;
  std::string werr;
  double write_s = 0;
  std::thread writer([&]() {
    std::vector<std::string> outs(threads);
    for (;;) {
      int hb;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return !ready.empty() || done; });
        if (ready.empty()) return;
        hb = ready.front();
        ready.pop_front();
      }
      const auto t0 = clk::now();
      try {
        const HostBuf& b = host[hb];
        if (kind == 0) {
          fk->write(b.keys, b.n * sizeof(uint64_t));
          fv->write(b.vals, b.n * (size_t)stride * sizeof(float));
        } else {
          const int T = (int)std::min<int64_t>(threads, std::max<int64_t>(1, b.n / 4096));
          std::vector<std::thread> ws;
          for (int w = 0; w < T; ++w) {
            ws.emplace_back([&, w]() {
              outs[w].clear();
              outs[w].reserve((size_t)(b.n / T + 1) * 160);
              format_rows(b, b.n * w / T, b.n * (w + 1) / T, odim, stride, l, sel, embedx_threshold, outs[w]);
            });
          }
          for (auto& th : ws) th.join();
          for (int w = 0; w < T; ++w) fk->write(outs[w].data(), outs[w].size());
        }
      } catch (const std::exception& e) {
        std::lock_guard<std::mutex> lk(mu);
        if (werr.empty()) werr = e.what();
      }
      write_s += std::chrono::duration<double>(clk::now() - t0).count();
      {
        std::lock_guard<std::mutex> lk(mu);
        free_bufs.push_back(hb);
      }
      cv.notify_all();
    }
  });
  auto stop_writer = [&]() {
    {
      std::lock_guard<std::mutex> lk(mu);
      done = true;
    }
    cv.notify_all();
    if (writer.joinable()) writer.join();
  };
  double gpu_s = 0;
  try {
    for (int64_t r0 = 0, c = 0; r0 < total_rows; r0 += chunk_rows, ++c) {
      const int64_t r1 = std::min(total_rows, r0 + chunk_rows);
      Dev& d = dev[c & 1];
      const auto t0 = clk::now();
      CK(hipMemsetAsync(d.count, 0, sizeof(unsigned long long), s));
      launch_save_chunk(t, r0, r1, sel, dec, d.keys, d.vals, d.count, s);
      CK(hipGetLastError());
      unsigned long long n = 0;
      CK(hipMemcpyAsync(&n, d.count, sizeof(n), hipMemcpyDeviceToHost, s));
      CK(hipStreamSynchronize(s));
      int hb;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return !free_bufs.empty() || !werr.empty(); });
        if (!werr.empty()) break;
        hb = free_bufs.front();
        free_bufs.pop_front();
      }
      HostBuf& h = host[hb];
      h.n = (int64_t)n;
      if (n) {
        CK(hipMemcpyAsync(h.keys, d.keys, n * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
        CK(hipMemcpyAsync(h.vals, d.vals, n * (size_t)stride * sizeof(float), hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
      }
      gpu_s += std::chrono::duration<double>(clk::now() - t0).count();
      if (saved_mixed)
        for (int64_t i = 0; i < (int64_t)n; ++i) saved_mixed->push_back(mix64(h.keys[i]));
      st.rows += (int64_t)n;
      st.chunks += 1;
      {
        std::lock_guard<std::mutex> lk(mu);
        ready.push_back(hb);
      }
      cv.notify_all();
    }
  } catch (...) {
    stop_writer();
    throw;
  }
  stop_writer();
  if (!werr.empty()) throw std::runtime_error(werr);
  if (kind == 0) {  // patch the shapes into the fixed-length headers
    for (int i = 0; i < 2; ++i) {
      File* f = i == 0 ? fk.get() : fv.get();
      const std::string h = i == 0 ? npy_header("<u8", st.rows, 0) : npy_header("<f4", st.rows, stride);
      if (fseek(f->f, 0, SEEK_SET) != 0) throw std::runtime_error("stream_save: seek failed");
      f->write(h.data(), kNpyHeader);
    }
    fv->close();
  }
  fk->close();
  st.gpu_s = gpu_s;
  st.write_s = write_s;
  st.total_s = std::chrono::duration<double>(clk::now() - t_start).count();
  return st;
}

}  // namespace pbx

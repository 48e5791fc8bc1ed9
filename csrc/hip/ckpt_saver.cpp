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

struct HostBuf {
  uint64_t* keys = nullptr;
  float* vals = nullptr;
  int64_t n = 0;
};

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
  std::unique_ptr<SaveFile> fk(new SaveFile(keys_path)), fv;
  if (kind == 0) {
    fv.reset(new SaveFile(vals_path));
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
              format_xbox_rows(b.keys, b.vals, b.n * w / T, b.n * (w + 1) / T, odim, stride, l, sel, embedx_threshold,
                               outs[w]);
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
      SaveFile* f = i == 0 ? fk.get() : fv.get();
      f->rewrite_head(i == 0 ? npy_header("<u8", st.rows, 0) : npy_header("<f4", st.rows, stride));
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

// Save of the tiered sparse model: the union of the host tier and the SSD
// log, written in the same files as the GPU streaming saver
// (csrc/common/ckpt_format.h), streamed so memory stays bounded whatever the
// table size:
//
//   host tier  shards in groups (one per pool thread, each under its lock,
//              groups narrowed to ~4M selected rows): selected rows copied
//              out and written shard by shard, delta_score reset in place
//   SSD log    SsdLog::rewrite -- sequential segment runs; the reset is
//              written back into the records' pages in place
//   writer     batch model: raw .npy appends; xbox: T formatter threads
//
// Every key lives in exactly one of the two tiers (staging moves SSD rows to
// the host, spills move host rows to SSD, write-back drops a key's SSD copy
// when it re-enters the host), so the union needs no dedup.
// Reference contract: BoxPS SaveBase / SaveDelta over the whole table
// (box_wrapper.cc:1286-1318); selection and reset ctr_accessor.cc:102-170.
#include "tier_save.h"

#include <algorithm>
#include <chrono>
#include <memory>
#include <thread>

#include "../common/ckpt_format.h"

namespace pbx {

namespace {

class PartWriter {
 public:
  PartWriter(int kind, int dim, int stride, const SaveSelect& sel, float embedx_threshold, const std::string& kp,
             const std::string& vp, int threads)
      : kind_(kind), dim_(dim), stride_(stride), sel_(sel), ex_thr_(embedx_threshold),
        threads_(std::max(1, threads)), l_(make_row_layout(dim)) {
    fk_.reset(new SaveFile(kp));
    if (kind_ == 0) {
      fv_.reset(new SaveFile(vp));
      fk_->write(npy_header("<u8", 0, 0).data(), kNpyHeader);
      fv_->write(npy_header("<f4", 0, stride_).data(), kNpyHeader);
    }
  }
  // rows staged for the next flush (feasigns, value rows)
  std::vector<uint64_t> keys;
  std::vector<float> vals;

  void flush() {
    write_rows(keys.data(), vals.data(), (int64_t)keys.size());
    keys.clear();
    vals.clear();
  }
  // rows straight from the caller's buffers (no staging copy)
  void write_rows(const uint64_t* keys, const float* vals, int64_t n) {
    if (n == 0) return;
    if (kind_ == 0) {
      fk_->write(keys, n * sizeof(uint64_t));
      fv_->write(vals, n * (size_t)stride_ * sizeof(float));
    } else {
      const int T = (int)std::min<int64_t>(threads_, std::max<int64_t>(1, n / 4096));
      std::vector<std::string> outs(T);
      std::vector<std::thread> ws;
      for (int w = 0; w < T; ++w)
        ws.emplace_back([&, w]() {
          outs[w].reserve((size_t)(n / T + 1) * 160);
          format_xbox_rows(keys, vals, n * w / T, n * (w + 1) / T, dim_, stride_, l_, sel_, ex_thr_, outs[w]);
        });
      for (auto& t : ws) t.join();
      for (auto& o : outs) fk_->write(o.data(), o.size());
    }
    rows_ += n;
  }
  int64_t finish() {
    flush();
    if (kind_ == 0) {
      fk_->rewrite_head(npy_header("<u8", rows_, 0));
      fv_->rewrite_head(npy_header("<f4", rows_, stride_));
      fv_->close();
    }
    fk_->close();
    return rows_;
  }

 private:
  int kind_, dim_, stride_;
  SaveSelect sel_;
  float ex_thr_;
  int threads_;
  RowLayout l_;
  std::unique_ptr<SaveFile> fk_, fv_;
  int64_t rows_ = 0;
};

}  // namespace

TierSaveStats save_tiers(HostTier* host, SsdLog* ssd, int kind, const SaveSelect& sel, int dim,
                         float embedx_threshold, const std::string& keys_path, const std::string& vals_path,
                         int threads, std::vector<uint64_t>* saved_mixed) {
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  if (!host && !ssd) throw std::runtime_error("save_tiers: no tier");
  const int stride = host ? host->stride() : ssd->stride();
  if (host && ssd && ssd->stride() != stride) throw std::runtime_error("save_tiers: tier strides differ");
  const RowLayout l = make_row_layout(dim);
  if (l.mf_size >= stride) throw std::runtime_error("save_tiers: row narrower than the layout of dim");
  PartWriter out(kind, dim, stride, sel, embedx_threshold, keys_path, vals_path, threads);
  TierSaveStats st;
  constexpr size_t kFlushRows = 1 << 20;
  if (host) {
    // groups of shards, one shard per pool thread: each shard's rows land in
    // its own list (no shared state in fn) and go to the writer straight from
    // it, shard by shard.  Memory bound: the selected rows of one group; the
    // group is narrowed so that it holds at most ~kGroupRows rows (the
    // shards are hash-balanced: size / kNumShards rows each).
    constexpr int64_t kGroupRows = 1 << 22;
    const int64_t per_shard = std::max<int64_t>(1, host->size() / HostTier::kNumShards);
    const int G = (int)std::max<int64_t>(1, std::min<int64_t>(host->threads(), kGroupRows / per_shard));
    std::vector<std::vector<uint64_t>> gk(HostTier::kNumShards);
    std::vector<std::vector<float>> gv(HostTier::kNumShards);
    for (int s0 = 0; s0 < HostTier::kNumShards; s0 += G) {
      const int s1 = std::min(HostTier::kNumShards, s0 + G);
      host->visit(s0, s1, [&](int si, uint64_t h, float* v) {
        if (!save_keep(sel, v, l)) return;
        gk[si].push_back(h);
        gv[si].insert(gv[si].end(), v, v + stride);
        if (sel.reset_delta) v[l.delta_score] = 0.f;
      });
      for (int si = s0; si < s1; ++si) {
        auto& k = gk[si];
        if (saved_mixed) saved_mixed->insert(saved_mixed->end(), k.begin(), k.end());
        for (auto& h : k) h = unmix64(h);
        out.write_rows(k.data(), gv[si].data(), (int64_t)k.size());
        st.host_rows += (int64_t)k.size();
        std::vector<uint64_t>().swap(k);
        std::vector<float>().swap(gv[si]);
      }
    }
  }
  if (ssd) {
    ssd->rewrite(
        [&](uint64_t h, float* v) {
          if (!save_keep(sel, v, l)) return (int)SsdLog::kKeep;
          out.keys.push_back(unmix64(h));
          out.vals.insert(out.vals.end(), v, v + stride);
          if (saved_mixed) saved_mixed->push_back(h);
          ++st.ssd_rows;
          if (sel.reset_delta && v[l.delta_score] != 0.f) {
            v[l.delta_score] = 0.f;
            return (int)SsdLog::kModified;
          }
          return (int)SsdLog::kKeep;
        },
        [&]() {
          if (out.keys.size() >= kFlushRows) out.flush();
        });
  }
  st.rows = out.finish();
  st.total_s = std::chrono::duration<double>(clk::now() - t0).count();
  return st;
}

}  // namespace pbx

// Sparse checkpoint formats shared by the GPU streaming saver
// (csrc/hip/ckpt_saver.cpp) and the host/SSD tier saver
// (csrc/host/tier_save.cc), so a model saved from HBM and one saved from the
// tiers are byte-identical:
//
//   batch model  part-R.keys.npy  uint64 [N]   feasigns (unmixed)
//                part-R.vals.npy  f32 [N, W]   value rows
//   xbox text    part-R.txt       "feasign\tslot unseen delta show click
//                                  embed_w g2sum [embedx.. embedx_g2sum]"
//
// Selection (SaveSelect, save_keep): mode 0 = every row, 1 = xbox base
// (score >= base_threshold and unseen_days <= delta_keep_days), 2 = xbox
// delta (additionally delta_score >= delta_threshold); the saved rows'
// delta_score is reset when reset_delta is set.  Semantics:
// distributed/ps/table/ctr_accessor.cc:102-170 (Save / UpdateStatAfterSave),
// text layout ctr_accessor.cc:310-341, call sites box_wrapper.cc:1286-1318.
#pragma once

#include <charconv>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>

#include "pbx_common.h"

namespace pbx {

struct SaveSelect {
  int mode = 0;
  int reset_delta = 0;
  float base_threshold = 0.f;
  float delta_threshold = 0.f;
  float delta_keep_days = 16.f;
  float nonclk_coeff = 0.1f;
  float clk_coeff = 1.f;
};

PBX_HD bool save_keep(const SaveSelect& sel, const float* v, const RowLayout& l) {
  if (sel.mode == 0) return true;
  const float score = (v[kShow] - v[kClick]) * sel.nonclk_coeff + v[kClick] * sel.clk_coeff;
  bool take = score >= sel.base_threshold && v[l.unseen_days] <= sel.delta_keep_days;
  if (take && sel.mode == 2) take = v[l.delta_score] >= sel.delta_threshold;
  return take;
}

// .npy header of a fixed 128-byte length (patched with the final shape once
// the row count is known)
constexpr size_t kNpyHeader = 128;

inline std::string npy_header(const char* descr, int64_t n, int64_t cols) {
  char dict[128];
  if (cols > 0)
    snprintf(dict, sizeof(dict), "{'descr': '%s', 'fortran_order': False, 'shape': (%lld, %lld), }", descr,
             (long long)n, (long long)cols);
  else
    snprintf(dict, sizeof(dict), "{'descr': '%s', 'fortran_order': False, 'shape': (%lld,), }", descr,
             (long long)n);
  std::string d(dict);
  const size_t body = kNpyHeader - 10;  // magic(6) + version(2) + length(2)
  if (d.size() + 1 > body) throw std::runtime_error("save: npy header too long");
  d.append(body - 1 - d.size(), ' ');
  d.push_back('\n');
  std::string h("\x93NUMPY\x01\x00", 8);
  h.push_back((char)(body & 0xff));
  h.push_back((char)(body >> 8));
  return h + d;
}

struct SaveFile {
  FILE* f = nullptr;
  explicit SaveFile(const std::string& p) {
    f = fopen(p.c_str(), "wb");
    if (!f) throw std::runtime_error("save: cannot open " + p);
    setvbuf(f, nullptr, _IOFBF, 1 << 22);
  }
  ~SaveFile() {
    if (f) fclose(f);
  }
  void write(const void* p, size_t n) {
    if (n && fwrite(p, 1, n, f) != n) throw std::runtime_error("save: write failed");
  }
  void rewrite_head(const std::string& h) {
    if (fseek(f, 0, SEEK_SET) != 0) throw std::runtime_error("save: seek failed");
    write(h.data(), h.size());
  }
  void close() {
    if (f && fclose(f) != 0) {
      f = nullptr;
      throw std::runtime_error("save: close failed");
    }
    f = nullptr;
  }
};

// xbox text lines of rows [i0, i1) (keys: feasigns; same bytes as the Python
// writer's f"{key}\t" + " ".join(f"{x:.6g}") + "\n")
inline void format_xbox_rows(const uint64_t* keys, const float* vals, int64_t i0, int64_t i1, int dim, int stride,
                             const RowLayout& l, const SaveSelect& sel, float embedx_threshold, std::string& out) {
  char tmp[48];
  auto put = [&](float x) {
    auto r = std::to_chars(tmp, tmp + sizeof(tmp), (double)x, std::chars_format::general, 6);
    out.append(tmp, r.ptr);
  };
  for (int64_t i = i0; i < i1; ++i) {
    const float* v = vals + i * (int64_t)stride;
    auto r = std::to_chars(tmp, tmp + sizeof(tmp), (unsigned long long)keys[i]);
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

}  // namespace pbx

// Example instance-parser plugin (ABI: csrc/host/parser_plugin.h): the raw
// Criteo display-ads TSV format
//
//   <label> \t I1 .. I13 (integer counts, may be empty) \t C1 .. C26 (32-bit hex, may be empty)
//
// Slot mapping, by the slot names the dataset registers:
//   label / click            the label (uint64 or float slot)
//   I1..I13                  one float each, log(1 + max(x, 0))
//   dense                    all 13 of them, same transform
//   C1..C26                  one uint64 feasign each: mix(slot, hex value), never 0
// other slots receive nothing.  Build:
//   g++ -O2 -shared -fPIC -Icsrc/host csrc/plugins/criteo_tsv_parser.cc -o criteo_tsv_parser.so
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "parser_plugin.h"

namespace {
enum Kind { kNone, kLabel, kInt, kDense, kCat };
struct Map {
  Kind kind;
  int idx;
  char type;
};
struct Parser {
  std::vector<Map> slots;
};

inline uint64_t mix(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return x;
}
}  // namespace

extern "C" {

void* pbx_parser_create(int n, const char* const* names, const char* types) {
  Parser* p = new (std::nothrow) Parser;
  if (!p) return nullptr;
  for (int i = 0; i < n; ++i) {
    const std::string s = names[i];
    Map m{kNone, 0, types[i]};
    if (s == "label" || s == "click") {
      m.kind = kLabel;
    } else if (s == "dense") {
      m.kind = kDense;
    } else if (s.size() >= 2 && (s[0] == 'I' || s[0] == 'C') && s.find_first_not_of("0123456789", 1) == std::string::npos) {
      const int k = atoi(s.c_str() + 1);
      if (s[0] == 'I' && k >= 1 && k <= 13) m = {kInt, k - 1, types[i]};
      if (s[0] == 'C' && k >= 1 && k <= 26) m = {kCat, k - 1, types[i]};
    }
    p->slots.push_back(m);
  }
  return p;
}

int pbx_parser_parse_line(void* h, const char* line, size_t len, const pbx_ins_sink* sink) {
  const Parser* p = (const Parser*)h;
  // split into 40 tab-separated fields
  const char* f[40];
  int fl[40];
  int nf = 0;
  const char* b = line;
  const char* end = line + len;
  while (end > line && (end[-1] == '\n' || end[-1] == '\r')) --end;
  for (const char* c = line; nf < 40; ++c) {
    if (c == end || *c == '\t') {
      f[nf] = b;
      fl[nf] = (int)(c - b);
      ++nf;
      b = c + 1;
      if (c == end) break;
    }
  }
  if (nf != 40 || fl[0] == 0) return -1;
  const int label = f[0][0] == '1';
  float ints[13];
  for (int k = 0; k < 13; ++k) {
    const double x = fl[1 + k] ? strtod(std::string(f[1 + k], fl[1 + k]).c_str(), nullptr) : 0.0;
    ints[k] = (float)std::log1p(x > 0 ? x : 0.0);
  }
  for (size_t i = 0; i < p->slots.size(); ++i) {
    const Map& m = p->slots[i];
    const int s = (int)i;
    switch (m.kind) {
      case kLabel:
        if (m.type == 'f') {
          const float v = (float)label;
          sink->add_f32(sink->ctx, s, &v, 1);
        } else {
          const uint64_t v = (uint64_t)label;
          sink->add_u64(sink->ctx, s, &v, 1);
        }
        break;
      case kInt:
        sink->add_f32(sink->ctx, s, &ints[m.idx], 1);
        break;
      case kDense:
        sink->add_f32(sink->ctx, s, ints, 13);
        break;
      case kCat: {
        const int k = 14 + m.idx;
        if (fl[k] == 0) break;
        const uint64_t v = strtoull(std::string(f[k], fl[k]).c_str(), nullptr, 16);
        uint64_t key = mix(((uint64_t)(m.idx + 1) << 40) ^ v);
        if (key == 0) key = 1;
        sink->add_u64(sink->ctx, s, &key, 1);
        break;
      }
      default:
        break;
    }
  }
  return sink->commit(sink->ctx);
}

void pbx_parser_destroy(void* h) { delete (Parser*)h; }

}  // extern "C"

// Example plugin for the replica-cache and input-index data feeds
// (reference SlotPaddleBoxDataFeedWithGpuReplicaCache / InputIndexDataFeed /
// InputTableDataFeed::ParseIndexData).  Instance line (whitespace separated):
//
//   label  qkey  n_cache c_1..c_n  [n_k id_1..id_nk]  for every further slot
//
// Slot roles by name: "label" (uint64), "cache_off" gets the replica-cache
// row offset of c_1..c_n, "qidx" gets the input-table offset of qkey (no
// feasign when the key is absent); every other slot takes the next counted
// group.  Index file line: "key v_1 .. v_D".
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "parser_plugin.h"

namespace {
struct Parser {
  std::vector<std::string> names;
  std::string types;
  int label = -1, cache = -1, qidx = -1;
};

const char* skip_ws(const char* p, const char* e) {
  while (p < e && (*p == ' ' || *p == '\t')) ++p;
  return p;
}
const char* token(const char* p, const char* e) {
  while (p < e && *p != ' ' && *p != '\t' && *p != '\n' && *p != '\r') ++p;
  return p;
}
}  // namespace

extern "C" {

void* pbx_parser_create(int n, const char* const* names, const char* types) {
  Parser* p = new Parser();
  for (int i = 0; i < n; ++i) {
    p->names.emplace_back(names[i]);
    if (p->names.back() == "label") p->label = i;
    if (p->names.back() == "cache_off") p->cache = i;
    if (p->names.back() == "qidx") p->qidx = i;
  }
  p->types = types;
  return p;
}

int pbx_parser_parse_line(void* h, const char* line, size_t len, const pbx_ins_sink* s) {
  const Parser* P = (const Parser*)h;
  const char* e = line + len;
  const char* p = skip_ws(line, e);
  char* q = nullptr;
  const uint64_t label = strtoull(p, &q, 10);
  if (q == p) return -1;
  p = skip_ws(q, e);
  const char* k0 = p;
  p = token(p, e);
  const std::string key(k0, p - k0);
  const long nc = strtol(p, &q, 10);
  if (q == p || nc < 0) return -1;
  p = q;
  std::vector<float> cvec((size_t)nc);
  for (long i = 0; i < nc; ++i) {
    cvec[i] = strtof(p, &q);
    if (q == p) return -1;
    p = q;
  }
  if (P->label >= 0) s->add_u64(s->ctx, P->label, &label, 1);
  if (P->cache >= 0 && s->add_cache) {
    const int64_t off = s->add_cache(s->ctx, cvec.data(), (int)nc);
    if (off >= 0) {
      const uint64_t v = (uint64_t)off;
      s->add_u64(s->ctx, P->cache, &v, 1);
    }
  }
  if (P->qidx >= 0 && s->index_offset) {
    const uint64_t off = s->index_offset(s->ctx, key.data(), (int)key.size());
    if (off != ~0ULL) s->add_u64(s->ctx, P->qidx, &off, 1);
  }
  std::vector<uint64_t> ids;
  for (int slot = 0; slot < (int)P->names.size(); ++slot) {
    if (slot == P->label || slot == P->cache || slot == P->qidx) continue;
    const long n = strtol(p, &q, 10);
    if (q == p) break;
    p = q;
    ids.clear();
    for (long i = 0; i < n; ++i) {
      ids.push_back(strtoull(p, &q, 10));
      p = q;
    }
    if (!ids.empty()) s->add_u64(s->ctx, slot, ids.data(), (int)ids.size());
  }
  return s->commit(s->ctx);
}

int pbx_parser_parse_index(void*, const char* line, size_t len, const pbx_index_sink* s) {
  const char* e = line + len;
  const char* p = skip_ws(line, e);
  const char* k0 = p;
  p = token(p, e);
  if (p == k0) return 0;
  std::vector<float> v;
  char* q = nullptr;
  for (;;) {
    const float f = strtof(p, &q);
    if (q == p) break;
    v.push_back(f);
    p = q;
  }
  s->add_index(s->ctx, k0, (int)(p - k0 < 0 ? 0 : (token(k0, e) - k0)), v.data(), (int)v.size());
  return 1;
}

void pbx_parser_destroy(void* h) { delete (Parser*)h; }
}

#include "slot_dataset.h"

#include <dlfcn.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <mutex>
#include <numeric>
#include <random>
#include <stdexcept>
#include <unordered_set>

#include "../common/pbx_common.h"
#include "dump.h"
#include "file_mgr.h"
#include "msg_service.h"
#include "parser_plugin.h"
#include "runtime.h"

namespace pbx {

// ---------------------------------------------------------------- store
void RecordStore::reset(int nu_, int nf_) {
  nu = nu_;
  nf = nf_;
  u64.clear();
  f32.clear();
  u64_off.assign(1, 0);
  f32_off.assign(1, 0);
  ins_id.clear();
  search_id.clear();
  cmatch.clear();
  rank.clear();
  ext.clear();
}

void RecordStore::ensure_ext(int d) {
  const size_t want = (size_t)nrec() * (size_t)(d > 0 ? d : 0);
  if (d != ext_dim) {
    ext.assign(want, 0.f);
    ext_dim = d;
  } else if (ext.size() != want) {
    ext.resize(want, 0.f);
  }
}

void RecordStore::append(const RecordStore& o) {
  const int d = std::max(ext_dim, o.ext_dim);
  if (d > 0) {
    ensure_ext(d);  // before the new records land: sized by the current count
    if (o.ext_dim == d && o.ext.size() == (size_t)o.nrec() * (size_t)d)
      ext.insert(ext.end(), o.ext.begin(), o.ext.end());
    else
      ext.insert(ext.end(), (size_t)o.nrec() * (size_t)d, 0.f);
  }
  const int64_t ub = (int64_t)u64.size(), fb = (int64_t)f32.size();
  u64.insert(u64.end(), o.u64.begin(), o.u64.end());
  f32.insert(f32.end(), o.f32.begin(), o.f32.end());
  for (size_t i = 1; i < o.u64_off.size(); ++i) u64_off.push_back(o.u64_off[i] + ub);
  for (size_t i = 1; i < o.f32_off.size(); ++i) f32_off.push_back(o.f32_off[i] + fb);
  ins_id.insert(ins_id.end(), o.ins_id.begin(), o.ins_id.end());
  search_id.insert(search_id.end(), o.search_id.begin(), o.search_id.end());
  cmatch.insert(cmatch.end(), o.cmatch.begin(), o.cmatch.end());
  rank.insert(rank.end(), o.rank.begin(), o.rank.end());
}

RecordStore RecordStore::select(const std::vector<int64_t>& idx) const {
  RecordStore r;
  r.reset(nu, nf);
  const bool has_ext = ext_dim > 0 && ext.size() == (size_t)nrec() * (size_t)ext_dim;
  if (has_ext) {
    r.ext_dim = ext_dim;
    r.ext.reserve(idx.size() * (size_t)ext_dim);
    for (int64_t i : idx)
      r.ext.insert(r.ext.end(), ext.begin() + i * ext_dim, ext.begin() + (i + 1) * ext_dim);
  }
  for (int64_t i : idx) {
    for (int j = 0; j < nu; ++j) {
      const int64_t b = u64_off[i * nu + j], e = u64_off[i * nu + j + 1];
      r.u64.insert(r.u64.end(), u64.begin() + b, u64.begin() + e);
      r.u64_off.push_back((int64_t)r.u64.size());
    }
    for (int j = 0; j < nf; ++j) {
      const int64_t b = f32_off[i * nf + j], e = f32_off[i * nf + j + 1];
      r.f32.insert(r.f32.end(), f32.begin() + b, f32.begin() + e);
      r.f32_off.push_back((int64_t)r.f32.size());
    }
    if (!ins_id.empty()) r.ins_id.push_back(ins_id[i]);
    r.search_id.push_back(search_id[i]);
    r.cmatch.push_back(cmatch[i]);
    r.rank.push_back(rank[i]);
  }
  return r;
}

// ---------------------------------------------------------------- dataset
SlotDataset::SlotDataset() {}
SlotDataset::~SlotDataset() {
  if (preload_ && preload_->joinable()) preload_->join();
}

void SlotDataset::set_slots(const std::vector<SlotDesc>& slots) {
  slots_ = slots;
  u_idx_.assign(slots.size(), -1);
  f_idx_.assign(slots.size(), -1);
  sparse_slots_.clear();
  dense_refs_.clear();
  int nu = 0, nf = 0, col = 0;
  for (size_t i = 0; i < slots.size(); ++i) {
    const auto& s = slots[i];
    if (!s.used) continue;
    if (s.type == 'u') {
      u_idx_[i] = nu;
      if (s.dense) {
        dense_refs_.push_back({'u', nu, s.dense_dim, col});
        col += s.dense_dim;
      } else {
        sparse_slots_.push_back(nu);
      }
      ++nu;
    } else {
      f_idx_[i] = nf;
      dense_refs_.push_back({'f', nf, s.dense ? s.dense_dim : std::max(1, s.dense_dim), col});
      col += s.dense ? s.dense_dim : std::max(1, s.dense_dim);
      ++nf;
    }
  }
  dense_width_ = col;
  store_.reset(nu, nf);
  ++version_;
}

std::vector<std::string> SlotDataset::sparse_slot_names() const {
  std::vector<std::string> out;
  for (size_t i = 0; i < slots_.size(); ++i)
    if (slots_[i].used && slots_[i].type == 'u' && !slots_[i].dense) out.push_back(slots_[i].name);
  return out;
}
std::vector<std::string> SlotDataset::dense_slot_names() const {
  std::vector<std::string> out;
  for (size_t i = 0; i < slots_.size(); ++i)
    if (slots_[i].used && (slots_[i].type == 'f' || slots_[i].dense)) out.push_back(slots_[i].name);
  return out;
}
std::vector<int> SlotDataset::dense_slot_dims() const {
  std::vector<int> out;
  for (auto& d : dense_refs_) out.push_back(d.dim);
  return out;
}

static bool parse_logkey(const char* s, size_t len, uint64_t* sid, uint32_t* cm, uint32_t* rk) {
  if (len < 32) return false;
  char buf[17];
  memcpy(buf, s + 16, 16);
  buf[16] = 0;
  *sid = strtoull(buf, nullptr, 16);
  memcpy(buf, s + 11, 3);
  buf[3] = 0;
  *cm = (uint32_t)strtoul(buf, nullptr, 16);
  memcpy(buf, s + 14, 2);
  buf[2] = 0;
  *rk = (uint32_t)strtoul(buf, nullptr, 16);
  return true;
}

// ---------------------------------------------------------------- plugin
struct SlotDataset::Plugin {
  void* so = nullptr;
  void* parser = nullptr;
  pbx_parser_parse_line_fn parse = nullptr;
  pbx_parser_destroy_fn destroy = nullptr;
  pbx_parser_parse_index_fn parse_index = nullptr;
  pbx_parser_unroll_fn unroll = nullptr;
  pbx_parser_parse_file_fn parse_file = nullptr;
  ~Plugin() {
    if (parser && destroy) destroy(parser);
    if (so) dlclose(so);
  }
};

namespace {
// per-instance staging handed to the plugin through pbx_ins_sink
struct SinkCtx {
  const std::vector<int>* u_idx;
  const std::vector<int>* f_idx;
  const std::vector<SlotDesc>* slots;
  bool keep_ins_id;
  bool need_sparse;
  RecordStore* st;
  ReplicaStore* replica = nullptr;
  const InputIndex* index = nullptr;
  std::vector<std::vector<uint64_t>> u;
  std::vector<std::vector<float>> f;
  std::string ins_id;
  uint64_t sid = 0;
  uint32_t cm = 0, rk = 0;
  int64_t sparse = 0;
  int kept = 0;
  void clear() {
    for (auto& v : u) v.clear();
    for (auto& v : f) v.clear();
    ins_id.clear();
    sid = 0;
    cm = rk = 0;
    sparse = 0;
  }
};

void sink_add_u64(void* c, int slot, const uint64_t* v, int n) {
  SinkCtx* s = (SinkCtx*)c;
  if (slot < 0 || slot >= (int)s->slots->size() || n <= 0) return;
  const int j = (*s->u_idx)[slot];
  if (j < 0) return;  // unused or float slot
  s->u[j].insert(s->u[j].end(), v, v + n);
  if (!(*s->slots)[slot].dense) s->sparse += n;
}

void sink_add_f32(void* c, int slot, const float* v, int n) {
  SinkCtx* s = (SinkCtx*)c;
  if (slot < 0 || slot >= (int)s->slots->size() || n <= 0) return;
  const int j = (*s->f_idx)[slot];
  if (j < 0) return;
  s->f[j].insert(s->f[j].end(), v, v + n);
}

void sink_set_meta(void* c, const char* id, int len, uint64_t sid, uint32_t cm, uint32_t rk) {
  SinkCtx* s = (SinkCtx*)c;
  if (id && len > 0) s->ins_id.assign(id, (size_t)len);
  s->sid = sid;
  s->cm = cm;
  s->rk = rk;
}

int64_t sink_add_cache(void* c, const float* v, int n) {
  SinkCtx* s = (SinkCtx*)c;
  return s->replica ? s->replica->add(v, n) : -1;
}

uint64_t sink_index_offset(void* c, const char* key, int len) {
  SinkCtx* s = (SinkCtx*)c;
  return s->index && key && len > 0 ? s->index->offset(key, (size_t)len) : InputIndex::kMissing;
}

void index_add(void* c, const char* key, int len, const float* v, int n) {
  if (key && len > 0) ((InputIndex*)c)->add(std::string(key, (size_t)len), v, n);
}

int sink_commit(void* c) {
  SinkCtx* s = (SinkCtx*)c;
  int ok = !(s->need_sparse && s->sparse == 0);
  if (ok) {
    RecordStore* st = s->st;
    for (auto& v : s->u) {
      st->u64.insert(st->u64.end(), v.begin(), v.end());
      st->u64_off.push_back((int64_t)st->u64.size());
    }
    for (auto& v : s->f) {
      st->f32.insert(st->f32.end(), v.begin(), v.end());
      st->f32_off.push_back((int64_t)st->f32.size());
    }
    if (s->keep_ins_id) st->ins_id.push_back(s->ins_id);
    st->search_id.push_back(s->sid);
    st->cmatch.push_back(s->cm);
    st->rank.push_back(s->rk);
    s->kept += 1;
  }
  s->clear();
  return ok;
}
}  // namespace

void SlotDataset::set_so_parser(const std::string& path) {
  plugin_.reset();
  if (path.empty()) return;
  auto pl = std::make_shared<Plugin>();
  pl->so = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
  if (!pl->so) throw std::runtime_error(std::string("so parser: dlopen failed: ") + dlerror());
  auto create = (pbx_parser_create_fn)dlsym(pl->so, "pbx_parser_create");
  pl->parse = (pbx_parser_parse_line_fn)dlsym(pl->so, "pbx_parser_parse_line");
  pl->destroy = (pbx_parser_destroy_fn)dlsym(pl->so, "pbx_parser_destroy");
  pl->parse_index = (pbx_parser_parse_index_fn)dlsym(pl->so, "pbx_parser_parse_index");  // optional
  pl->unroll = (pbx_parser_unroll_fn)dlsym(pl->so, "pbx_parser_unroll");                // optional
  pl->parse_file = (pbx_parser_parse_file_fn)dlsym(pl->so, "pbx_parser_parse_file");    // optional
  if (!create || !pl->parse || !pl->destroy)
    throw std::runtime_error("so parser " + path + ": missing pbx_parser_{create,parse_line,destroy}");
  std::vector<const char*> names;
  std::string types;
  for (auto& s : slots_) {
    names.push_back(s.name.c_str());
    types.push_back(s.type);
  }
  pl->parser = create((int)slots_.size(), names.data(), types.c_str());
  if (!pl->parser) throw std::runtime_error("so parser " + path + ": pbx_parser_create returned null");
  plugin_ = pl;
}

bool SlotDataset::parse_plugin_line(const char* line, size_t len, RecordStore* st) const {
  thread_local SinkCtx ctx;
  ctx.u_idx = &u_idx_;
  ctx.f_idx = &f_idx_;
  ctx.slots = &slots_;
  ctx.keep_ins_id = parse_.parse_ins_id || parse_.parse_logkey;
  ctx.need_sparse = !sparse_slots_.empty();
  ctx.st = st;
  ctx.replica = replica_.get();
  ctx.index = input_index_.get();
  ctx.u.resize(store_.nu);
  ctx.f.resize(store_.nf);
  ctx.clear();
  ctx.kept = 0;
  pbx_ins_sink sink{&ctx,          sink_add_u64,
                    sink_add_f32,  sink_set_meta,
                    sink_commit,   replica_ ? sink_add_cache : nullptr,
                    input_index_ ? sink_index_offset : nullptr};
  const int n = plugin_->parse(plugin_->parser, line, len, &sink);
  ctx.clear();  // an instance the plugin never committed is discarded
  return n > 0 && ctx.kept > 0;
}

namespace {
int64_t file_read(void* ctx, char* buf, int64_t len) {
  return (int64_t)fread(buf, 1, (size_t)len, (FILE*)ctx);
}
}  // namespace

int64_t SlotDataset::parse_plugin_file(const std::string& path, FILE* fp, RecordStore* st) const {
  SinkCtx ctx;
  ctx.u_idx = &u_idx_;
  ctx.f_idx = &f_idx_;
  ctx.slots = &slots_;
  ctx.keep_ins_id = parse_.parse_ins_id || parse_.parse_logkey;
  ctx.need_sparse = !sparse_slots_.empty();
  ctx.st = st;
  ctx.replica = replica_.get();
  ctx.index = input_index_.get();
  ctx.u.resize(store_.nu);
  ctx.f.resize(store_.nf);
  ctx.clear();
  const pbx_ins_sink sink{&ctx,         sink_add_u64,
                          sink_add_f32, sink_set_meta,
                          sink_commit,  replica_ ? sink_add_cache : nullptr,
                          input_index_ ? sink_index_offset : nullptr};
  const bool with_path = Flags::ins().get_bool_or("enable_ins_parser_add_file_path", false);
  return plugin_->parse_file(plugin_->parser, with_path ? path.c_str() : nullptr, file_read, fp, &sink);
}

int64_t SlotDataset::load_index_files(const std::vector<std::string>& files, InputIndex* t) const {
  if (!plugin_ || !plugin_->parse_index) return t->load_text(files, threads_);
  std::atomic<size_t> next{0};
  std::atomic<int64_t> n{0};
  std::vector<std::thread> th;
  const int T = std::max(1, std::min<int>(threads_, (int)files.size()));
  for (int k = 0; k < T; ++k)
    th.emplace_back([&] {
      const pbx_index_sink sink{t, index_add};
      for (;;) {
        const size_t fi = next++;
        if (fi >= files.size()) break;
        bool is_pipe = false;
        FILE* fp = default_file_mgr().open_read(files[fi], "", &is_pipe);
        if (!fp) continue;
        char* line = nullptr;
        size_t cap = 0;
        ssize_t len;
        while ((len = getline(&line, &cap, fp)) > 0) {
          const int r = plugin_->parse_index(plugin_->parser, line, (size_t)len, &sink);
          if (r > 0) n += r;
        }
        free(line);
        FileMgr::close(fp, is_pipe);
      }
    });
  for (auto& x : th) x.join();
  return n.load();
}

bool SlotDataset::parse_line(const char* str, size_t len, RecordStore* st) const {
  if (plugin_) return parse_plugin_line(str, len, st);
  const char* end = str + len;
  char* p = const_cast<char*>(str);
  std::string ins_id;
  uint64_t sid = 0;
  uint32_t cm = 0, rk = 0;
  auto read_token = [&](std::string* out) -> bool {
    long n = strtol(p, &p, 10);
    if (n != 1) return false;
    while (p < end && *p == ' ') ++p;
    const char* b = p;
    while (p < end && *p != ' ' && *p != '\n' && *p != '\t') ++p;
    out->assign(b, p - b);
    return true;
  };
  if (parse_.parse_ins_id) {
    if (!read_token(&ins_id)) return false;
  }
  if (parse_.parse_logkey) {
    std::string lk;
    if (!read_token(&lk)) return false;
    parse_logkey(lk.data(), lk.size(), &sid, &cm, &rk);
    ins_id = lk;
  }
  if (parse_.sample_rate < 1.0f) {
    const uint64_t hh = mix64(std::hash<std::string>()(std::string(str, std::min<size_t>(len, 64))) ^ parse_.sample_seed);
    if ((float)(hh >> 40) / 16777216.0f >= parse_.sample_rate) return false;
  }
  const int nu = store_.nu, nf = store_.nf;
  thread_local std::vector<std::vector<uint64_t>> uvals;
  thread_local std::vector<std::vector<float>> fvals;
  uvals.resize(nu);
  fvals.resize(nf);
  for (auto& v : uvals) v.clear();
  for (auto& v : fvals) v.clear();
  int64_t total_sparse = 0;
  for (size_t i = 0; i < slots_.size(); ++i) {
    const SlotDesc& s = slots_[i];
    char* q = p;
    long num = strtol(p, &q, 10);
    if (q == p || num <= 0) return false;  // reference: the number of ids can not be zero
    p = q;
    if (s.used && s.type == 'u') {
      auto& v = uvals[u_idx_[i]];
      for (long j = 0; j < num; ++j) {
        const uint64_t x = strtoull(p, &q, 10);
        if (q == p) return false;
        p = q;
        if (x == 0 && !s.dense) continue;
        v.push_back(x);
        if (!s.dense) ++total_sparse;
      }
    } else if (s.used && s.type == 'f') {
      auto& v = fvals[f_idx_[i]];
      for (long j = 0; j < num; ++j) {
        const float x = strtof(p, &q);
        if (q == p) return false;
        p = q;
        if (std::fabs(x) < 1e-6f && !s.dense) continue;
        v.push_back(x);
      }
    } else {
      for (long j = 0; j < num; ++j) {
        while (p < end && *p == ' ') ++p;
        while (p < end && *p != ' ' && *p != '\n') ++p;
      }
    }
  }
  if (total_sparse == 0 && !sparse_slots_.empty()) return false;
  for (int j = 0; j < nu; ++j) {
    st->u64.insert(st->u64.end(), uvals[j].begin(), uvals[j].end());
    st->u64_off.push_back((int64_t)st->u64.size());
  }
  for (int j = 0; j < nf; ++j) {
    st->f32.insert(st->f32.end(), fvals[j].begin(), fvals[j].end());
    st->f32_off.push_back((int64_t)st->f32.size());
  }
  if (parse_.parse_ins_id || parse_.parse_logkey) st->ins_id.push_back(ins_id);
  st->search_id.push_back(sid);
  st->cmatch.push_back(cm);
  st->rank.push_back(rk);
  return true;
}

int64_t SlotDataset::load_files(const std::vector<std::string>& files, RecordStore* out) {
  const int T = std::max(1, std::min<int>(threads_, (int)files.size()));
  // FLAGS_enable_ins_parser_file: the plugin parses whole files
  const bool file_mode = plugin_ && plugin_->parse_file && Flags::ins().get_bool_or("enable_ins_parser_file", false);
  std::vector<RecordStore> parts(T);
  std::atomic<size_t> next{0};
  std::atomic<int64_t> bad{0};
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t) {
    parts[t].reset(store_.nu, store_.nf);
    th.emplace_back([&, t] {
      std::unique_ptr<KeyAgent::Stage> stg;
      if (agent_) stg.reset(new KeyAgent::Stage(agent_.get()));
      for (;;) {
        const size_t fi = next++;
        if (fi >= files.size()) break;
        const std::string& f = files[fi];
        // local / remote (hdfs://, afs://), plain / .gz, through the converter
        bool is_pipe = false;
        FILE* fp = default_file_mgr().open_read(f, pipe_command_, &is_pipe);
        if (!fp) {
          bad += 1;
          continue;
        }
        const int64_t r0 = parts[t].nrec();
        if (file_mode) {
          if (parse_plugin_file(f, fp, &parts[t]) < 0) bad += 1;
        } else {
          char* line = nullptr;
          size_t cap = 0;
          ssize_t n;
          while ((n = getline(&line, &cap, fp)) > 0) {
            if (n <= 1) continue;
            if (!parse_line(line, (size_t)n, &parts[t])) bad += 1;
          }
          free(line);
        }
        if (stg) register_keys(parts[t], r0, parts[t].nrec(), stg.get());
        FileMgr::close(fp, is_pipe);
      }
    });
  }
  for (auto& x : th) x.join();
  for (auto& pt : parts) out->append(pt);
  bad_lines_ += bad.load();
  return out->nrec();
}

int64_t SlotDataset::load_into_memory() {
  RecordStore st;
  st.reset(store_.nu, store_.nf);
  load_files(files_, &st);
  store_.append(st);
  ++version_;
  order_.resize(store_.nrec());
  std::iota(order_.begin(), order_.end(), 0);
  return store_.nrec();
}

void SlotDataset::preload_into_memory() {
  if (preload_ && preload_->joinable()) preload_->join();
  preload_store_.reset(store_.nu, store_.nf);
  auto files = files_;
  preload_.reset(new std::thread([this, files] { load_files(files, &preload_store_); }));
}

int64_t SlotDataset::wait_preload_done() {
  if (preload_ && preload_->joinable()) preload_->join();
  store_.append(preload_store_);
  ++version_;
  preload_store_.reset(store_.nu, store_.nf);
  order_.resize(store_.nrec());
  std::iota(order_.begin(), order_.end(), 0);
  return store_.nrec();
}

int64_t SlotDataset::add_lines(const std::vector<std::string>& lines) {
  int64_t ok = 0;
  const int64_t r0 = store_.nrec();
  for (auto& l : lines) {
    if (parse_line(l.data(), l.size(), &store_)) ++ok; else ++bad_lines_;
  }
  if (agent_) {
    KeyAgent::Stage stg(agent_.get());
    register_keys(store_, r0, store_.nrec(), &stg);
  }
  ++version_;
  order_.resize(store_.nrec());
  std::iota(order_.begin(), order_.end(), 0);
  return ok;
}

void SlotDataset::release_memory() {
  store_.reset(store_.nu, store_.nf);
  ++version_;
  order_.clear();
  store_.u64.shrink_to_fit();
  store_.f32.shrink_to_fit();
}

void SlotDataset::register_keys(const RecordStore& st, int64_t r0, int64_t r1, KeyAgent::Stage* stg) const {
  const int nu = st.nu;
  for (int64_t i = r0; i < r1; ++i)
    for (int j : sparse_slots_)
      for (int64_t e = st.u64_off[i * nu + j]; e < st.u64_off[i * nu + j + 1]; ++e) stg->push(st.u64[e]);
}

std::vector<uint64_t> SlotDataset::collect_keys(bool unique) const {
  const int64_t n = store_.nrec();
  if (unique) {
    // parallel registration into a sharded set (the loader-thread path)
    KeyAgent agent;
    const int T = std::max(1, std::min(threads_ * 2, 16));
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t] {
        KeyAgent::Stage stg(&agent);
        register_keys(store_, n * t / T, n * (t + 1) / T, &stg);
      });
    for (auto& x : th) x.join();
    return agent.keys();
  }
  std::vector<uint64_t> keys;
  const int nu = store_.nu;
  for (int64_t i = 0; i < n; ++i)
    for (int j : sparse_slots_) {
      const int64_t b = store_.u64_off[i * nu + j], e = store_.u64_off[i * nu + j + 1];
      keys.insert(keys.end(), store_.u64.begin() + b, store_.u64.begin() + e);
    }
  return keys;
}

void SlotDataset::shuffle(uint64_t seed) {
  std::mt19937_64 rng(seed);
  std::shuffle(order_.begin(), order_.end(), rng);
}

std::vector<int64_t> SlotDataset::merge_by_search_id() {
  std::stable_sort(order_.begin(), order_.end(),
                   [this](int64_t a, int64_t b) { return store_.search_id[a] < store_.search_id[b]; });
  std::vector<int64_t> off{0};
  for (size_t i = 1; i < order_.size(); ++i)
    if (store_.search_id[order_[i]] != store_.search_id[order_[i - 1]]) off.push_back((int64_t)i);
  off.push_back((int64_t)order_.size());
  return off;
}

SlotDataset::BatchDims SlotDataset::batch_dims(int64_t begin, int64_t count) const {
  BatchDims d;
  d.B = (int)count;
  const int nu = store_.nu;
  for (int64_t r = begin; r < begin + count; ++r) {
    const int64_t i = order_[r];
    for (int j : sparse_slots_) d.L += store_.u64_off[i * nu + j + 1] - store_.u64_off[i * nu + j];
  }
  return d;
}

// batch assembly pool: condition-variable workers (no OpenMP spin-waiting that
// would steal cores from the training loop's own threads)
static ThreadPool& assembly_pool() {
  static ThreadPool pool([] {
    const char* e = std::getenv("PBX_BATCH_THREADS");
    const int n = e ? std::atoi(e) : 8;
    return n < 1 ? 1 : n;
  }());
  return pool;
}

void SlotDataset::build_batch(int64_t begin, int64_t count, int64_t* keys, int64_t* lod, float* dense) const {
  build_batch_impl(begin, count, [keys](int64_t) { return keys; }, lod, dense);
}

void SlotDataset::build_batch_impl(int64_t begin, int64_t count, const std::function<int64_t*(int64_t)>& keys_for,
                                   int64_t* lod, float* dense) const {
  const int nu = store_.nu, nf = store_.nf;
  const int B = (int)count;
  const int S = (int)sparse_slots_.size();
  ThreadPool& pool = assembly_pool();
  // record-major passes: every record's slots are contiguous in the store, so
  // each record is read once, sequentially (a slot-major walk would stride
  // over every record once per slot).  Pass 1 writes per-slot lengths into
  // the lod rows and per-chunk slot totals; a tiny serial scan over (slot,
  // chunk) gives every chunk its starting offset per slot; pass 2 (same static
  // chunks) turns its lengths into offsets, copies each record's keys to its
  // slot-major positions and fills the dense row.
  const int T = pool.size();
  std::vector<int64_t> csum((size_t)T * S, 0);
  pool.parallel_range(B, [&](int t, int64_t bb, int64_t be) {
    int64_t* cs = &csum[(size_t)t * S];
    for (int64_t b = bb; b < be; ++b) {
      const int64_t i = order_[begin + b];
      const int64_t* off = &store_.u64_off[i * nu];
      for (int s = 0; s < S; ++s) {
        const int j = sparse_slots_[s];
        const int64_t n = off[j + 1] - off[j];
        lod[(int64_t)s * (B + 1) + b] = n;
        cs[s] += n;
      }
    }
  });
  int64_t k = 0;
  for (int s = 0; s < S; ++s) {
    for (int t = 0; t < T; ++t) {
      const int64_t n = csum[(size_t)t * S + s];
      csum[(size_t)t * S + s] = k;
      k += n;
    }
    lod[(int64_t)s * (B + 1) + B] = k;
  }
  int64_t* keys = keys_for(k);
  const bool do_dense = dense && dense_width_ > 0;
  pool.parallel_range(B, [&](int t, int64_t bb, int64_t be) {
    int64_t* run = &csum[(size_t)t * S];
    for (int64_t b = bb; b < be; ++b) {
      const int64_t i = order_[begin + b];
      const int64_t* off = &store_.u64_off[i * nu];
      for (int s = 0; s < S; ++s) {
        const int j = sparse_slots_[s];
        int64_t& l = lod[(int64_t)s * (B + 1) + b];
        const int64_t n = l;
        l = run[s];
        int64_t* dst = keys + run[s];
        const uint64_t* src = store_.u64.data() + off[j];
        for (int64_t e = 0; e < n; ++e) dst[e] = (int64_t)src[e];
        run[s] += n;
      }
      if (!do_dense) continue;
      float* row = dense + b * dense_width_;
      for (const auto& d : dense_refs_) {
        int64_t e0, e1;
        if (d.type == 'u') {
          e0 = store_.u64_off[i * nu + d.idx];
          e1 = store_.u64_off[i * nu + d.idx + 1];
        } else {
          e0 = store_.f32_off[i * nf + d.idx];
          e1 = store_.f32_off[i * nf + d.idx + 1];
        }
        for (int c = 0; c < d.dim; ++c) {
          const int64_t e = e0 + c;
          float v = 0.f;
          if (e < e1) v = d.type == 'u' ? (float)store_.u64[e] : store_.f32[e];
          row[d.col + c] = v;
        }
      }
    }
  });
}

int64_t SlotDataset::build_batch_staged(int64_t begin, int64_t count, int64_t* keys, int64_t keys_cap, int64_t* lod,
                                       float* dense) const {
  thread_local std::vector<int64_t> sk, sl;
  thread_local std::vector<float> sd;
  const int64_t S = (int64_t)sparse_slots_.size();
  const int64_t nl = S * (count + 1), nd = dense ? count * dense_width_ : 0;
  if ((int64_t)sl.size() < nl) sl.resize(nl);
  if ((int64_t)sd.size() < nd) sd.resize(nd);
  int64_t L = 0;
  build_batch_impl(
      begin, count,
      [&](int64_t n) {
        // lengths are known before any key is written: refuse an oversized batch
        if (n > keys_cap) throw std::runtime_error("build_batch: batch has more keys than its buffer");
        if ((int64_t)sk.size() < n) sk.resize(n);
        L = n;
        return sk.data();
      },
      sl.data(), nd ? sd.data() : nullptr);
  // (thread_local names inside the pool's lambdas would resolve to the
  // workers' own, empty, scratch: hand them this thread's pointer)
  const int64_t* src = sk.data();
  assembly_pool().parallel_range(keys_cap, [&](int, int64_t a, int64_t b) {
    const int64_t e = std::min(b, L);
    if (a < e) std::memcpy(keys + a, src + a, (e - a) * sizeof(int64_t));
    for (int64_t i = std::max(a, L); i < b; ++i) keys[i] = -1;
  });
  std::memcpy(lod, sl.data(), nl * sizeof(int64_t));
  if (nd) std::memcpy(dense, sd.data(), nd * sizeof(float));
  return L;
}

std::vector<int32_t> SlotDataset::dense_refs() const {
  std::vector<int32_t> out;
  for (const auto& d : dense_refs_) {
    out.push_back(d.type == 'u' ? 0 : 1);
    out.push_back(d.idx);
    out.push_back(d.dim);
    out.push_back(d.col);
  }
  return out;
}

void SlotDataset::build_rank_offset(int64_t begin, int64_t count, int max_rank, int32_t* out) const {
  const int col = 2 * max_rank + 1;
  for (int64_t i = 0; i < count * col; ++i) out[i] = -1;
  auto rank_of = [&](int64_t r) -> int {
    const int64_t i = order_[begin + r];
    const uint32_t cm = store_.cmatch[i], rk = store_.rank[i];
    if ((cm == 222 || cm == 223) && rk <= (uint32_t)max_rank && rk != 0) return (int)rk;
    return -1;
  };
  int64_t g0 = 0;
  while (g0 < count) {
    int64_t g1 = g0 + 1;
    const uint64_t sid = store_.search_id[order_[begin + g0]];
    while (g1 < count && store_.search_id[order_[begin + g1]] == sid) ++g1;
    for (int64_t j = g0; j < g1; ++j) {
      const int rank = rank_of(j);
      out[j * col] = rank;
      if (rank > 0) {
        for (int64_t k = g0; k < g1; ++k) {
          const int fr = rank_of(k);
          if (fr > 0) {
            const int m = fr - 1;
            out[j * col + 2 * m + 1] = fr;
            out[j * col + 2 * m + 2] = (int32_t)k;
          }
        }
      }
    }
    g0 = g1;
  }
}

// ---------------------------------------------------------------- archive
static const uint64_t kArchiveMagic = 0x50425841524348ULL;  // "PBXARCH"

template <typename T>
static void wvec(FILE* f, const std::vector<T>& v) {
  const uint64_t n = v.size();
  fwrite(&n, 8, 1, f);
  if (n) fwrite(v.data(), sizeof(T), n, f);
}
template <typename T>
static bool rvec(FILE* f, std::vector<T>* v) {
  uint64_t n = 0;
  if (fread(&n, 8, 1, f) != 1) return false;
  v->resize(n);
  return n == 0 || fread(v->data(), sizeof(T), n, f) == n;
}

void SlotDataset::save_archive(const std::string& path) const {
  FILE* f = fopen(path.c_str(), "wb");
  if (!f) throw std::runtime_error("cannot open archive for write: " + path);
  fwrite(&kArchiveMagic, 8, 1, f);
  const int32_t hdr[2] = {store_.nu, store_.nf};
  fwrite(hdr, 4, 2, f);
  wvec(f, store_.u64);
  wvec(f, store_.u64_off);
  wvec(f, store_.f32);
  wvec(f, store_.f32_off);
  wvec(f, store_.search_id);
  wvec(f, store_.cmatch);
  wvec(f, store_.rank);
  const uint64_t ni = store_.ins_id.size();
  fwrite(&ni, 8, 1, f);
  for (auto& s : store_.ins_id) {
    const uint32_t l = (uint32_t)s.size();
    fwrite(&l, 4, 1, f);
    fwrite(s.data(), 1, l, f);
  }
  const int32_t ed = store_.ext.size() == (size_t)store_.nrec() * (size_t)store_.ext_dim ? store_.ext_dim : 0;
  if (ed > 0) {  // optional tail: extension floats (older archives end here)
    fwrite(&ed, 4, 1, f);
    wvec(f, store_.ext);
  }
  fclose(f);
}

int64_t SlotDataset::load_archive(const std::string& path, bool append) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) throw std::runtime_error("cannot open archive: " + path);
  uint64_t magic = 0;
  int32_t hdr[2];
  if (fread(&magic, 8, 1, f) != 1 || magic != kArchiveMagic || fread(hdr, 4, 2, f) != 2) {
    fclose(f);
    throw std::runtime_error("bad archive: " + path);
  }
  if (hdr[0] != store_.nu || hdr[1] != store_.nf) {
    fclose(f);
    throw std::runtime_error("archive slot layout mismatch: " + path);
  }
  RecordStore st;
  st.nu = hdr[0];
  st.nf = hdr[1];
  bool ok = rvec(f, &st.u64) && rvec(f, &st.u64_off) && rvec(f, &st.f32) && rvec(f, &st.f32_off) &&
            rvec(f, &st.search_id) && rvec(f, &st.cmatch) && rvec(f, &st.rank);
  uint64_t ni = 0;
  ok = ok && fread(&ni, 8, 1, f) == 1;
  for (uint64_t i = 0; ok && i < ni; ++i) {
    uint32_t l = 0;
    ok = fread(&l, 4, 1, f) == 1;
    std::string s(l, '\0');
    ok = ok && (l == 0 || fread(&s[0], 1, l, f) == l);
    st.ins_id.push_back(s);
  }
  int32_t ed = 0;
  if (ok && fread(&ed, 4, 1, f) == 1 && ed > 0) {
    st.ext_dim = ed;
    ok = rvec(f, &st.ext);
  }
  fclose(f);
  if (!ok) throw std::runtime_error("truncated archive: " + path);
  if (!append) store_.reset(store_.nu, store_.nf);
  store_.append(st);
  ++version_;
  if (agent_) {
    KeyAgent::Stage stg(agent_.get());
    register_keys(st, 0, st.nrec(), &stg);
  }
  order_.resize(store_.nrec());
  std::iota(order_.begin(), order_.end(), 0);
  return st.nrec();
}

// ---------------------------------------------------------------- UnrollInstance
namespace {
struct ViewCtx {
  const RecordStore* st;
  const std::vector<int>* u_idx;
  const std::vector<int>* f_idx;
};
int view_get_u64(void* c, int64_t rec, int slot, const uint64_t** v) {
  const ViewCtx* x = (const ViewCtx*)c;
  if (rec < 0 || rec >= x->st->nrec() || slot < 0 || slot >= (int)x->u_idx->size()) return 0;
  const int j = (*x->u_idx)[slot];
  if (j < 0) return 0;
  const int64_t b = x->st->u64_off[rec * x->st->nu + j], e = x->st->u64_off[rec * x->st->nu + j + 1];
  *v = x->st->u64.data() + b;
  return (int)(e - b);
}
int view_get_f32(void* c, int64_t rec, int slot, const float** v) {
  const ViewCtx* x = (const ViewCtx*)c;
  if (rec < 0 || rec >= x->st->nrec() || slot < 0 || slot >= (int)x->f_idx->size()) return 0;
  const int j = (*x->f_idx)[slot];
  if (j < 0) return 0;
  const int64_t b = x->st->f32_off[rec * x->st->nf + j], e = x->st->f32_off[rec * x->st->nf + j + 1];
  *v = x->st->f32.data() + b;
  return (int)(e - b);
}
void view_get_meta(void* c, int64_t rec, const char** id, int* id_len, uint64_t* sid, uint32_t* cm, uint32_t* rk) {
  const ViewCtx* x = (const ViewCtx*)c;
  const RecordStore& st = *x->st;
  const bool has_id = (size_t)rec < st.ins_id.size();
  *id = has_id ? st.ins_id[(size_t)rec].data() : "";
  *id_len = has_id ? (int)st.ins_id[(size_t)rec].size() : 0;
  *sid = st.search_id[(size_t)rec];
  *cm = st.cmatch[(size_t)rec];
  *rk = st.rank[(size_t)rec];
}
}  // namespace

int64_t SlotDataset::unroll_instances() {
  if (!plugin_ || !plugin_->unroll) return store_.nrec();  // reference default: records unchanged
  ViewCtx vc{&store_, &u_idx_, &f_idx_};
  const pbx_record_view view{&vc, store_.nrec(), view_get_u64, view_get_f32, view_get_meta};
  RecordStore out;
  out.reset(store_.nu, store_.nf);
  SinkCtx ctx;
  ctx.u_idx = &u_idx_;
  ctx.f_idx = &f_idx_;
  ctx.slots = &slots_;
  ctx.keep_ins_id = true;
  ctx.need_sparse = !sparse_slots_.empty();
  ctx.st = &out;
  ctx.u.resize(store_.nu);
  ctx.f.resize(store_.nf);
  ctx.clear();
  const pbx_ins_sink sink{&ctx, sink_add_u64, sink_add_f32, sink_set_meta, sink_commit, nullptr, nullptr};
  const int64_t n = plugin_->unroll(plugin_->parser, &view, &sink);
  if (n < 0) return -1;
  store_ = std::move(out);
  ++version_;
  if (agent_) {
    KeyAgent::Stage stg(agent_.get());
    register_keys(store_, 0, store_.nrec(), &stg);
  }
  order_.resize((size_t)store_.nrec());
  std::iota(order_.begin(), order_.end(), 0);
  return store_.nrec();
}

// ---------------------------------------------------------------- PCOC q values
void SlotDataset::batch_ext(int64_t begin, int64_t count, int d, float* out) {
  store_.ensure_ext(d);
  for (int64_t i = 0; i < count; ++i) {
    const int64_t r = order_.empty() ? begin + i : order_[(size_t)(begin + i)];
    memcpy(out + i * d, store_.ext.data() + r * d, sizeof(float) * (size_t)d);
  }
}

void SlotDataset::store_ext(int64_t begin, int64_t count, int d, int col, const float* q) {
  if (col < 0 || col >= d) throw std::out_of_range("store_ext: column");
  store_.ensure_ext(d);
  for (int64_t i = 0; i < count; ++i) {
    const int64_t r = order_.empty() ? begin + i : order_[(size_t)(begin + i)];
    store_.ext[(size_t)(r * d + col)] = q[i];
  }
}

// ---------------------------------------------------------------- shuffle
namespace {
template <typename T>
void put_vec(std::string* o, const std::vector<T>& v) {
  const uint64_t n = v.size();
  o->append(reinterpret_cast<const char*>(&n), 8);
  if (n) o->append(reinterpret_cast<const char*>(v.data()), n * sizeof(T));
}
template <typename T>
bool get_vec(const char*& p, const char* end, std::vector<T>* v) {
  uint64_t n;
  if (end - p < 8) return false;
  memcpy(&n, p, 8);
  p += 8;
  if ((uint64_t)(end - p) / sizeof(T) < n) return false;
  v->resize(n);
  if (n) memcpy(v->data(), p, n * sizeof(T));
  p += n * sizeof(T);
  return true;
}
}  // namespace

void RecordStore::serialize(std::string* out) const {
  const int32_t hdr[2] = {nu, nf};
  out->append(reinterpret_cast<const char*>(hdr), 8);
  put_vec(out, u64);
  put_vec(out, u64_off);
  put_vec(out, f32);
  put_vec(out, f32_off);
  put_vec(out, search_id);
  put_vec(out, cmatch);
  put_vec(out, rank);
  const uint64_t ni = ins_id.size();
  out->append(reinterpret_cast<const char*>(&ni), 8);
  for (const auto& s : ins_id) {
    const uint32_t l = (uint32_t)s.size();
    out->append(reinterpret_cast<const char*>(&l), 4);
    out->append(s);
  }
  const int32_t ed = ext.size() == (size_t)nrec() * (size_t)ext_dim ? ext_dim : 0;
  out->append(reinterpret_cast<const char*>(&ed), 4);
  if (ed > 0) put_vec(out, ext);
}

bool RecordStore::parse(const char* buf, size_t len) {
  const char* p = buf;
  const char* end = buf + len;
  int32_t hdr[2];
  if (len < 8) return false;
  memcpy(hdr, p, 8);
  p += 8;
  if (hdr[0] != nu || hdr[1] != nf) return false;
  RecordStore st;
  st.nu = nu;
  st.nf = nf;
  bool ok = get_vec(p, end, &st.u64) && get_vec(p, end, &st.u64_off) && get_vec(p, end, &st.f32) &&
            get_vec(p, end, &st.f32_off) && get_vec(p, end, &st.search_id) && get_vec(p, end, &st.cmatch) &&
            get_vec(p, end, &st.rank);
  uint64_t ni = 0;
  ok = ok && end - p >= 8;
  if (ok) {
    memcpy(&ni, p, 8);
    p += 8;
  }
  for (uint64_t i = 0; ok && i < ni; ++i) {
    uint32_t l;
    ok = end - p >= 4;
    if (!ok) break;
    memcpy(&l, p, 4);
    p += 4;
    ok = (uint64_t)(end - p) >= l;
    if (ok) st.ins_id.emplace_back(p, l);
    p += ok ? l : 0;
  }
  int32_t ed = 0;
  ok = ok && end - p >= 4;
  if (ok) {
    memcpy(&ed, p, 4);
    p += 4;
  }
  if (ok && ed > 0) {
    st.ext_dim = ed;
    ok = get_vec(p, end, &st.ext);
  }
  ok = ok && p == end && st.u64_off.size() >= 1 && st.f32_off.size() >= 1;
  if (ok) append(st);
  return ok;
}

int64_t SlotDataset::global_shuffle(MsgService& svc, int mode, uint64_t seed, int64_t chunk, int threads) {
  const int W = svc.world(), R = svc.rank();
  if (chunk < 1) chunk = 1;
  const RecordStore& st = store_;
  const int64_t n = st.nrec();
  std::vector<std::vector<int64_t>> dest((size_t)W);
  std::mt19937_64 rng(seed * 1000003ULL + (uint64_t)R);
  for (int64_t i = 0; i < n; ++i) {
    uint64_t h;
    if (mode == 1) {
      h = mix64(st.search_id[(size_t)i]);
    } else if (mode == 2) {
      const std::string& id = (size_t)i < st.ins_id.size() ? st.ins_id[(size_t)i] : std::string();
      if (id.size() < 32) throw std::runtime_error("global_shuffle: ins_id shorter than 32 bytes: " + id);
      h = xxh64(id.data(), 32, 0);
    } else {
      h = rng();
    }
    dest[(size_t)(h % (uint64_t)W)].push_back(i);
  }

  std::mutex mu;
  std::condition_variable cv;
  int finished = 0;
  bool bad = false;
  std::vector<char> lost_peer((size_t)W, 0), done_peer((size_t)W, 0);  // lost connections, end markers seen
  std::string send_err;
  RecordStore incoming;
  incoming.reset(st.nu, st.nf);
  const int lid = svc.add_loss_listener([&](int peer) {
    std::lock_guard<std::mutex> g(mu);
    lost_peer[(size_t)peer] = 1;
    cv.notify_all();
  });
  // a peer lost before its end marker arrived: its records never will (mu held)
  auto lost_unfinished = [&]() {
    for (int r = 0; r < W; ++r)
      if (lost_peer[(size_t)r] && !done_peer[(size_t)r]) return r;
    return -1;
  };
  const int sid = svc.register_handler([&](int src, const char* buf, int64_t len) {
    if (len == 0) {  // end of this peer's stream (FIFO per peer: after its data)
      std::lock_guard<std::mutex> g(mu);
      ++finished;
      if (src >= 0 && src < W) done_peer[(size_t)src] = 1;
      cv.notify_all();
      return;
    }
    RecordStore part;
    part.reset(st.nu, st.nf);
    const bool ok = part.parse(buf, (size_t)len);
    std::lock_guard<std::mutex> g(mu);
    if (ok) {
      incoming.append(part);
    } else {
      bad = true;
    }
  });
  // stream the outgoing records, one message per chunk; `threads` workers
  // (FLAGS_padbox_dataset_shuffle_thread_num) serialize chunks in parallel,
  // each owning whole destinations so a destination's chunks stay in order
  std::vector<std::thread> workers;
  const int T = std::max(1, std::min(threads, W - 1));
  for (int t = 0; t < T; ++t)
    workers.emplace_back([&, t] {
      std::string msg;
      for (int r = 0, k = 0; r < W; ++r) {
        if (r == R) continue;
        if (k++ % T != t) continue;
        const auto& idx = dest[(size_t)r];
        for (size_t b = 0; b < idx.size(); b += (size_t)chunk) {
          std::vector<int64_t> part(idx.begin() + b, idx.begin() + std::min(idx.size(), b + (size_t)chunk));
          msg.clear();
          st.select(part).serialize(&msg);
          try {
            svc.send_message((sid << 16) | r, msg.data(), (int64_t)msg.size(), nullptr);
          } catch (const std::exception& e) {  // destination lost: stop sending to it
            std::lock_guard<std::mutex> g(mu);
            if (send_err.empty()) send_err = e.what();
            break;
          }
        }
      }
    });
  for (auto& w : workers) w.join();
  std::string err;
  try {
    for (int r = 0; r < W; ++r)
      if (r != R) svc.send_message((sid << 16) | r, nullptr, 0, nullptr);
    svc.wait_done(sid);  // every message of ours handled by its receiver (throws if a peer was lost)
  } catch (const std::exception& e) {
    err = e.what();
  }
  {
    const std::vector<int> already = svc.broken_peers();  // lost before the listener existed
    std::unique_lock<std::mutex> g(mu);
    for (int r : already) lost_peer[(size_t)r] = 1;
    cv.wait(g, [&] { return finished == W - 1 || lost_unfinished() >= 0; });
    if (err.empty() && !send_err.empty()) err = send_err;
    const int lu = lost_unfinished();
    if (err.empty() && lu >= 0) err = "rank " + std::to_string(lu) + " was lost before finishing its stream";
  }
  svc.remove_loss_listener(lid);
  svc.unregister_consumer(sid);
  if (!err.empty()) throw std::runtime_error("global_shuffle: " + err);
  if (bad) throw std::runtime_error("global_shuffle: malformed shuffle message");

  RecordStore kept = st.select(dest[(size_t)R]);
  kept.append(incoming);
  store_ = std::move(kept);
  ++version_;
  if (agent_ && incoming.nrec()) {
    // the feed pass keys of the records that arrived (MergeInsKeys runs after
    // the shuffle in the reference, data_set.cc:2293-2349)
    KeyAgent::Stage stg(agent_.get());
    register_keys(incoming, 0, incoming.nrec(), &stg);
  }
  order_.resize((size_t)store_.nrec());
  std::iota(order_.begin(), order_.end(), 0);
  return incoming.nrec();
}

}  // namespace pbx

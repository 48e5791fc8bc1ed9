// In-memory slot dataset for pass-based CTR training.
//
// Behaviour reproduced (not code): SlotRecord CSR storage (fw/data_feed.h:96-240),
// the MultiSlot text parser with optional ins_id/logkey prefix and zero-feasign
// dropping (fw/data_feed.cc:4024-4134, parser_log_key :2385-2395),
// PadBoxSlotDataset load / feed-pass key collection / PrepareTrain batching
// (fw/data_set.cc:1905-2860), dense-slot expansion (ExpandSlotRecord
// :3244-3303), page-view merge by search_id (:2648-2688), rank_offset build
// (data_feed.cu:1319-1369), and the O_DIRECT-style binary archive for
// "load into disk" mode (data_feed.cc:2824-2992).
//
// MI355X-first: records are stored columnar (one CSR per pass, not one heap
// object per instance), so building a batch is a handful of memcpy's into
// pinned staging buffers that go to HBM in a single H2D copy per tensor.
#pragma once
#include <cstdint>
#include <cstdio>
#include <functional>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "key_agent.h"
#include "side_tables.h"

namespace pbx {

struct SlotDesc {
  std::string name;
  char type = 'u';  // 'u' = uint64 feasigns, 'f' = float
  bool used = true;
  bool dense = false;  // dense slot: fixed width, zeros kept
  int dense_dim = 1;
};

struct ParseConfig {
  bool parse_ins_id = false;
  bool parse_logkey = false;
  float sample_rate = 1.0f;
  uint64_t sample_seed = 0;
};

// Columnar CSR store of a pass.
struct RecordStore {
  int nu = 0, nf = 0;  // used uint64 / float slot counts
  std::vector<uint64_t> u64;
  std::vector<int64_t> u64_off{0};  // [nrec*nu + 1]
  std::vector<float> f32;
  std::vector<int64_t> f32_off{0};  // [nrec*nf + 1]
  std::vector<std::string> ins_id;
  std::vector<uint64_t> search_id;
  std::vector<uint32_t> cmatch, rank;
  // per-record extension floats (FLAGS_padbox_slotrecord_extend_dim: PCOC q
  // values written by store_q_value, read back by the next batch over the
  // record; data_feed.h:195-240 trailing float[extend_dim])
  int ext_dim = 0;
  std::vector<float> ext;  // [nrec * ext_dim] when ext_dim > 0
  void ensure_ext(int d);
  int64_t nrec() const { return nu ? (int64_t)(u64_off.size() - 1) / nu : (nf ? (int64_t)(f32_off.size() - 1) / nf : (int64_t)search_id.size()); }
  void reset(int nu_, int nf_);
  void append(const RecordStore& o);
  RecordStore select(const std::vector<int64_t>& idx) const;
  // flat byte image (shuffle messages): appends to *out; parse() appends the
  // decoded records to *this and returns false on a malformed image
  void serialize(std::string* out) const;
  bool parse(const char* buf, size_t len);
};

class MsgService;

class SlotDataset {
 public:
  SlotDataset();
  ~SlotDataset();
  void set_slots(const std::vector<SlotDesc>& slots);
  void set_filelist(const std::vector<std::string>& files) { files_ = files; }
  void set_pipe_command(const std::string& cmd) { pipe_command_ = cmd; }
  void set_thread_num(int n) { threads_ = n < 1 ? 1 : n; }
  void set_parse(const ParseConfig& c) { parse_ = c; }
  // dlopen an instance-parser plugin (parser_plugin.h); "" = built-in parser
  void set_so_parser(const std::string& path);
  bool has_so_parser() const { return plugin_ != nullptr; }

  // parse one line into store (returns false if dropped / no sparse feasign)
  bool parse_line(const char* line, size_t len, RecordStore* st) const;
  int64_t load_into_memory();      // blocking
  void preload_into_memory();      // async
  int64_t wait_preload_done();
  int64_t add_lines(const std::vector<std::string>& lines);  // in-memory lines (tests)
  void release_memory();

  int64_t size() const { return store_.nrec(); }
  const RecordStore& store() const { return store_; }
  // any non-const access may change the records: bump the store version the
  // device-resident pass copy (data/device_pass.py) is keyed on
  RecordStore& mutable_store() {
    ++version_;
    return store_;
  }
  uint64_t version() const { return version_; }

  // feed-pass keys: every feasign of sparse uint64 slots (optionally unique)
  std::vector<uint64_t> collect_keys(bool unique) const;
  // feed-pass agent: while set, the loader threads register the sparse
  // feasigns of every record they parse (load / preload / add_lines / archive)
  void set_key_agent(std::shared_ptr<KeyAgent> a) { agent_ = std::move(a); }
  // side tables a parser plugin fills / queries while loading (replica-cache
  // and input-index data feeds)
  void set_replica_cache(std::shared_ptr<ReplicaStore> r) { replica_ = std::move(r); }
  void set_input_index(std::shared_ptr<InputIndex> t) { input_index_ = std::move(t); }
  // index files into `t` (InputTableDataFeed): the plugin's parse_index when
  // it has one, else "key v1 ... vD" text lines
  int64_t load_index_files(const std::vector<std::string>& files, InputIndex* t) const;

  // order of records for this pass (shuffle: Fisher-Yates with seed)
  void shuffle(uint64_t seed);
  void set_order(const std::vector<int64_t>& order) { order_ = order; }
  const std::vector<int64_t>& order() const { return order_; }

  // page-view merge: group consecutive records by search_id (after sorting
  // by search_id); returns pv group offsets into order_
  std::vector<int64_t> merge_by_search_id();

  // Batch assembly over order_[begin, begin+count): writes
  //  keys  [L]            sparse slots, slot-major
  //  lod   [S*(B+1)]
  //  dense [B, dense_width] (dense slots, padded/truncated)
  // returns L.  sizes via batch_sizes().
  struct BatchDims {
    int64_t L = 0;
    int B = 0;
  };
  BatchDims batch_dims(int64_t begin, int64_t count) const;
  void build_batch(int64_t begin, int64_t count, int64_t* keys, int64_t* lod, float* dense) const;
  // build_batch into this thread's pageable scratch, then stream it into the
  // (pinned) targets with sequential copies; keys[L..keys_cap) = -1.  Pinned
  // host memory is write-combined: the assembly's scattered stores into it ran
  // 4x slower than into pageable memory (measured 1.75 vs 0.43 ms per batch).
  // Returns L; throws when L > keys_cap.
  int64_t build_batch_staged(int64_t begin, int64_t count, int64_t* keys, int64_t keys_cap, int64_t* lod,
                             float* dense) const;

 private:
  // keys_for(L) is called once the batch's key count is known and returns the
  // key target (it may throw to refuse the batch)
  void build_batch_impl(int64_t begin, int64_t count, const std::function<int64_t*(int64_t)>& keys_for,
                        int64_t* lod, float* dense) const;

 public:
  // rank_offset [B, 2*max_rank+1] for PV batches (data_feed.cu:1319-1369)
  void build_rank_offset(int64_t begin, int64_t count, int max_rank, int32_t* out) const;

  int num_sparse_slots() const { return (int)sparse_slots_.size(); }
  int dense_width() const { return dense_width_; }
  std::vector<std::string> sparse_slot_names() const;
  // used-uint64 index of each sparse slot (order of sparse_slot_names)
  const std::vector<int>& sparse_slot_u64_index() const { return sparse_slots_; }
  std::vector<std::string> dense_slot_names() const;
  std::vector<int> dense_slot_dims() const;
  // dense slot sources as rows (type 0 = uint64 / 1 = float, used-slot idx,
  // width, first column) for the on-device batch builder
  std::vector<int32_t> dense_refs() const;

  // Inter-rank record shuffle over the message service (PaddleShuffler flow,
  // data_set.cc:2422-2604): every record goes to rank hash % world, where
  // hash = random (mode 0), mix64(search_id) (1, pv merge /
  // enable_shuffle_by_searchid) or xxh64 of the first 32 ins_id bytes (2,
  // merge_by_insid); records travel in messages of up to `chunk` records
  // while the receivers append them, then one empty message per peer marks
  // the end.  Returns the number of records received from peers.
  int64_t global_shuffle(MsgService& svc, int mode, uint64_t seed, int64_t chunk = 4096, int threads = 1);

  // PCOC q values (MiniBatchGpuPack::pack_qvalue / store_qvalue,
  // data_feed.cc:4945-4984): the extension floats of the batch's records
  // [count, d] in batch order, and the write-back of one column from a
  // computed q tensor.  Neither bumps the store version (the device-resident
  // pass does not hold extension floats).
  void batch_ext(int64_t begin, int64_t count, int d, float* out);
  void store_ext(int64_t begin, int64_t count, int d, int col, const float* q);

  // UnrollInstance (FLAGS_padbox_dataset_enable_unrollinstance): the parser
  // plugin's optional pbx_parser_unroll rewrites the loaded pass (any number
  // of instances per record).  Returns the new record count (-1: the plugin
  // failed and the pass is unchanged); without the hook the pass is kept.
  int64_t unroll_instances();

  // binary archive ("load into disk" mode)
  void save_archive(const std::string& path) const;
  int64_t load_archive(const std::string& path, bool append);

  int64_t bad_lines() const { return bad_lines_; }

 private:
  struct Plugin;
  bool parse_plugin_line(const char* line, size_t len, RecordStore* st) const;
  int64_t parse_plugin_file(const std::string& path, FILE* fp, RecordStore* st) const;
  std::shared_ptr<Plugin> plugin_;
  int64_t load_files(const std::vector<std::string>& files, RecordStore* out);
  std::vector<SlotDesc> slots_;
  // index mapping: slot i -> used uint64 idx / used float idx (-1 = unused)
  std::vector<int> u_idx_, f_idx_;
  std::vector<int> sparse_slots_;  // used uint64 idx of sparse slots
  struct DenseRef {
    char type;
    int idx;
    int dim;
    int col;
  };
  std::vector<DenseRef> dense_refs_;
  int dense_width_ = 0;
  std::vector<std::string> files_;
  std::string pipe_command_ = "cat";
  int threads_ = 4;
  ParseConfig parse_;
  RecordStore store_;
  std::vector<int64_t> order_;
  std::unique_ptr<std::thread> preload_;
  RecordStore preload_store_;
  int64_t bad_lines_ = 0;
  uint64_t version_ = 0;
  std::shared_ptr<KeyAgent> agent_;
  std::shared_ptr<ReplicaStore> replica_;
  std::shared_ptr<InputIndex> input_index_;
  void register_keys(const RecordStore& st, int64_t r0, int64_t r1, KeyAgent::Stage* stg) const;
};

}  // namespace pbx

// Launcher API for the hand-written gfx950 kernels.  The .hip translation
// units include only HIP headers (fast to build); the torch-facing glue in
// csrc/hip/bindings.cpp calls these with raw pointers + the current stream.
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>
#include <cstddef>
#include <cstdint>

#include "../common/pbx_common.h"
#include "../common/ckpt_format.h"

namespace pbx {

// ---------------------------------------------------------------- hash table
struct TableDev {
  uint64_t* keys = nullptr;   // [nb*16] mixed keys, kEmptyKey = free
  uint32_t* fill = nullptr;   // [nb] occupied prefix length of each bucket
  float* values = nullptr;    // [(nb*16 + stash_cap) * stride]
  uint64_t nb = 0;            // number of buckets
  uint64_t* stash_keys = nullptr;  // [stash_cap]
  uint32_t* stash_n = nullptr;     // device scalar
  uint32_t stash_cap = 0;
  int stride = 16;  // floats per row
  int dim = 8;      // embedx dim
  // sticky guard bits (device int32): an index a kernel is about to follow
  // that lies outside its buffer -- a table row past the table, a unique id
  // past the batch -- is skipped and recorded here instead of becoming a
  // wild access; SparseEngine.check_overflow raises on it (bits: 1 table row
  // of a push, 2 dedup unique id, 4 dedup perm slot, 8 push occurrence / id)
  int32_t* err = nullptr;
};
PBX_HD int64_t table_rows(const TableDev& t) { return (int64_t)t.nb * kBucketSlots + (int64_t)t.stash_cap; }

// rows[i] = row id of h[i] or -1.  n_dev (optional) = device-side count.
void launch_table_probe(const TableDev& t, const uint64_t* h, int64_t n, const int32_t* n_dev,
                        int64_t* rows, hipStream_t s);
// Owner side of the sharded pull: rows[i] = row of h[i] (or -1) and out[i] =
// its pull record (zero padded to out_stride floats), no dedup needed.
void launch_probe_gather(const TableDev& t, const uint64_t* h, int64_t n, int64_t* rows, float* out, int out_stride,
                         hipStream_t s);
// Owner side of the sharded push without a dedup of the received keys:
// entries with the same table row elect a leader through lock[row] (int32,
// -1 = free, reset by the apply), the others add their record into the
// leader's (slot field excepted); then each leader applies sparse Adagrad.
bool launch_owner_push(const TableDev& t, const int64_t* rows, float* rec, int rec_stride, int64_t n,
                       int32_t* lock, int32_t* lead, const SparseSGDConfig& cfg, uint64_t seed, hipStream_t s);
// Insert unique keys h[i] whose rows[i] < 0.  Overflowing keys are appended to
// ovf_keys (count in ovf_n) for launch_table_resolve_overflow.
void launch_table_insert(const TableDev& t, const uint64_t* h, int64_t n, const int32_t* n_dev,
                         const int64_t* rows, const SparseSGDConfig& cfg, uint64_t seed,
                         int init_embedx, uint64_t* ovf_keys, uint32_t* ovf_n, hipStream_t s);
void launch_table_clamp_fill(const TableDev& t, hipStream_t s);
// Serial cuckoo displacement for the (rare) keys that did not fit; falls back
// to the stash.  fail_n counts keys that could not be placed anywhere.
void launch_table_resolve_overflow(const TableDev& t, const uint64_t* ovf_keys,
                                   const uint32_t* ovf_n, const SparseSGDConfig& cfg, uint64_t seed,
                                   int init_embedx, uint32_t* fail_n, hipStream_t s);
// Compact every bucket to a prefix and delete rows flagged in del (by row id).
void launch_table_count(const TableDev& t, unsigned long long* count, hipStream_t s);
// Write (h, value row) of every occupied slot into out arrays starting at
// atomic cursor; used for save / rehash / host write-back.
void launch_table_export(const TableDev& t, uint64_t* out_keys, float* out_vals,
                         unsigned long long* cursor, hipStream_t s);
// Overwrite value rows for rows[i] >= 0 with vals[i].
void launch_table_assign(const TableDev& t, const int64_t* rows, const float* vals, int64_t n,
                         int vals_stride, hipStream_t s);
// Shrink: decay show/click, age unseen_days, delete rows below thresholds.
struct ShrinkConfig {
  float show_click_decay_rate = 0.98f;
  float delete_threshold = 0.8f;
  float delete_after_unseen_days = 30.f;
  float nonclk_coeff = 0.1f;
  float clk_coeff = 1.0f;
};
void launch_table_shrink(const TableDev& t, const ShrinkConfig& c, unsigned long long* deleted,
                         hipStream_t s);

// ---------------------------------------------------------------- dedup
// Temp-storage sizing for the hipCUB radix sort / scan used by dedup.
size_t dedup_temp_bytes(int64_t n);
// From keys (uint64 feasigns) of length n (padded entries == kEmptyKey are
// ignored): h_sorted (unique-first), perm (sorted position -> original index),
// uid[i] (original index -> unique id, -1 for padding), uniq_h[U], seg[U+1]
// (segment starts into perm), u_count (device scalar U).
void launch_dedup(const uint64_t* keys, int64_t n, bool keys_are_mixed, uint64_t* h_tmp,
                  uint64_t* h_sorted, int32_t* idx_tmp, int32_t* perm, int32_t* flags,
                  int32_t* scan, int32_t* uid, uint64_t* uniq_h, int32_t* seg, int32_t* u_count,
                  void* temp, size_t temp_bytes, hipStream_t s);

// Sort-free dedup (same outputs; uniq_h in insertion order, perm grouped by
// unique id).  Scratch table tk/tu [tmask+1] must start as kEmptyKey / -1 and
// cnt [cap+1] as 0; the launch cleans what the previous run used.
struct HashDedupArgs {
  const uint64_t* keys = nullptr;
  int64_t n = 0, cap = 0;
  int mixed = 0;
  uint64_t* tk = nullptr;
  int32_t* tu = nullptr;
  uint64_t tmask = 0;
  int32_t* slot = nullptr;       // [cap]
  int32_t* slot_of_u = nullptr;  // [cap]
  int32_t* cnt = nullptr;        // [cap+1]
  int32_t* rank = nullptr;       // [cap]
  int32_t* uid = nullptr;
  int32_t* perm = nullptr;
  uint64_t* uniq_h = nullptr;
  int32_t* seg = nullptr;  // [cap+1]
  int32_t* u_count = nullptr;
  int32_t* zero_extra = nullptr;  // optional: zeroed by the first launch (e.g. the shard pack's per-owner counts)
  int zero_n = 0;
};
size_t hash_dedup_temp_bytes(int64_t cap);
void launch_dedup_hash(const HashDedupArgs& a, void* temp, size_t temp_bytes, hipStream_t s);

// ---------------------------------------------------------------- slot metadata
// Flat slot-major key layout: keys of slot s for instance b are
// [lod[s*(B+1)+b], lod[s*(B+1)+b+1]).  Writes occ_slot / occ_ins per key.
void launch_fill_occurrence(const int64_t* lod, int S, int B, int32_t* occ_slot, int32_t* occ_ins,
                            hipStream_t s);

// ---------------------------------------------------------------- pull
// out[u, 0:P] = table row (rows[u]) head (P = 3 + D), zeros if row < 0.
void launch_gather_pull(const TableDev& t, const int64_t* rows, const int32_t* n_dev, int64_t n,
                        float* out, int out_stride, hipStream_t s);

// Fused seqpool + CVM over the pull record source.
struct SeqpoolCvmArgs {
  const float* src = nullptr;   // record base
  int src_stride = 0;           // floats per record
  const int64_t* src_index = nullptr;  // unique id -> record index (nullable: identity)
  const int32_t* uid = nullptr;        // occurrence -> unique id
  const int64_t* lod = nullptr;        // [S*(B+1)]
  int S = 0, B = 0;
  int E = 11;                 // pulled record width used (cvm_offset + ...)
  float* out = nullptr;       // [B, out_stride], slot s at column col_offset + s*Eo
  int out_stride = 0;
  int col_offset = 0;
  int use_cvm = 1;
  int cvm_offset = 2;
  int clk_filter = 0;
  float pad_value = 0.f;
  int need_filter = 0;
  float show_coeff = 0.2f, clk_coeff = 1.0f, threshold = 0.96f;
  int quant_ratio = 0;
  int embed_threshold_filter = 0;
  float embed_threshold = 0.f;
  int embed_thres_size = 0;
  // optional dense features copied into out[b, dense_col : dense_col + dense_dim]
  // by the same launch (the concat of the pooled slots with the dense slots)
  const float* dense = nullptr;
  int dense_dim = 0;
  int dense_col = 0;
  int dense_stride = 0;  // floats between dense rows (0: dense_dim; a column slice of a wider block)
  // optional occurrence map (occ_slot[k] = s, occ_ins[k] = b) written as the
  // keys are walked, so the push needs no separate fill launch
  int32_t* occ_slot = nullptr;
  int32_t* occ_ins = nullptr;
  // optional fused probe (split pull, single shard): occurrence k's row is
  // probed here from its raw feasign probe_keys[k] and written to rows_out[k]
  // (for the side-stream dedup) instead of read through uid / src_index
  const uint64_t* probe_keys = nullptr;
  TableDev probe_t;
  int64_t* rows_out = nullptr;
  // optional fused table-dedup scatter (launch_table_dedup with
  // do_scatter = false before it): for every occurrence k with a row,
  // uid[k] = uid_row[row], perm[seg[uid] + rank[k]] = k; threads 0..3
  // publish the dedup counters (u_count = acc, acc = 0)
  const int32_t* sc_uid_row = nullptr;
  const int32_t* sc_seg = nullptr;
  const int32_t* sc_rank = nullptr;
  int32_t* sc_uid = nullptr;
  int32_t* sc_perm = nullptr;
  int32_t* sc_acc = nullptr;
  int32_t* sc_u_count = nullptr;
  // index guards (0: unchecked): occurrence k < n_occ, unique id < n_index
  // (src_index length), record < src_rows; a violating occurrence is skipped
  // and sets a kSeqpoolGuard* bit of *err (sticky; read by check_guards)
  int64_t n_occ = 0, n_index = 0, src_rows = 0;
  int32_t* err = nullptr;
};
constexpr int32_t kSeqpoolGuardOcc = 16;  // lod walks past the occurrence buffers
constexpr int32_t kSeqpoolGuardUid = 32;  // unique id past src_index
constexpr int32_t kSeqpoolGuardRow = 64;  // record past src
int seqpool_cvm_out_width(const SeqpoolCvmArgs& a);
void launch_seqpool_cvm_fwd(const SeqpoolCvmArgs& a, hipStream_t s);

// ---------------------------------------------------------------- push
// Segmented merge of per-occurrence gradients into per-unique push records.
// Gradient source for occurrence k (instance b, slot s):
//   cvm cols      <- cvm[b*cvm_offset + c]
//   embed cols    <- dout[b*out_stride + col_offset + s*Eo + (c - cvm_offset + (use_cvm?cvm_offset:0))]
// push[uidx(u)] = [slot_id, show, click, -bs*embed_g, -bs*embedx_g...]
struct PushMergeArgs {
  const float* dout = nullptr;
  int out_stride = 0, col_offset = 0;
  const float* cvm = nullptr;
  int cvm_offset = 2;
  int use_cvm = 1;
  int clk_filter = 0;
  int E = 11;  // pull record width (3 + D)
  const int32_t* perm = nullptr;     // sorted position -> occurrence
  const int32_t* uid = nullptr;      // occurrence -> unique
  const int32_t* occ_slot = nullptr;
  const int32_t* occ_ins = nullptr;
  const float* slot_ids = nullptr;   // [S] slot id (as float, BoxPS convention)
  const int32_t* n_valid = nullptr;  // device: number of valid (non-pad) occurrences
  int64_t n = 0;                     // upper bound of occurrences (launch size)
  float* push = nullptr;             // [U_cap, push_stride]
  int push_stride = 12;
  const int64_t* push_index = nullptr;  // unique -> push row (nullable: identity)
  float bs_scale = 1.f;              // multiply embed grads by -bs_scale
  int dim = 8;
  int embed_thres_size = 0;          // use_cvm = 0: leading embed columns dropped from the output
  int32_t* err = nullptr;            // guard bits (TableDev::err)
};
void launch_push_merge(const PushMergeArgs& a, hipStream_t s);
// Owner-side merge of received push records rec[j] (j over n entries) keyed by
// uid_r[j] (sorted by perm_r) into out[u].
void launch_push_merge_records(const float* rec, int rec_stride, const int32_t* perm,
                               const int32_t* uid, const int32_t* n_valid, int64_t n, int dim,
                               float* out, int out_stride, hipStream_t s);
// Sparse Adagrad (+show/click stats, embedx creation) on table rows.
void launch_push_adagrad(const TableDev& t, const int64_t* rows, const float* push,
                         int push_stride, const int32_t* n_dev, int64_t n,
                         const SparseSGDConfig& cfg, uint64_t seed, hipStream_t s);
// Zero the first U rows (U from device) of a [cap, stride] buffer.
void launch_zero_rows(float* buf, int stride, const int32_t* n_dev, int64_t cap, hipStream_t s);
// graph-safe 32-bit fill (use instead of hipMemsetAsync in capturable code)
void launch_fill32(void* p, uint32_t v, int64_t n_words, hipStream_t s);

// IPC mesh collectives (ipc.hip): peer pointers of one node's ranks
constexpr int kIpcMaxRanks = 8;
constexpr int kIpcCountBits = 28;  // flag word count field (ipc.hip)
struct IpcPeers {
  unsigned char* inbox[kIpcMaxRanks];  // each rank's inbox [depth][2][world][slot_bytes]
  uint64_t* flags[kIpcMaxRanks];       // each rank's flag words [2][world] = epoch << kIpcCountBits | count
  int64_t slot_bytes;
  int world, rank, depth;  // depth = inbox slots (a call uses slot epoch % depth)
  int64_t spin_limit;    // s_sleep(2) polls before a wait gives up (sticky err)
  uint64_t* epoch;       // own, device
  unsigned int* arrive;  // own, device
  unsigned int* depart;  // own, device
  int* err;              // own, device: 1 = a wait timed out (sticky)
  int fence;             // 1: a system-scope release / acquire per block (always on)
};
// send / dst [world][slot_bytes]; counts (device [world], nullable = whole
// slots) of rec_bytes records go to each peer; the received records land in
// dst, rcounts (device [world], nullable) gets the received counts and
// fill_tail writes 0xFF over the rest of each dst slot
void launch_ipc_exchange(const IpcPeers& pt, const void* send, void* dst, const int32_t* counts, int64_t rec_bytes,
                         bool fill_tail, int32_t* rcounts, int blocks, hipStream_t s);
// the sharded pull's key exchange with the owner pack fused in (ipc.hip
// k_ipc_pack_exchange): uniq_h [*u_count] keys -> owners' inbox slots, send_index
// [u] = owner * cap + position, ocnt (zeroed on entry) = per-owner counts, dst
// [world][cap] keys received (tail -1), rcounts [world] received counts
void launch_ipc_pack_exchange(const IpcPeers& pt, const uint64_t* uniq_h, const int32_t* u_count, int64_t cap,
                              int64_t* send_index, int32_t* ocnt, int32_t* overflow, uint64_t* dst, int32_t* rcounts,
                              int blocks, hipStream_t s);
// the sharded pull's answer exchange with the owner probe + gather fused in
// (ipc.hip k_ipc_answer_exchange): recv [world][cap] keys of rcnt[src] valid
// each -> rows [world * cap] (-1 past the counts), answers of rec floats into
// the askers' inboxes, dst [world][cap][rec] the answers to this rank's keys
void launch_ipc_answer_exchange(const IpcPeers& pt, const TableDev& t, const uint64_t* recv, const int32_t* rcnt,
                                int64_t cap, int rec, int64_t* rows, float* dst, int blocks, hipStream_t s);
// out = scale * sum over ranks of src (n floats; out may alias src)
void launch_ipc_allreduce(const IpcPeers& pt, const float* src, float* out, int64_t n, float scale, bool two_phase,
                          int blocks, hipStream_t s);

// device-resident pass (batch_ops.hip): the record store's CSR arrays + the
// pass order on the GPU
struct BatchSrc {
  const int64_t* u64;   // uint64 slot values (as int64)
  const int64_t* uoff;  // [nrec*nu + 1]
  const float* f32;
  const int64_t* foff;  // [nrec*nf + 1]
  const int64_t* order;
  const int32_t* sparse_idx;  // [S] used-uint64 index of each sparse slot
  const int32_t* drefs;       // [ndref][4] (0=u64/1=f32, idx, dim, col)
  int nu, nf, S, ndref, Dw;
};
void launch_batch_assemble(const BatchSrc& src, int64_t begin, int B, int64_t* lod, int64_t* tot, int64_t* keys,
                           int64_t keys_cap, float* dense, int32_t* overflow, hipStream_t st);
int batch_assemble_max_slots();

// ---------------------------------------------------------------- sharding
// Unique mixed keys (sorted) -> per-owner fixed-capacity send buffer [N, C]
// (kEmptyKey padded) + send_index[u] = o*C + (u - start_o) + overflow flag.
void launch_shard_pack(const uint64_t* uniq_h, const int32_t* u_count, int64_t u_cap, int nranks,
                       int64_t cap, uint64_t* send, int64_t* send_index, int32_t* overflow,
                       hipStream_t s);
// resp[j] = pulled[uid_r[j]] for received entries (invalid -> zeros).
void launch_gather_by_uid(const float* src, int src_stride, const int32_t* uid, int64_t n,
                          float* out, int out_stride, int width, hipStream_t s);
// Owner pack after the sort-free dedup: unique keys (any order) -> per-owner
// fixed-capacity segments of send [nranks*cap] (kEmptyKey padded) and
// send_index[u]; ocnt [nranks] scratch; overflow flag is sticky.
void launch_shard_pack_hash(const uint64_t* uniq_h, const int32_t* u_count, int64_t u_cap, int nranks, int64_t cap,
                            uint64_t* send, int64_t* send_index, int32_t* ocnt, int32_t* overflow, bool prezeroed,
                            hipStream_t s);
// out[j] = pull head of table row rows[uid[j]] (zeros if uid/row < 0);
// out_stride % 4 == 0 and <= table stride.
void launch_gather_rows_by_uid(const TableDev& t, const int64_t* rows, const int32_t* uid, int64_t n, float* out,
                               int out_stride, hipStream_t s);
// Fused owner-side merge + Adagrad: unique u's records are
// rec[perm[seg[u] + j]], j < cnt[u].  Returns false if the dim/stride has no
// vectorised instantiation (caller falls back to merge + launch_push_adagrad).
bool launch_push_adagrad_seg(const TableDev& t, const int64_t* rows, const float* rec, int rec_stride,
                             const int32_t* perm, const int32_t* seg, const int32_t* cnt, const int32_t* n_dev,
                             int64_t n, const SparseSGDConfig& cfg, uint64_t seed, hipStream_t s);

// Single-shard fused push: merge the batch gradients per unique key and apply
// Adagrad in place (a.push = acc scratch [U_cap, stride], kept all-zero;
// inc [ceil(n/64)] scratch).  False if the dim/stride/layout has no fused
// instantiation (caller falls back to launch_push_merge + launch_push_adagrad).
// inc: int32 per wave (two launches: merge + k_push_finish) or, with ctr set
// (int64 per unique, zero between pushes), one fused launch (inc unused)
bool launch_push_merge_apply(const PushMergeArgs& a, const TableDev& t, const int64_t* rows, int32_t* inc,
                             unsigned long long* ctr,
                             const SparseSGDConfig& cfg, uint64_t seed, hipStream_t s);
// Sharded push: the same merge, each unique's summed record written to
// send[send_index[u]] (rows with send_index -1 dropped); a.push / a.push_stride
// = the all-zero straddle accumulator [>= U_cap rows]; no memset of send.
// No-dedup single-shard push: rows[k] = table row of occurrence k (a.n of
// them); a.push / a.push_stride = all-zero accumulator [>= kOccRep * n rows]
// (kept zero); lock = per-table-row int32 (-1 = free), lead = [n] scratch.
constexpr int kOccRep = 8;
bool launch_push_occ(const PushMergeArgs& a, const TableDev& t, const int64_t* rows, int32_t* lock, int32_t* lead,
                     const SparseSGDConfig& cfg, uint64_t seed, hipStream_t s);
// Streaming checkpoint (ckpt.hip / ckpt_saver.cpp).  mode 0 = every row
// (batch model), 1 = xbox base, 2 = xbox delta (ctr_accessor.cc:102-170).
// Output row of a save: the table row as stored (n = 0), or a decoded row of
// n floats (feature-type codec tables: the canonical fp32 layout of
// ps/feature_types.py FeatureCodec.decode) -- map[j] >= 0: stored float
// column, -1: zero, <= -2: int16 element (-2 - map[j]) of the row's
// embedding block (stored from float column 3) times scale.
constexpr int kSaveMaxCols = 1024;  // 2 KB of kernel arguments
struct SaveDecode {
  int n = 0;
  float scale = 1.f;
  int16_t map[kSaveMaxCols];
};
// Compact the selected rows of flat row range [r0, r1) (buckets then stash)
// into okeys (unmixed feasigns) / ovals (out_stride floats per row: stride,
// or dec.n when decoding) at positions atomically taken from *count; resets
// delta_score if asked.
void launch_save_chunk(const TableDev& t, int64_t r0, int64_t r1, const SaveSelect& sel, const SaveDecode& dec,
                       uint64_t* okeys, float* ovals, unsigned long long* count, hipStream_t s);
struct SaveStats {
  int64_t rows = 0;
  int64_t chunks = 0;
  double gpu_s = 0, write_s = 0, total_s = 0;
};
// Host driver: walks the table in chunks of chunk_rows row slots through two
// device buffers and pinned host buffers into writer threads.  kind 0: numpy
// batch model (keys_path .npy uint64 [N], vals_path .npy f32 [N, stride]);
// kind 1: xbox text (keys_path, "feasign\tslot unseen delta show click
// embed_w g2sum [embedx.. embedx_g2sum]", embedx only when score >=
// embedx_threshold and mf_size != 0).  saved_mixed (optional): the mixed keys
// of the saved rows are appended (for tiers that mirror the delta reset).
// dec.n > 0: rows are decoded to the canonical layout of embedding width
// out_dim (text and .npy use it).
SaveStats stream_save_table(const TableDev& t, int64_t total_rows, int kind, const SaveSelect& sel,
                            const SaveDecode& dec, int out_dim, float embedx_threshold, const std::string& keys_path,
                            const std::string& vals_path, int64_t chunk_rows, int threads,
                            std::vector<uint64_t>* saved_mixed, int device, hipStream_t s);
// Single-shard dedup through the table itself: rows_occ[i] = row of raw key
// keys[i] (-1: padding / absent), rows_u[u] = row of unique u, uid / perm /
// seg / u_count as the hash dedup (u_count = [U, n_valid, -, cursor]).
// cnt_row / uid_row: int32 per table row; cnt_row all-zero between calls
// (re-zeroed by the call), uid_row needs no reset.
void launch_table_dedup(const TableDev& t, const int64_t* keys, int64_t n, int64_t* rows_occ, int32_t* rank,
                        int32_t* cnt_row, int64_t cnt_rs, int32_t* uid_row, int64_t* rows_u, int32_t* uid,
                        int32_t* perm, int32_t* seg, int32_t* u_count, int32_t* acc, bool rows_given,
                        hipStream_t s, bool do_scatter = true, int stage = 0);
// stage: 0 = the whole dedup; 1 = the probe + rank launch only (rows_occ /
// rows_u / per-row counts ready: what the pooling needs); 2 = run starts +
// scatter only (uid / perm / u_count: what the push needs), which may then
// run on a side stream beside the pooling
// Probe raw feasigns (mixed in the kernel, -1 = padding -> row -1).
void launch_probe_raw(const TableDev& t, const int64_t* keys, int64_t n, int64_t* rows, hipStream_t s);
bool launch_push_merge_send(const PushMergeArgs& a, int dim, float* send, int send_stride, const int64_t* send_index,
                            int32_t* inc, unsigned long long* ctr, hipStream_t s);

// ---------------------------------------------------------------- dense ops
void launch_data_norm_fwd(const float* x, int N, int C, const float* bsize, const float* bsum,
                          const float* bsq, float* y, float* means, float* scales,
                          const float* scale_w, const float* bias, hipStream_t s);
void launch_data_norm_bwd(const float* x, const float* dy, int N, int C, const float* means,
                          const float* scales, float eps, float* dx, float* stats /*[3,C]*/,
                          float* acc /*[2,C] scratch*/, const float* scale_w, hipStream_t s);
void launch_data_norm_update(float* bsize, float* bsum, float* bsq, const float* stats, int C,
                             float decay, hipStream_t s);

// bf16 MFMA GEMM for the MLP (csrc/hip/gemm.hip): C[M,N] = A'[M,K] B'[K,N]
// with A'(m,k) at A[m*lda+k] (a_kcontig) or A[k*lda+m]; B'(k,n) at
// B[n*ldb+k] (b_kcontig) or B[k*ldb+n].
enum GemmEpi { EPI_BIAS_RELU_BF16 = 0, EPI_BIAS_BF16 = 1, EPI_BF16 = 2, EPI_F32_SLAB = 3 };
struct GemmArgs {
  const unsigned short* A = nullptr;
  const unsigned short* maskA = nullptr;  // relu' mask in A's layout (bf16), optional
  const unsigned short* B = nullptr;
  void* C = nullptr;
  const float* bias = nullptr;
  int M = 0, N = 0, K = 0;
  int lda = 0, ldb = 0, ldc = 0;
  bool a_kcontig = true, b_kcontig = true;
  int ones_col_b = -1;  // virtual all-ones B column at n == ones_col_b (bias grad)
  int epi = EPI_BF16;
  int k_per_split = 1 << 30;
  int64_t slab_stride = 0;
};
void launch_gemm(const GemmArgs& g, hipStream_t s);
// DCN-V2 cross head (cross.hip): s[m] = x[m, :N] . w ; and the top of its
// backward: g[m,n] = ds[m] w[n] (f32), u = bf16(x0 * g) and u^T [n][ldt],
// acc = z * g, dw[n] += sum_m ds[m] x[m,n].  x, x0, z, g, u, acc share ld.
void launch_cross_dot(const float* x, int M, int N, int ld, const float* w, float* out, hipStream_t s);
int cross_top_blocks(int M);
void launch_cross_top_bwd(const float* x, const unsigned short* x0, const float* z, const float* w, const float* ds,
                          int M, int N, int ld, float* g, unsigned short* u, unsigned short* ut, int ldt, float* acc,
                          float* part, float* dw, hipStream_t s);
void launch_slab_reduce(const float* slab, int splits, int64_t slab_stride, int M, int N, int ldc, float* dW,
                        float* db, float scale, hipStream_t s);
void launch_gemv_out(const unsigned short* h, int M, int K, int ldh, const float* w, const float* b, float* out,
                     hipStream_t s);
// out[c] += sum_r part[r, c] for c < split_col, out2[c - split_col] += ... otherwise
void launch_colsum_acc(const float* part, int R, int W, float* out, int split_col, float* out2, hipStream_t s);
int gemv_out_bwd_blocks(int M);
// part: scratch [gemv_out_bwd_blocks(M), K+1] f32 (per-block partial sums)
void launch_gemv_out_bwd(const unsigned short* h, int M, int K, int ldh, const float* w, const float* dout,
                         unsigned short* dh, float* dw, float* db, float* part, hipStream_t s);
void launch_f32_to_bf16(const float* x, unsigned short* y, int64_t n, hipStream_t s);

// Fused data_norm + first-order + FM head (csrc/hip/head_ops.hip).
struct HeadArgs {
  const float* x = nullptr;  // [B, C] fp32 (pooled slot blocks | dense)
  int B = 0, C = 0, Cp = 0;  // Cp = C padded to a multiple of 8 (GEMM K)
  int S = 0, Eo = 11, ew_col = 2, D = 8;
  const float* bsize = nullptr;  // data_norm summaries (null = no data_norm)
  const float* bsum = nullptr;
  const float* bsq = nullptr;
  float* means = nullptr;   // [C] out (fwd)
  float* scales = nullptr;  // [C] out (fwd) / in (bwd)
  unsigned short* y = nullptr;  // [B, ldy] bf16 out (fwd), columns >= Cp untouched
  int ldy = 0;                  // row stride of y / dy (0 = Cp)
  unsigned short* yT = nullptr; // optional [Cp][ldyt] transposed copy of y (fwd)
  int ldyt = 0;
  float* lin = nullptr;         // [B] first + FM out (fwd)
  const unsigned short* dy = nullptr;  // [B, ldy] bf16 in (bwd)
  const float* dlin = nullptr;         // [B] in (bwd), nullable (= 0)
  const float* dlin_scale = nullptr;   // optional device scalar multiplying dlin (bwd)
  float* dx = nullptr;                 // [B, C] out (bwd)
  float* stat_acc = nullptr;           // [head_blocks(B), 2C] per-block partial sums (bwd)
  unsigned short* ymp = nullptr;       // optional m-packed copy of y (fwd; Cp % 32 == 0, B rows padded to 16)
  float* stat_part = nullptr;          // optional [head_blocks(B), 2C] batch-stat partials computed in fwd
  // fp32 MLP input (the fp32 tower): used instead of y / ymp / dy when set
  float* yf = nullptr;         // [B, ldy] fp32 out (fwd)
  float* ympf = nullptr;       // MP32 copy of y (fwd; Cp % 16 == 0)
  const float* dyf = nullptr;  // [B, ldy] fp32 in (bwd)
};
size_t head_lds_bytes(int C, int D, int Cp);
int head_blocks(int B);
void launch_head_fwd(const HeadArgs& a, hipStream_t s);
void launch_head_bwd(const HeadArgs& a, hipStream_t s);
// acc: scratch [2C]
void launch_dn_stats(const float* part, int nrows, int C, int N, float eps, float* stats, float* acc,
                     hipStream_t s);

// DeepFM second-order FM over S fields of dim D read from x[b, col0 + s*fstride + d].
void launch_fm_fwd(const float* x, int B, int S, int D, int row_stride, int col0, int fstride,
                   float* out, hipStream_t s);
void launch_fm_bwd(const float* x, const float* dout, int B, int S, int D, int row_stride,
                   int col0, int fstride, float* dx, int dx_stride, int accumulate, hipStream_t s);

// Fused sigmoid + log-loss (+ grad of mean loss).
void launch_sigmoid_logloss(const float* logit, const float* label, int B, float* pred,
                            float* loss_sum, float* dlogit, float grad_scale, hipStream_t s);

// z = a + b (b nullable); pred = sigmoid(z), dz = (pred - y)/B, loss_mean = mean BCE.
// ws: caller-owned uint32 [1 + kLogitLossMaxBlocks], zero before the first
// launch (the kernel re-arms it); one workspace per stream
constexpr int kLogitLossMaxBlocks = 1024;
void launch_logit_loss(const float* a, const float* b, const float* label, int B, float* pred, float* dz,
                       float* loss_mean, uint32_t* ws, hipStream_t s);

// Streaming AUC histogram: table[label][bucket] += 1 and error sums
// (stats: [abserr, sqrerr, pred_sum, label_sum, count]) in double.
void launch_auc_accumulate(const float* pred, const float* label, const float* mask, int B,
                           int nbuckets, double* table /*[2,nbuckets]*/, double* stats,
                           hipStream_t s);

// Flat Adam over a contiguous fp32 buffer; pows = device [beta1^t, beta2^t]
// (advanced in-stream, graph-replayable).
void launch_adam_flat(float* p, float* g, float* m, float* v, int64_t n, float lr, float b1,
                      float b2, float eps, float* pows, float grad_scale, float weight_decay,
                      bool clear_grad, hipStream_t s);

// ---------------------------------------------------------------- fused MLP engine (mlp.hip)
enum MlpEpi {
  MLP_EPI_FWD = 0,
  MLP_EPI_DX = 1,
  MLP_EPI_DW = 2,
  // DCN-V2 cross layer x_{l+1} = x0 * (x_l W^T + b) + x_l: fout = x_{l+1},
  // zout = z_l (f32 [M][ldf]); C / CT = bf16 x_{l+1} and its transpose
  MLP_EPI_CROSS_FWD = 3,
  // cross backward: g_l = acc + gin.  With zprev (layer l > 0): fout = g_l,
  // accum += zprev * g_l, C / CT = bf16(x0 * g_l) (= u_{l-1});
  // without (layer 0): C = bf16(g_l + accum), the gradient of x0
  MLP_EPI_CROSS_DX = 4
};
struct MlpGemmArgs {
  const unsigned short* A = nullptr;  // [M rows][lda] k-contiguous bf16
  const unsigned short* B = nullptr;  // [N rows][ldb] k-contiguous bf16
  int lda = 0, ldb = 0;
  int M = 0, N = 0, K = 0;  // K: multiple of 64, zero padded in both operands
  int k_per_split = 1 << 30;
  // FWD / DX
  unsigned short* C = nullptr;  // [M][ldc]
  int ldc = 0;
  unsigned short* CT = nullptr;  // optional transposed copy [ncols_valid][ldct]
  int ldct = 0;
  int ncols_valid = 0;  // FWD/DX: real output width (bias / CT rows); DW: real K (col == it -> db)
  int nrows_valid = 0;  // DW: real N of dW
  const float* bias = nullptr;
  int relu = 0;
  const unsigned short* mask = nullptr;  // DX: [M][ldmask], zero the output where mask <= 0
  int ldmask = 0;
  // DW
  float* dW = nullptr;  // [nrows_valid][lddw] fp32 (atomic accumulate)
  int lddw = 0;
  float* db = nullptr;
  // CROSS_FWD / CROSS_DX (x0 bf16 [M][ldx0]; f32 buffers [M][ldf])
  const unsigned short* x0 = nullptr;
  int ldx0 = 0;
  const float* xin = nullptr;
  const float* gin = nullptr;
  const float* zprev = nullptr;
  float* fout = nullptr;
  float* zout = nullptr;
  float* accum = nullptr;
  int ldf = 0;
  int add_c = 0;  // CROSS_DX layer 0: C += (the gradient of x0 is added to C's bf16 contents)
};
void launch_mlp_gemm(const MlpGemmArgs& g, int epi, hipStream_t s);
constexpr int kMaxMlpLayers = 8;
struct CastWtBatch {  // all layers' fp32 -> bf16 (W, W^T) casts in one launch
  const float* w[kMaxMlpLayers];
  unsigned short* wb[kMaxMlpLayers];
  unsigned short* wtb[kMaxMlpLayers];
  int N[kMaxMlpLayers], K[kMaxMlpLayers], pN[kMaxMlpLayers], pK[kMaxMlpLayers];
  int tile_off[kMaxMlpLayers + 1];  // prefix sum of 32x32 tiles per layer
  int n = 0;
};
void launch_cast_wt(const CastWtBatch& c, hipStream_t s);
// DCN-V2 cross stack forward fused into one launch (tower.hip k_cross_fwd):
// per 32-row tile x_0 and x_l stay in LDS (bf16 MFMA operand + fp32
// residual) across all L layers, the packed bf16 weights stream from L2
// (tower wp layout, Np = pad32(D), Kp = pad16(D)), and only what the
// backward reads goes to HBM: z_l (f32), m-packed x_l (bf16, the dW GEMM
// operand), x_L (f32) and s = x_L . w_c.  Same epilogue as MLP_EPI_CROSS_FWD.
struct CrossFwdArgs {
  const unsigned short* x0 = nullptr;  // [M][ldx0] bf16
  int ldx0 = 0;
  const unsigned short* wp[kMaxMlpLayers] = {};
  const float* bias[kMaxMlpLayers] = {};
  float* z[kMaxMlpLayers] = {};            // [M][ldf]
  unsigned short* xmp[kMaxMlpLayers] = {};  // m-packed x_l, l < L (tower MP layout, NB = Np/32): dW B operand
  float* xlast = nullptr;  // [M][ldf]
  int ldf = 0;
  const float* wc = nullptr;
  float* s = nullptr;  // [M]
  int M = 0, D = 0, L = 0, Np = 0, Kp = 0;
};
size_t cross_fwd_lds_bytes(int Np, int Kp);  // 0 if the tile does not fit in LDS
void launch_cross_fwd(const CrossFwdArgs& a, hipStream_t s);
// fp32 W_l [D][D] -> packed bf16 W_l (tower wp layout, Kp) and, when wtp is
// given, packed W_l^T (tower wtp layout, Np = pad32(D)); pad entries untouched
void launch_cross_pack(const float* const* w, unsigned short* const* wp, unsigned short* const* wtp, int L, int D,
                       int Kp, int Np, hipStream_t s);
// DCN-V2 cross backward chain fused into one launch (tower.hip k_cross_bwd):
// per 32-row tile g (f32), the dx_0 accumulator (f32) and u = bf16(x_0 * g)
// stay in LDS across the layers; top (g_L = ds w_c), dX chain
// g_l = u_l W_l + g_{l+1}, dx_0 = g_0 + sum_l z_l * g_{l+1} -> dy (bf16),
// m-packed u_l for the grouped dW launch (k_tower_dw over the cross layers)
// and per-tile db / dw_c partials.  Same math as k_cross_top_bwd +
// MLP_EPI_CROSS_DX.
struct CrossBwdArgs {
  const unsigned short* x0 = nullptr;  // [M][ldx0] bf16
  int ldx0 = 0;
  const unsigned short* wtp[kMaxMlpLayers] = {};
  const float* z[kMaxMlpLayers] = {};  // [M][ldf]
  const float* xlast = nullptr;        // x_L [M][ldf]
  int ldf = 0;
  const float* ds = nullptr;  // [M]
  const float* ds_scale = nullptr;  // scalar multiplier of ds (the upstream loss grad; nullable = 1)
  const float* wc = nullptr;  // [D]
  unsigned short* ump[kMaxMlpLayers] = {};  // m-packed u_l (dW GEMM A operand)
  unsigned short* dy = nullptr;  // [M][ldy]
  int ldy = 0, add_dy = 0;
  // per-tile column partials [Mp/32][bias_ld]: db_l at l*Np (sum of u_l),
  // dw_c at L*Np (sum of ds x_L) -- reduced by the grouped dW launch
  float* bias_part = nullptr;
  int bias_ld = 0;
  int M = 0, D = 0, L = 0, Np = 0;
};
void launch_cross_bwd(const CrossBwdArgs& a, hipStream_t s);
int cross_bwd_blocks(int M);
void launch_mlp_gemv_fwd(const unsigned short* h, int M, int K, int ld, const float* w, const float* b, float* out,
                         hipStream_t s);
int mlp_gemv_bwd_blocks(int M);
void launch_mlp_gemv_bwd(const unsigned short* h, int M, int K, int ld, const float* w, const float* dout,
                         unsigned short* dz, unsigned short* dzt, int ldt, float* part, float* dw, float* db,
                         hipStream_t s);

// ---------------------------------------------------------------- fused dense tower (tower.hip)
// Whole CTR MLP (ReLU layers + 1-logit output + sigmoid/log-loss + AUC) as
// three launches: a row-tile-resident forward, a row-tile-resident backward
// (dX chain) and one grouped dW GEMM (+ bias / data_norm column reductions).
//
// Layouts (all bf16 = unsigned short; dims padded to multiples of 32, Mp =
// pad32(M)):
//  * "MP" (m-packed) activations Z[M][N]: 1 KB chunks [Mp/16][Np/32][64][8];
//    lane l, element j of chunk (mb, nb) = Z[16mb + 8(l/32) + j][32nb + l%32]
//    -- exactly the MFMA 32x32x16 operand fragment with m as the reduction
//    dim, so the dW GEMM streams both operands 1 KB at a time.
//  * packed W  [Np/32][Kp/16][64][8]: lane l, j = W[32nb + l%32][16kb + 8(l/32) + j]
//  * packed Wt [Kp/32][Np/16][64][8]: lane l, j = W[16nb + 8(l/32) + j][32kb + l%32]
constexpr int kMaxTowerLayers = 8;
struct TowerLayerDev {
  const unsigned short* wp = nullptr;   // packed W
  const unsigned short* wtp = nullptr;  // packed W^T
  const float* bias = nullptr;          // [N]
  int K = 0, N = 0, Kp = 0, Np = 0;
  unsigned short* xmp = nullptr;   // MP of this layer's output X_{l+1}
  unsigned short* dzmp = nullptr;  // MP of dZ_{l+1}
  float* dw = nullptr;             // [N][K] fp32 grad (accumulated)
  float* db = nullptr;             // [N]
  int bias_off = 0;                // column of this layer's db partials in a bias_part row
  // fp32 tower (tower32.hip): packed fp32 weights and fp32 MP32 activations
  const float* wpf = nullptr;   // packed W  [Np/16][Kp/16][64][4]
  const float* wtpf = nullptr;  // packed W^T [Kp/16][Np/16][64][4]
  float* xmpf = nullptr;        // MP32 of X_{l+1}
  float* dzmpf = nullptr;       // MP32 of dZ_{l+1}
};
struct TowerArgs {
  int M = 0, Mp = 0, L = 0;
  int lds_ld = 0;  // LDS row stride in elements (max padded width + 8)
  int t32_part = 0;  // fp32 tower: LDS scratch of the wave-stream remainder partials present (set by the launcher)
  const unsigned short* x0 = nullptr;  // row-major input [M][ld0] (>= Kp_0 cols, pad cols 0)
  int ld0 = 0;
  const unsigned short* x0mp = nullptr;  // MP(X0)
  TowerLayerDev ly[kMaxTowerLayers];
  const float* w_out = nullptr;  // [N_L]
  const float* b_out = nullptr;  // [1]
  const float* lin = nullptr;    // [M] extra logit part (first-order + FM), nullable
  const float* label = nullptr;  // [M], element m at label[m * label_stride]
  int label_stride = 1;          // a label column of the batch's dense block (no copy)
  float* pred = nullptr;         // [M]
  float* dz = nullptr;           // [M] d(mean loss)/d logit
  float* loss = nullptr;         // [1] mean loss
  float* part = nullptr;         // [nwg][8] per-WG partials (loss, 5 AUC sums)
  unsigned int* ticket = nullptr;  // zero between launches
  double* auc_table = nullptr;   // [2, auc_buckets] (nullable = no AUC)
  double* auc_stats = nullptr;   // [5]
  int auc_buckets = 0;
  const float* auc_mask = nullptr;
  // backward
  const float* dloss = nullptr;  // scalar upstream grad of the loss (nullable = 1)
  unsigned short* dx0 = nullptr;  // row-major [M][lddx0] grad wrt X0
  int lddx0 = 0;
  int need_dx0 = 1;
  float* bias_part = nullptr;  // [nwg][bias_ld]: db partials per layer, dw_out, db_out
  int bias_ld = 0, dwout_off = 0, dbout_off = 0;
  float* dw_out = nullptr;
  float* db_out = nullptr;
  // data_norm batch statistics, reduced by the dW launch: part [dn_rows][2C]
  // (sum x, sum (x-mean)^2) -> stats [3][C] (1, sum/N, sq/N + eps)
  const float* dn_part = nullptr;
  int dn_rows = 0, dn_C = 0;
  float dn_eps = 0.f;
  float* dn_stats = nullptr;
  // optional: the summaries updated in place from those stats by the same
  // workgroup (bsize = bsize * decay + 1, ...), instead of a k_dn_update launch
  float* dn_bsize = nullptr;
  float* dn_bsum = nullptr;
  float* dn_bsq = nullptr;
  float dn_decay = 1.f;
  int dw_splits = 2;
  // fp32 dW split-M partials, reduced in split order (no float atomics: the
  // update is bit-reproducible): slab [tiles][dw_splits][64 x 64] and one
  // arrival counter per 64x64 output tile (zero between launches)
  float* dw_slab = nullptr;
  int* dw_cnt = nullptr;
  int debug = 0;  // timing experiments only (PBX_TOWER_DEBUG): 1 no loss reduction, 2 no dW reductions, 4 no dW GEMM,
                  // 8 no fwd m-packed stores (fp32: no MP32 stores in the fwd / bwd layer epilogues), 16 no output layer / loss, 32 fp32 tower: no s_setprio on waves 4-7,
                  // 64 fp32 fwd/bwd: no weight loads in the k-loop, 256 fp32 fwd/bwd: plain (not
                  // non-temporal) MP32 stores / loads
  // fp32 tower (f32 = 1): fp32 X0 row-major / MP32, fp32 dX0; widths padded to 16
  int f32 = 0;
  long long* stamps = nullptr;  // timing experiments only: per-wave s_memtime stamps (fp32 fwd)
  const float* x0f = nullptr;
  const float* x0mpf = nullptr;
  float* dx0f = nullptr;
  // x3 tower: the DeepFM head backward fused into the dX0 epilogue (k_head_bwd
  // semantics): hdx[m][c] = dX0[m][c] * hscales[c] (+ d lin terms of the
  // first-order / FM columns when hlin); hx: the head input rows [M][hC]
  const float* hx = nullptr;
  float* hdx = nullptr;
  const float* hscales = nullptr;
  int hC = 0, hS = 0, hEo = 0, hew = 0, hD = 0, hlin = 0;
  int x3_rot = 5;  // x3 tower: k-step rotation multiplier per workgroup (start = blockIdx * x3_rot mod KS)
};
int tower_nwg(int M);
size_t tower_lds_bytes(const TowerArgs& a);
void launch_tower_fwd(const TowerArgs& a, hipStream_t s);
void launch_tower_bwd(const TowerArgs& a, hipStream_t s);
void launch_tower_dw(const TowerArgs& a, hipStream_t s);
// fp32 [N][K] -> packed W / W^T (pads zero), all layers in one launch
void launch_tower_pack(const TowerArgs& a, const float* const* w, hipStream_t s);

// fp32 tower (tower32.hip): the same three launches on v_mfma_f32_16x16x4_f32
// (exact fp32, the reference fc precision).  Layouts (floats, widths padded
// to 16, Mp a multiple of 256):
//  * MP32 activations Z[M][N]: 1 KB chunks [Mp/16][Np/16][64][4]; lane l,
//    element t of chunk (mb, nb) = Z[16mb + 4(l/16) + t][16nb + l%16] -- the
//    16x16x4 accumulator layout, and the operand fragment of the dW GEMM
//  * packed W  [Np/16][Kp/16][64][4]: lane l, t = W[16nb + l%16][16kb + 4(l/16) + t]
//  * packed Wt [Kp/16][Np/16][64][4]: lane l, t = W[16nb + 4(l/16) + t][16kb + l%16]
constexpr int kTower32MaxWidth = 512;
constexpr size_t kTower32LdsTotal = 160 * 1024;  // LDS per CU
constexpr size_t kTower32BwdStatic = 8704;       // k_t32_bwd's static LDS (gs + csum), rounded up
int tower32_lds_ld(int maxw);
size_t tower32_lds_bytes(const TowerArgs& a);
size_t tower32_lds_bytes_for(int lds_ld, bool part, int bias_floats);
void launch_tower32_fwd(const TowerArgs& a, hipStream_t s);
void launch_tower32_bwd(const TowerArgs& a, hipStream_t s);
void launch_tower32_dw(const TowerArgs& a, hipStream_t s);
void launch_tower32_pack(const TowerArgs& a, const float* const* w, hipStream_t s);

// fp32-precision tower on bf16 MFMA (tower_x3.hip): the bf16 tower's layouts
// with a lo twin after every bf16 buffer (packed W / W^T: + Np Kp; MP
// activations / dZ: + Mp Np; MP(X0): + Mp K0p), fp32 X0 rows in (x0f), fp32
// dX0 rows out (dx0f); 4 LDS planes of 32 x lds_ld bf16
size_t tower_x3_lds_bytes(int lds_ld);
void launch_tower_x3_fwd(const TowerArgs& a, hipStream_t s);
void launch_tower_x3_bwd(const TowerArgs& a, hipStream_t s);
void launch_tower_x3_dw(const TowerArgs& a, hipStream_t s);
void launch_tower_x3_pack(const TowerArgs& a, const float* const* w, hipStream_t s);

// Flat Adam with fused extras: beta powers advanced by the last workgroup
// (ticket), weight regions re-packed to bf16 tower layouts, data_norm
// summaries updated from their batch statistics.
constexpr int kMaxPackRegions = 8;
constexpr int kMaxDnUpdates = 4;
struct AdamExtras {
  int n_pack = 0;
  int64_t pack_off[kMaxPackRegions];  // arena element offset of W [N][K]
  int pack_N[kMaxPackRegions], pack_K[kMaxPackRegions], pack_Np[kMaxPackRegions], pack_Kp[kMaxPackRegions];
  unsigned short* pack_wp[kMaxPackRegions];
  unsigned short* pack_wtp[kMaxPackRegions];
  float* pack_wp32[kMaxPackRegions];   // fp32 tower regions (pack_wp / pack_wtp null)
  float* pack_wtp32[kMaxPackRegions];
  // fp32: group position tables [Np/16][Kp/16] and [Kp/16][Np/16] (tower_wp32_index_pos)
  const int* pack_pos32[kMaxPackRegions];
  const int* pack_posT32[kMaxPackRegions];
  // x3 tower regions: the bf16 copies also get their lo halves, Np Kp after
  int pack_x3[kMaxPackRegions] = {};
  int n_dn = 0;
  const float* dn_stats[kMaxDnUpdates];
  float* dn_bsize[kMaxDnUpdates];
  float* dn_bsum[kMaxDnUpdates];
  float* dn_bsq[kMaxDnUpdates];
  int dn_C[kMaxDnUpdates];
  float dn_decay[kMaxDnUpdates];
  unsigned int* ticket = nullptr;
};
void launch_adam_fused(float* p, float* g, float* m, float* v, int64_t n, float lr, float b1, float b2, float eps,
                       float* pows, float grad_scale, float weight_decay, bool clear_grad, const AdamExtras& x,
                       hipStream_t s);

// ---------------------------------------------------------------- CTR op family (ctr_ext.hip)
// C[b](m, n) = alpha * sum_k A[b](m, k) B[b](k, n) (+ bias[b][n] * bias_scale)
// (+ C_old when accumulate); A(m,k) = A[b*sA + m*rsA + k*csA], B(k,n) =
// B[b*sB + k*rsB + n*csB], C row-major with ldc.  fp32 throughout.
struct SgemmArgs {
  const float* A = nullptr;
  const float* B = nullptr;
  float* C = nullptr;
  const float* bias = nullptr;
  int M = 0, N = 0, K = 0, batch = 1;
  int64_t sA = 0, rsA = 0, csA = 0;
  int64_t sB = 0, rsB = 0, csB = 0;
  int64_t sC = 0, ldc = 0, sBias = 0;
  float bias_scale = 1.f, alpha = 1.f;
  int accumulate = 0;
  int ksplit = 1;  // set by launch_sgemm: K slices per output tile (fp32 atomics)
};
void launch_sgemm(const SgemmArgs& g, hipStream_t s);
// batch_fc with every slot's fc at most 64 x 64 (the CTR shapes): one block
// per (slot, run of 64-row tiles) keeps W_p in LDS and streams x / dy tiles
// through it.  Operands are (slot stride, row stride) with unit columns:
// x, dx (sx, rx); W, dW (sw, rw); y, dy (sy, ry); b, db (sb).  The backward
// computes dx, dW and db from one read of x and dy: every block writes its
// dW / db partial to ws ([P][G][64*64 + 64], G = batch_fc_bwd_groups) and an
// ordered second pass sums them (deterministic, no atomics).  Both return
// false when the shapes or alignment do not fit (the caller runs the generic
// k_mgemm path).
struct BfcArgs {
  const float* x = nullptr;
  const float* W = nullptr;
  const float* b = nullptr;
  float* y = nullptr;
  const float* dy = nullptr;
  float* dx = nullptr;
  float* dW = nullptr;
  float* db = nullptr;
  int P = 0, N = 0, I = 0, O = 0;
  int64_t sx = 0, rx = 0, sw = 0, rw = 0, sy = 0, ry = 0, sb = 0;
  float* ws = nullptr;  // backward partials, batch_fc_bwd_groups(P, N) * P * kBfcPart floats
  int tiles = 1;        // 64-row tiles per block (set by the launcher)
};
constexpr int kBfcPart = 64 * 64 + 64;
// 64-row tiles per block: about `blocks` blocks over the launch
inline int batch_fc_tiles(int P, int N, int blocks) {
  const int ntile = (N + 63) / 64;
  const int want = blocks / (P > 0 ? P : 1) > 0 ? blocks / (P > 0 ? P : 1) : 1;
  const int t = (ntile + want - 1) / want;
  return t > 0 ? t : 1;
}
inline int batch_fc_bwd_groups(int P, int N) {
  const int tiles = batch_fc_tiles(P, N, 768);
  return ((N + 63) / 64 + tiles - 1) / tiles;
}
bool launch_batch_fc_fwd(const BfcArgs& a, hipStream_t s);
bool launch_batch_fc_bwd(const BfcArgs& a, hipStream_t s);
// scaled_fc's fp16 GEMMs with the reference's rounding points
// (scaled_fc_op.cu:144-330): operands a_scale * A, b_scale * B rounded to
// fp16, fp32-accumulated MFMA (v_mfma_f32_16x16x32_f16), then
//   v = fp16(alpha16 * acc); if bias: v = fp16(v + fp16(fp16(bias) * bs16));
//   C = float(v) * out_scale, inf -> NaN
// (alpha16 / bs16 = the fp16 values of alpha / bias_scale).  Split-K adds
// fp32 partials into the zeroed scratch ws (M x N per batch) and a second
// pass applies the fp16 epilogue.
struct HgemmArgs {
  const float* A = nullptr;
  const float* B = nullptr;
  float* C = nullptr;
  const float* bias = nullptr;
  float* ws = nullptr;
  int M = 0, N = 0, K = 0;
  int64_t rsA = 0, csA = 0, rsB = 0, csB = 0, ldc = 0;
  float a_scale = 1.f, b_scale = 1.f, alpha = 1.f, bias_scale = 1.f, out_scale = 1.f;
  int ksplit = 1;
};
// scaled_fc's fp16 epilogue over an fp32 accumulator [M][N] (library GEMM path); out may alias acc
// scaled_fc fused fp16 GEMM: out = h16_epi(fp16(A * a_scale) @ Bk^T), Bk fp16 [Nd][Kd]
// (false: Kd % 8 != 0 or misaligned operands -- the caller takes the library path)
bool launch_sfc(const float* A, const void* Bk_, int M, int Nd, int Kd, float a_scale, const float* bias,
                float alpha, float bias_scale, float out_scale, float* out, hipStream_t s);
void launch_h16_epi(const float* acc, const float* bias, int M, int N, float alpha, float bias_scale, float out_scale,
                    float* out, hipStream_t s);
void launch_hgemm(const HgemmArgs& g, hipStream_t s);
// scaled_fc weight + bias gradient in one launch (k_sfc_dw): dW [K][O] =
// h16_epi(fp16(x * a_scale)^T fp16(d * b_scale)) over n < N, db [O] = colsum(d)
// (db may be null).  80 x 80 tiles split S ways over n (chunk rows each, a
// multiple of 64); slab: ntk * nto * S * 6400 + nto * S * 80 floats; cnt:
// ntk * nto zeroed ints, left zeroed by the launch.  (false: K or O not a
// multiple of 4, or operands not 16-B aligned -- the caller takes k_hgemm.)
struct SfcDwArgs {
  const float* x = nullptr;
  const float* d = nullptr;
  float* dW = nullptr;
  float* db = nullptr;
  float* slab = nullptr;
  float* db_slab = nullptr;
  int* cnt = nullptr;
  int N = 0, K = 0, O = 0;
  int64_t ldx = 0, ldd = 0;
  int ntk = 0, nto = 0, S = 1, chunk = 0;
  float a_scale = 1.f, b_scale = 1.f, alpha = 1.f, out_scale = 1.f;
  int mode = 0;  // 0: scaled_fc fp16 chain; 1: fp32 as three bf16 products (scales / epilogue unused)
};
inline int sfc_dw_tiles(int K, int O) { return ((K + 79) / 80) * ((O + 79) / 80); }
inline int sfc_dw_chunk(int N, int S) { return ((N + S - 1) / S + 63) / 64 * 64; }
bool launch_sfc_dw(const SfcDwArgs& a, hipStream_t s);
// out [M][Nd] = A [M][Kd] fp32 @ (Bh + Bl)^T with B's bf16 split [Nd][Kd] (k_f3gemm_nt:
// three bf16 MFMA products, fp32 accumulate; false: Kd % 8 != 0 or misaligned operands)
bool launch_f3gemm_nt(const float* A, const void* Bh, const void* Bl, int M, int Nd, int Kd, float* out,
                      hipStream_t s);
void launch_colsum_strided(const float* x, int batch, int M, int N, int64_t sb, int64_t ld, float* out, int64_t so,
                           bool accumulate, hipStream_t s);
void launch_i8_quant(const float* x, int R, int C, int ldo, float expand, float clip, float range, bool transpose,
                     signed char* out, hipStream_t s);
void launch_i8_gemm(const signed char* qx, const signed char* qwt, int M, int N, int Kp, float scale,
                    const float* bias, float* y, int ldy, hipStream_t s);
// rank_attention, rank-bucketed (ctr_ext.hip): the forward counting-sorts the
// instances by rank into `bucket` (rank_attention_bucket_ints(B, R) ints:
// permutation + tile table), which the backward reuses.
int rank_attention_bucket_ints(int B, int R);
void launch_rank_attention_fwd(const float* x, const int* ro, int ld, const float* W, int B, int C, int P, int R,
                               int* bucket, float* out, hipStream_t s);
// dexp: scratch [B][R][C] (the G rows); dx overwritten; dW accumulated (atomics: zero it first)
void launch_rank_attention_bwd(const float* x, const float* dout, const int* ro, int ld, const float* W, int B, int C,
                               int P, int R, const int* bucket, float* dexp, float* dx, float* dW, hipStream_t s);
void launch_cvm_fwd(const float* x, int64_t n, int W, bool use_cvm, float* y, hipStream_t s);
void launch_cvm_bwd(const float* dy, const float* cvm, int64_t n, int W, bool use_cvm, int cvm_rows, float* dx,
                    hipStream_t s);
int mdn_blocks(int N);
void launch_masked_dn_fwd(const float* x, const float* mask, int N, int C, const float* bsize, const float* bsum,
                          const float* bsq, const float* sw, const float* bias, float* y, float* part /*[blocks][3][C]*/,
                          hipStream_t s);
void launch_masked_dn_bwd(const float* x, const float* dy, const float* mask, int N, int C, const float* bsize,
                          const float* bsum, const float* bsq, const float* sw, float* dx,
                          float* part /*[blocks][2][C] or null*/, hipStream_t s);
void launch_mdn_stats(const float* part, int rows, int C, float eps, float* stats, hipStream_t s);
int cnh_blocks(int B);
void launch_cnh_fwd(const float* x, int B, int F, int E, const float* summary, float* y, float* part /*[blocks][2][W]*/,
                    hipStream_t s);
void launch_cnh_bwd(const float* x, const float* dy, int B, int F, int E, const float* summary, float* dx,
                    hipStream_t s);
struct ColAffine {
  float mul[4] = {1.f, 1.f, 1.f, 1.f};
  float add[4] = {0.f, 0.f, 0.f, 0.f};
};
void launch_colsum_rows(const float* part, int rows, int Q, int C, const ColAffine& f, float* out, hipStream_t s);

// ---------------------------------------------------------------- feature types
// Row codec of the GPU PS (feature_ops.hip): kind 0 fp32 Adagrad, 1 int16
// embedx/expand Adagrad, 2 fp32 SparseAdam; De = expand (NNCross) columns.
struct CodecDev {
  int kind = 0;
  int D = 8, De = 0;
  int Wx = 8, We = 0;  // storage words of embedx / expand
  float qscale = 1.f;
  float beta1 = 0.9f, beta2 = 0.999f, eps = 1e-8f;
  int g2 = 0, xg2 = 0, delta = 0, slot = 0, unseen = 0, mf = 0;
  int eg2 = 0;   // expand g2sum (Adagrad, De > 0)
  int adam = 0;  // first SparseAdam state word
  int xsz = 0;   // kind 3: the row's embedding size (0, D or De) as a float
  int extra = 0;  // floats after the standard tail
  // kind 3: bitmap over slot ids of the slots whose features are created
  // with De columns (the slots pulled into an expand output)
  const uint32_t* vslots = nullptr;
  int vslot_bits = 0;
};
// fills storage widths and field offsets for (kind, D, De)
inline CodecDev make_codec(int kind, int D, int De, float qscale, float beta1, float beta2, float eps) {
  CodecDev c;
  c.kind = kind;
  c.D = D;
  c.De = De;
  // kind 3 (variable): one block of max(D, De) columns, the first `size` live
  c.Wx = kind == 1 ? (D + 1) / 2 : (kind == 3 ? (D > De ? D : De) : D);
  c.We = kind == 1 ? (De + 1) / 2 : (kind == 3 ? 0 : De);
  c.qscale = qscale;
  c.beta1 = beta1;
  c.beta2 = beta2;
  c.eps = eps;
  const RowLayout l = make_row_layout(c.Wx + c.We);
  c.g2 = l.embed_g2sum;
  c.xg2 = l.embedx_g2sum;
  c.delta = l.delta_score;
  c.slot = l.slot;
  c.unseen = l.unseen_days;
  c.mf = l.mf_size;
  int used = l.mf_size + 1;
  c.eg2 = used;
  if (De > 0 && kind != 3) used += 1;
  c.xsz = used;
  if (kind == 3) used += 1;
  c.adam = used;
  if (kind == 2) used += 6 + 2 * (D + De);
  c.extra = used - (l.mf_size + 1);
  return c;
}
void launch_codec_pull(const TableDev& t, const CodecDev& c, const int64_t* rows, const int32_t* uid,
                       const int32_t* n_dev, int64_t n, float* out, int out_stride, hipStream_t s);
void launch_codec_update(const TableDev& t, const CodecDev& c, const int64_t* rows, const float* push,
                         int push_stride, const int32_t* n_dev, int64_t n, const SparseSGDConfig& cfg, uint64_t seed,
                         hipStream_t s);
void launch_codec_init(const TableDev& t, const CodecDev& c, const int64_t* rows, const uint64_t* keys, int64_t n,
                       const SparseSGDConfig& cfg, uint64_t seed, int init_embedx, hipStream_t s);

// fused_seqpool_cvm variant family (seqpool_variants.hip).  The per-variant
// CVM epilogue and its gradient are column tables built on the host:
//   ftab[c]  (op << 24) | (s1 << 12) | s2, op: 0 copy p[s1], 1 log(p[s1]+1),
//            2 log(p[s1]+1) - log(p[s2]+1)
//   btab[e]  (op << 24) | idx, op: 0 zero, 1 cvm[b][idx], 2 qv[b][idx], 3 dout[idx]
struct SpvArgs {
  const float* x = nullptr;  // records [L_total][E]
  int E = 0;
  const int* row_base = nullptr;  // [S] first record of slot s
  const int* off = nullptr;       // [S][B+1] instance offsets within the slot
  int S = 0, B = 0;
  int need_filter = 0;
  float show_coeff = 0.f, clk_coeff = 1.f;
  const float* thr = nullptr;  // [S] show/click threshold per slot
  int embed_filter = 0;
  float embed_threshold = 0.f;
  int ets = 0;  // width of the embedding scored by the embed filter
  int co = 2;
  int quant = 0, mcol = 2;
  int tradew = 0, tn = 0, tid = -1;
  int ecs = 1;
  float pad = 0.f;
  int Epool = 0, Eo = 0;
  const int* ftab = nullptr;
  const int* btab = nullptr;
  float* out = nullptr;  // [S][B][ecs*Eo]
  const float* dout = nullptr;
  const float* cvm = nullptr;
  int ncv = 0;
  const float* qv = nullptr;
  int nq = 0;
  float* dx = nullptr;  // [L_total][E]
};
void launch_spv_fwd(const SpvArgs& a, hipStream_t s);
void launch_spv_bwd(const SpvArgs& a, hipStream_t s);
// fused_seq_tensor: x [ins][bc][S][T][E], ad [ins][bc][A][E] -> din
// [bc][ins][T][4][A][E], mask [bc][ins][T], side [bc][ins][T][S-A][E],
// sess [bc][ins][T][A][E]
void launch_fused_seq_tensor(const float* x, const float* ad, int ins, int bc, int T, int E, int S, int A,
                             int ad_off, float* din, float* mask, float* side, float* sess, hipStream_t s);

}  // namespace pbx

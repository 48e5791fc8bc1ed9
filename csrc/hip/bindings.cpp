// torch-facing glue for the gfx950 kernels (module paddlebox_amd._pbx_hip).
// Everything here is shape checking + pointer plumbing; no compute.
#include <ATen/hip/HIPContext.h>
#include <torch/extension.h>

#include <cstring>

#include <stdexcept>

#include "kernels.h"

namespace py = pybind11;
using torch::Tensor;

namespace pbx {

static hipStream_t cur_stream() { return at::hip::getCurrentHIPStream().stream(); }

#define PBX_CHECK(cond, msg)                                     \
  do {                                                           \
    if (!(cond)) throw std::runtime_error(std::string("pbx: ") + msg); \
  } while (0)

static void check_cuda(const Tensor& t, const char* name) {
  PBX_CHECK(t.is_cuda(), std::string(name) + " must be a GPU tensor");
  PBX_CHECK(t.is_contiguous(), std::string(name) + " must be contiguous");
}
template <typename T>
static T* ptr(const Tensor& t) {
  return reinterpret_cast<T*>(t.data_ptr());
}
template <typename T>
static T* optr(const c10::optional<Tensor>& t) {
  return t.has_value() && t->defined() ? reinterpret_cast<T*>(t->data_ptr()) : nullptr;
}

// --------------------------------------------------------------- GPU table
class GpuTable {
 public:
  GpuTable(int dim, int64_t capacity, int64_t stash_cap, int device, int extra = 0)
      : dim_(dim), device_(device) {
    PBX_CHECK(dim >= 1 && dim <= 128, "embedx dim must be in [1,128]");
    PBX_CHECK(extra >= 0 && extra <= 1024, "extra row floats");
    const RowLayout l = make_row_layout(dim);
    // codec state (feature_ops.hip) follows the standard tail
    stride_ = extra > 0 ? ((l.mf_size + 1 + extra) + 3) & ~3 : l.stride;
    // PBX_TD_INROW=1: a plain row's first padding word (after the layout's
    // last field) holds the table dedup's per-row occurrence counter -- zero
    // between dedups -- on the row's own page instead of a separate
    // table-sized array.  Opt-in: a dedup running CONCURRENTLY with a push
    // (PBX_SPLIT_PREFETCH modes) races the push's whole-row float4 stores and
    // faulted; never combined with them.
    const char* inrow = getenv("PBX_TD_INROW");
    const char* split = getenv("PBX_SPLIT_PREFETCH");
    const bool split_on = split && split[0] != '\0' && split[0] != '0';
    pad_col_ = (extra == 0 && stride_ > l.mf_size + 1 && inrow && inrow[0] == '1' && !split_on) ? l.mf_size + 1 : -1;
    nb_ = (uint64_t)((capacity + kBucketSlots - 1) / kBucketSlots);
    if (nb_ < 1) nb_ = 1;
    stash_cap_ = stash_cap;
    auto opt8 = torch::TensorOptions().dtype(torch::kInt64).device(torch::kCUDA, device);
    auto opt4 = torch::TensorOptions().dtype(torch::kInt32).device(torch::kCUDA, device);
    auto optf = torch::TensorOptions().dtype(torch::kFloat32).device(torch::kCUDA, device);
    keys_ = torch::full({(int64_t)nb_ * kBucketSlots}, -1, opt8);  // kEmptyKey
    fill_ = torch::zeros({(int64_t)nb_}, opt4);
    values_ = torch::zeros({(int64_t)nb_ * kBucketSlots + stash_cap_, stride_}, optf);
    stash_keys_ = torch::full({std::max<int64_t>(stash_cap_, 1)}, -1, opt8);
    scratch_ = torch::zeros({8}, opt8);  // [stash_n, ovf_n, fail_n, count, cursor...]
    err_ = torch::zeros({1}, opt4);       // guard bits (TableDev::err), sticky until clear_error
  }
  TableDev view() const {
    TableDev t;
    t.keys = ptr<uint64_t>(keys_);
    t.fill = ptr<uint32_t>(fill_);
    t.values = ptr<float>(values_);
    t.nb = nb_;
    t.stash_keys = ptr<uint64_t>(stash_keys_);
    t.stash_n = reinterpret_cast<uint32_t*>(ptr<int64_t>(scratch_) + 0);
    t.stash_cap = (uint32_t)stash_cap_;
    t.stride = stride_;
    t.dim = dim_;
    t.err = ptr<int32_t>(err_);
    return t;
  }
  // guard bits the kernels recorded (a device read: call outside captures)
  int64_t error_bits() const { return err_.cpu().item<int32_t>(); }
  void clear_error() { err_.zero_(); }
  Tensor probe(const Tensor& h, const c10::optional<Tensor>& n_dev) {
    check_cuda(h, "h");
    auto rows = torch::empty({h.numel()}, h.options().dtype(torch::kInt64));
    launch_table_probe(view(), ptr<uint64_t>(h), h.numel(), optr<int32_t>(n_dev), ptr<int64_t>(rows), cur_stream());
    return rows;
  }
  // probe into a caller-owned (persistent) row buffer: graph-captured
  // prefetches need the rows at a fixed address
  void probe_into(const Tensor& h, const c10::optional<Tensor>& n_dev, Tensor rows) {
    check_cuda(h, "h");
    check_cuda(rows, "rows");
    PBX_CHECK(rows.scalar_type() == torch::kInt64 && rows.is_contiguous() && rows.numel() >= h.numel(),
              "probe_into: rows must be contiguous int64 with >= h.numel() entries");
    launch_table_probe(view(), ptr<uint64_t>(h), h.numel(), optr<int32_t>(n_dev), ptr<int64_t>(rows), cur_stream());
  }
  // Insert unique mixed keys (those not present). Returns number of keys that
  // could not be placed (0 normally).  Synchronises (build phase only).
  int64_t insert(const Tensor& h, const c10::optional<Tensor>& n_dev, const SparseSGDConfig& cfg,
                 uint64_t seed, bool init_embedx) {
    check_cuda(h, "h");
    const int64_t n = h.numel();
    if (n == 0) return 0;
    auto s = cur_stream();
    Tensor rows = probe(h, n_dev);
    auto ovf = torch::empty({n}, h.options());
    auto ctr = torch::zeros({4}, h.options().dtype(torch::kInt32));
    launch_table_insert(view(), ptr<uint64_t>(h), n, optr<int32_t>(n_dev), ptr<int64_t>(rows), cfg, seed,
                        init_embedx ? 1 : 0, ptr<uint64_t>(ovf), reinterpret_cast<uint32_t*>(ptr<int32_t>(ctr)), s);
    launch_table_clamp_fill(view(), s);
    launch_table_resolve_overflow(view(), ptr<uint64_t>(ovf), reinterpret_cast<uint32_t*>(ptr<int32_t>(ctr)), cfg,
                                  seed, init_embedx ? 1 : 0, reinterpret_cast<uint32_t*>(ptr<int32_t>(ctr) + 1), s);
    auto host = ctr.cpu();
    last_overflow_ = host[0].item<int32_t>();
    return host[1].item<int32_t>();
  }
  int64_t last_overflow() const { return last_overflow_; }
  int64_t size() {
    auto c = torch::zeros({1}, keys_.options());
    launch_table_count(view(), reinterpret_cast<unsigned long long*>(ptr<int64_t>(c)), cur_stream());
    int64_t stash = stash_n();
    return c.cpu().item<int64_t>() + stash;
  }
  int64_t stash_n() { return scratch_.narrow(0, 0, 1).cpu().item<int64_t>() & 0xFFFFFFFF; }
  // Export all (mixed key, value row) pairs.
  std::pair<Tensor, Tensor> export_all(bool with_values) {
    const int64_t n = size();
    auto k = torch::empty({n}, keys_.options());
    Tensor v = with_values ? torch::empty({n, stride_}, values_.options()) : Tensor();
    auto cur = torch::zeros({1}, keys_.options());
    if (n > 0)
      launch_table_export(view(), ptr<uint64_t>(k), with_values ? ptr<float>(v) : nullptr,
                          reinterpret_cast<unsigned long long*>(ptr<int64_t>(cur)), cur_stream());
    return {k, v};
  }
  void assign(const Tensor& rows, const Tensor& vals) {
    check_cuda(rows, "rows");
    check_cuda(vals, "vals");
    PBX_CHECK(vals.dim() == 2 && vals.size(0) == rows.numel(), "assign: shape");
    launch_table_assign(view(), ptr<int64_t>(rows), ptr<float>(vals), rows.numel(), (int)vals.size(1), cur_stream());
  }
  int64_t shrink(const ShrinkConfig& c) {
    auto d = torch::zeros({1}, keys_.options());
    launch_table_shrink(view(), c, reinterpret_cast<unsigned long long*>(ptr<int64_t>(d)), cur_stream());
    return d.cpu().item<int64_t>();
  }
  Tensor gather_pull(const Tensor& rows, const c10::optional<Tensor>& n_dev, int out_stride) {
    check_cuda(rows, "rows");
    auto out = torch::empty({rows.numel(), out_stride}, values_.options());
    launch_gather_pull(view(), ptr<int64_t>(rows), optr<int32_t>(n_dev), rows.numel(), ptr<float>(out), out_stride,
                       cur_stream());
    return out;
  }
  void push_adagrad(const Tensor& rows, const Tensor& push, const c10::optional<Tensor>& n_dev,
                    const SparseSGDConfig& cfg, uint64_t seed) {
    check_cuda(rows, "rows");
    check_cuda(push, "push");
    PBX_CHECK(push.dim() == 2 && push.size(1) >= push_width(dim_), "push record width");
    launch_push_adagrad(view(), ptr<int64_t>(rows), ptr<float>(push), (int)push.size(1), optr<int32_t>(n_dev),
                        rows.numel(), cfg, seed, cur_stream());
  }
  // owner side of the sharded pull: out[j] = pull head of rows[uid[j]]
  void gather_rows_by_uid(const Tensor& rows, const Tensor& uid, Tensor out) {
    check_cuda(rows, "rows");
    check_cuda(uid, "uid");
    check_cuda(out, "out");
    PBX_CHECK(out.dim() == 2 && out.size(0) == uid.numel(), "gather_rows_by_uid: out rows");
    PBX_CHECK(out.size(1) % 4 == 0 && out.size(1) <= stride_, "gather_rows_by_uid: out stride");
    launch_gather_rows_by_uid(view(), ptr<int64_t>(rows), ptr<int32_t>(uid), uid.numel(), ptr<float>(out),
                              (int)out.size(1), cur_stream());
  }
  // owner side of the sharded push: merge each unique's received records and
  // apply Adagrad in one pass; false if not vectorisable for this dim
  bool push_adagrad_seg(const Tensor& rows, const Tensor& rec, const Tensor& perm, const Tensor& seg,
                        const Tensor& cnt, const Tensor& n_dev, const SparseSGDConfig& cfg, uint64_t seed) {
    check_cuda(rows, "rows");
    check_cuda(rec, "rec");
    PBX_CHECK(rec.dim() == 2 && rec.size(1) >= push_width(dim_), "push record width");
    return launch_push_adagrad_seg(view(), ptr<int64_t>(rows), ptr<float>(rec), (int)rec.size(1),
                                   ptr<int32_t>(perm), ptr<int32_t>(seg), ptr<int32_t>(cnt), ptr<int32_t>(n_dev),
                                   rows.numel(), cfg, seed, cur_stream());
  }
  // owner side of the sharded pull, one launch: rows[i] = row of h[i] (-1 if
  // absent) and out[i] = its pull record; h may hold -1 padding (skipped)
  void probe_gather(const Tensor& h, Tensor rows, Tensor out) {
    check_cuda(h, "h");
    check_cuda(rows, "rows");
    check_cuda(out, "out");
    PBX_CHECK(rows.scalar_type() == torch::kInt64 && rows.is_contiguous() && rows.numel() >= h.numel(),
              "probe_gather: rows");
    PBX_CHECK(out.dim() == 2 && out.is_contiguous() && out.size(0) >= h.numel() && out.size(1) % 4 == 0 &&
                  out.size(1) <= stride_,
              "probe_gather: out must be contiguous [>= n, stride % 4 == 0, <= row stride]");
    launch_probe_gather(view(), ptr<uint64_t>(h), h.numel(), ptr<int64_t>(rows), ptr<float>(out), (int)out.size(1),
                        cur_stream());
  }
  // the sharded pull's answer exchange with this owner's probe + gather fused
  // in (ipc.hip k_ipc_answer_exchange) over the IPC mesh whose peer table is
  // at peers (IpcComm.peers_ptr): recv [world * cap] keys (rcnt [world]
  // valid per peer), rows [world * cap] out, dst [world * cap, rec] answers
  void answer_exchange(int64_t peers, int64_t blocks, const Tensor& recv, const Tensor& rcnt, int64_t cap,
                       Tensor rows, Tensor dst) {
    check_cuda(recv, "recv");
    check_cuda(rcnt, "rcnt");
    check_cuda(rows, "rows");
    check_cuda(dst, "dst");
    const IpcPeers& pt = *reinterpret_cast<const IpcPeers*>((uintptr_t)peers);
    PBX_CHECK(peers != 0 && blocks > 0, "answer_exchange: mesh");
    PBX_CHECK(recv.scalar_type() == torch::kInt64 && recv.is_contiguous() && recv.numel() == pt.world * cap,
              "answer_exchange: recv must be [world * cap] int64");
    PBX_CHECK(rcnt.scalar_type() == torch::kInt32 && rcnt.numel() >= pt.world, "answer_exchange: rcnt");
    PBX_CHECK(rows.scalar_type() == torch::kInt64 && rows.is_contiguous() && rows.numel() >= recv.numel(),
              "answer_exchange: rows");
    PBX_CHECK(dst.dim() == 2 && dst.is_contiguous() && dst.size(0) == recv.numel() && dst.size(1) % 4 == 0 &&
                  dst.size(1) <= stride_ && stride_ % 4 == 0,
              "answer_exchange: dst must be contiguous [world * cap, rec], rec % 4 == 0, <= row stride");
    PBX_CHECK(dst.size(1) * 4 <= pt.slot_bytes, "answer_exchange: record larger than the mesh slot");
    launch_ipc_answer_exchange(pt, view(), ptr<uint64_t>(recv), ptr<int32_t>(rcnt), cap, (int)dst.size(1),
                               ptr<int64_t>(rows), ptr<float>(dst), (int)blocks, cur_stream());
  }
  // no-dedup pull: rows[k] = row of raw feasign keys[k] (-1: padding / absent)
  void probe_raw(const Tensor& keys, Tensor rows) {
    check_cuda(keys, "keys");
    check_cuda(rows, "rows");
    PBX_CHECK(keys.scalar_type() == torch::kInt64 && keys.is_contiguous(), "probe_raw: keys must be int64");
    PBX_CHECK(rows.scalar_type() == torch::kInt64 && rows.is_contiguous() && rows.numel() >= keys.numel(),
              "probe_raw: rows");
    launch_probe_raw(view(), ptr<int64_t>(keys), keys.numel(), ptr<int64_t>(rows), cur_stream());
  }
  Tensor& owner_lock() {
    if (!lock_.defined()) {
      auto opt4 = torch::TensorOptions().dtype(torch::kInt32).device(torch::kCUDA, device_);
      lock_ = torch::full({values_.size(0)}, -1, opt4);  // free; every apply resets what it took
    }
    return lock_;
  }
  // per-row scratch of the table dedup (launch_table_dedup): occurrence
  // counts (kept all-zero between batches) and the batch's unique id of a row
  // (cnt base, cnt stride in int32 words, uid_row)
  std::tuple<int32_t*, int64_t, int32_t*> dedup_rows() {
    if (!uid_row_.defined()) {
      PBX_CHECK(values_.size(0) < (int64_t)INT32_MAX, "table dedup: table rows must fit int32");
      auto opt4 = torch::TensorOptions().dtype(torch::kInt32).device(torch::kCUDA, device_);
      if (pad_col_ < 0) cnt_row_ = torch::zeros({values_.size(0)}, opt4);
      uid_row_ = torch::empty({values_.size(0)}, opt4);
    }
    if (pad_col_ >= 0) return {reinterpret_cast<int32_t*>(ptr<float>(values_)) + pad_col_, (int64_t)stride_, ptr<int32_t>(uid_row_)};
    return {ptr<int32_t>(cnt_row_), (int64_t)1, ptr<int32_t>(uid_row_)};
  }
  Tensor& lead_buf(int64_t n) {
    if (!lead_.defined() || lead_.numel() < n) lead_ = torch::empty({n}, owner_lock().options());
    return lead_;
  }
  // no-dedup push (one record per occurrence, merged per row by leader
  // election, then Adagrad); acc: all-zero scratch [>= n, stride], kept zero.
  // False if not vectorisable for this dim / layout.
  bool push_occ(const Tensor& dout, int col_offset, const Tensor& cvm, bool use_cvm, bool clk_filter, int E,
                const Tensor& occ_slot, const Tensor& occ_ins, const Tensor& slot_ids, const Tensor& rows, Tensor acc,
                float bs_scale, const SparseSGDConfig& cfg, uint64_t seed, int embed_thres_size) {
    check_cuda(dout, "dout");
    check_cuda(cvm, "cvm");
    check_cuda(rows, "rows");
    check_cuda(acc, "acc");
    const int64_t n = rows.numel();
    if (cvm.dim() != 2 || cvm.size(1) != 2 || E != 3 + dim_) return false;
    PBX_CHECK(acc.dim() == 2 && acc.is_contiguous() && acc.size(0) >= n * kOccRep, "push_occ: acc rows (kOccRep x n)");
    PBX_CHECK(occ_slot.numel() >= n && occ_ins.numel() >= n, "push_occ: occurrence maps");
    PBX_CHECK(n < (int64_t)INT32_MAX, "push_occ: too many occurrences");
    PBX_CHECK(values_.size(0) < (int64_t)0xFFFFFFFFll, "push_occ: table rows must fit 32 bits");
    PushMergeArgs a;
    a.dout = ptr<float>(dout);
    a.out_stride = (int)dout.size(1);
    a.col_offset = col_offset;
    a.cvm = ptr<float>(cvm);
    a.cvm_offset = 2;
    a.use_cvm = use_cvm;
    a.clk_filter = clk_filter;
    a.E = E;
    a.perm = nullptr;
    a.uid = nullptr;
    a.occ_slot = ptr<int32_t>(occ_slot);
    a.occ_ins = ptr<int32_t>(occ_ins);
    a.slot_ids = ptr<float>(slot_ids);
    a.n_valid = nullptr;
    a.n = n;
    a.push = ptr<float>(acc);
    a.push_stride = (int)acc.size(1);
    a.push_index = nullptr;
    a.bs_scale = bs_scale;
    a.dim = dim_;
    a.embed_thres_size = use_cvm ? 0 : embed_thres_size;
    return launch_push_occ(a, view(), ptr<int64_t>(rows), ptr<int32_t>(owner_lock()), ptr<int32_t>(lead_buf(n)), cfg,
                           seed, cur_stream());
  }
  // streaming checkpoint of this table (ckpt.hip / ckpt_saver.cpp): kind 0 =
  // numpy batch model (keys_path / vals_path), 1 = xbox text (keys_path);
  // mode 0 all / 1 base / 2 delta.  Returns (rows, chunks, gpu_s, write_s,
  // total_s, saved mixed keys (int64 CPU tensor) or None).
  py::tuple save_stream(int kind, int mode, bool reset_delta, float base_threshold, float delta_threshold,
                        float delta_keep_days, float nonclk_coeff, float clk_coeff, float embedx_threshold,
                        const std::string& keys_path, const std::string& vals_path, int64_t chunk_rows, int threads,
                        bool collect, std::vector<int64_t> decode_map, float decode_scale, int out_dim) {
    SaveDecode dec;
    PBX_CHECK(decode_map.size() <= (size_t)kSaveMaxCols, "save_stream: decoded row wider than kSaveMaxCols");
    dec.n = (int)decode_map.size();
    dec.scale = decode_scale;
    for (size_t i = 0; i < decode_map.size(); ++i) {
      PBX_CHECK(decode_map[i] >= -(int64_t)(2 * values_.size(1)) - 2 && decode_map[i] < values_.size(1),
                "save_stream: decode map column out of the row");
      dec.map[i] = (int16_t)decode_map[i];
    }
    SaveSelect sel;
    sel.mode = mode;
    sel.reset_delta = reset_delta ? 1 : 0;
    sel.base_threshold = base_threshold;
    sel.delta_threshold = delta_threshold;
    sel.delta_keep_days = delta_keep_days;
    sel.nonclk_coeff = nonclk_coeff;
    sel.clk_coeff = clk_coeff;
    std::vector<uint64_t> mixed;
    SaveStats st;
    {
      py::gil_scoped_release nogil;
      st = stream_save_table(view(), values_.size(0), kind, sel, dec, out_dim, embedx_threshold, keys_path,
                             vals_path, chunk_rows, threads, collect ? &mixed : nullptr, device_, cur_stream());
    }
    py::object keys = py::none();
    if (collect) {
      auto k = torch::empty({(int64_t)mixed.size()}, torch::TensorOptions().dtype(torch::kInt64));
      if (!mixed.empty()) std::memcpy(k.data_ptr(), mixed.data(), mixed.size() * sizeof(uint64_t));
      keys = py::cast(k);
    }
    return py::make_tuple(st.rows, st.chunks, st.gpu_s, st.write_s, st.total_s, keys);
  }
  // owner side of the sharded push without a dedup of the received keys
  // (entries sharing a row elect a leader through a per-row lock word, see
  // launch_owner_push); rec is modified (records summed into the leaders').
  // False if not vectorisable for this dim / record stride.
  bool owner_push(const Tensor& rows, Tensor rec, const SparseSGDConfig& cfg, uint64_t seed) {
    check_cuda(rows, "rows");
    check_cuda(rec, "rec");
    const int64_t n = rows.numel();
    PBX_CHECK(rec.dim() == 2 && rec.is_contiguous() && rec.size(0) >= n && rec.size(1) >= push_width(dim_),
              "owner_push: rec");
    PBX_CHECK(n < (int64_t)INT32_MAX, "owner_push: too many records");
    return launch_owner_push(view(), ptr<int64_t>(rows), ptr<float>(rec), (int)rec.size(1), n,
                             ptr<int32_t>(owner_lock()), ptr<int32_t>(lead_buf(n)), cfg, seed, cur_stream());
  }
  // single-shard push: merge per unique key + Adagrad in one pass (acc: all-zero
  // scratch [>= U_cap, stride], kept zero; inc: [>= ceil(n/64)] int32 scratch)
  bool push_merge_apply(const Tensor& dout, int col_offset, const Tensor& cvm, bool use_cvm, bool clk_filter, int E,
                        const Tensor& perm, const Tensor& uid, const Tensor& occ_slot, const Tensor& occ_ins,
                        const Tensor& slot_ids, const Tensor& n_valid, Tensor acc, Tensor inc, float bs_scale,
                        const Tensor& rows, const SparseSGDConfig& cfg, uint64_t seed, int embed_thres_size) {
    check_cuda(dout, "dout");
    check_cuda(cvm, "cvm");
    check_cuda(acc, "acc");
    check_cuda(rows, "rows");
    PBX_CHECK(E == 3 + dim_, "push_merge_apply: E must be 3 + dim");
    PBX_CHECK(cvm.dim() == 2 && cvm.size(1) == 2, "push_merge_apply: cvm must be [B, 2]");
    PBX_CHECK(acc.dim() == 2 && acc.size(0) >= perm.numel() && acc.size(0) >= rows.numel(), "push_merge_apply: acc rows");
    const bool fused = inc.scalar_type() == torch::kInt64;  // per-unique arrival counters: one launch
    PBX_CHECK(fused ? inc.numel() >= perm.numel() : (inc.scalar_type() == torch::kInt32 && inc.numel() * 64 >= perm.numel()),
              "push_merge_apply: inc too small");
    PushMergeArgs a;
    a.dout = ptr<float>(dout);
    a.out_stride = (int)dout.size(1);
    a.col_offset = col_offset;
    a.cvm = ptr<float>(cvm);
    a.cvm_offset = 2;
    a.use_cvm = use_cvm;
    a.clk_filter = clk_filter;
    a.E = E;
    a.perm = ptr<int32_t>(perm);
    a.uid = ptr<int32_t>(uid);
    a.occ_slot = ptr<int32_t>(occ_slot);
    a.occ_ins = ptr<int32_t>(occ_ins);
    a.slot_ids = ptr<float>(slot_ids);
    a.n_valid = ptr<int32_t>(n_valid);
    a.n = perm.numel();
    a.push = ptr<float>(acc);
    a.push_stride = (int)acc.size(1);
    a.push_index = nullptr;
    a.bs_scale = bs_scale;
    a.dim = dim_;
    a.embed_thres_size = use_cvm ? 0 : embed_thres_size;
    a.err = ptr<int32_t>(err_);
    return launch_push_merge_apply(a, view(), ptr<int64_t>(rows), fused ? nullptr : ptr<int32_t>(inc),
                                   fused ? reinterpret_cast<unsigned long long*>(ptr<int64_t>(inc)) : nullptr, cfg,
                                   seed, cur_stream());
  }
  // ---- feature-type codec (feature_ops.hip)
  void codec_check(const CodecDev& c) const {
    PBX_CHECK(c.Wx + c.We == dim_, "codec storage width != table dim");
    PBX_CHECK(c.mf + 1 + c.extra <= stride_, "codec state exceeds the row stride");
  }
  Tensor codec_pull(const CodecDev& c, const Tensor& rows, const c10::optional<Tensor>& uid,
                    const c10::optional<Tensor>& n_dev, int64_t n, Tensor out) {
    codec_check(c);
    check_cuda(rows, "rows");
    check_cuda(out, "out");
    const int need = 3 + (c.kind == 3 ? c.Wx : c.D + c.De);  // variable: one block of max(D, De)
    PBX_CHECK(out.dim() == 2 && out.size(0) >= n && out.size(1) >= need, "codec_pull: out shape");
    if (uid.has_value() && uid->defined()) PBX_CHECK(uid->numel() >= n, "codec_pull: uid");
    else PBX_CHECK(rows.numel() >= n, "codec_pull: rows");
    launch_codec_pull(view(), c, ptr<int64_t>(rows), optr<int32_t>(uid), optr<int32_t>(n_dev), n, ptr<float>(out),
                      (int)out.size(1), cur_stream());
    return out;
  }
  void codec_update(const CodecDev& c, const Tensor& rows, const Tensor& push, const c10::optional<Tensor>& n_dev,
                    const SparseSGDConfig& cfg, uint64_t seed) {
    codec_check(c);
    check_cuda(rows, "rows");
    check_cuda(push, "push");
    PBX_CHECK(push.dim() == 2 && push.size(0) >= rows.numel() && push.size(1) >= 4 + (c.kind == 3 ? c.Wx : c.D + c.De),
              "codec_update: push record width");
    launch_codec_update(view(), c, ptr<int64_t>(rows), ptr<float>(push), (int)push.size(1), optr<int32_t>(n_dev),
                        rows.numel(), cfg, seed, cur_stream());
  }
  void codec_init(const CodecDev& c, const Tensor& rows, const Tensor& h, const SparseSGDConfig& cfg, uint64_t seed,
                  bool init_embedx) {
    codec_check(c);
    check_cuda(rows, "rows");
    check_cuda(h, "h");
    PBX_CHECK(h.numel() == rows.numel(), "codec_init: one key per row");
    launch_codec_init(view(), c, ptr<int64_t>(rows), ptr<uint64_t>(h), rows.numel(), cfg, seed, init_embedx ? 1 : 0,
                      cur_stream());
  }
  // copy another table's full state (same geometry) into this one's storage,
  // on the current stream: the tiered store swaps a staged pass working set
  // into the live table without moving its device addresses (captured
  // graphs keep pointing at the live table)
  void copy_from(const GpuTable& o) {
    PBX_CHECK(o.nb_ == nb_ && o.stash_cap_ == stash_cap_ && o.stride_ == stride_ && o.dim_ == dim_,
              "copy_from: table geometry differs");
    keys_.copy_(o.keys_, true);
    fill_.copy_(o.fill_, true);
    values_.copy_(o.values_, true);
    stash_keys_.copy_(o.stash_keys_, true);
    scratch_.copy_(o.scratch_, true);
  }
  void clear() {
    keys_.fill_(-1);
    fill_.zero_();
    scratch_.zero_();
    stash_keys_.fill_(-1);
  }
  Tensor keys() const { return keys_; }
  Tensor values() const { return values_; }
  Tensor fill() const { return fill_; }
  int dim() const { return dim_; }
  int stride() const { return stride_; }
  int64_t capacity() const { return (int64_t)nb_ * kBucketSlots; }
  int64_t nbuckets() const { return (int64_t)nb_; }

 private:
  int dim_;
  int device_;
  int stride_;
  uint64_t nb_;
  int64_t stash_cap_;
  int64_t last_overflow_ = 0;
  Tensor keys_, fill_, values_, stash_keys_, scratch_, err_;
  Tensor lock_, lead_;  // owner_push: per-row leader word (-1 = free), per-record leader
  Tensor cnt_row_, uid_row_;  // table dedup scratch (dedup_rows)
  int pad_col_ = -1;          // in-row dedup counter column (-1: cnt_row_)
};

// --------------------------------------------------------------- dedup
struct DedupWorkspace {
  int64_t cap;
  Tensor h_tmp, h_sorted, idx_tmp, perm, flags, scan, uid, uniq_h, seg, u_count, temp;
  size_t temp_bytes;
  bool hash = false;
  Tensor tk, tu, slot, slot_of_u, cnt, rank;
  uint64_t tmask = 0;
  DedupWorkspace(int64_t cap_, int device, bool hash_) : cap(cap_), hash(hash_) {
    auto o8 = torch::TensorOptions().dtype(torch::kInt64).device(torch::kCUDA, device);
    auto o4 = torch::TensorOptions().dtype(torch::kInt32).device(torch::kCUDA, device);
    if (hash) {
      int64_t tcap = 1024;
      while (tcap < 2 * cap) tcap <<= 1;  // load <= 0.5
      tmask = (uint64_t)tcap - 1;
      tk = torch::full({tcap}, -1, o8);  // kEmptyKey
      tu = torch::full({tcap}, -1, o4);
      slot = torch::empty({cap}, o4);
      slot_of_u = torch::empty({cap}, o4);
      cnt = torch::zeros({cap + 1}, o4);
      rank = torch::empty({cap}, o4);
    }
    h_tmp = torch::empty({cap}, o8);
    h_sorted = torch::empty({cap}, o8);
    idx_tmp = torch::empty({cap}, o4);
    perm = torch::empty({cap}, o4);
    flags = torch::empty({cap}, o4);
    scan = torch::empty({cap}, o4);
    uid = torch::empty({cap}, o4);
    uniq_h = torch::empty({cap}, o8);
    seg = torch::empty({cap + 1}, o4);
    u_count = torch::zeros({4}, o4);  // [U, n_valid, U of the previous hash run, segment cursor]
    temp_bytes = hash ? hash_dedup_temp_bytes(cap) : dedup_temp_bytes(cap);
    temp = torch::empty({(int64_t)temp_bytes}, torch::TensorOptions().dtype(torch::kUInt8).device(torch::kCUDA, device));
  }
  // keys: int64 tensor (n <= cap).  Results live in this workspace.
  // zero (optional, hash mode): int32 counters zeroed by the first launch
  void run(const Tensor& keys, bool mixed, const c10::optional<Tensor>& zero) {
    check_cuda(keys, "keys");
    const int64_t n = keys.numel();
    PBX_CHECK(n <= cap, "dedup: more keys than workspace capacity");
    if (hash) {
      HashDedupArgs a;
      if (zero.has_value() && zero->defined()) {
        PBX_CHECK(zero->is_cuda() && zero->scalar_type() == torch::kInt32 && zero->numel() <= 256, "dedup zero");
        a.zero_extra = ptr<int32_t>(*zero);
        a.zero_n = (int)zero->numel();
      }
      a.keys = ptr<uint64_t>(keys);
      a.n = n; a.cap = cap; a.mixed = mixed ? 1 : 0;
      a.tk = ptr<uint64_t>(tk); a.tu = ptr<int32_t>(tu); a.tmask = tmask;
      a.slot = ptr<int32_t>(slot); a.slot_of_u = ptr<int32_t>(slot_of_u);
      a.cnt = ptr<int32_t>(cnt); a.rank = ptr<int32_t>(rank);
      a.uid = ptr<int32_t>(uid); a.perm = ptr<int32_t>(perm); a.uniq_h = ptr<uint64_t>(uniq_h);
      a.seg = ptr<int32_t>(seg); a.u_count = ptr<int32_t>(u_count);
      launch_dedup_hash(a, temp.data_ptr(), temp_bytes, cur_stream());
      last_n = n;
      return;
    }
    launch_dedup(ptr<uint64_t>(keys), n, mixed, ptr<uint64_t>(h_tmp), ptr<uint64_t>(h_sorted), ptr<int32_t>(idx_tmp),
                 ptr<int32_t>(perm), ptr<int32_t>(flags), ptr<int32_t>(scan), ptr<int32_t>(uid), ptr<uint64_t>(uniq_h),
                 ptr<int32_t>(seg), ptr<int32_t>(u_count), temp.data_ptr(), temp_bytes, cur_stream());
    last_n = n;
  }
  // Single-shard dedup through the GPU table (launch_table_dedup): keys are
  // raw feasigns; rows_u[u] = table row of unique u (st.rows), rows_occ the
  // row of every occurrence.  Same uid / perm / seg / u_count contract.
  // rows_given: rows_occ[:n] already holds the rows (probed by the split
  // pull); keys then only give n.
  Tensor rows_u, rows_occ, u_acc;
  Tensor& table_rows_occ() {
    if (!rows_u.defined()) {
      auto o8 = perm.options().dtype(torch::kInt64);
      rows_u = torch::empty({cap}, o8);
      rows_occ = torch::full({cap}, -1, o8);  // kept all -1 between split pulls (k_table_scatter resets it)
      u_acc = torch::zeros({4}, perm.options());  // the dedup's private counters (zero between dedups)
      if (!rank.defined()) rank = torch::empty({cap}, perm.options());
    }
    return rows_occ;
  }
  // rows_occ holds rows after a probing dedup (rows_given = false: the
  // pipelined pull's seqpool reads them); the split pull needs it all -1
  // outside the lod, so it cleans a dirty workspace first
  bool rows_occ_dirty = false;
  void clean_rows_occ() {
    if (!rows_occ_dirty) return;
    rows_occ.fill_(-1);
    rows_occ_dirty = false;
  }
  // defer_scatter: the per-occurrence scatter (uid, perm) and the counter
  // publish are left to the seqpool launch that follows (seqpool_cvm_fwd
  // scatter_ws = this workspace)
  const int32_t* sc_uid_row = nullptr;
  // stage (launch_table_dedup): 0 all, 1 probe + rank, 2 run starts + scatter
  // of the stage-1 call before it on the same keys (may be another stream)
  void run_table(const Tensor& keys, GpuTable& t, bool rows_given, bool defer_scatter = false, int stage = 0) {
    check_cuda(keys, "keys");
    const int64_t n = keys.numel();
    PBX_CHECK(n <= cap, "dedup: more keys than workspace capacity");
    PBX_CHECK(keys.scalar_type() == torch::kInt64 && keys.is_contiguous(), "run_table: keys must be int64");
    PBX_CHECK(stage >= 0 && stage <= 2 && !(stage != 0 && defer_scatter), "run_table: stage");
    table_rows_occ();
    auto rc = t.dedup_rows();
    PBX_CHECK(!(defer_scatter && rows_given), "run_table: a deferred scatter needs the probing dedup");
    launch_table_dedup(t.view(), ptr<int64_t>(keys), n, ptr<int64_t>(rows_occ), ptr<int32_t>(rank), std::get<0>(rc),
                       std::get<1>(rc), std::get<2>(rc), ptr<int64_t>(rows_u), ptr<int32_t>(uid), ptr<int32_t>(perm),
                       ptr<int32_t>(seg), ptr<int32_t>(u_count), ptr<int32_t>(u_acc), rows_given, cur_stream(),
                       !(defer_scatter && n > 0), stage);
    sc_uid_row = (defer_scatter && n > 0) ? std::get<2>(rc) : nullptr;
    last_n = n;
    if (!rows_given) rows_occ_dirty = true;  // rows_given: k_table_scatter hands rows_occ back all -1
  }
  int64_t last_n = 0;
};

// --------------------------------------------------------------- free ops
// process-wide sticky guard word of the kernels without a table of their own
// (seqpool): kSeqpoolGuard* bits, read by SparseEngine.check_guards
static Tensor& guard_tensor(const c10::Device& dev) {
  static Tensor* t = new Tensor();  // never destroyed: no device free after the runtime's teardown
  if (!t->defined() || t->device() != dev) *t = torch::zeros({1}, torch::dtype(torch::kInt32).device(dev));
  return *t;
}
static int32_t* guard_word(const c10::Device& dev) { return ptr<int32_t>(guard_tensor(dev)); }
static int64_t guard_bits_get(const std::string& device) {
  Tensor& t = guard_tensor(c10::Device(device));
  return (int64_t)t.item<int32_t>();
}
static void guard_bits_clear(const std::string& device) { guard_tensor(c10::Device(device)).zero_(); }

static void fill_occurrence(const Tensor& lod, int S, int B, Tensor occ_slot, Tensor occ_ins) {
  check_cuda(lod, "lod");
  PBX_CHECK(lod.numel() == (int64_t)S * (B + 1), "lod shape");
  launch_fill_occurrence(ptr<int64_t>(lod), S, B, ptr<int32_t>(occ_slot), ptr<int32_t>(occ_ins), cur_stream());
}

static void seqpool_cvm_fwd(const Tensor& src, const c10::optional<Tensor>& src_index, const c10::optional<Tensor>& uid,
                            const Tensor& lod, int S, int B, int E, Tensor out, int col_offset, bool use_cvm,
                            int cvm_offset, bool clk_filter, float pad_value, bool need_filter, float show_coeff,
                            float clk_coeff, float threshold, int quant_ratio, bool embed_threshold_filter,
                            float embed_threshold, int embed_thres_size, const c10::optional<Tensor>& dense,
                            int dense_col, const c10::optional<Tensor>& occ_slot,
                            const c10::optional<Tensor>& occ_ins, const c10::optional<Tensor>& probe_keys,
                            GpuTable* probe_table, const c10::optional<Tensor>& rows_out,
                            DedupWorkspace* scatter_ws) {
  check_cuda(src, "src");
  check_cuda(lod, "lod");
  check_cuda(out, "out");
  PBX_CHECK(src.dim() == 2 && src.size(1) >= E, "src width < E");
  // uid None: record index = occurrence index (no-dedup pull; the caller
  // sizes the occurrence maps to its key buffer -- no device read here, the
  // call is graph-captured)
  const int64_t L = uid.has_value() && uid->defined() ? uid->numel() : 0;
  PBX_CHECK(out.dim() == 2 && out.size(0) == B, "out shape");
  SeqpoolCvmArgs a;
  a.src = ptr<float>(src);
  a.src_stride = (int)src.size(1);
  a.src_index = optr<int64_t>(src_index);
  a.uid = optr<int32_t>(uid);
  a.lod = ptr<int64_t>(lod);
  a.S = S;
  a.B = B;
  a.E = E;
  a.out = ptr<float>(out);
  a.out_stride = (int)out.size(1);
  a.col_offset = col_offset;
  a.use_cvm = use_cvm;
  a.cvm_offset = cvm_offset;
  a.clk_filter = clk_filter;
  a.pad_value = pad_value;
  a.need_filter = need_filter;
  a.show_coeff = show_coeff;
  a.clk_coeff = clk_coeff;
  a.threshold = threshold;
  a.quant_ratio = quant_ratio;
  a.embed_threshold_filter = embed_threshold_filter;
  a.embed_threshold = embed_threshold;
  a.embed_thres_size = embed_thres_size;
  PBX_CHECK(col_offset + (int64_t)S * seqpool_cvm_out_width(a) <= out.size(1), "out too narrow");
  if (scatter_ws != nullptr && scatter_ws->sc_uid_row != nullptr) {
    // the deferred table-dedup scatter of scatter_ws rides on this launch:
    // occurrence k's row must be read directly (src_index = rows_occ, no uid)
    PBX_CHECK(!(uid.has_value() && uid->defined()) && a.src_index == scatter_ws->rows_occ.data_ptr<int64_t>(),
              "fused scatter: src_index must be the workspace's rows_occ and uid None");
    PBX_CHECK(E == 11 || E == 12 || E == 19 || E == 35, "fused scatter: needs a specialised seqpool width");
    a.sc_uid_row = scatter_ws->sc_uid_row;
    a.sc_seg = ptr<int32_t>(scatter_ws->seg);
    a.sc_rank = ptr<int32_t>(scatter_ws->rank);
    a.sc_uid = ptr<int32_t>(scatter_ws->uid);
    a.sc_perm = ptr<int32_t>(scatter_ws->perm);
    a.sc_acc = ptr<int32_t>(scatter_ws->u_acc);
    a.sc_u_count = ptr<int32_t>(scatter_ws->u_count);
    scatter_ws->sc_uid_row = nullptr;  // one pooling per dedup
  }
  if (occ_slot.has_value() && occ_slot->defined()) {  // occurrence map written by the same launch
    PBX_CHECK(occ_ins.has_value() && occ_ins->defined(), "occ_ins required with occ_slot");
    PBX_CHECK(occ_slot->numel() >= L && occ_ins->numel() >= L, "occ buffers too small");
    a.occ_slot = ptr<int32_t>(*occ_slot);
    a.occ_ins = ptr<int32_t>(*occ_ins);
  }
  if (dense.has_value() && dense->defined()) {
    PBX_CHECK(dense->is_cuda(), "dense must be a GPU tensor");
    PBX_CHECK(dense->dim() == 2 && dense->size(0) == B && dense->scalar_type() == torch::kFloat32,
              "dense must be f32 [B, Dd]");
    PBX_CHECK(S > 0 && dense_col >= 0 && dense_col + dense->size(1) <= out.size(1), "dense columns out of range");
    PBX_CHECK(dense->stride(1) == 1 || dense->size(1) == 1, "dense: rows must be unit-stride");
    PBX_CHECK(dense->stride(0) >= dense->size(1) || dense->size(0) == 1, "dense: overlapping rows (expanded view)");
    a.dense = ptr<float>(*dense);
    a.dense_dim = (int)dense->size(1);
    a.dense_col = dense_col;
    a.dense_stride = (int)dense->stride(0);  // a column slice of the batch's dense block: read in place
  }
  if (probe_keys.has_value() && probe_keys->defined()) {  // fused probe of the split pull
    PBX_CHECK(probe_table != nullptr && rows_out.has_value() && rows_out->defined(),
              "fused probe needs the table and rows_out");
    check_cuda(*probe_keys, "probe_keys");
    PBX_CHECK(probe_keys->scalar_type() == torch::kInt64 && probe_keys->is_contiguous(), "probe_keys: int64");
    PBX_CHECK(rows_out->scalar_type() == torch::kInt64 && rows_out->numel() >= probe_keys->numel(), "rows_out");
    PBX_CHECK(!uid.has_value() || !uid->defined(), "fused probe replaces uid / src_index");
    PBX_CHECK(a.src_stride % 4 == 0 && (E == 11 || E == 12 || E == 19 || E == 35),
              "fused probe: vectorised record widths only");
    PBX_CHECK(!occ_slot.has_value() || !occ_slot->defined() || occ_slot->numel() >= probe_keys->numel(),
              "occ buffers too small");
    a.probe_keys = reinterpret_cast<const uint64_t*>(probe_keys->data_ptr<int64_t>());
    a.probe_t = probe_table->view();
    a.rows_out = ptr<int64_t>(*rows_out);
  }
  // index guards: the buffers the lod's occurrence indices, the unique ids
  // and the record indices may address (a violation is skipped and flagged)
  {
    int64_t n_occ = INT64_MAX;
    if (a.uid) n_occ = std::min<int64_t>(n_occ, uid->numel());
    if (a.occ_slot) n_occ = std::min<int64_t>(n_occ, std::min(occ_slot->numel(), occ_ins->numel()));
    if (a.probe_keys) n_occ = std::min<int64_t>(n_occ, probe_keys->numel());
    if (a.src_index && !a.uid && !a.probe_keys) n_occ = std::min<int64_t>(n_occ, src_index->numel());
    a.n_occ = n_occ == INT64_MAX ? 0 : std::max<int64_t>(n_occ, 1);
    a.n_index = (a.src_index && a.uid) ? std::max<int64_t>(src_index->numel(), 1) : 0;
    a.src_rows = std::max<int64_t>(src.size(0), 1);
    a.err = guard_word(src.device());
  }
  launch_seqpool_cvm_fwd(a, cur_stream());
}

static void push_merge(const Tensor& dout, int col_offset, const Tensor& cvm, int cvm_offset, bool use_cvm,
                       bool clk_filter, int E, const Tensor& perm, const Tensor& uid, const Tensor& occ_slot,
                       const Tensor& occ_ins, const Tensor& slot_ids, const Tensor& n_valid, Tensor push,
                       const c10::optional<Tensor>& push_index, float bs_scale, int dim, int embed_thres_size) {
  check_cuda(dout, "dout");
  check_cuda(cvm, "cvm");
  check_cuda(push, "push");
  PBX_CHECK(cvm_offset == 2, "fused push merge requires cvm_offset == 2");
  PBX_CHECK(E == 3 + dim, "E must be 3 + dim");
  PBX_CHECK(dim == 4 || dim == 8 || dim == 16 || dim == 32, "fused push merge: dim in {4,8,16,32}");
  PBX_CHECK(push.dim() == 2 && push.size(1) >= push_width(dim), "push width");
  PushMergeArgs a;
  a.dout = ptr<float>(dout);
  a.out_stride = (int)dout.size(1);
  a.col_offset = col_offset;
  a.cvm = ptr<float>(cvm);
  a.cvm_offset = cvm_offset;
  a.use_cvm = use_cvm;
  a.clk_filter = clk_filter;
  a.E = E;
  a.perm = ptr<int32_t>(perm);
  a.uid = ptr<int32_t>(uid);
  a.occ_slot = ptr<int32_t>(occ_slot);
  a.occ_ins = ptr<int32_t>(occ_ins);
  a.slot_ids = ptr<float>(slot_ids);
  a.n_valid = ptr<int32_t>(n_valid);
  a.n = perm.numel();
  a.push = ptr<float>(push);
  a.push_stride = (int)push.size(1);
  a.push_index = optr<int64_t>(push_index);
  a.bs_scale = bs_scale;
  a.dim = dim;
  a.embed_thres_size = use_cvm ? 0 : embed_thres_size;
  launch_push_merge(a, cur_stream());
}

// Sharded push, fused: per-unique merged records written straight into their
// send slots (send[send_index[u]]); acc = all-zero straddle scratch [>= U_cap,
// stride] (kept zero), inc = [>= ceil(n/64)] int32 scratch.  False when the
// dim / layout has no fused instantiation (caller: zero + push_merge).
static bool push_merge_send(const Tensor& dout, int col_offset, const Tensor& cvm, bool use_cvm, bool clk_filter,
                            int E, const Tensor& perm, const Tensor& uid, const Tensor& occ_slot, const Tensor& occ_ins,
                            const Tensor& slot_ids, const Tensor& n_valid, Tensor acc, Tensor inc, Tensor send,
                            const Tensor& send_index, float bs_scale, int dim, int embed_thres_size) {
  check_cuda(dout, "dout");
  check_cuda(cvm, "cvm");
  check_cuda(acc, "acc");
  check_cuda(send, "send");
  check_cuda(send_index, "send_index");
  if (cvm.dim() != 2 || cvm.size(1) != 2 || E != 3 + dim) return false;
  PBX_CHECK(acc.dim() == 2 && acc.is_contiguous() && acc.size(0) >= perm.numel(), "push_merge_send: acc rows");
  PBX_CHECK(send.dim() == 2 && send.is_contiguous(), "push_merge_send: send");
  PBX_CHECK(send_index.scalar_type() == torch::kInt64 && send_index.numel() >= perm.numel(),
            "push_merge_send: send_index");
  const bool fused = inc.scalar_type() == torch::kInt64;  // per-unique arrival counters: one launch
  PBX_CHECK(fused ? inc.numel() >= perm.numel() : (inc.scalar_type() == torch::kInt32 && inc.numel() * 64 >= perm.numel()),
            "push_merge_send: inc too small");
  PushMergeArgs a;
  a.dout = ptr<float>(dout);
  a.out_stride = (int)dout.size(1);
  a.col_offset = col_offset;
  a.cvm = ptr<float>(cvm);
  a.cvm_offset = 2;
  a.use_cvm = use_cvm;
  a.clk_filter = clk_filter;
  a.E = E;
  a.perm = ptr<int32_t>(perm);
  a.uid = ptr<int32_t>(uid);
  a.occ_slot = ptr<int32_t>(occ_slot);
  a.occ_ins = ptr<int32_t>(occ_ins);
  a.slot_ids = ptr<float>(slot_ids);
  a.n_valid = ptr<int32_t>(n_valid);
  a.n = perm.numel();
  a.push = ptr<float>(acc);
  a.push_stride = (int)acc.size(1);
  a.push_index = nullptr;
  a.bs_scale = bs_scale;
  a.dim = dim;
  a.embed_thres_size = use_cvm ? 0 : embed_thres_size;
  return launch_push_merge_send(a, dim, ptr<float>(send), (int)send.size(1), ptr<int64_t>(send_index),
                                fused ? nullptr : ptr<int32_t>(inc),
                                fused ? reinterpret_cast<unsigned long long*>(ptr<int64_t>(inc)) : nullptr, cur_stream());
}

static void push_merge_records(const Tensor& rec, const Tensor& perm, const Tensor& uid, const Tensor& n_valid,
                               int dim, Tensor out) {
  check_cuda(rec, "rec");
  check_cuda(out, "out");
  // records are merged over dim rounded up to a multiple of 4 (the padding
  // columns of a record are zero); the record strides must cover it
  PBX_CHECK(dim >= 1 && dim <= 60, "merge records: dim in [1, 60]");
  const int dim4 = (dim + 3) & ~3;
  PBX_CHECK(rec.size(1) >= dim4 + 4 && out.size(1) >= dim4 + 4, "merge records: record stride < 4 + round4(dim)");
  dim = dim4;
  launch_push_merge_records(ptr<float>(rec), (int)rec.size(1), ptr<int32_t>(perm), ptr<int32_t>(uid),
                            ptr<int32_t>(n_valid), perm.numel(), dim, ptr<float>(out), (int)out.size(1), cur_stream());
}

static void shard_pack(const Tensor& uniq_h, const Tensor& u_count, int nranks, int64_t cap, Tensor send,
                       Tensor send_index, Tensor overflow) {
  check_cuda(uniq_h, "uniq_h");
  PBX_CHECK(send.numel() == nranks * cap, "send shape");
  launch_shard_pack(ptr<uint64_t>(uniq_h), ptr<int32_t>(u_count), send_index.numel(), nranks, cap,
                    ptr<uint64_t>(send), ptr<int64_t>(send_index), ptr<int32_t>(overflow), cur_stream());
}

// prezeroed: ocnt was zeroed by an earlier launch (the dedup's) and the send
// slots' tails need no -1 fill (the IPC exchange fills them at the receiver)
static void shard_pack_hash(const Tensor& uniq_h, const Tensor& u_count, int nranks, int64_t cap, Tensor send,
                            Tensor send_index, Tensor ocnt, Tensor overflow, bool prezeroed) {
  check_cuda(uniq_h, "uniq_h");
  check_cuda(send, "send");
  PBX_CHECK(send.numel() == nranks * cap, "send shape");
  PBX_CHECK(nranks >= 1 && nranks <= 64, "shard_pack_hash: 1..64 ranks");
  PBX_CHECK(ocnt.numel() >= nranks && ocnt.scalar_type() == torch::kInt32, "ocnt");
  PBX_CHECK(send_index.numel() >= uniq_h.numel(), "send_index too short");
  launch_shard_pack_hash(ptr<uint64_t>(uniq_h), ptr<int32_t>(u_count), uniq_h.numel(), nranks, cap,
                         ptr<uint64_t>(send), ptr<int64_t>(send_index), ptr<int32_t>(ocnt), ptr<int32_t>(overflow),
                         prezeroed, cur_stream());
}

static void gather_by_uid(const Tensor& src, const Tensor& uid, Tensor out, int width) {
  check_cuda(src, "src");
  check_cuda(out, "out");
  launch_gather_by_uid(ptr<float>(src), (int)src.size(1), ptr<int32_t>(uid), uid.numel(), ptr<float>(out),
                       (int)out.size(1), width, cur_stream());
}

static std::vector<Tensor> data_norm_fwd(const Tensor& x, const Tensor& bsize, const Tensor& bsum, const Tensor& bsq,
                                         const c10::optional<Tensor>& scale_w, const c10::optional<Tensor>& bias) {
  check_cuda(x, "x");
  const int N = (int)x.size(0), C = (int)x.size(1);
  auto y = torch::empty_like(x);
  auto means = torch::empty({C}, x.options());
  auto scales = torch::empty({C}, x.options());
  launch_data_norm_fwd(ptr<float>(x), N, C, ptr<float>(bsize), ptr<float>(bsum), ptr<float>(bsq), ptr<float>(y),
                       ptr<float>(means), ptr<float>(scales), optr<float>(scale_w), optr<float>(bias), cur_stream());
  return {y, means, scales};
}

static std::vector<Tensor> data_norm_bwd(const Tensor& x, const Tensor& dy, const Tensor& means, const Tensor& scales,
                                         float eps, bool need_dx, const c10::optional<Tensor>& scale_w) {
  check_cuda(x, "x");
  check_cuda(dy, "dy");
  const int N = (int)x.size(0), C = (int)x.size(1);
  Tensor dx = need_dx ? torch::empty_like(x) : Tensor();
  auto stats = torch::empty({3, C}, x.options());
  auto acc = torch::empty({2, C}, x.options());
  launch_data_norm_bwd(ptr<float>(x), ptr<float>(dy), N, C, ptr<float>(means), ptr<float>(scales), eps,
                       need_dx ? ptr<float>(dx) : nullptr, ptr<float>(stats), ptr<float>(acc), optr<float>(scale_w),
                       cur_stream());
  return {dx, stats};
}

// ---------------------------------------------------------------- MLP (MFMA GEMM)
static void check_bf16(const Tensor& t, const char* n) {
  check_cuda(t, n);
  PBX_CHECK(t.scalar_type() == torch::kBFloat16 && t.dim() == 2, std::string(n) + " must be bf16 2-D");
}

// y = act(x w^T + b): x bf16 [M,K], w bf16 [N,K], b f32 [N] -> y bf16 [M,N]
static Tensor linear_fwd(const Tensor& x, const Tensor& w, const c10::optional<Tensor>& bias, bool relu) {
  check_bf16(x, "x");
  check_bf16(w, "w");
  const int M = (int)x.size(0), K = (int)x.size(1), N = (int)w.size(0);
  PBX_CHECK(w.size(1) == K, "linear_fwd: K mismatch");
  PBX_CHECK(K % 8 == 0, "linear_fwd: K must be a multiple of 8 (pad the input)");
  auto y = torch::empty({M, N}, x.options());
  GemmArgs g;
  g.A = reinterpret_cast<const unsigned short*>(x.data_ptr());
  g.B = reinterpret_cast<const unsigned short*>(w.data_ptr());
  g.C = y.data_ptr();
  g.bias = optr<float>(bias);
  g.M = M; g.N = N; g.K = K;
  g.lda = K; g.ldb = K; g.ldc = N;
  g.a_kcontig = true; g.b_kcontig = true;
  g.epi = relu ? EPI_BIAS_RELU_BF16 : EPI_BIAS_BF16;
  launch_gemm(g, cur_stream());
  return y;
}

// Backward of linear_fwd.  dy bf16 [M,N] (grad wrt the layer output),
// ymask (the layer output when relu was applied), x bf16 [M,K], w bf16 [N,K].
// Accumulates dW f32 [N,K] and db f32 [N]; returns dx bf16 [M,K] (or undefined).
static Tensor linear_bwd(const Tensor& dy, const c10::optional<Tensor>& ymask, const Tensor& x, const Tensor& w,
                         Tensor dW, Tensor db, bool need_dx, int k_split) {
  check_bf16(dy, "dy");
  check_bf16(x, "x");
  check_bf16(w, "w");
  const int M = (int)dy.size(0), N = (int)dy.size(1), K = (int)x.size(1);
  PBX_CHECK(w.size(0) == N && w.size(1) == K && x.size(0) == M, "linear_bwd shapes");
  PBX_CHECK(N % 8 == 0 && K % 8 == 0, "linear_bwd: N, K must be multiples of 8");
  auto s = cur_stream();
  const unsigned short* mk = ymask.has_value() ? reinterpret_cast<const unsigned short*>(ymask->data_ptr()) : nullptr;
  Tensor dx;
  if (need_dx) {
    dx = torch::empty({M, K}, x.options());
    GemmArgs g;
    g.A = reinterpret_cast<const unsigned short*>(dy.data_ptr());
    g.maskA = mk;
    g.B = reinterpret_cast<const unsigned short*>(w.data_ptr());
    g.C = dx.data_ptr();
    g.M = M; g.N = K; g.K = N;
    g.lda = N; g.ldb = K; g.ldc = K;
    g.a_kcontig = true; g.b_kcontig = false;
    g.epi = EPI_BF16;
    launch_gemm(g, s);
  }
  // dW (+db via the virtual ones column), split-K over the batch
  const int ks = k_split > 0 ? k_split : 512;
  const int splits = (M + ks - 1) / ks;
  auto slab = torch::empty({splits, N, K + 1}, dW.options());
  GemmArgs g;
  g.A = reinterpret_cast<const unsigned short*>(dy.data_ptr());
  g.maskA = mk;
  g.B = reinterpret_cast<const unsigned short*>(x.data_ptr());
  g.C = slab.data_ptr();
  g.M = N; g.N = K; g.K = M;
  g.lda = N; g.ldb = K; g.ldc = K + 1;
  g.a_kcontig = false; g.b_kcontig = false;
  g.ones_col_b = K;
  g.epi = EPI_F32_SLAB;
  g.k_per_split = ks;
  g.slab_stride = (int64_t)N * (K + 1);
  launch_gemm(g, s);
  launch_slab_reduce(ptr<float>(slab), splits, g.slab_stride, N, K, K + 1, ptr<float>(dW), ptr<float>(db), 1.f, s);
  return dx;
}

static Tensor gemv_out(const Tensor& h, const Tensor& w, const c10::optional<Tensor>& b) {
  check_bf16(h, "h");
  const int M = (int)h.size(0), K = (int)h.size(1);
  auto out = torch::empty({M}, h.options().dtype(torch::kFloat32));
  launch_gemv_out(reinterpret_cast<const unsigned short*>(h.data_ptr()), M, K, K, ptr<float>(w), optr<float>(b),
                  ptr<float>(out), cur_stream());
  return out;
}

static Tensor gemv_out_bwd(const Tensor& h, const Tensor& w, const Tensor& dout, Tensor dw, Tensor db) {
  check_bf16(h, "h");
  const int M = (int)h.size(0), K = (int)h.size(1);
  auto dh = torch::empty_like(h);
  auto d = dout.contiguous();
  auto part = torch::empty({gemv_out_bwd_blocks(M), K + 1}, dw.options());
  launch_gemv_out_bwd(reinterpret_cast<const unsigned short*>(h.data_ptr()), M, K, K, ptr<float>(w), ptr<float>(d),
                      reinterpret_cast<unsigned short*>(dh.data_ptr()), ptr<float>(dw), ptr<float>(db),
                      ptr<float>(part), cur_stream());
  return dh;
}

static void cast_bf16(const Tensor& x, Tensor y) {
  check_cuda(x, "x");
  PBX_CHECK(y.scalar_type() == torch::kBFloat16 && y.numel() == x.numel(), "cast_bf16");
  launch_f32_to_bf16(ptr<float>(x), reinterpret_cast<unsigned short*>(y.data_ptr()), x.numel(), cur_stream());
}

// Fused data_norm + first/FM head.  Returns (y bf16 [B,Cp], lin [B], means, scales).
static std::vector<Tensor> head_fwd(const Tensor& x, int S, int Eo, int ew_col, int D, int Cp,
                                    const c10::optional<Tensor>& bsize, const c10::optional<Tensor>& bsum,
                                    const c10::optional<Tensor>& bsq, const c10::optional<Tensor>& y_out,
                                    const c10::optional<Tensor>& yT_out, const c10::optional<Tensor>& ymp_out,
                                    const c10::optional<Tensor>& stat_part) {
  check_cuda(x, "x");
  PBX_CHECK(x.scalar_type() == torch::kFloat32 && x.dim() == 2, "head: x must be fp32 [B, C]");
  const int B = (int)x.size(0), C = (int)x.size(1);
  PBX_CHECK(Cp >= C && Cp <= (C + 31) / 32 * 32 + 8 && S * Eo <= C, "head: bad widths");
  PBX_CHECK(head_lds_bytes(C, D, Cp) <= 160 * 1024, "head: row slab exceeds LDS");
  HeadArgs a;
  a.x = ptr<float>(x);
  a.B = B; a.C = C; a.Cp = Cp; a.S = S; a.Eo = Eo; a.ew_col = ew_col; a.D = D;
  Tensor y;
  bool yf32 = false;
  if (y_out.has_value() && y_out->defined()) {
    y = *y_out;
    check_cuda(y, "y_out");
    yf32 = y.scalar_type() == torch::kFloat32;
    PBX_CHECK((yf32 || y.scalar_type() == torch::kBFloat16) && y.size(0) == B && y.size(1) >= Cp,
              "head: y_out must be bf16 or fp32 [B, >= Cp]");
    a.ldy = (int)y.size(1);
  } else {
    y = torch::empty({B, Cp}, x.options().dtype(torch::kBFloat16));
  }
  if (yT_out.has_value() && yT_out->defined()) {
    check_cuda(*yT_out, "yT_out");
    PBX_CHECK(yT_out->size(0) >= Cp && yT_out->size(1) >= B, "head: yT_out shape");
    a.yT = reinterpret_cast<unsigned short*>(yT_out->data_ptr());
    a.ldyt = (int)yT_out->size(1);
  }
  if (ymp_out.has_value() && ymp_out->defined()) {
    check_cuda(*ymp_out, "ymp_out");
    if (ymp_out->scalar_type() == torch::kFloat32) {
      PBX_CHECK(yf32 && Cp % 16 == 0 && ymp_out->numel() >= (int64_t)(B + 15) / 16 * 16 * Cp,
                "head: fp32 ymp_out needs an fp32 y_out, Cp % 16 == 0 and pad16(B) * Cp floats");
      a.ympf = ptr<float>(*ymp_out);
    } else {
      PBX_CHECK(!yf32 && Cp % 32 == 0 && ymp_out->numel() >= (int64_t)(B + 15) / 16 * 16 * Cp,
                "head: ymp_out size / Cp % 32");
      a.ymp = reinterpret_cast<unsigned short*>(ymp_out->data_ptr());
    }
  }
  PBX_CHECK(!(yf32 && yT_out.has_value() && yT_out->defined()), "head: yT_out is a bf16-path output");
  if (stat_part.has_value() && stat_part->defined()) {
    check_cuda(*stat_part, "stat_part");
    PBX_CHECK(stat_part->numel() >= (int64_t)head_blocks(B) * 2 * C, "head: stat_part size");
    a.stat_part = ptr<float>(*stat_part);
  }
  auto lin = torch::empty({B}, x.options());
  Tensor means, scales;
  if (bsize.has_value()) {
    means = torch::empty({C}, x.options());
    scales = torch::empty({C}, x.options());
    a.bsize = ptr<float>(*bsize); a.bsum = ptr<float>(*bsum); a.bsq = ptr<float>(*bsq);
    a.means = ptr<float>(means); a.scales = ptr<float>(scales);
  }
  if (yf32) a.yf = ptr<float>(y);
  else a.y = reinterpret_cast<unsigned short*>(y.data_ptr());
  a.lin = ptr<float>(lin);
  launch_head_fwd(a, cur_stream());
  return {y, lin, means, scales};
}

// Backward: returns (dx fp32 [B,C], stats [3,C] or undefined).
static std::vector<Tensor> head_bwd(const Tensor& x, const c10::optional<Tensor>& dy,
                                    const c10::optional<Tensor>& dlin, int S, int Eo, int ew_col, int D, int Cp,
                                    const c10::optional<Tensor>& means, const c10::optional<Tensor>& scales,
                                    float eps, const c10::optional<Tensor>& dlin_scale, bool want_stats) {
  check_cuda(x, "x");
  const int B = (int)x.size(0), C = (int)x.size(1);
  HeadArgs a;
  a.x = ptr<float>(x);
  a.B = B; a.C = C; a.Cp = Cp; a.S = S; a.Eo = Eo; a.ew_col = ew_col; a.D = D;
  auto dx = torch::empty_like(x);
  Tensor stats, acc;
  if (dy.has_value()) {
    PBX_CHECK((dy->scalar_type() == torch::kBFloat16 || dy->scalar_type() == torch::kFloat32) &&
                  dy->size(1) >= Cp && dy->is_contiguous(), "head: dy");
    if (dy->scalar_type() == torch::kFloat32) a.dyf = ptr<float>(*dy);
    else a.dy = reinterpret_cast<const unsigned short*>(dy->data_ptr());
    a.ldy = (int)dy->size(1);
  }
  Tensor dl;
  if (dlin.has_value() && dlin->defined()) {
    dl = dlin->contiguous();
    PBX_CHECK(dl.numel() == B, "head: dlin size");
    a.dlin = ptr<float>(dl);
  }
  a.dlin_scale = optr<float>(dlin_scale);
  a.dx = ptr<float>(dx);
  if (means.has_value() && means->defined() && scales.has_value() && scales->defined()) {
    a.means = ptr<float>(*means);
    a.scales = ptr<float>(*scales);
  }
  if (want_stats && means.has_value() && means->defined()) {
    acc = torch::empty({head_blocks(B), 2 * C}, x.options());
    stats = torch::empty({3, C}, x.options());
    a.stat_acc = ptr<float>(acc);
  }
  launch_head_bwd(a, cur_stream());
  if (a.stat_acc) {
    auto sums = torch::empty({2 * C}, x.options());
    launch_dn_stats(ptr<float>(acc), head_blocks(B), C, B, eps, ptr<float>(stats), ptr<float>(sums), cur_stream());
  }
  return {dx, stats};
}

// --------------------------------------------------------------- fused MLP workspace
// Persistent, zero-initialised buffers in the layout contract of mlp.hip, for
// a fixed batch M and layer widths dims = [K0, H1, ..., Hn] (multiples of 8).
class MlpWorkspace {
 public:
  MlpWorkspace(int64_t M, std::vector<int64_t> dims, int device, int64_t k_split)
      : M_(M), dims_(dims), ksplit_(k_split) {
    PBX_CHECK(dims.size() >= 2, "mlp: need at least one hidden layer");
    for (auto d : dims) PBX_CHECK(d > 0 && d % 8 == 0, "mlp: widths must be multiples of 8");
    PBX_CHECK(k_split % 64 == 0 && k_split > 0, "mlp: k_split must be a positive multiple of 64");
    auto ob = torch::TensorOptions().dtype(torch::kBFloat16).device(torch::kCUDA, device);
    auto of = torch::TensorOptions().dtype(torch::kFloat32).device(torch::kCUDA, device);
    ldM_ = p64(M);
    const int n = (int)dims.size() - 1;
    for (int i = 0; i <= n; ++i) {
      X_.push_back(torch::zeros({M, p64(dims[i])}, ob));
      auto xt = torch::zeros({p64(dims[i] + 1), ldM_}, ob);
      xt[dims[i]].narrow(0, 0, M).fill_(1.0);  // bias ones row
      XT_.push_back(xt);
    }
    for (int l = 0; l < n; ++l) {
      dZ_.push_back(torch::zeros({M, p64(dims[l + 1])}, ob));
      dZT_.push_back(torch::zeros({p64(dims[l + 1]), ldM_}, ob));
      Wb_.push_back(torch::zeros({p64(dims[l + 1]), p64(dims[l])}, ob));
      WTb_.push_back(torch::zeros({p64(dims[l]), p64(dims[l + 1])}, ob));
    }
    dX0_ = torch::zeros({M, p64(dims[0])}, ob);
    logits_ = torch::zeros({M}, of);
    part_ = torch::zeros({mlp_gemv_bwd_blocks((int)M), dims[n] + 1}, of);
  }
  static int64_t p64(int64_t v) { return (v + 63) / 64 * 64; }

  Tensor forward(const std::vector<Tensor>& W, const std::vector<Tensor>& b, const Tensor& wout, const Tensor& bout) {
    const int n = (int)dims_.size() - 1;
    PBX_CHECK((int)W.size() == n && (int)b.size() == n, "mlp.forward: layer count");
    auto s = cur_stream();
    PBX_CHECK(n <= kMaxMlpLayers, "mlp: too many layers");
    CastWtBatch cb;
    cb.n = n;
    cb.tile_off[0] = 0;
    for (int l = 0; l < n; ++l) {
      const int K = (int)dims_[l], N = (int)dims_[l + 1];
      check_cuda(W[l], "W");
      PBX_CHECK(W[l].size(0) == N && W[l].size(1) == K, "mlp.forward: W shape");
      cb.w[l] = ptr<float>(W[l]);
      cb.wb[l] = bptr(Wb_[l]);
      cb.wtb[l] = bptr(WTb_[l]);
      cb.N[l] = N; cb.K[l] = K; cb.pN[l] = (int)p64(N); cb.pK[l] = (int)p64(K);
      cb.tile_off[l + 1] = cb.tile_off[l] + (cb.pN[l] / 32) * (cb.pK[l] / 32);
    }
    launch_cast_wt(cb, s);
    for (int l = 0; l < n; ++l) {
      const int K = (int)dims_[l], N = (int)dims_[l + 1];
      MlpGemmArgs g;
      g.A = bptr(X_[l]); g.lda = (int)p64(K);
      g.B = bptr(Wb_[l]); g.ldb = (int)p64(K);
      g.M = (int)M_; g.N = (int)p64(N); g.K = (int)p64(K);
      g.C = bptr(X_[l + 1]); g.ldc = (int)p64(N);
      g.CT = bptr(XT_[l + 1]); g.ldct = (int)ldM_;
      g.ncols_valid = N;
      g.bias = ptr<float>(b[l]);
      g.relu = 1;
      launch_mlp_gemm(g, MLP_EPI_FWD, s);
    }
    launch_mlp_gemv_fwd(bptr(X_[n]), (int)M_, (int)dims_[n], (int)p64(dims_[n]), ptr<float>(wout), ptr<float>(bout),
                        ptr<float>(logits_), s);
    return logits_;
  }

  // Accumulates parameter grads into dW/db/dwout/dbout; returns dX0 when need_dx.
  Tensor backward(const Tensor& dlogit, const std::vector<Tensor>& dW, const std::vector<Tensor>& db,
                  const Tensor& wout, Tensor dwout, Tensor dbout, bool need_dx) {
    const int n = (int)dims_.size() - 1;
    auto s = cur_stream();
    auto dl = dlogit.contiguous();
    const int H = (int)dims_[n];
    launch_mlp_gemv_bwd(bptr(X_[n]), (int)M_, H, (int)p64(H), ptr<float>(wout), ptr<float>(dl), bptr(dZ_[n - 1]),
                        bptr(dZT_[n - 1]), (int)ldM_, ptr<float>(part_), ptr<float>(dwout), ptr<float>(dbout), s);
    for (int l = n - 1; l >= 0; --l) {
      const int K = (int)dims_[l], N = (int)dims_[l + 1];
      check_cuda(dW[l], "dW");
      MlpGemmArgs g;  // dW_l += dZ_l^T [X_l | 1]
      g.A = bptr(dZT_[l]); g.lda = (int)ldM_;
      g.B = bptr(XT_[l]); g.ldb = (int)ldM_;
      g.M = N; g.N = K + 1; g.K = (int)ldM_;
      g.k_per_split = (int)ksplit_;
      g.dW = ptr<float>(dW[l]); g.lddw = K; g.db = ptr<float>(db[l]);
      g.ncols_valid = K; g.nrows_valid = N;
      launch_mlp_gemm(g, MLP_EPI_DW, s);
      if (l > 0 || need_dx) {
        MlpGemmArgs d;  // dZ_{l-1} = (dZ_l W_l) . [X_l > 0]
        d.A = bptr(dZ_[l]); d.lda = (int)p64(N);
        d.B = bptr(WTb_[l]); d.ldb = (int)p64(N);
        d.M = (int)M_; d.N = (int)p64(K); d.K = (int)p64(N);
        d.C = l > 0 ? bptr(dZ_[l - 1]) : bptr(dX0_);
        d.ldc = (int)p64(K);
        d.CT = l > 0 ? bptr(dZT_[l - 1]) : nullptr;
        d.ldct = (int)ldM_;
        d.ncols_valid = K;
        d.mask = l > 0 ? bptr(X_[l]) : nullptr;
        d.ldmask = (int)p64(K);
        launch_mlp_gemm(d, MLP_EPI_DX, s);
      }
    }
    return need_dx ? dX0_ : Tensor();
  }
  Tensor x(int i) const { return X_.at(i); }
  Tensor xt(int i) const { return XT_.at(i); }
  Tensor dz(int i) const { return dZ_.at(i); }
  Tensor dx0() const { return dX0_; }
  int64_t M() const { return M_; }

 private:
  static unsigned short* bptr(const Tensor& t) { return reinterpret_cast<unsigned short*>(t.data_ptr()); }
  int64_t M_, ldM_;
  std::vector<int64_t> dims_;
  int64_t ksplit_;
  std::vector<Tensor> X_, XT_, dZ_, dZT_, Wb_, WTb_;
  Tensor dX0_, logits_, part_;
};

static void data_norm_update(Tensor bsize, Tensor bsum, Tensor bsq, const Tensor& stats, float decay) {
  launch_data_norm_update(ptr<float>(bsize), ptr<float>(bsum), ptr<float>(bsq), ptr<float>(stats),
                          (int)bsize.numel(), decay, cur_stream());
}

static Tensor fm_fwd(const Tensor& x, int S, int D, int col0, int fstride) {
  check_cuda(x, "x");
  auto out = torch::empty({x.size(0)}, x.options());
  launch_fm_fwd(ptr<float>(x), (int)x.size(0), S, D, (int)x.size(1), col0, fstride, ptr<float>(out), cur_stream());
  return out;
}

static void fm_bwd(const Tensor& x, const Tensor& dout, int S, int D, int col0, int fstride, Tensor dx,
                   bool accumulate) {
  check_cuda(x, "x");
  check_cuda(dx, "dx");
  PBX_CHECK(dx.size(1) == x.size(1), "fm_bwd: dx must match x layout");
  launch_fm_bwd(ptr<float>(x), ptr<float>(dout), (int)x.size(0), S, D, (int)x.size(1), col0, fstride, ptr<float>(dx),
                (int)dx.size(1), accumulate ? 1 : 0, cur_stream());
}

static std::vector<Tensor> sigmoid_logloss(const Tensor& logit, const Tensor& label, float grad_scale) {
  check_cuda(logit, "logit");
  const int B = (int)logit.numel();
  auto pred = torch::empty_like(logit);
  auto dz = torch::empty_like(logit);
  auto loss = torch::zeros({1}, logit.options());
  launch_sigmoid_logloss(ptr<float>(logit), ptr<float>(label), B, ptr<float>(pred), ptr<float>(loss), ptr<float>(dz),
                         grad_scale, cur_stream());
  return {pred, loss, dz};
}

static std::vector<Tensor> logit_loss(const Tensor& a, const c10::optional<Tensor>& b, const Tensor& label,
                                      const Tensor& ws) {
  check_cuda(a, "a");
  check_cuda(label, "label");
  const int B = (int)a.numel();
  PBX_CHECK(label.numel() == B && a.scalar_type() == torch::kFloat32 && label.scalar_type() == torch::kFloat32,
            "logit_loss: a/label must be f32 [B]");
  if (b.has_value() && b->defined()) {
    check_cuda(*b, "b");
    PBX_CHECK(b->numel() == B && b->scalar_type() == torch::kFloat32, "logit_loss: b must be f32 [B]");
  }
  auto pred = torch::empty({B}, a.options());
  auto dz = torch::empty({B}, a.options());
  auto loss = torch::empty({1}, a.options());
  check_cuda(ws, "ws");
  PBX_CHECK(ws.scalar_type() == torch::kInt32 && ws.numel() >= 1 + kLogitLossMaxBlocks && ws.is_contiguous(),
            "logit_loss: ws must be int32 [1 + 1024] (zeroed once)");
  launch_logit_loss(ptr<float>(a), optr<float>(b), ptr<float>(label), B, ptr<float>(pred), ptr<float>(dz),
                    ptr<float>(loss), reinterpret_cast<uint32_t*>(ws.data_ptr()), cur_stream());
  return {loss, pred, dz};
}

static void auc_accumulate(const Tensor& pred, const Tensor& label, const c10::optional<Tensor>& mask, Tensor table,
                           Tensor stats) {
  check_cuda(pred, "pred");
  check_cuda(table, "table");
  PBX_CHECK(table.scalar_type() == torch::kFloat64 && stats.scalar_type() == torch::kFloat64, "auc tables are f64");
  launch_auc_accumulate(ptr<float>(pred), ptr<float>(label), optr<float>(mask), (int)pred.numel(),
                        (int)(table.numel() / 2), ptr<double>(table), ptr<double>(stats), cur_stream());
}

static void adam_flat(Tensor p, Tensor g, Tensor m, Tensor v, Tensor pows, float lr, float b1, float b2,
                      float eps, float grad_scale, float wd, bool clear_grad) {
  check_cuda(p, "p");
  PBX_CHECK(p.numel() == g.numel() && p.numel() == m.numel() && p.numel() == v.numel(), "adam sizes");
  PBX_CHECK(pows.is_cuda() && pows.numel() >= 2 && pows.scalar_type() == torch::kFloat32, "adam pows");
  launch_adam_flat(ptr<float>(p), ptr<float>(g), ptr<float>(m), ptr<float>(v), p.numel(), lr, b1, b2, eps,
                   ptr<float>(pows), grad_scale, wd, clear_grad, cur_stream());
}

}  // namespace pbx

namespace pbx {
void bind_tower(py::module& m);
void bind_ctr(py::module& m);
void bind_cross(py::module& m);
void bind_ipc(py::module& m);
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  using namespace pbx;
  bind_tower(m);
  bind_ctr(m);
  bind_cross(m);
  bind_ipc(m);
  m.doc() = "PaddleBox-capability engine: hand-written gfx950 (MI355X) kernels";
  py::class_<SparseSGDConfig>(m, "SparseSGDConfig")
      .def(py::init<>())
      .def_readwrite("nonclk_coeff", &SparseSGDConfig::nonclk_coeff)
      .def_readwrite("clk_coeff", &SparseSGDConfig::clk_coeff)
      .def_readwrite("min_bound", &SparseSGDConfig::min_bound)
      .def_readwrite("max_bound", &SparseSGDConfig::max_bound)
      .def_readwrite("learning_rate", &SparseSGDConfig::learning_rate)
      .def_readwrite("initial_g2sum", &SparseSGDConfig::initial_g2sum)
      .def_readwrite("initial_range", &SparseSGDConfig::initial_range)
      .def_readwrite("mf_create_thresholds", &SparseSGDConfig::mf_create_thresholds)
      .def_readwrite("mf_learning_rate", &SparseSGDConfig::mf_learning_rate)
      .def_readwrite("mf_initial_g2sum", &SparseSGDConfig::mf_initial_g2sum)
      .def_readwrite("mf_initial_range", &SparseSGDConfig::mf_initial_range)
      .def_readwrite("mf_min_bound", &SparseSGDConfig::mf_min_bound)
      .def_readwrite("mf_max_bound", &SparseSGDConfig::mf_max_bound)
      .def_readwrite("nodeid_slot", &SparseSGDConfig::nodeid_slot)
      .def_readwrite("feature_learning_rate", &SparseSGDConfig::feature_learning_rate)
      .def_readwrite("use_feature_lr", &SparseSGDConfig::use_feature_lr);
  py::class_<ShrinkConfig>(m, "ShrinkConfig")
      .def(py::init<>())
      .def_readwrite("show_click_decay_rate", &ShrinkConfig::show_click_decay_rate)
      .def_readwrite("delete_threshold", &ShrinkConfig::delete_threshold)
      .def_readwrite("delete_after_unseen_days", &ShrinkConfig::delete_after_unseen_days)
      .def_readwrite("nonclk_coeff", &ShrinkConfig::nonclk_coeff)
      .def_readwrite("clk_coeff", &ShrinkConfig::clk_coeff);
  py::class_<CodecDev>(m, "Codec")
      .def(py::init([](int kind, int D, int De, float qscale, float beta1, float beta2, float eps) {
             PBX_CHECK(kind >= 0 && kind <= 3, "codec kind 0/1/2/3");
             PBX_CHECK(D >= 1 && De >= 0 && D + De <= 256, "codec dims");
             return make_codec(kind, D, De, qscale, beta1, beta2, eps);
           }),
           py::arg("kind"), py::arg("D"), py::arg("De") = 0, py::arg("qscale") = 1.f, py::arg("beta1") = 0.9f,
           py::arg("beta2") = 0.999f, py::arg("eps") = 1e-8f)
      .def_readonly("kind", &CodecDev::kind)
      .def_readonly("D", &CodecDev::D)
      .def_readonly("De", &CodecDev::De)
      .def_readonly("Wx", &CodecDev::Wx)
      .def_readonly("We", &CodecDev::We)
      .def_readonly("qscale", &CodecDev::qscale)
      .def_readonly("mf", &CodecDev::mf)
      .def_readonly("eg2", &CodecDev::eg2)
      .def_readonly("adam", &CodecDev::adam)
      .def_readonly("xsz", &CodecDev::xsz)
      // kind 3: bitmap (int32 device tensor, kept alive by the caller) of
      // the slot ids whose new features get De columns
      .def("set_expand_slots",
           [](CodecDev& c, const Tensor& bm) {
             check_cuda(bm, "bitmap");
             PBX_CHECK(bm.scalar_type() == torch::kInt32 && bm.is_contiguous(), "bitmap must be int32");
             c.vslots = reinterpret_cast<const uint32_t*>(bm.data_ptr());
             c.vslot_bits = (int)bm.numel() * 32;
           })
      .def_readonly("extra", &CodecDev::extra)
      .def_property_readonly("storage_dim", [](const CodecDev& c) { return c.Wx + c.We; });
  py::class_<GpuTable>(m, "GpuTable")
      .def(py::init<int, int64_t, int64_t, int, int>(), py::arg("dim"), py::arg("capacity"),
           py::arg("stash_cap") = 4096, py::arg("device") = 0, py::arg("extra") = 0)
      .def("probe", &GpuTable::probe, py::arg("h"), py::arg("n_dev") = py::none())
      .def("insert", &GpuTable::insert, py::arg("h"), py::arg("n_dev"), py::arg("cfg"), py::arg("seed"),
           py::arg("init_embedx"))
      .def("last_overflow", &GpuTable::last_overflow)
      .def("size", &GpuTable::size)
      .def("stash_n", &GpuTable::stash_n)
      .def("error_bits", &GpuTable::error_bits)
      .def("clear_error", &GpuTable::clear_error)
      .def("probe_into", &GpuTable::probe_into)
      .def("export_all", &GpuTable::export_all)
      .def("assign", &GpuTable::assign)
      .def("shrink", &GpuTable::shrink)
      .def("gather_pull", &GpuTable::gather_pull, py::arg("rows"), py::arg("n_dev"), py::arg("out_stride"))
      .def("push_adagrad", &GpuTable::push_adagrad)
      .def("gather_rows_by_uid", &GpuTable::gather_rows_by_uid)
      .def("push_adagrad_seg", &GpuTable::push_adagrad_seg)
      .def("push_merge_apply", &GpuTable::push_merge_apply)
      .def("probe_gather", &GpuTable::probe_gather)
      .def("answer_exchange", &GpuTable::answer_exchange)
      .def("probe_raw", &GpuTable::probe_raw)
      .def("save_stream", &GpuTable::save_stream)
      .def_property_readonly_static("occ_replicas", [](py::object) { return kOccRep; })
      .def("push_occ", &GpuTable::push_occ)
      .def("owner_push", &GpuTable::owner_push)
      .def("codec_pull", &GpuTable::codec_pull, py::arg("codec"), py::arg("rows"), py::arg("uid"), py::arg("n_dev"),
           py::arg("n"), py::arg("out"))
      .def("codec_update", &GpuTable::codec_update)
      .def("codec_init", &GpuTable::codec_init)
      .def_property_readonly("stride", &GpuTable::stride)
      .def("copy_from", &GpuTable::copy_from)
      .def("clear", &GpuTable::clear)
      .def_property_readonly("keys", &GpuTable::keys)
      .def_property_readonly("values", &GpuTable::values)
      .def_property_readonly("fill", &GpuTable::fill)
      .def_property_readonly("dim", &GpuTable::dim)
      .def_property_readonly("stride", &GpuTable::stride)
      .def_property_readonly("capacity", &GpuTable::capacity)
      .def_property_readonly("nbuckets", &GpuTable::nbuckets);
  py::class_<DedupWorkspace>(m, "DedupWorkspace")
      .def(py::init<int64_t, int, bool>(), py::arg("cap"), py::arg("device"), py::arg("hash") = true)
      .def("run", &DedupWorkspace::run, py::arg("keys"), py::arg("mixed") = false, py::arg("zero") = py::none())
      .def("run_table", &DedupWorkspace::run_table, py::arg("keys"), py::arg("table"), py::arg("rows_given") = false,
           py::arg("defer_scatter") = false, py::arg("stage") = 0)
      .def("table_rows_occ", &DedupWorkspace::table_rows_occ)
      .def("clean_rows_occ", &DedupWorkspace::clean_rows_occ)
      .def_readonly("rows_occ_dirty", &DedupWorkspace::rows_occ_dirty)
      .def_readonly("rows_u", &DedupWorkspace::rows_u)
      .def_readonly("rows_occ", &DedupWorkspace::rows_occ)
      .def_readonly("hash", &DedupWorkspace::hash)
      .def_readonly("cap", &DedupWorkspace::cap)
      .def_readonly("h_sorted", &DedupWorkspace::h_sorted)
      .def_readonly("perm", &DedupWorkspace::perm)
      .def_readonly("uid", &DedupWorkspace::uid)
      .def_readonly("uniq_h", &DedupWorkspace::uniq_h)
      .def_readonly("seg", &DedupWorkspace::seg)
      .def_readonly("cnt", &DedupWorkspace::cnt)
      .def_readonly("u_count", &DedupWorkspace::u_count);
  py::class_<MlpWorkspace>(m, "MlpWorkspace")
      .def(py::init<int64_t, std::vector<int64_t>, int, int64_t>(), py::arg("M"), py::arg("dims"),
           py::arg("device"), py::arg("k_split") = 1024)
      .def("forward", &MlpWorkspace::forward)
      .def("backward", &MlpWorkspace::backward)
      .def("x", &MlpWorkspace::x)
      .def("xt", &MlpWorkspace::xt)
      .def("dz", &MlpWorkspace::dz)
      .def("dx0", &MlpWorkspace::dx0)
      .def_property_readonly("M", &MlpWorkspace::M);
  m.attr("kSaveMaxCols") = kSaveMaxCols;
  m.def("fill_occurrence", &fill_occurrence);
  m.def("guard_bits", &guard_bits_get);
  m.def("clear_guard_bits", &guard_bits_clear);
  m.def("seqpool_cvm_fwd", &seqpool_cvm_fwd, py::arg("src"), py::arg("src_index"), py::arg("uid"), py::arg("lod"),
        py::arg("S"), py::arg("B"), py::arg("E"), py::arg("out"), py::arg("col_offset"), py::arg("use_cvm"),
        py::arg("cvm_offset"), py::arg("clk_filter"), py::arg("pad_value"), py::arg("need_filter"),
        py::arg("show_coeff"), py::arg("clk_coeff"), py::arg("threshold"), py::arg("quant_ratio"),
        py::arg("embed_threshold_filter"), py::arg("embed_threshold"), py::arg("embed_thres_size"),
        py::arg("dense") = py::none(), py::arg("dense_col") = 0, py::arg("occ_slot") = py::none(),
        py::arg("occ_ins") = py::none(), py::arg("probe_keys") = py::none(),
        py::arg("probe_table") = static_cast<GpuTable*>(nullptr), py::arg("rows_out") = py::none(),
        py::arg("scatter_ws") = static_cast<DedupWorkspace*>(nullptr));
  m.def("push_merge", &push_merge, py::arg("dout"), py::arg("col_offset"), py::arg("cvm"), py::arg("cvm_offset"),
        py::arg("use_cvm"), py::arg("clk_filter"), py::arg("E"), py::arg("perm"), py::arg("uid"), py::arg("occ_slot"),
        py::arg("occ_ins"), py::arg("slot_ids"), py::arg("n_valid"), py::arg("push"), py::arg("push_index"),
        py::arg("bs_scale"), py::arg("dim"), py::arg("embed_thres_size") = 0);
  m.def("push_merge_send", &push_merge_send);
  m.def("push_merge_records", &push_merge_records);
  m.def("shard_pack", &shard_pack);
  m.def("shard_pack_hash", &shard_pack_hash, py::arg("uniq_h"), py::arg("u_count"), py::arg("nranks"), py::arg("cap"),
        py::arg("send"), py::arg("send_index"), py::arg("ocnt"), py::arg("overflow"), py::arg("prezeroed") = false);
  m.def("gather_by_uid", &gather_by_uid);
  m.def("data_norm_fwd", &data_norm_fwd);
  m.def("data_norm_bwd", &data_norm_bwd);
  m.def("data_norm_update", &data_norm_update);
  m.def("head_fwd", &head_fwd, py::arg("x"), py::arg("S"), py::arg("Eo"), py::arg("ew_col"), py::arg("D"),
        py::arg("Cp"), py::arg("bsize"), py::arg("bsum"), py::arg("bsq"), py::arg("y_out") = py::none(),
        py::arg("yT_out") = py::none(), py::arg("ymp_out") = py::none(), py::arg("stat_part") = py::none());
  m.def("head_blocks", &head_blocks);
  m.def("head_bwd", &head_bwd, py::arg("x"), py::arg("dy"), py::arg("dlin"), py::arg("S"), py::arg("Eo"),
        py::arg("ew_col"), py::arg("D"), py::arg("Cp"), py::arg("means"), py::arg("scales"), py::arg("eps"),
        py::arg("dlin_scale") = py::none(), py::arg("want_stats") = true);
  m.def("linear_fwd", &linear_fwd);
  m.def("linear_bwd", &linear_bwd);
  m.def("gemv_out", &gemv_out);
  m.def("gemv_out_bwd", &gemv_out_bwd);
  m.def("cast_bf16", &cast_bf16);
  m.def("fm_fwd", &fm_fwd);
  m.def("fm_bwd", &fm_bwd);
  m.def("sigmoid_logloss", &sigmoid_logloss);
  m.def("auc_accumulate", &auc_accumulate);
  m.def("logit_loss", &logit_loss, py::arg("a"), py::arg("b"), py::arg("label"), py::arg("ws"));
  m.def("adam_flat", &adam_flat, py::arg("p"), py::arg("g"), py::arg("m"), py::arg("v"), py::arg("pows"),
        py::arg("lr"), py::arg("b1"), py::arg("b2"), py::arg("eps"), py::arg("grad_scale"), py::arg("wd"),
        py::arg("clear_grad") = false);
  m.def("mix64", [](uint64_t k) { return mix64(k); });
  m.def("unmix64", [](uint64_t k) { return unmix64(k); });
}

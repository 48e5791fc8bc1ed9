// torch glue for the fused dense tower (tower.hip) and the fused Adam.
// Buffers live in a persistent TowerWorkspace (fixed batch M and widths), so
// a captured training step replays against stable addresses.
#include <ATen/hip/HIPContext.h>
#include <torch/extension.h>

#include <cstdlib>
#include <stdexcept>

#include "kernels.h"
#include "tower32_sched.h"

namespace py = pybind11;
using torch::Tensor;

namespace pbx {
namespace {

hipStream_t stream() { return at::hip::getCurrentHIPStream().stream(); }

#define TW_CHECK(cond, msg)                                                 \
  do {                                                                      \
    if (!(cond)) throw std::runtime_error(std::string("pbx tower: ") + msg); \
  } while (0)

template <typename T>
T* P(const Tensor& t) {
  return reinterpret_cast<T*>(t.data_ptr());
}
template <typename T>
T* OP(const c10::optional<Tensor>& t) {
  return t.has_value() && t->defined() ? reinterpret_cast<T*>(t->data_ptr()) : nullptr;
}
unsigned short* BP(const Tensor& t) { return reinterpret_cast<unsigned short*>(t.data_ptr()); }
int64_t pad(int64_t v, int64_t a) { return (v + a - 1) / a * a; }

void check_f32(const Tensor& t, int64_t numel, const char* what) {
  TW_CHECK(t.is_cuda() && t.is_contiguous() && t.scalar_type() == torch::kFloat32, std::string(what) + ": f32 GPU");
  TW_CHECK(numel < 0 || t.numel() == numel, std::string(what) + ": size");
}

}  // namespace

class TowerWorkspace {
 public:
  // fp32 = true: the exact-fp32 tower (tower32.hip, reference fc precision):
  // fp32 activations / weights, widths padded to 16, Mp to 256
  // x3 = true (with fp32 = false): fp32 precision on bf16 MFMA (tower_x3.hip):
  // the bf16 layouts with lo twins, fp32 X0 / dX0 rows, dW one writer per tile
  TowerWorkspace(int64_t M, std::vector<int64_t> dims, int device, int64_t dw_splits, bool fp32, bool x3)
      : M_(M), dims_(dims), splits_(dw_splits), fp32_(fp32), x3_(x3) {
    TW_CHECK(!(fp32 && x3), "fp32 and x3 are different towers");
    if (x3) TW_CHECK(dw_splits == 1 || dw_splits == 2 || dw_splits == 4, "x3 dw_splits in {1, 2, 4}");
    TW_CHECK(dims.size() >= 2 && dims.size() - 1 <= (size_t)kMaxTowerLayers, "1..8 hidden layers");
    TW_CHECK(M > 0, "M > 0");
    if (fp32) TW_CHECK(dw_splits == 1 || dw_splits == 2 || dw_splits == 4 || dw_splits == 8, "dw_splits in {1,2,4,8}");
    else TW_CHECK(dw_splits == 1 || dw_splits == 2 || dw_splits == 4, "dw_splits in {1, 2, 4}");
    const int64_t wmax = fp32 ? kTower32MaxWidth : 2048;
    for (auto d : dims) TW_CHECK(d > 0 && d <= wmax, "layer widths exceed the fused tower's limit");
    auto ob = torch::TensorOptions().dtype(fp32 ? torch::kFloat32 : torch::kBFloat16).device(torch::kCUDA, device);
    const int64_t tw = x3 ? 2 : 1;  // x3: hi + lo halves of every bf16 buffer
    auto of = torch::TensorOptions().dtype(torch::kFloat32).device(torch::kCUDA, device);
    auto oi = torch::TensorOptions().dtype(torch::kInt32).device(torch::kCUDA, device);
    wpad_ = fp32 ? 16 : 32;
    L_ = (int)dims.size() - 1;
    int64_t maxw = 0;
    for (auto d : dims) maxw = std::max(maxw, pad(d, wpad_));
    if (fp32) {
      Mp_ = pad(M, 256);  // the dW splits walk whole 2-step (32-row) ring stages
      lds_ld_ = tower32_lds_ld((int)maxw);
      bool part = false;  // wave-stream remainder scratch (tower32.hip): some column count not a multiple of 128
      for (auto d : dims) part = part || (pad(d, 16) / 16) % 8 != 0;
      int64_t nbias = 0;
      for (size_t l = 1; l < dims.size(); ++l) nbias += pad(dims[l], 16);
      TW_CHECK(tower32_lds_bytes_for(lds_ld_, part, 0) + kTower32BwdStatic <= kTower32LdsTotal &&
                   tower32_lds_bytes_for(lds_ld_, part, (int)nbias) + 512 <= kTower32LdsTotal,
               "widths exceed the fp32 LDS tile budget");
    } else {
      Mp_ = tower_nwg((int)M) * 32;
      // each split walks a whole number of 4-step (64-row) ring stages; a small
      // batch that cannot be cut in 4 falls back to 2 (always valid: Mp % 128 == 0)
      if ((Mp_ / 16) % (4 * splits_) != 0) splits_ = 2;
      lds_ld_ = (int)maxw + 8;
      TW_CHECK((size_t)2 * tw * 32 * lds_ld_ * 2 <= 150 * 1024, "widths exceed the LDS tile budget");
    }
    const int64_t K0p = pad(dims[0], wpad_);
    x0_ = torch::zeros({M, K0p}, x3 ? of : ob);
    x0mp_ = torch::zeros({tw * Mp_ * K0p}, ob);
    dx0_ = torch::zeros({M, K0p}, x3 ? of : ob);
    int64_t boff = 0;
    for (int l = 0; l < L_; ++l) {
      const int64_t Kp = pad(dims[l], wpad_), Np = pad(dims[l + 1], wpad_);
      // fp32: the wave-stream layout (tower32_sched.h: per-wave streams,
      // units / segments padded to the ring depth) + slack for the weight
      // ring, which loads kT32Ring steps (2 KB each) past a stream's end
      const int64_t slack = 256 * 2 * 2 * kT32Ring;
      const int64_t n_wp = fp32 ? t32_stream_groups((int)(Np / 16), (int)(Kp / 16)) * 256 + slack : tw * Np * Kp;
      const int64_t n_wtp = fp32 ? t32_stream_groups((int)(Kp / 16), (int)(Np / 16)) * 256 + slack : tw * Np * Kp;
      wp_.push_back(torch::zeros({n_wp}, ob));
      wtp_.push_back(torch::zeros({n_wtp}, ob));
      if (fp32) {
        // group position of every (column block, k-group) of the wave-stream
        // layout, for the per-step re-pack in the fused Adam (the closed form
        // walks the schedule: ~100s of integer ops per element)
        const int nb = (int)(Np / 16), kb = (int)(Kp / 16);
        auto pos = torch::empty({(int64_t)nb * kb}, torch::kInt32), posT = torch::empty({(int64_t)kb * nb}, torch::kInt32);
        for (int c = 0; c < nb; ++c)
          for (int g = 0; g < kb; ++g) pos.data_ptr<int>()[c * kb + g] = (int)t32_group_pos(nb, kb, c, g);
        for (int c = 0; c < kb; ++c)
          for (int g = 0; g < nb; ++g) posT.data_ptr<int>()[c * nb + g] = (int)t32_group_pos(kb, nb, c, g);
        pos_.push_back(pos.to(x0_.device()));
        posT_.push_back(posT.to(x0_.device()));
      }
      xmp_.push_back(torch::zeros({tw * Mp_ * Np}, ob));
      dzmp_.push_back(torch::zeros({tw * Mp_ * Np}, ob));
      boff_.push_back(boff);
      boff += Np;
    }
    dwout_off_ = (int)boff;
    dbout_off_ = (int)(boff + pad(dims[L_], wpad_));
    bias_ld_ = dbout_off_ + 1;
    const int nwg = (int)(Mp_ / 32);
    bias_part_ = torch::zeros({nwg, bias_ld_}, of);
    pred_ = torch::zeros({M}, of);
    dz_ = torch::zeros({M}, of);
    loss_ = torch::zeros({1}, of);
    part_ = torch::zeros({nwg * 8}, of);
    ticket_ = torch::zeros({1}, oi);
    if (x3 && splits_ > 1) {
      // split-M dW slabs + per-tile arrival counters (tower_x3.hip k_tx3_dw)
      int64_t tiles = 0;
      for (int l = 0; l < L_; ++l) tiles += ((pad(dims[l + 1], 32) + 63) / 64) * ((pad(dims[l], 32) + 63) / 64);
      dw_slab_ = torch::empty({tiles * splits_ * 4096}, of);
      dw_cnt_ = torch::zeros({tiles}, oi);
    }
    if (fp32 && splits_ > 1) {
      // split-M dW slabs + per-tile arrival counters (tower32.hip t32_dw_combine)
      int64_t tiles = 0;
      for (int l = 0; l < L_; ++l)
        tiles += ((pad(dims[l + 1], 16) / 16 + 3) / 4) * ((pad(dims[l], 16) / 16 + 3) / 4);
      dw_slab_ = torch::empty({tiles * splits_ * 4096}, of);
      dw_cnt_ = torch::zeros({tiles}, oi);
    }
  }

  // fp32 master weights W_l [N_l][K_l] -> packed bf16 copies (one launch)
  void pack(const std::vector<Tensor>& W) {
    TW_CHECK((int)W.size() == L_, "pack: layer count");
    TowerArgs a = base();
    const float* w[kMaxTowerLayers];
    for (int l = 0; l < L_; ++l) {
      check_f32(W[l], dims_[l + 1] * dims_[l], "W");
      w[l] = P<float>(W[l]);
    }
    if (fp32_) launch_tower32_pack(a, w, stream());
    else if (x3_) launch_tower_x3_pack(a, w, stream());
    else launch_tower_pack(a, w, stream());
  }

  std::vector<Tensor> forward(const std::vector<Tensor>& b, const Tensor& w_out, const Tensor& b_out,
                              const c10::optional<Tensor>& lin, const Tensor& label,
                              const c10::optional<Tensor>& auc_table, const c10::optional<Tensor>& auc_stats,
                              const c10::optional<Tensor>& auc_mask) {
    TW_CHECK((int)b.size() == L_, "forward: layer count");
    TowerArgs a = base();
    for (int l = 0; l < L_; ++l) {
      check_f32(b[l], dims_[l + 1], "bias");
      a.ly[l].bias = P<float>(b[l]);
    }
    check_f32(w_out, dims_[L_], "w_out");
    check_f32(b_out, 1, "b_out");
    // the label may be a column view of the batch's dense block: [M] or
    // [M, 1] with any row stride (read strided by the loss tail, no copy)
    TW_CHECK(label.is_cuda() && label.scalar_type() == torch::kFloat32 && label.numel() == M_ &&
                 (label.dim() == 1 || (label.dim() == 2 && label.size(1) == 1)),
             "label: f32 GPU [M] / [M, 1]");
    a.w_out = P<float>(w_out);
    a.b_out = P<float>(b_out);
    if (lin.has_value() && lin->defined()) check_f32(*lin, M_, "lin");
    a.lin = OP<float>(lin);
    a.label = P<float>(label);
    a.label_stride = (int)label.stride(0);
    if (auc_table.has_value() && auc_table->defined()) {
      TW_CHECK(auc_table->scalar_type() == torch::kFloat64 && auc_stats.has_value() &&
                   auc_stats->scalar_type() == torch::kFloat64 && auc_stats->numel() >= 5,
               "auc tables are f64 [2, T] / [5]");
      a.auc_table = OP<double>(auc_table);
      a.auc_stats = OP<double>(auc_stats);
      a.auc_buckets = (int)(auc_table->numel() / 2);
      a.auc_mask = OP<float>(auc_mask);
    }
    if (stamps_.defined()) a.stamps = reinterpret_cast<long long*>(stamps_.data_ptr());
    if (fp32_) launch_tower32_fwd(a, stream());
    else if (x3_) launch_tower_x3_fwd(a, stream());
    else launch_tower_fwd(a, stream());
    return {loss_, pred_, dz_};
  }

  // Parameter grads are ACCUMULATED (+=) into dW/db/dw_out/db_out.  Optional
  // data_norm stat partials [dn_rows][2C] are reduced into dn_stats [3, C].
  Tensor backward(const c10::optional<Tensor>& dloss, const Tensor& w_out, const std::vector<Tensor>& dW,
                  const std::vector<Tensor>& db, const Tensor& dw_out, const Tensor& db_out, bool need_dx,
                  const c10::optional<Tensor>& dn_part,
                  int64_t dn_rows, double dn_eps, const c10::optional<Tensor>& dn_stats, int64_t parts,
                  const c10::optional<Tensor>& dn_bsize, const c10::optional<Tensor>& dn_bsum,
                  const c10::optional<Tensor>& dn_bsq, double dn_decay, const c10::optional<Tensor>& head_x,
                  const c10::optional<Tensor>& head_scales, int64_t hS, int64_t hEo, int64_t hew, int64_t hD,
                  bool hlin) {
    TW_CHECK((int)dW.size() == L_ && (int)db.size() == L_, "backward: layer count");
    TowerArgs a = base();
    Tensor hdx;
    if (head_x.has_value() && head_x->defined() && (parts & 1)) {
      // x3: the DeepFM head backward fused into the dX0 epilogue
      TW_CHECK(x3_ && need_dx, "fused head backward: x3 tower with dX0 only");
      check_f32(*head_x, -1, "head_x");
      TW_CHECK(head_x->dim() == 2 && head_x->size(0) == M_ && head_x->size(1) <= pad(dims_[0], wpad_) &&
                   hD >= 0 && hD <= 16 && hS >= 0 && hS * hEo <= head_x->size(1) && (hS == 0 || hew + hD < hEo),
               "head_x: [M, C <= K0p], D <= 16, slot blocks inside the row");
      hdx = torch::empty_like(*head_x);
      a.hx = P<float>(*head_x);
      a.hdx = P<float>(hdx);
      a.hC = (int)head_x->size(1);
      if (head_scales.has_value() && head_scales->defined()) {
        check_f32(*head_scales, a.hC, "head_scales");
        a.hscales = P<float>(*head_scales);
      }
      a.hS = (int)hS;
      a.hEo = (int)hEo;
      a.hew = (int)hew;
      a.hD = (int)hD;
      a.hlin = hlin ? 1 : 0;
    }
    for (int l = 0; l < L_; ++l) {
      check_f32(dW[l], dims_[l + 1] * dims_[l], "dW");
      check_f32(db[l], dims_[l + 1], "db");
      a.ly[l].dw = P<float>(dW[l]);
      a.ly[l].db = P<float>(db[l]);
    }
    check_f32(w_out, dims_[L_], "w_out");
    check_f32(dw_out, dims_[L_], "dw_out");
    check_f32(db_out, 1, "db_out");
    a.w_out = P<float>(w_out);  // dX_L = g w_out^T
    a.dw_out = P<float>(dw_out);
    a.db_out = P<float>(db_out);
    a.dloss = OP<float>(dloss);
    a.need_dx0 = need_dx ? 1 : 0;
    if (fp32_ || x3_) a.dx0f = P<float>(dx0_);
    else a.dx0 = BP(dx0_);
    a.lddx0 = (int)dx0_.size(1);
    if (dn_part.has_value() && dn_part->defined()) {
      TW_CHECK(dn_stats.has_value() && dn_stats->defined(), "dn_stats required with dn_part");
      const int C = (int)(dn_stats->numel() / 3);
      TW_CHECK(dn_part->numel() >= dn_rows * 2 * C, "dn_part size");
      a.dn_part = OP<float>(dn_part);
      a.dn_rows = (int)dn_rows;
      a.dn_C = C;
      a.dn_eps = (float)dn_eps;
      a.dn_stats = OP<float>(dn_stats);
      if (dn_bsize.has_value() && dn_bsize->defined()) {
        check_f32(*dn_bsize, C, "dn_bsize");
        check_f32(*dn_bsum, C, "dn_bsum");
        check_f32(*dn_bsq, C, "dn_bsq");
        a.dn_bsize = P<float>(*dn_bsize);
        a.dn_bsum = P<float>(*dn_bsum);
        a.dn_bsq = P<float>(*dn_bsq);
        a.dn_decay = (float)dn_decay;
      }
    }
    // parts: bit 0 = dX chain (k_tower_bwd), bit 1 = dW / bias / data_norm
    // reductions (k_tower_dw); the caller may issue them on different streams
    // (dW overlapped with the head backward + sparse push), bwd first
    auto s = stream();
    if (fp32_) {
      if (parts & 1) launch_tower32_bwd(a, s);
      if (parts & 2) launch_tower32_dw(a, s);
    } else if (x3_) {
      if (parts & 1) launch_tower_x3_bwd(a, s);
      if (parts & 2) launch_tower_x3_dw(a, s);
    } else {
      if (parts & 1) launch_tower_bwd(a, s);
      if (parts & 2) launch_tower_dw(a, s);
    }
    if (hdx.defined()) return hdx;
    return need_dx ? dx0_ : Tensor();
  }

  // (wp, wtp, N, K, Np, Kp) per layer, for the optimizer's fused re-pack
  std::vector<py::tuple> pack_regions() const {
    std::vector<py::tuple> r;
    for (int l = 0; l < L_; ++l)
      r.push_back(py::make_tuple(wp_[l], wtp_[l], dims_[l + 1], dims_[l], pad(dims_[l + 1], wpad_), pad(dims_[l], wpad_),
                                 fp32_ ? py::object(py::cast(pos_[l])) : py::object(py::none()),
                                 fp32_ ? py::object(py::cast(posT_[l])) : py::object(py::none()), x3_));
    return r;
  }

  Tensor x0() const { return x0_; }
  Tensor x0mp() const { return x0mp_; }
  Tensor xmp(int l) const { return xmp_.at(l); }
  Tensor dzmp(int l) const { return dzmp_.at(l); }
  Tensor dx0() const { return dx0_; }
  Tensor wp(int l) const { return wp_.at(l); }
  Tensor wtp(int l) const { return wtp_.at(l); }
  int64_t M() const { return M_; }
  int64_t Mp() const { return Mp_; }
  int64_t K0p() const { return pad(dims_[0], wpad_); }
  // timing experiments: per-wave s_memtime stamps of the fp32 forward
  void set_stamps(const Tensor& t) { stamps_ = t; }
  bool fp32() const { return fp32_; }
  bool x3() const { return x3_; }
  int64_t dw_splits() const { return splits_; }
  int64_t lds_ld() const { return lds_ld_; }

 private:
  TowerArgs base() const {
    TowerArgs a;
    a.M = (int)M_;
    a.Mp = (int)Mp_;
    a.L = L_;
    a.lds_ld = lds_ld_;
    a.ld0 = (int)x0_.size(1);
    a.f32 = fp32_ ? 1 : 0;
    if (fp32_) {
      a.x0f = P<float>(x0_);
      a.x0mpf = P<float>(x0mp_);
    } else if (x3_) {
      a.x0f = P<float>(x0_);
      a.x0mp = BP(x0mp_);
    } else {
      a.x0 = BP(x0_);
      a.x0mp = BP(x0mp_);
    }
    for (int l = 0; l < L_; ++l) {
      TowerLayerDev& d = a.ly[l];
      if (fp32_) {
        d.wpf = P<float>(wp_[l]);
        d.wtpf = P<float>(wtp_[l]);
        d.xmpf = P<float>(xmp_[l]);
        d.dzmpf = P<float>(dzmp_[l]);
      } else {
        d.wp = BP(wp_[l]);
        d.wtp = BP(wtp_[l]);
        d.xmp = BP(xmp_[l]);
        d.dzmp = BP(dzmp_[l]);
      }
      d.K = (int)dims_[l];
      d.N = (int)dims_[l + 1];
      d.Kp = (int)pad(dims_[l], wpad_);
      d.Np = (int)pad(dims_[l + 1], wpad_);
      d.bias_off = (int)boff_[l];
    }
    a.pred = P<float>(pred_);
    a.dz = P<float>(dz_);
    a.loss = P<float>(loss_);
    a.part = P<float>(part_);
    a.ticket = reinterpret_cast<unsigned int*>(ticket_.data_ptr());
    a.bias_part = P<float>(bias_part_);
    a.bias_ld = bias_ld_;
    a.dwout_off = dwout_off_;
    a.dbout_off = dbout_off_;
    a.dw_splits = (int)splits_;
    if (dw_slab_.defined()) {
      a.dw_slab = P<float>(dw_slab_);
      a.dw_cnt = P<int>(dw_cnt_);
    }
    static const int dbg = [] {
      const char* e = getenv("PBX_TOWER_DEBUG");
      return e ? atoi(e) : 0;
    }();
    a.debug = dbg;
    return a;
  }

  int64_t M_, Mp_ = 0;
  std::vector<int64_t> dims_;
  int64_t splits_;
  bool fp32_ = false, x3_ = false;
  int64_t wpad_ = 32;
  int L_ = 0, lds_ld_ = 0, bias_ld_ = 0, dwout_off_ = 0, dbout_off_ = 0;
  std::vector<int64_t> boff_;
  Tensor x0_, x0mp_, dx0_, bias_part_, pred_, dz_, loss_, part_, ticket_, stamps_, dw_slab_, dw_cnt_;
  std::vector<Tensor> wp_, wtp_, xmp_, dzmp_;
  std::vector<Tensor> pos_, posT_;  // fp32: wave-stream group position per (column block, k-group), W and W^T
};

// Adam over the flat arena + fused extras (see kernels.h AdamExtras).
// pack: [(arena_offset, wp, wtp, N, K, Np, Kp)], dn: [(stats, bsize, bsum, bsq, decay)]
static void adam_fused(Tensor p, Tensor g, Tensor m, Tensor v, Tensor pows, Tensor ticket, double lr, double b1,
                       double b2, double eps, double grad_scale, double wd, bool clear_grad,
                       const std::vector<py::tuple>& pack, const std::vector<py::tuple>& dn) {
  check_f32(p, -1, "p");
  TW_CHECK(g.numel() >= p.numel() && m.numel() == p.numel() && v.numel() == p.numel(), "adam sizes");
  TW_CHECK(pows.is_cuda() && pows.numel() >= 2 && pows.scalar_type() == torch::kFloat32, "adam pows");
  TW_CHECK(ticket.is_cuda() && ticket.scalar_type() == torch::kInt32, "adam ticket");
  TW_CHECK(pack.size() <= (size_t)kMaxPackRegions && dn.size() <= (size_t)kMaxDnUpdates, "too many extras");
  AdamExtras x;
  x.n_pack = (int)pack.size();
  for (size_t i = 0; i < pack.size(); ++i) {
    const auto& t = pack[i];
    x.pack_off[i] = t[0].cast<int64_t>();
    auto wpt = t[1].cast<Tensor>(), wtpt = t[2].cast<Tensor>();
    if (wpt.scalar_type() == torch::kFloat32) {  // fp32 tower region
      x.pack_wp[i] = x.pack_wtp[i] = nullptr;
      x.pack_wp32[i] = P<float>(wpt);
      x.pack_wtp32[i] = P<float>(wtpt);
    } else {
      x.pack_wp[i] = BP(wpt);
      x.pack_wtp[i] = BP(wtpt);
      x.pack_wp32[i] = x.pack_wtp32[i] = nullptr;
    }
    x.pack_pos32[i] = x.pack_posT32[i] = nullptr;
    if (t.size() >= 9 && !t[7].is_none()) {
      x.pack_pos32[i] = P<int>(t[7].cast<Tensor>());
      x.pack_posT32[i] = P<int>(t[8].cast<Tensor>());
    }
    x.pack_x3[i] = (t.size() >= 10 && !t[9].is_none() && t[9].cast<bool>()) ? 1 : 0;
    x.pack_N[i] = t[3].cast<int>();
    x.pack_K[i] = t[4].cast<int>();
    x.pack_Np[i] = t[5].cast<int>();
    x.pack_Kp[i] = t[6].cast<int>();
    TW_CHECK(x.pack_off[i] >= 0 && x.pack_off[i] + (int64_t)x.pack_N[i] * x.pack_K[i] <= p.numel(), "pack range");
  }
  x.n_dn = (int)dn.size();
  for (size_t i = 0; i < dn.size(); ++i) {
    const auto& t = dn[i];
    auto st = t[0].cast<Tensor>();
    auto bs = t[1].cast<Tensor>();
    x.dn_C[i] = (int)bs.numel();
    TW_CHECK(st.numel() == 3 * bs.numel(), "dn stats must be [3, C]");
    x.dn_stats[i] = P<float>(st);
    x.dn_bsize[i] = P<float>(bs);
    x.dn_bsum[i] = P<float>(t[2].cast<Tensor>());
    x.dn_bsq[i] = P<float>(t[3].cast<Tensor>());
    x.dn_decay[i] = t[4].cast<float>();
  }
  x.ticket = reinterpret_cast<unsigned int*>(ticket.data_ptr());
  launch_adam_fused(P<float>(p), P<float>(g), P<float>(m), P<float>(v), p.numel(), (float)lr, (float)b1, (float)b2,
                    (float)eps, P<float>(pows), (float)grad_scale, (float)wd, clear_grad, x, stream());
}

// Raw async H2D copy on the current stream.  torch's copy_ from pinned memory
// records a fresh event in the caching host allocator for every copy and only
// reclaims them on allocation; a training loop that re-uses the same pinned
// batches never allocates, the events pile up and every few dozen copies the
// runtime stalls the host for milliseconds (profiles/r2_h2d_stall.txt).  Buffer
// reuse is ordered by the caller's own events instead.
static void memcpy_h2d(Tensor dst, const Tensor& src) {
  TW_CHECK(dst.is_cuda() && dst.is_contiguous(), "memcpy_h2d: dst must be a contiguous GPU tensor");
  TW_CHECK(!src.is_cuda() && src.is_contiguous() && src.is_pinned(), "memcpy_h2d: src must be contiguous pinned host memory");
  const size_t n = (size_t)dst.numel() * dst.element_size();
  TW_CHECK((size_t)src.numel() * src.element_size() == n, "memcpy_h2d: size mismatch");
  if (hipMemcpyAsync(dst.data_ptr(), src.data_ptr(), n, hipMemcpyHostToDevice, stream()) != hipSuccess)
    throw std::runtime_error("pbx: hipMemcpyAsync H2D failed");
}

void bind_tower(py::module& m) {
  m.def("memcpy_h2d", &memcpy_h2d, py::arg("dst"), py::arg("src"));
  py::class_<TowerWorkspace>(m, "TowerWorkspace")
      .def(py::init<int64_t, std::vector<int64_t>, int, int64_t, bool, bool>(), py::arg("M"), py::arg("dims"),
           py::arg("device"), py::arg("dw_splits") = 2, py::arg("fp32") = false, py::arg("x3") = false)
      .def("pack", &TowerWorkspace::pack)
      .def("forward", &TowerWorkspace::forward, py::arg("b"), py::arg("w_out"), py::arg("b_out"), py::arg("lin"),
           py::arg("label"), py::arg("auc_table") = py::none(), py::arg("auc_stats") = py::none(),
           py::arg("auc_mask") = py::none())
      .def("backward", &TowerWorkspace::backward, py::arg("dloss"), py::arg("w_out"), py::arg("dW"), py::arg("db"),
           py::arg("dw_out"),
           py::arg("db_out"), py::arg("need_dx"), py::arg("dn_part") = py::none(), py::arg("dn_rows") = 0,
           py::arg("dn_eps") = 0.0, py::arg("dn_stats") = py::none(), py::arg("parts") = 3,
           py::arg("dn_bsize") = py::none(), py::arg("dn_bsum") = py::none(), py::arg("dn_bsq") = py::none(),
           py::arg("dn_decay") = 1.0, py::arg("head_x") = py::none(), py::arg("head_scales") = py::none(),
           py::arg("hS") = 0, py::arg("hEo") = 0, py::arg("hew") = 0, py::arg("hD") = 0, py::arg("hlin") = false)
      .def("pack_regions", &TowerWorkspace::pack_regions)
      .def("set_stamps", &TowerWorkspace::set_stamps)
      .def("x0", &TowerWorkspace::x0)
      .def("x0mp", &TowerWorkspace::x0mp)
      .def("xmp", &TowerWorkspace::xmp)
      .def("dzmp", &TowerWorkspace::dzmp)
      .def("dx0", &TowerWorkspace::dx0)
      .def("wp", &TowerWorkspace::wp)
      .def("wtp", &TowerWorkspace::wtp)
      .def_property_readonly("M", &TowerWorkspace::M)
      .def_property_readonly("Mp", &TowerWorkspace::Mp)
      .def_property_readonly("K0p", &TowerWorkspace::K0p)
      .def_property_readonly("fp32", &TowerWorkspace::fp32)
      .def_property_readonly("x3", &TowerWorkspace::x3)
      .def_property_readonly("dw_splits", &TowerWorkspace::dw_splits)
      .def_property_readonly("lds_ld", &TowerWorkspace::lds_ld);
  m.def("adam_fused", &adam_fused, py::arg("p"), py::arg("g"), py::arg("m"), py::arg("v"), py::arg("pows"),
        py::arg("ticket"), py::arg("lr"), py::arg("b1"), py::arg("b2"), py::arg("eps"), py::arg("grad_scale"),
        py::arg("wd"), py::arg("clear_grad"), py::arg("pack"), py::arg("dn"));
}

}  // namespace pbx

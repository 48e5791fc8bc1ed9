// CrossWorkspace: DCN-V2 cross network.  Default (the 32-row tile fits in
// LDS): forward = weight pack + ONE launch for all layers and the w_c dot
// (tower.hip k_cross_fwd), backward = ONE launch for the top + dX chain
// (k_cross_bwd) + ONE grouped dW launch for all layers, db and dw_c
// (tower.hip k_tower_dw on m-packed operands).  Fallback
// (PBX_CROSS_FUSED=0 or wide D): the per-layer LDS-DMA MFMA GEMMs (mlp.hip,
// MLP_EPI_CROSS_* epilogues) + cross.hip: forward = 1 weight cast + L GEMMs +
// 1 dot, backward = top kernel + colsum + 2 GEMMs per layer.  Persistent
// padded buffers, all shapes checked here.
#include <ATen/hip/HIPContext.h>
#include <torch/extension.h>

#include <cstdlib>
#include <stdexcept>

#include "kernels.h"

namespace py = pybind11;
using torch::Tensor;

namespace pbx {
namespace {

hipStream_t xs() { return at::hip::getCurrentHIPStream().stream(); }

#define CR_CHECK(cond, msg)                                                   \
  do {                                                                        \
    if (!(cond)) throw std::runtime_error(std::string("pbx cross: ") + msg); \
  } while (0)

unsigned short* bp(const Tensor& t) { return reinterpret_cast<unsigned short*>(t.data_ptr()); }
float* fp(const Tensor& t) { return reinterpret_cast<float*>(t.data_ptr()); }

// Layout (matches the MlpWorkspace whose input it shares): D = the MLP input
// width (multiple of 8), ld = pad64(D), ldM = pad64(M).
//   x0 = MLP X_0 [M][ld] bf16, x0^T = MLP X_0^T [pad64(D+1)][ldM] (ones row D)
//   W_l, W_l^T bf16 [ld][ld] (cast from the fp32 masters [D][D] every step)
//   x_{l+1}: f32 [M][ld], bf16 [M][ld] + bf16^T [pad64(D+1)][ldM] (l+1 < L)
//   z_l f32; backward g (f32) / u (bf16 + u^T) ping-pong pairs, acc f32
class CrossWorkspace {
 public:
  CrossWorkspace(int64_t M, int64_t D, int64_t L, int device, int64_t k_split)
      : M_(M), D_(D), L_(L), ks_(k_split) {
    CR_CHECK(M > 0 && D > 0 && D % 8 == 0 && L >= 1 && L <= kMaxMlpLayers, "bad shape");
    CR_CHECK(k_split > 0 && k_split % 64 == 0, "k_split must be a positive multiple of 64");
    ld_ = p64(D);
    ldM_ = p64(M);
    auto ob = torch::TensorOptions().dtype(torch::kBFloat16).device(torch::kCUDA, device);
    auto of = torch::TensorOptions().dtype(torch::kFloat32).device(torch::kCUDA, device);
    for (int l = 0; l < L; ++l) {
      wb_.push_back(torch::zeros({ld_, ld_}, ob));
      wtb_.push_back(torch::zeros({ld_, ld_}, ob));
      xf_.push_back(torch::zeros({M, ld_}, of));
      z_.push_back(torch::zeros({M, ld_}, of));
      if (l + 1 < L) {
        xb_.push_back(torch::zeros({M, ld_}, ob));
        auto t = torch::zeros({p64(D + 1), ldM_}, ob);
        t[D].narrow(0, 0, M).fill_(1.0);  // bias ones row
        xt_.push_back(t);
      }
    }
    for (int i = 0; i < 2; ++i) {
      g_.push_back(torch::zeros({M, ld_}, of));
      u_.push_back(torch::zeros({M, ld_}, ob));
      ut_.push_back(torch::zeros({ld_, ldM_}, ob));
    }
    // fused forward (k_cross_fwd) when its 32-row tile fits in LDS
    np_ = (D + 31) / 32 * 32;
    kp_ = (D + 15) / 16 * 16;
    const char* fe = getenv("PBX_CROSS_FUSED");
    fused_ = (!fe || atoi(fe) != 0) && cross_fwd_lds_bytes((int)np_, (int)kp_) > 0;
    if (fused_) {
      mp_ = (M + 127) / 128 * 128;  // the grouped dW launch walks M in 128-row stages
      for (int l = 0; l < L; ++l) {
        wp_.push_back(torch::zeros({np_ * kp_}, ob));
        wtp_.push_back(torch::zeros({np_ * np_}, ob));
        xmp_.push_back(torch::zeros({mp_ * np_}, ob));  // m-packed x_l (dW B operand)
        ump_.push_back(torch::zeros({mp_ * np_}, ob));  // m-packed u_l (dW A operand)
      }
      bias_ld_ = L * np_ + (D + 31) / 32 * 32;
      biasp_ = torch::zeros({mp_ / 32, bias_ld_}, of);
    }
    acc_ = torch::zeros({M, ld_}, of);
    dy_ = torch::zeros({M, ld_}, ob);
    s_ = torch::zeros({M}, of);
    part_ = torch::zeros({cross_top_blocks((int)M), D}, of);
  }
  static int64_t p64(int64_t v) { return (v + 63) / 64 * 64; }

  Tensor forward(const Tensor& y, const std::vector<Tensor>& W, const std::vector<Tensor>& b, const Tensor& wc) {
    check_x0(y);
    CR_CHECK((int64_t)W.size() == L_ && (int64_t)b.size() == L_, "layer count");
    CR_CHECK(wc.is_cuda() && wc.numel() == D_ && wc.scalar_type() == torch::kFloat32 && wc.is_contiguous(), "w_c");
    auto s = xs();
    CastWtBatch cb;
    cb.n = (int)L_;
    cb.tile_off[0] = 0;
    for (int l = 0; l < L_; ++l) {
      CR_CHECK(W[l].is_cuda() && W[l].is_contiguous() && W[l].scalar_type() == torch::kFloat32 &&
                   W[l].size(0) == D_ && W[l].size(1) == D_,
               "W must be contiguous f32 [D, D]");
      CR_CHECK(b[l].is_cuda() && b[l].numel() == D_ && b[l].scalar_type() == torch::kFloat32 && b[l].is_contiguous(),
               "b must be f32 [D]");
      cb.w[l] = fp(W[l]);
      cb.wb[l] = bp(wb_[l]);
      cb.wtb[l] = bp(wtb_[l]);
      cb.N[l] = cb.K[l] = (int)D_;
      cb.pN[l] = cb.pK[l] = (int)ld_;
      cb.tile_off[l + 1] = cb.tile_off[l] + (int)((ld_ / 32) * (ld_ / 32));
    }
    if (fused_) {  // one launch for the whole stack + the w_c dot (weights packed for it and the fused backward)
      const float* wl[kMaxMlpLayers];
      unsigned short* wpl[kMaxMlpLayers];
      unsigned short* wtpl[kMaxMlpLayers];
      CrossFwdArgs a;
      a.x0 = bp(y);
      a.ldx0 = (int)ld_;
      for (int l = 0; l < L_; ++l) {
        wl[l] = fp(W[l]);
        wpl[l] = bp(wp_[l]);
        wtpl[l] = bp(wtp_[l]);
        a.wp[l] = bp(wp_[l]);
        a.bias[l] = fp(b[l]);
        a.z[l] = fp(z_[l]);
        a.xmp[l] = bp(xmp_[l]);
      }
      // the packed bf16 copies: re-packed by the fused Adam after each update
      // when the optimizer owns them (FlatAdam.fuse), else every forward
      if (!pack_by_opt_ || !packed_) {
        launch_cross_pack(wl, wpl, wtpl, (int)L_, (int)D_, (int)kp_, (int)np_, s);
        packed_ = true;
      }
      a.xlast = fp(xf_[L_ - 1]);
      a.ldf = (int)ld_;
      a.wc = fp(wc);
      a.s = fp(s_);
      a.M = (int)M_;
      a.D = (int)D_;
      a.L = (int)L_;
      a.Np = (int)np_;
      a.Kp = (int)kp_;
      launch_cross_fwd(a, s);
      return s_;
    }
    launch_cast_wt(cb, s);
    for (int l = 0; l < L_; ++l) {
      const bool last = l + 1 == L_;
      MlpGemmArgs g;
      g.A = l == 0 ? bp(y) : bp(xb_[l - 1]);
      g.lda = (int)ld_;
      g.B = bp(wb_[l]);
      g.ldb = (int)ld_;
      g.M = (int)M_;
      g.N = (int)ld_;
      g.K = (int)ld_;
      g.C = last ? nullptr : bp(xb_[l]);
      g.ldc = (int)ld_;
      g.CT = last ? nullptr : bp(xt_[l]);
      g.ldct = (int)ldM_;
      g.ncols_valid = (int)D_;
      g.bias = fp(b[l]);
      g.x0 = bp(y);
      g.ldx0 = (int)ld_;
      g.xin = l == 0 ? nullptr : fp(xf_[l - 1]);
      g.fout = fp(xf_[l]);
      g.zout = fp(z_[l]);
      g.ldf = (int)ld_;
      launch_mlp_gemm(g, MLP_EPI_CROSS_FWD, s);
    }
    launch_cross_dot(fp(xf_[L_ - 1]), (int)M_, (int)D_, (int)ld_, fp(wc), fp(s_), s);
    return s_;
  }

  // grads accumulate into dW[l] / db[l] / dwc (dense-arena views); returns
  // d(loss)/d(x0) as bf16 [M, ld] (pad columns zero)
  // dy_out (optional): a bf16 [M, ld] gradient buffer the x0 gradient is
  // ADDED to (e.g. the fused tower's dX0, before its data_norm backward)
  Tensor backward(const Tensor& y, const Tensor& yt, const Tensor& ds, const std::vector<Tensor>& dW,
                  const std::vector<Tensor>& db, const Tensor& wc, const Tensor& dwc,
                  const c10::optional<Tensor>& dy_out, int64_t parts, const c10::optional<Tensor>& ds_scale) {
    check_x0(y);
    if (ds_scale.has_value() && ds_scale->defined())
      CR_CHECK(fused_ && ds_scale->is_cuda() && ds_scale->numel() == 1 && ds_scale->scalar_type() == torch::kFloat32,
               "ds_scale: one f32 on the GPU, fused stack only");
    CR_CHECK(yt.is_cuda() && yt.scalar_type() == torch::kBFloat16 && yt.is_contiguous() && yt.dim() == 2 &&
                 yt.size(0) >= D_ + 1 && yt.size(1) == ldM_,
             "x0^T must be the MLP's bf16 [pad64(D+1), pad64(M)] transposed input");
    CR_CHECK(ds.is_cuda() && ds.numel() == M_ && ds.scalar_type() == torch::kFloat32 && ds.is_contiguous(), "ds");
    CR_CHECK((int64_t)dW.size() == L_ && (int64_t)db.size() == L_, "grad count");
    for (int l = 0; l < L_; ++l) {
      CR_CHECK(dW[l].is_cuda() && dW[l].is_contiguous() && dW[l].numel() == D_ * D_ &&
                   dW[l].scalar_type() == torch::kFloat32,
               "dW must be contiguous f32 [D, D]");
      CR_CHECK(db[l].is_cuda() && db[l].is_contiguous() && db[l].numel() == D_ && db[l].scalar_type() == torch::kFloat32,
               "db");
    }
    CR_CHECK(wc.is_cuda() && wc.numel() == D_ && wc.is_contiguous(), "w_c");
    CR_CHECK(dwc.is_cuda() && dwc.numel() == D_ && dwc.scalar_type() == torch::kFloat32 && dwc.is_contiguous(), "dwc");
    auto s = xs();
    // parts (fused stack only): bit 0 = top + dX chain (k_cross_bwd), bit 1 =
    // the grouped dW + db / dw_c reductions -- the caller may issue them on
    // different streams (the dW after the chain, beside the head backward)
    CR_CHECK(parts == 3 || (fused_ && (parts == 1 || parts == 2)), "parts: 3, or 1 / 2 with the fused stack");
    if (fused_) return backward_fused(y, yt, ds, dW, db, wc, dwc, dy_out, s, (int)parts, ds_scale);
    int cur = 0;  // ping-pong index holding g_{l+1}, u_l, u_l^T
    launch_cross_top_bwd(fp(xf_[L_ - 1]), bp(y), fp(z_[L_ - 1]), fp(wc), fp(ds), (int)M_, (int)D_, (int)ld_,
                         fp(g_[cur]), bp(u_[cur]), bp(ut_[cur]), (int)ldM_, fp(acc_), fp(part_), fp(dwc), s);
    for (int l = (int)L_ - 1; l >= 0; --l) {
      MlpGemmArgs w;  // dW_l += u_l^T [x_l | 1]   (split-K over the batch)
      w.A = bp(ut_[cur]);
      w.lda = (int)ldM_;
      w.B = l == 0 ? bp(yt) : bp(xt_[l - 1]);
      w.ldb = (int)ldM_;
      w.M = (int)D_;
      w.N = (int)D_ + 1;
      w.K = (int)ldM_;
      w.k_per_split = (int)ks_;
      w.dW = fp(dW[l]);
      w.lddw = (int)D_;
      w.db = fp(db[l]);
      w.ncols_valid = (int)D_;
      w.nrows_valid = (int)D_;
      launch_mlp_gemm(w, MLP_EPI_DW, s);
      MlpGemmArgs d;  // g_l = u_l W_l + g_{l+1}
      d.A = bp(u_[cur]);
      d.lda = (int)ld_;
      d.B = bp(wtb_[l]);
      d.ldb = (int)ld_;
      d.M = (int)M_;
      d.N = (int)ld_;
      d.K = (int)ld_;
      d.ncols_valid = (int)D_;
      d.ldc = (int)ld_;
      d.ldct = (int)ldM_;
      d.x0 = bp(y);
      d.ldx0 = (int)ld_;
      d.gin = fp(g_[cur]);
      d.accum = fp(acc_);
      d.ldf = (int)ld_;
      if (l > 0) {
        d.C = bp(u_[cur ^ 1]);
        d.CT = bp(ut_[cur ^ 1]);
        d.fout = fp(g_[cur ^ 1]);
        d.zprev = fp(z_[l - 1]);
      } else if (dy_out.has_value() && dy_out->defined()) {
        CR_CHECK(dy_out->is_cuda() && dy_out->scalar_type() == torch::kBFloat16 && dy_out->is_contiguous() &&
                     dy_out->dim() == 2 && dy_out->size(0) == M_ && dy_out->size(1) == ld_,
                 "dy_out must be bf16 [M, ld]");
        d.C = bp(*dy_out);
        d.CT = nullptr;
        d.add_c = 1;
      } else {
        d.C = bp(dy_);
        d.CT = nullptr;
      }
      launch_mlp_gemm(d, MLP_EPI_CROSS_DX, s);
      cur ^= 1;
    }
    return dy_out.has_value() && dy_out->defined() ? *dy_out : dy_;
  }

  // one launch for the top + dX chain (k_cross_bwd), then ONE grouped dW
  // launch over all layers (k_tower_dw on the m-packed u_l / x_l) whose extra
  // workgroups reduce the db and dw_c column partials
  Tensor backward_fused(const Tensor& y, const Tensor& yt, const Tensor& ds, const std::vector<Tensor>& dW,
                        const std::vector<Tensor>& db, const Tensor& wc, const Tensor& dwc,
                        const c10::optional<Tensor>& dy_out, hipStream_t s, int parts,
                        const c10::optional<Tensor>& ds_scale) {
    (void)yt;
    const bool add = dy_out.has_value() && dy_out->defined();
    if (add)
      CR_CHECK(dy_out->is_cuda() && dy_out->scalar_type() == torch::kBFloat16 && dy_out->is_contiguous() &&
                   dy_out->dim() == 2 && dy_out->size(0) == M_ && dy_out->size(1) == ld_,
               "dy_out must be bf16 [M, ld]");
    CrossBwdArgs a;
    a.x0 = bp(y);
    a.ldx0 = (int)ld_;
    for (int l = 0; l < L_; ++l) {
      a.wtp[l] = bp(wtp_[l]);
      a.z[l] = fp(z_[l]);
      a.ump[l] = bp(ump_[l]);
    }
    a.xlast = fp(xf_[L_ - 1]);
    a.ldf = (int)ld_;
    a.ds = fp(ds);
    a.ds_scale = ds_scale.has_value() && ds_scale->defined() ? fp(*ds_scale) : nullptr;
    a.wc = fp(wc);
    a.dy = add ? bp(*dy_out) : bp(dy_);
    a.ldy = (int)ld_;
    a.add_dy = add ? 1 : 0;
    a.bias_part = fp(biasp_);
    a.bias_ld = (int)bias_ld_;
    a.M = (int)M_;
    a.D = (int)D_;
    a.L = (int)L_;
    a.Np = (int)np_;
    if (parts & 1) launch_cross_bwd(a, s);
    if (!(parts & 2)) return add ? *dy_out : dy_;
    TowerArgs t;
    t.M = (int)M_;
    t.Mp = (int)mp_;
    t.L = (int)L_;
    t.x0mp = bp(xmp_[0]);
    for (int l = 0; l < L_; ++l) {
      TowerLayerDev& d = t.ly[l];
      d.N = d.K = (int)D_;
      d.Np = d.Kp = (int)np_;
      d.dzmp = bp(ump_[l]);
      d.xmp = l + 1 < L_ ? bp(xmp_[l + 1]) : nullptr;  // X_{l+1}: the B operand of layer l+1
      d.dw = fp(dW[l]);
      d.db = fp(db[l]);
      d.bias_off = (int)(l * np_);
    }
    t.bias_part = fp(biasp_);
    t.bias_ld = (int)bias_ld_;
    t.dwout_off = (int)(L_ * np_);
    t.dbout_off = (int)bias_ld_;  // no output-layer bias here
    t.dw_out = fp(dwc);
    t.dw_splits = 2;
    launch_tower_dw(t, s);
    return add ? *dy_out : dy_;
  }

  Tensor x_out() const { return xf_[L_ - 1].narrow(1, 0, D_); }
  bool fused() const { return fused_; }
  // (wp, wtp, N, K, Np, Kp, None, None) per layer: the bf16 pack regions of
  // the fused Adam (the tower's bf16 layout, wp_index / wtp_index)
  std::vector<py::tuple> pack_regions() const {
    std::vector<py::tuple> r;
    if (!fused_) return r;
    for (int l = 0; l < L_; ++l)
      r.push_back(py::make_tuple(wp_[l], wtp_[l], D_, D_, np_, kp_, py::none(), py::none()));
    return r;
  }
  void set_pack_by_optimizer(bool v) { pack_by_opt_ = v; }
  void invalidate_pack() { packed_ = false; }

 private:
  void check_x0(const Tensor& y) const {
    CR_CHECK(y.is_cuda() && y.scalar_type() == torch::kBFloat16 && y.is_contiguous() && y.dim() == 2 &&
                 y.size(0) == M_ && y.size(1) == ld_,
             "x0 must be the MLP's contiguous bf16 [M, pad64(D)] input");
  }
  int64_t M_, D_, L_, ks_, ld_ = 0, ldM_ = 0, np_ = 0, kp_ = 0, mp_ = 0, bias_ld_ = 0;
  bool fused_ = false;
  bool pack_by_opt_ = false, packed_ = false;
  std::vector<Tensor> wb_, wtb_, xf_, xb_, xt_, z_, g_, u_, ut_, wp_, wtp_, xmp_, ump_;
  Tensor acc_, dy_, s_, part_, biasp_;
};

}  // namespace

void bind_cross(py::module& m) {
  py::class_<CrossWorkspace>(m, "CrossWorkspace")
      .def(py::init<int64_t, int64_t, int64_t, int, int64_t>())
      .def("forward", &CrossWorkspace::forward)
      .def("backward", &CrossWorkspace::backward, py::arg("y"), py::arg("yt"), py::arg("ds"), py::arg("dW"),
           py::arg("db"), py::arg("wc"), py::arg("dwc"), py::arg("dy_out") = py::none(), py::arg("parts") = 3,
           py::arg("ds_scale") = py::none())
      .def("x_out", &CrossWorkspace::x_out)
      .def("pack_regions", &CrossWorkspace::pack_regions)
      .def("set_pack_by_optimizer", &CrossWorkspace::set_pack_by_optimizer)
      .def("invalidate_pack", &CrossWorkspace::invalidate_pack)
      .def_property_readonly("fused_forward", [](const CrossWorkspace& w) { return w.fused(); });
}

}  // namespace pbx

// CrossWorkspace: DCN-V2 cross network on the hand-written MFMA GEMM
// (gemm.hip EPI_CROSS_* epilogues + cross.hip).  Persistent padded buffers,
// all shapes checked here; the forward is L GEMMs + 1 dot, the backward
// 1 top kernel + 3 launches per layer (dW GEMM, slab reduce, dX GEMM).
#include <ATen/hip/HIPContext.h>
#include <torch/extension.h>

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

class CrossWorkspace {
 public:
  CrossWorkspace(int64_t M, int64_t C, int64_t L, int64_t ldx0, int device, int64_t k_split)
      : M_(M), C_(C), L_(L), ldx0_(ldx0), ks_(k_split) {
    CR_CHECK(M > 0 && C > 0 && L >= 1 && L <= kMaxMlpLayers, "bad shape");
    CR_CHECK(ldx0 >= C && ldx0 % 8 == 0, "x0 row stride must be >= C and a multiple of 8");
    CR_CHECK(k_split > 0 && k_split % 64 == 0, "k_split must be a positive multiple of 64");
    Cp_ = (C + 7) / 8 * 8;
    auto ob = torch::TensorOptions().dtype(torch::kBFloat16).device(torch::kCUDA, device);
    auto of = torch::TensorOptions().dtype(torch::kFloat32).device(torch::kCUDA, device);
    for (int l = 0; l < L; ++l) {
      wb_.push_back(torch::zeros({Cp_, Cp_}, ob));
      wtb_.push_back(torch::zeros({Cp_, Cp_}, ob));
      xf_.push_back(torch::zeros({M, Cp_}, of));
      xb_.push_back(torch::zeros({M, Cp_}, ob));
      z_.push_back(torch::zeros({M, Cp_}, of));
    }
    for (int i = 0; i < 2; ++i) {
      g_.push_back(torch::zeros({M, Cp_}, of));
      u_.push_back(torch::zeros({M, Cp_}, ob));
    }
    acc_ = torch::zeros({M, Cp_}, of);
    dy_ = torch::zeros({M, ldx0}, ob);
    s_ = torch::zeros({M}, of);
    splits_ = (M + k_split - 1) / k_split;
    slab_ = torch::zeros({splits_, C, C + 1}, of);
    part_ = torch::zeros({cross_top_blocks((int)M), C}, of);
  }

  Tensor forward(const Tensor& y, const std::vector<Tensor>& W, const std::vector<Tensor>& b, const Tensor& wc) {
    check_x0(y);
    CR_CHECK((int64_t)W.size() == L_ && (int64_t)b.size() == L_, "layer count");
    CR_CHECK(wc.is_cuda() && wc.numel() == C_ && wc.scalar_type() == torch::kFloat32, "w_c");
    auto s = xs();
    CastWtBatch cb;
    cb.n = (int)L_;
    cb.tile_off[0] = 0;
    for (int l = 0; l < L_; ++l) {
      CR_CHECK(W[l].is_cuda() && W[l].is_contiguous() && W[l].scalar_type() == torch::kFloat32 &&
                   W[l].size(0) == C_ && W[l].size(1) == C_,
               "W must be contiguous f32 [C, C]");
      CR_CHECK(b[l].is_cuda() && b[l].numel() == C_ && b[l].scalar_type() == torch::kFloat32, "b must be f32 [C]");
      cb.w[l] = fp(W[l]);
      cb.wb[l] = bp(wb_[l]);
      cb.wtb[l] = bp(wtb_[l]);
      cb.N[l] = cb.K[l] = (int)C_;
      cb.pN[l] = cb.pK[l] = (int)Cp_;
      const int t = (int)((Cp_ + 31) / 32);
      cb.tile_off[l + 1] = cb.tile_off[l] + t * t;
    }
    launch_cast_wt(cb, s);
    for (int l = 0; l < L_; ++l) {
      GemmArgs g;
      g.A = l == 0 ? bp(y) : bp(xb_[l - 1]);
      g.lda = l == 0 ? (int)ldx0_ : (int)Cp_;
      g.B = bp(wb_[l]);
      g.ldb = (int)Cp_;
      g.M = (int)M_;
      g.N = (int)C_;
      g.K = (int)C_;
      g.C = fp(xf_[l]);
      g.ldc = (int)Cp_;
      g.bias = fp(b[l]);
      g.epi = EPI_CROSS_FWD;
      g.x0 = bp(y);
      g.ldx0 = (int)ldx0_;
      g.xin = l == 0 ? nullptr : fp(xf_[l - 1]);
      g.out2 = fp(z_[l]);
      g.outb = l + 1 < L_ ? bp(xb_[l]) : nullptr;
      launch_gemm(g, s);
    }
    launch_cross_dot(fp(xf_[L_ - 1]), (int)M_, (int)C_, (int)Cp_, fp(wc), fp(s_), s);
    return s_;
  }

  // grads accumulate into dW[l] / db[l] / dwc (dense-arena views); returns
  // d(loss)/d(x0) as bf16 [M, ldx0] (pad columns zero)
  Tensor backward(const Tensor& y, const Tensor& ds, const std::vector<Tensor>& dW, const std::vector<Tensor>& db,
                  const Tensor& wc, const Tensor& dwc) {
    check_x0(y);
    CR_CHECK(ds.is_cuda() && ds.numel() == M_ && ds.scalar_type() == torch::kFloat32 && ds.is_contiguous(), "ds");
    CR_CHECK((int64_t)dW.size() == L_ && (int64_t)db.size() == L_, "grad count");
    for (int l = 0; l < L_; ++l) {
      CR_CHECK(dW[l].is_cuda() && dW[l].is_contiguous() && dW[l].numel() == C_ * C_ &&
                   dW[l].scalar_type() == torch::kFloat32,
               "dW must be contiguous f32 [C, C]");
      CR_CHECK(db[l].is_cuda() && db[l].is_contiguous() && db[l].numel() == C_ && db[l].scalar_type() == torch::kFloat32,
               "db");
    }
    CR_CHECK(dwc.is_cuda() && dwc.numel() == C_ && dwc.scalar_type() == torch::kFloat32 && dwc.is_contiguous(), "dwc");
    auto s = xs();
    int cur = 0;  // g_/u_ ping-pong index holding g_{l+1}, u_l
    launch_cross_top_bwd(fp(xf_[L_ - 1]), bp(y), (int)ldx0_, fp(z_[L_ - 1]), fp(wc), fp(ds), (int)M_, (int)C_,
                         (int)Cp_, fp(g_[cur]), bp(u_[cur]), fp(acc_), fp(part_), fp(dwc), s);
    for (int l = (int)L_ - 1; l >= 0; --l) {
      // dW_l = u_l^T x_l, db_l = colsum(u_l) (virtual ones column), split-K over the batch
      GemmArgs w;
      w.A = bp(u_[cur]);
      w.lda = (int)Cp_;
      w.a_kcontig = false;
      w.B = l == 0 ? bp(y) : bp(xb_[l - 1]);
      w.ldb = l == 0 ? (int)ldx0_ : (int)Cp_;
      w.b_kcontig = false;
      w.M = (int)C_;
      w.N = (int)C_;
      w.K = (int)M_;
      w.ones_col_b = (int)C_;
      w.C = fp(slab_);
      w.ldc = (int)C_ + 1;
      w.epi = EPI_F32_SLAB;
      w.k_per_split = (int)ks_;
      w.slab_stride = C_ * (C_ + 1);
      launch_gemm(w, s);
      launch_slab_reduce(fp(slab_), (int)splits_, C_ * (C_ + 1), (int)C_, (int)C_, (int)C_ + 1, fp(dW[l]), fp(db[l]),
                         1.f, s);
      // g_l = u_l W_l + g_{l+1}
      GemmArgs d;
      d.A = bp(u_[cur]);
      d.lda = (int)Cp_;
      d.B = bp(wtb_[l]);
      d.ldb = (int)Cp_;
      d.M = (int)M_;
      d.N = (int)C_;
      d.K = (int)C_;
      d.epi = EPI_CROSS_DX;
      d.gin = fp(g_[cur]);
      d.x0 = bp(y);
      d.ldx0 = (int)ldx0_;
      d.ldc = (int)Cp_;
      d.out2 = fp(acc_);
      if (l > 0) {
        d.C = fp(g_[cur ^ 1]);
        d.zprev = fp(z_[l - 1]);
        d.outb = bp(u_[cur ^ 1]);
      } else {
        d.C = nullptr;
        d.zprev = nullptr;
        d.outb = bp(dy_);
      }
      launch_gemm(d, s);
      cur ^= 1;
    }
    return dy_;
  }

  Tensor x_out() const { return xf_[L_ - 1].narrow(1, 0, C_); }

 private:
  void check_x0(const Tensor& y) const {
    CR_CHECK(y.is_cuda() && y.scalar_type() == torch::kBFloat16 && y.is_contiguous() && y.dim() == 2 &&
                 y.size(0) == M_ && y.size(1) == ldx0_,
             "x0 must be the contiguous bf16 [M, ldx0] MLP input");
  }
  int64_t M_, C_, L_, ldx0_, ks_, Cp_ = 0, splits_ = 1;
  std::vector<Tensor> wb_, wtb_, xf_, xb_, z_, g_, u_;
  Tensor acc_, dy_, s_, slab_, part_;
};

}  // namespace

void bind_cross(py::module& m) {
  py::class_<CrossWorkspace>(m, "CrossWorkspace")
      .def(py::init<int64_t, int64_t, int64_t, int64_t, int, int64_t>())
      .def("forward", &CrossWorkspace::forward)
      .def("backward", &CrossWorkspace::backward)
      .def("x_out", &CrossWorkspace::x_out);
}

}  // namespace pbx

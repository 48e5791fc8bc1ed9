// torch glue for the CTR op-family kernels (ctr_ext.hip): shape checks and
// pointer plumbing only.
#include <ATen/hip/HIPContext.h>
#include <torch/extension.h>

#include <stdexcept>
#include <unordered_map>

#include "kernels.h"

namespace py = pybind11;
using torch::Tensor;

namespace pbx {
namespace {

hipStream_t cs() { return at::hip::getCurrentHIPStream().stream(); }

#define CX_CHECK(cond, msg)                                               \
  do {                                                                    \
    if (!(cond)) throw std::runtime_error(std::string("pbx ctr: ") + msg); \
  } while (0)

void f32(const Tensor& t, const char* n) {
  CX_CHECK(t.is_cuda() && t.scalar_type() == torch::kFloat32, std::string(n) + " must be an f32 GPU tensor");
}
template <typename T>
T* P(const Tensor& t) {
  return reinterpret_cast<T*>(t.data_ptr());
}
template <typename T>
T* OP(const c10::optional<Tensor>& t) {
  return t.has_value() && t->defined() ? reinterpret_cast<T*>(t->data_ptr()) : nullptr;
}

// generic strided batched fp32 GEMM: C = alpha A B (+ bias * bias_scale) (+ C)
void sgemm(const Tensor& A, const Tensor& B, Tensor C, const c10::optional<Tensor>& bias, int64_t M, int64_t N,
           int64_t K, int64_t batch, std::vector<int64_t> a_strides, std::vector<int64_t> b_strides, int64_t sC,
           int64_t ldc, int64_t sBias, double bias_scale, double alpha, bool accumulate) {
  f32(A, "A");
  f32(B, "B");
  f32(C, "C");
  CX_CHECK(a_strides.size() == 3 && b_strides.size() == 3, "strides are (batch, row, col)");
  SgemmArgs g;
  g.A = P<float>(A);
  g.B = P<float>(B);
  g.C = P<float>(C);
  g.bias = OP<float>(bias);
  g.M = (int)M; g.N = (int)N; g.K = (int)K; g.batch = (int)batch;
  g.sA = a_strides[0]; g.rsA = a_strides[1]; g.csA = a_strides[2];
  g.sB = b_strides[0]; g.rsB = b_strides[1]; g.csB = b_strides[2];
  g.sC = sC; g.ldc = ldc; g.sBias = sBias;
  g.bias_scale = (float)bias_scale;
  g.alpha = (float)alpha;
  g.accumulate = accumulate ? 1 : 0;
  // bounds of the furthest element touched by each operand
  auto span = [](int64_t b, int64_t sb, int64_t r, int64_t sr, int64_t c, int64_t sc) {
    return (b - 1) * sb + (r - 1) * sr + (c - 1) * sc;
  };
  CX_CHECK(span(batch, g.sA, M, g.rsA, K, g.csA) < A.numel(), "A too small for its strides");
  CX_CHECK(span(batch, g.sB, K, g.rsB, N, g.csB) < B.numel(), "B too small for its strides");
  CX_CHECK(span(batch, sC, M, ldc, N, 1) < C.numel(), "C too small for its strides");
  launch_sgemm(g, cs());
}

// batch_fc with slots of at most 64 x 64 (launch_batch_fc_fwd / _bwd).
// strides = (sx, rx, sw, rw, sy, ry, sb); False when the shape / alignment
// does not fit the dedicated kernels (nothing launched).
BfcArgs bfc_args(const Tensor& x, const Tensor& W, const Tensor& yy, int64_t Pn, int64_t N, int64_t I, int64_t O,
                 const std::vector<int64_t>& st) {
  f32(x, "x");
  f32(W, "W");
  f32(yy, "y/dy");
  CX_CHECK(st.size() == 7, "strides are (sx, rx, sw, rw, sy, ry, sb)");
  BfcArgs a;
  a.P = (int)Pn; a.N = (int)N; a.I = (int)I; a.O = (int)O;
  a.sx = st[0]; a.rx = st[1]; a.sw = st[2]; a.rw = st[3]; a.sy = st[4]; a.ry = st[5]; a.sb = st[6];
  auto span = [](int64_t b, int64_t sb, int64_t r, int64_t sr, int64_t c) { return (b - 1) * sb + (r - 1) * sr + c - 1; };
  if (Pn > 0 && N > 0) {
    CX_CHECK(span(Pn, a.sx, N, a.rx, I) < x.numel(), "x too small for its strides");
    CX_CHECK(span(Pn, a.sw, I, a.rw, O) < W.numel(), "W too small for its strides");
    CX_CHECK(span(Pn, a.sy, N, a.ry, O) < yy.numel(), "y too small for its strides");
  }
  return a;
}

bool batch_fc_fwd(const Tensor& x, const Tensor& W, const Tensor& b, Tensor y, int64_t Pn, int64_t N, int64_t I,
                  int64_t O, std::vector<int64_t> st) {
  BfcArgs a = bfc_args(x, W, y, Pn, N, I, O, st);
  f32(b, "b");
  CX_CHECK(Pn == 0 || (Pn - 1) * a.sb + O <= b.numel(), "b too small for its stride");
  a.x = P<float>(x);
  a.W = P<float>(W);
  a.b = P<float>(b);
  a.y = P<float>(y);
  return launch_batch_fc_fwd(a, cs());
}

bool batch_fc_bwd(const Tensor& x, const Tensor& W, const Tensor& dy, Tensor dx, Tensor dW, Tensor db, int64_t Pn,
                  int64_t N, int64_t I, int64_t O, std::vector<int64_t> st) {
  BfcArgs a = bfc_args(x, W, dy, Pn, N, I, O, st);
  f32(dx, "dx");
  f32(dW, "dW");
  f32(db, "db");
  CX_CHECK(dx.numel() == x.numel() && dW.numel() == W.numel(), "dx / dW must have x / W's layout");
  CX_CHECK(Pn == 0 || (Pn - 1) * a.sb + O <= db.numel(), "db too small for its stride");
  a.x = P<float>(x);
  a.W = P<float>(W);
  a.dy = P<float>(dy);
  a.dx = P<float>(dx);
  a.dW = P<float>(dW);
  a.db = P<float>(db);
  const int64_t G = batch_fc_bwd_groups(a.P, a.N);
  Tensor ws = torch::empty({std::max<int64_t>(1, G * Pn * kBfcPart)}, x.options());
  a.ws = P<float>(ws);
  return launch_batch_fc_bwd(a, cs());
}

// scaled_fc's fp16 GEMM (launch_hgemm): C [M, ldc] fp32 from strided fp32
// A [M x K] (rsA, csA) and B [K x N] (rsB, csB) with the reference rounding
void hgemm(const Tensor& A, const Tensor& B, Tensor C, const c10::optional<Tensor>& bias, int64_t M, int64_t N,
           int64_t K, std::vector<int64_t> a_strides, std::vector<int64_t> b_strides, int64_t ldc, double a_scale,
           double b_scale, double alpha, double bias_scale, double out_scale, int64_t ksplit) {
  f32(A, "A");
  f32(B, "B");
  f32(C, "C");
  CX_CHECK(a_strides.size() == 2 && b_strides.size() == 2, "strides are (row, col)");
  HgemmArgs g;
  g.A = P<float>(A);
  g.B = P<float>(B);
  g.C = P<float>(C);
  g.bias = OP<float>(bias);
  g.M = (int)M; g.N = (int)N; g.K = (int)K;
  g.rsA = a_strides[0]; g.csA = a_strides[1];
  g.rsB = b_strides[0]; g.csB = b_strides[1];
  g.ldc = ldc;
  g.a_scale = (float)a_scale; g.b_scale = (float)b_scale; g.alpha = (float)alpha;
  g.bias_scale = (float)bias_scale; g.out_scale = (float)out_scale;
  g.ksplit = (int)std::max<int64_t>(1, std::min<int64_t>(ksplit, (K + 31) / 32));
  CX_CHECK((M - 1) * g.rsA + (K - 1) * g.csA < A.numel(), "A too small for its strides");
  CX_CHECK((K - 1) * g.rsB + (N - 1) * g.csB < B.numel(), "B too small for its strides");
  CX_CHECK((M - 1) * ldc + N - 1 < C.numel(), "C too small");
  if (g.bias) CX_CHECK(bias->numel() >= N, "bias");
  Tensor ws;
  if (g.ksplit > 1) {
    ws = torch::empty({M * N}, C.options());
    g.ws = P<float>(ws);
  }
  launch_hgemm(g, cs());
}

// in place: acc [M, N] fp32 -> the reference fp16 rounding chain of scaled_fc
void h16_epi(Tensor acc, const c10::optional<Tensor>& bias, double alpha, double bias_scale, double out_scale) {
  f32(acc, "acc");
  CX_CHECK(acc.dim() == 2 && acc.is_contiguous(), "acc must be a contiguous [M, N] tensor");
  const int M = (int)acc.size(0), N = (int)acc.size(1);
  if (bias.has_value() && bias->defined()) CX_CHECK(bias->numel() >= N && bias->is_contiguous(), "bias");
  launch_h16_epi(P<float>(acc), OP<float>(bias), M, N, (float)alpha, (float)bias_scale, (float)out_scale, P<float>(acc),
                 cs());
}

// scaled_fc fused fp16 GEMM (forward / dx): out [M, Nd] = h16_epi(fp16(A * a_scale) @ Bk^T),
// Bk fp16 [Nd, Kd] contiguous.  Returns an undefined tensor when the shapes do not fit the kernel.
Tensor sfc(const Tensor& A, const Tensor& Bk, const c10::optional<Tensor>& bias, double a_scale, double alpha,
           double bias_scale, double out_scale) {
  f32(A, "A");
  CX_CHECK(A.dim() == 2 && A.is_contiguous(), "A must be a contiguous [M, Kd] tensor");
  CX_CHECK(Bk.is_cuda() && Bk.scalar_type() == torch::kHalf && Bk.dim() == 2 && Bk.is_contiguous() &&
               Bk.size(1) == A.size(1), "Bk must be a contiguous fp16 [Nd, Kd] tensor");
  const int M = (int)A.size(0), Kd = (int)A.size(1), Nd = (int)Bk.size(0);
  if (bias.has_value() && bias->defined()) {
    f32(*bias, "bias");
    CX_CHECK(bias->numel() >= Nd && bias->is_contiguous(), "bias");
  }
  auto out = torch::empty({M, Nd}, A.options());
  if (!launch_sfc(P<float>(A), static_cast<const void*>(Bk.data_ptr<at::Half>()), M, Nd, Kd, (float)a_scale,
                  OP<float>(bias), (float)alpha, (float)bias_scale, (float)out_scale, P<float>(out), cs()))
    return Tensor();
  return out;
}

// scaled_fc weight + bias gradient (launch_sfc_dw): dW [K, O] and db [O] from
// x [N, K], d [N, O] (contiguous fp32) split S ways over N.  The tile counters
// come from a per-device ring of zeroed slots (the kernel leaves its slot
// zeroed), so back-to-back launches -- and launches on different streams, up
// to kSfcDwSlots in flight -- never share a counter.  false: the shapes do
// not fit the kernel (the caller takes the k_hgemm path).
constexpr int kSfcDwSlots = 64, kSfcDwSlotInts = 1024;
bool sfc_dw(const Tensor& x, const Tensor& d, Tensor dW, const c10::optional<Tensor>& db, double a_scale,
            double b_scale, double alpha, double out_scale, int64_t splits, int64_t mode) {
  f32(x, "x");
  f32(d, "d");
  f32(dW, "dW");
  CX_CHECK(x.dim() == 2 && d.dim() == 2 && x.is_contiguous() && d.is_contiguous() && x.size(0) == d.size(0),
           "sfc_dw: x [N, K], d [N, O] contiguous");
  SfcDwArgs a;
  a.N = (int)x.size(0);
  a.K = (int)x.size(1);
  a.O = (int)d.size(1);
  CX_CHECK(dW.is_contiguous() && dW.numel() == (int64_t)a.K * a.O, "dW must be a contiguous [K, O] tensor");
  a.x = P<float>(x);
  a.d = P<float>(d);
  a.dW = P<float>(dW);
  a.ldx = a.K;
  a.ldd = a.O;
  if (db.has_value() && db->defined()) {
    f32(*db, "db");
    CX_CHECK(db->is_contiguous() && db->numel() == a.O, "db must be a contiguous [O] tensor");
    a.db = P<float>(*db);
  }
  const int tiles = sfc_dw_tiles(a.K, a.O);
  int S = (int)std::max<int64_t>(1, splits);
  if (S > 1) {
    a.chunk = sfc_dw_chunk(a.N, S);
    S = (a.N + a.chunk - 1) / a.chunk;  // no empty splits
  }
  if (S <= 1 || tiles > kSfcDwSlotInts) S = 1;
  a.S = S;
  Tensor slab;
  if (S > 1) {
    const int nto = (a.O + 79) / 80;
    slab = torch::empty({(int64_t)tiles * S * 6400 + (int64_t)nto * S * 80}, x.options());
    a.slab = P<float>(slab);
    a.db_slab = a.slab + (int64_t)tiles * S * 6400;
    // device -> (slots, next slot); never destroyed (no tensor release after the runtime's teardown)
    static auto* ring = new std::unordered_map<int, std::pair<Tensor, int>>();
    auto& r = (*ring)[x.get_device()];
    if (!r.first.defined()) r.first = torch::zeros({kSfcDwSlots * kSfcDwSlotInts}, x.options().dtype(torch::kInt));
    a.cnt = r.first.data_ptr<int>() + (int64_t)r.second * kSfcDwSlotInts;
    r.second = (r.second + 1) % kSfcDwSlots;
  }
  a.a_scale = (float)a_scale;
  a.b_scale = (float)b_scale;
  a.alpha = (float)alpha;
  a.out_scale = (float)out_scale;
  a.mode = (int)mode;
  return launch_sfc_dw(a, cs());
}

// out [M, Nd] = A [M, Kd] @ (Bh + Bl)^T: fp32 A, B as its bf16 split (two
// contiguous [Nd, Kd] bf16 tensors) -- launch_f3gemm_nt.  Undefined tensor
// when the shapes do not fit the kernel.
Tensor f3gemm_nt(const Tensor& A, const Tensor& Bh, const Tensor& Bl) {
  f32(A, "A");
  CX_CHECK(A.dim() == 2 && A.is_contiguous(), "A must be a contiguous [M, Kd] tensor");
  for (const Tensor* b : {&Bh, &Bl})
    CX_CHECK(b->is_cuda() && b->scalar_type() == torch::kBFloat16 && b->dim() == 2 && b->is_contiguous() &&
                 b->size(1) == A.size(1) && b->size(0) == Bh.size(0),
             "Bh / Bl must be contiguous bf16 [Nd, Kd] tensors");
  const int M = (int)A.size(0), Kd = (int)A.size(1), Nd = (int)Bh.size(0);
  auto out = torch::empty({M, Nd}, A.options());
  if (!launch_f3gemm_nt(P<float>(A), Bh.data_ptr(), Bl.data_ptr(), M, Nd, Kd, P<float>(out), cs())) return Tensor();
  return out;
}

void colsum_strided(const Tensor& x, int64_t batch, int64_t M, int64_t N, int64_t sb, int64_t ld, Tensor out,
                    int64_t so, bool accumulate) {
  f32(x, "x");
  f32(out, "out");
  launch_colsum_strided(P<float>(x), (int)batch, (int)M, (int)N, sb, ld, P<float>(out), so, accumulate, cs());
}

// scaled_int8fc forward: y = int8(x) . int8(W) * interval / (ie * we) + b
Tensor int8_fc(const Tensor& x, const Tensor& W, const Tensor& b, double ie, double ic, double we, double wc,
               double range) {
  f32(x, "x");
  f32(W, "W");
  f32(b, "b");
  CX_CHECK(x.dim() == 2 && W.dim() == 2 && x.size(1) == W.size(0), "int8_fc: x [N, K], W [K, O]");
  const int N = (int)x.size(0), K = (int)x.size(1), O = (int)W.size(1);
  const int Kp = (K + 31) / 32 * 32;
  auto oi = x.options().dtype(torch::kInt8);
  auto qx = torch::zeros({N, Kp}, oi);
  auto qwt = torch::zeros({O, Kp}, oi);
  auto xc = x.contiguous(), Wc = W.contiguous();
  launch_i8_quant(P<float>(xc), N, K, Kp, (float)ie, (float)ic, (float)range, false, P<signed char>(qx), cs());
  launch_i8_quant(P<float>(Wc), K, O, Kp, (float)we, (float)wc, (float)range, true, P<signed char>(qwt), cs());
  auto y = torch::empty({N, O}, x.options());
  const float scale = (float)(2.0 * ic / range / (ie * we));
  auto bc = b.contiguous();
  launch_i8_gemm(P<signed char>(qx), P<signed char>(qwt), N, O, Kp, scale, P<float>(bc), P<float>(y), O, cs());
  return y;
}

// returns (out, bucket): bucket = the rank permutation + tile table the backward reuses
std::vector<Tensor> rank_attention_fwd(const Tensor& x, const Tensor& ro, const Tensor& W, int64_t R) {
  f32(x, "x");
  f32(W, "W");
  CX_CHECK(ro.is_cuda() && ro.scalar_type() == torch::kInt32 && ro.dim() == 2 && ro.size(1) >= 2 * R + 1,
           "rank_offset must be int32 [B, 2R+1]");
  CX_CHECK(R >= 1 && R <= 8, "max_rank in 1..8");
  const int B = (int)x.size(0), C = (int)x.size(1), P_ = (int)W.size(1);
  CX_CHECK(W.size(0) == R * R * C, "W must be [R*R*C, P]");
  auto xc = x.contiguous(), Wc = W.contiguous(), roc = ro.contiguous();
  auto out = torch::empty({B, P_}, x.options());
  auto bucket = torch::empty({rank_attention_bucket_ints(B, (int)R)}, roc.options());
  launch_rank_attention_fwd(P<float>(xc), P<int>(roc), (int)roc.size(1), P<float>(Wc), B, C, P_, (int)R,
                            P<int>(bucket), P<float>(out), cs());
  return {out, bucket};
}

// part 0: dx and dW; 1: dx only (dexp + the gather merge); 2: dW only --
// parts 1 and 2 are independent (both read dout): the caller may run them on
// two streams
std::vector<Tensor> rank_attention_bwd(const Tensor& x, const Tensor& ro, const Tensor& W, const Tensor& dout,
                                       const Tensor& bucket, int64_t R, int64_t part) {
  f32(x, "x");
  f32(dout, "dout");
  CX_CHECK(bucket.scalar_type() == torch::kInt32 && bucket.numel() == rank_attention_bucket_ints((int)x.size(0), (int)R),
           "bucket must come from rank_attention_fwd with the same B and R");
  const int B = (int)x.size(0), C = (int)x.size(1), P_ = (int)W.size(1);
  auto xc = x.contiguous(), Wc = W.contiguous(), roc = ro.contiguous(), dc = dout.contiguous();
  CX_CHECK(part >= 0 && part <= 2, "rank_attention_bwd: part");
  Tensor dexp, dx, dW;
  if (part != 2) {
    dexp = torch::empty({B, R, C}, x.options());
    dx = torch::empty_like(xc);
  }
  if (part != 1) dW = torch::zeros_like(Wc);
  launch_rank_attention_bwd(P<float>(xc), P<float>(dc), P<int>(roc), (int)roc.size(1), P<float>(Wc), B, C, P_,
                            (int)R, P<int>(bucket), part != 2 ? P<float>(dexp) : nullptr,
                            part != 2 ? P<float>(dx) : nullptr, part != 1 ? P<float>(dW) : nullptr, cs());
  return {dx, dW};
}

Tensor cvm_fwd(const Tensor& x, bool use_cvm) {
  f32(x, "x");
  auto xc = x.contiguous();
  const int W = (int)xc.size(-1);
  const int64_t n = xc.numel() / W;
  auto sizes = xc.sizes().vec();
  if (!use_cvm) sizes.back() = W - 2;
  auto y = torch::empty(sizes, x.options());
  launch_cvm_fwd(P<float>(xc), n, W, use_cvm, P<float>(y), cs());
  return y;
}

Tensor cvm_bwd(const Tensor& dy, const Tensor& cvm, int64_t W, bool use_cvm) {
  f32(dy, "dy");
  f32(cvm, "cvm");
  auto dyc = dy.contiguous(), cc = cvm.contiguous();
  const int Wo = use_cvm ? (int)W : (int)W - 2;
  const int64_t n = dyc.numel() / Wo;
  const int64_t crow = cc.numel() / 2;
  CX_CHECK(crow == n || crow == 1, "cvm rows must match dy rows (or be 1)");
  auto dx = torch::empty({n, W}, dy.options());
  launch_cvm_bwd(P<float>(dyc), P<float>(cc), n, (int)W, use_cvm, (int)crow, P<float>(dx), cs());
  return dx;
}

std::vector<Tensor> masked_dn_fwd(const Tensor& x, const Tensor& mask, const Tensor& bsize, const Tensor& bsum,
                                  const Tensor& bsq, const c10::optional<Tensor>& sw,
                                  const c10::optional<Tensor>& bias, double eps) {
  f32(x, "x");
  f32(mask, "mask");
  auto xc = x.contiguous(), mc = mask.contiguous();
  const int N = (int)xc.size(0), C = (int)xc.size(1);
  auto y = torch::empty_like(xc);
  const int rows = mdn_blocks(N);
  auto part = torch::empty({rows, 3, C}, x.options());
  launch_masked_dn_fwd(P<float>(xc), P<float>(mc), N, C, P<float>(bsize), P<float>(bsum), P<float>(bsq),
                       OP<float>(sw), OP<float>(bias), P<float>(y), P<float>(part), cs());
  auto stats = torch::empty({3, C}, x.options());
  launch_mdn_stats(P<float>(part), rows, C, (float)eps, P<float>(stats), cs());
  return {y, stats};
}

std::vector<Tensor> masked_dn_bwd(const Tensor& x, const Tensor& dy, const Tensor& mask, const Tensor& bsize,
                                  const Tensor& bsum, const Tensor& bsq, const c10::optional<Tensor>& sw) {
  f32(x, "x");
  f32(dy, "dy");
  auto xc = x.contiguous(), dc = dy.contiguous(), mc = mask.contiguous();
  const int N = (int)xc.size(0), C = (int)xc.size(1);
  auto dx = torch::empty_like(xc);
  const bool has_sw = sw.has_value() && sw->defined();
  const int rows = mdn_blocks(N);
  Tensor part, dsw, dbias;
  if (has_sw) part = torch::empty({rows, 2, C}, x.options());
  launch_masked_dn_bwd(P<float>(xc), P<float>(dc), P<float>(mc), N, C, P<float>(bsize), P<float>(bsum), P<float>(bsq),
                       OP<float>(sw), P<float>(dx), has_sw ? P<float>(part) : nullptr, cs());
  if (has_sw) {
    auto g = torch::empty({2, C}, x.options());
    launch_colsum_rows(P<float>(part), rows, 2, C, ColAffine(), P<float>(g), cs());
    dsw = g[0];
    dbias = g[1];
  }
  return {dx, dsw, dbias};
}

std::vector<Tensor> cnh_fwd(const Tensor& x, const Tensor& summary, int64_t F, int64_t E, double eps) {
  f32(x, "x");
  f32(summary, "summary");
  auto xc = x.contiguous();
  const int B = (int)xc.size(0);
  const int W = (int)(F * (3 * E + 1));
  CX_CHECK(xc.size(1) == F * 2 * E && summary.numel() == 3 * W, "cross_norm_hadamard shapes");
  CX_CHECK((size_t)2 * W * sizeof(float) <= 64 * 1024, "cross_norm_hadamard: too many output columns");
  auto y = torch::empty({B, W}, x.options());
  const int rows = cnh_blocks(B);
  auto part = torch::empty({rows, 2, W}, x.options());
  auto sc = summary.contiguous();
  launch_cnh_fwd(P<float>(xc), B, (int)F, (int)E, P<float>(sc), P<float>(y), P<float>(part), cs());
  // batch stats [1, mean raw, mean (raw-mean)^2 + eps]: rows 1 and 2 of the reduced partials
  auto stats = torch::empty({3, W}, x.options());
  ColAffine f;
  f.mul[0] = 1.f / (float)B;
  f.mul[1] = 1.f / (float)B;
  f.add[1] = (float)eps;
  launch_colsum_rows(P<float>(part), rows, 2, W, f, P<float>(stats) + W, cs());
  stats[0].fill_(1.0);
  return {y, stats};
}

Tensor cnh_bwd(const Tensor& x, const Tensor& dy, const Tensor& summary, int64_t F, int64_t E) {
  f32(x, "x");
  f32(dy, "dy");
  auto xc = x.contiguous(), dc = dy.contiguous(), sc = summary.contiguous();
  auto dx = torch::empty_like(xc);
  launch_cnh_bwd(P<float>(xc), P<float>(dc), (int)xc.size(0), (int)F, (int)E, P<float>(sc), P<float>(dx), cs());
  return dx;
}

// ints: need_filter, embed_filter, ets, co, quant, mcol, tradew, tn, tid, ecs, Epool, Eo
// floats: show_coeff, clk_coeff, embed_threshold, pad
SpvArgs spv_args(const Tensor& x, const Tensor& row_base, const Tensor& off, int64_t S, int64_t B,
                 const std::vector<int64_t>& ints, const std::vector<double>& fl) {
  f32(x, "x");
  CX_CHECK(ints.size() == 12 && fl.size() == 4, "spv: 12 int and 4 float attributes");
  CX_CHECK(row_base.scalar_type() == torch::kInt32 && row_base.numel() == S, "row_base int32 [S]");
  CX_CHECK(off.scalar_type() == torch::kInt32 && off.numel() == S * (B + 1), "offsets int32 [S][B+1]");
  SpvArgs a;
  a.x = P<float>(x);
  a.E = (int)x.size(1);
  a.row_base = P<int>(row_base);
  a.off = P<int>(off);
  a.S = (int)S;
  a.B = (int)B;
  a.need_filter = (int)ints[0];
  a.embed_filter = (int)ints[1];
  a.ets = (int)ints[2];
  a.co = (int)ints[3];
  a.quant = (int)ints[4];
  a.mcol = (int)ints[5];
  a.tradew = (int)ints[6];
  a.tn = (int)ints[7];
  a.tid = (int)ints[8];
  a.ecs = (int)ints[9];
  a.Epool = (int)ints[10];
  a.Eo = (int)ints[11];
  a.show_coeff = (float)fl[0];
  a.clk_coeff = (float)fl[1];
  a.embed_threshold = (float)fl[2];
  a.pad = (float)fl[3];
  CX_CHECK(a.Epool <= 4095 && a.Epool + (a.tradew ? a.tn : 0) == a.E, "spv: pool width");
  CX_CHECK((size_t)4 * a.ecs * a.Epool * sizeof(float) <= 64 * 1024, "spv: ecs * pool width too large");
  CX_CHECK(!a.embed_filter || a.co + a.ets <= a.E, "spv: embed filter width");
  CX_CHECK(!a.tradew || a.tid < a.tn, "spv: trade_id out of range");
  return a;
}

Tensor spv_fwd(const Tensor& x, const Tensor& row_base, const Tensor& off, const Tensor& thr, const Tensor& ftab,
               int64_t S, int64_t B, std::vector<int64_t> ints, std::vector<double> fl) {
  SpvArgs a = spv_args(x, row_base, off, S, B, ints, fl);
  CX_CHECK(ftab.scalar_type() == torch::kInt32 && ftab.numel() == a.Eo, "ftab int32 [Eo]");
  f32(thr, "thr");
  CX_CHECK(thr.numel() == S, "thr [S]");
  a.thr = P<float>(thr);
  a.ftab = P<int>(ftab);
  auto out = torch::empty({S, B, (int64_t)a.ecs * a.Eo}, x.options());
  a.out = P<float>(out);
  launch_spv_fwd(a, cs());
  return out;
}

Tensor spv_bwd(const Tensor& x, const Tensor& row_base, const Tensor& off, const Tensor& btab, const Tensor& dout,
               const Tensor& cvm, const c10::optional<Tensor>& qv, int64_t S, int64_t B, std::vector<int64_t> ints,
               std::vector<double> fl) {
  SpvArgs a = spv_args(x, row_base, off, S, B, ints, fl);
  CX_CHECK(btab.scalar_type() == torch::kInt32 && btab.numel() == a.Epool, "btab int32 [Epool]");
  f32(dout, "dout");
  f32(cvm, "cvm");
  CX_CHECK(dout.numel() == S * B * a.ecs * a.Eo, "dout [S][B][ecs*Eo]");
  a.btab = P<int>(btab);
  a.dout = P<float>(dout);
  a.cvm = P<float>(cvm);
  a.ncv = (int)(cvm.numel() / B);
  if (qv.has_value() && qv->defined() && qv->numel() > 0) {
    f32(*qv, "qv");
    a.qv = P<float>(*qv);
    a.nq = (int)(qv->numel() / B);
  }
  auto dx = torch::empty_like(x);
  a.dx = P<float>(dx);
  launch_spv_bwd(a, cs());
  return dx;
}

std::vector<Tensor> fused_seq_tensor(const Tensor& x, const Tensor& ad, int64_t bc, int64_t T, int64_t E, int64_t S,
                                     int64_t A, int64_t ad_off) {
  f32(x, "x");
  f32(ad, "ad");
  auto xc = x.contiguous(), ac = ad.contiguous();
  const int64_t ins = xc.size(0);
  CX_CHECK(xc.numel() == ins * bc * S * T * E && ac.numel() == ins * bc * A * E, "fused_seq_tensor shapes");
  CX_CHECK(A <= S && ad_off >= 0 && ad_off + A <= S, "fused_seq_tensor ad slots");
  auto o = x.options();
  auto din = torch::empty({bc, ins * T, 4 * A * E}, o);
  auto mask = torch::empty({bc, ins, T}, o);
  auto side = torch::empty({bc, ins * T, (S - A) * E}, o);
  auto sess = torch::empty({bc, ins * T, A, E}, o);
  launch_fused_seq_tensor(P<float>(xc), P<float>(ac), (int)ins, (int)bc, (int)T, (int)E, (int)S, (int)A, (int)ad_off,
                          P<float>(din), P<float>(mask), P<float>(side), P<float>(sess), cs());
  return {din, mask, side, sess};
}

}  // namespace

// device-resident pass batch assembly (batch_ops.hip).  Every index the
// kernels follow is checked here: order values against nrec, offset array
// lengths, output shapes.
int64_t batch_assemble(const Tensor& u64, const Tensor& uoff, const Tensor& f32v, const Tensor& foff,
                       const Tensor& order, const Tensor& sparse_idx, const Tensor& drefs, int64_t nu, int64_t nf,
                       int64_t Dw, int64_t nrec, int64_t begin, int64_t B, Tensor lod, Tensor tot, Tensor keys,
                       Tensor dense, Tensor overflow) {
  auto i64 = [](const Tensor& t, const char* n) {
    CX_CHECK(t.is_cuda() && t.is_contiguous() && t.scalar_type() == torch::kInt64,
             std::string(n) + " must be a contiguous int64 GPU tensor");
  };
  i64(u64, "u64");
  i64(uoff, "uoff");
  i64(foff, "foff");
  i64(order, "order");
  i64(lod, "lod");
  i64(tot, "tot");
  i64(keys, "keys");
  f32(f32v, "f32");
  f32(dense, "dense");
  CX_CHECK(sparse_idx.is_cuda() && sparse_idx.scalar_type() == torch::kInt32, "sparse_idx must be int32 GPU");
  CX_CHECK(drefs.is_cuda() && drefs.scalar_type() == torch::kInt32 && drefs.is_contiguous(), "drefs int32 GPU");
  CX_CHECK(overflow.is_cuda() && overflow.scalar_type() == torch::kInt32 && overflow.numel() >= 1, "overflow");
  const int64_t S = sparse_idx.numel();
  CX_CHECK(S >= 1 && S <= batch_assemble_max_slots(), "sparse slot count out of range");
  CX_CHECK(uoff.numel() == nrec * nu + 1 && foff.numel() == nrec * nf + 1, "offset arrays do not match nrec");
  CX_CHECK(begin >= 0 && B >= 1 && begin + B <= order.numel(), "batch range outside the pass order");
  CX_CHECK(lod.numel() == S * (B + 1) && tot.numel() >= S, "lod / tot shape");
  CX_CHECK(dense.numel() == B * Dw, "dense shape");
  CX_CHECK(drefs.dim() == 2 && drefs.size(1) == 4, "drefs must be [n, 4]");
  BatchSrc src;
  src.u64 = P<int64_t>(u64);
  src.uoff = P<int64_t>(uoff);
  src.f32 = P<float>(f32v);
  src.foff = P<int64_t>(foff);
  src.order = P<int64_t>(order);
  src.sparse_idx = P<int32_t>(sparse_idx);
  src.drefs = P<int32_t>(drefs);
  src.nu = (int)nu;
  src.nf = (int)nf;
  src.S = (int)S;
  src.ndref = (int)drefs.size(0);
  src.Dw = (int)Dw;
  launch_batch_assemble(src, begin, (int)B, P<int64_t>(lod), P<int64_t>(tot), P<int64_t>(keys), keys.numel(),
                        P<float>(dense), P<int32_t>(overflow), cs());
  return keys.numel();
}

void bind_ctr(py::module& m) {
  m.def("batch_assemble", &batch_assemble);
  m.def("spv_fwd", &spv_fwd);
  m.def("spv_bwd", &spv_bwd);
  m.def("fused_seq_tensor", &fused_seq_tensor);
  m.def("sgemm", &sgemm, py::arg("A"), py::arg("B"), py::arg("C"), py::arg("bias"), py::arg("M"), py::arg("N"),
        py::arg("K"), py::arg("batch"), py::arg("a_strides"), py::arg("b_strides"), py::arg("sC"), py::arg("ldc"),
        py::arg("sBias") = 0, py::arg("bias_scale") = 1.0, py::arg("alpha") = 1.0, py::arg("accumulate") = false);
  m.def("colsum_strided", &colsum_strided);
  m.def("hgemm", &hgemm);
  m.def("sfc_dw", &sfc_dw, py::arg("x"), py::arg("d"), py::arg("dW"), py::arg("db"), py::arg("a_scale"),
        py::arg("b_scale"), py::arg("alpha"), py::arg("out_scale"), py::arg("splits"), py::arg("mode") = 0);
  m.def("f3gemm_nt", &f3gemm_nt);
  m.def("h16_epi", &h16_epi);
  m.def("sfc", &sfc);
  m.def("int8_fc", &int8_fc);
  m.def("rank_attention_fwd", &rank_attention_fwd);
  m.def("batch_fc_fwd", &batch_fc_fwd);
  m.def("batch_fc_bwd", &batch_fc_bwd);
  m.def("rank_attention_bwd", &rank_attention_bwd, py::arg("x"), py::arg("ro"), py::arg("W"), py::arg("dout"),
        py::arg("bucket"), py::arg("R"), py::arg("part") = 0);
  m.def("cvm_fwd", &cvm_fwd);
  m.def("cvm_bwd", &cvm_bwd);
  m.def("masked_dn_fwd", &masked_dn_fwd);
  m.def("masked_dn_bwd", &masked_dn_bwd);
  m.def("cnh_fwd", &cnh_fwd);
  m.def("cnh_bwd", &cnh_bwd);
}

}  // namespace pbx

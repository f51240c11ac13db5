// Torch bindings: implicit-GEMM convolution (+ BN-statistics epilogue) and BN from partials.
#include <algorithm>

#include "bindings/common.h"
#include "bindings/registry.h"

namespace hypbind {
namespace {

// Effective split-K count for a conv of nk reduction steps (conv_fwd's own rounding: no empty splits).
int plan_splits(int M, int K, int nk, int bm, int bn, int64_t splits_req) {
  int sp = splits_req > 0 ? (int)splits_req : (splits_req == 0 ? 1 : hyp::conv_fwd_splits(M, K, nk, bm, bn));
  sp = std::max(1, std::min(sp, nk));
  const int steps = (nk + sp - 1) / sp;
  return (nk + steps - 1) / steps;
}

// x [N,C,H,W] channels-last, w [K,C,R,S] channels-last -> (y [N,K,P,Q] channels-last, Σy, Σy² as
// [kStatSlots, K] slot partials).  The statistics are ADDED into `sums` ([kStatSlots*2*K] fp64, zeroed).
std::vector<at::Tensor> conv_fwd(const at::Tensor& x, const at::Tensor& w, int64_t sh, int64_t sw, int64_t ph,
                                 int64_t pw, bool stats, int64_t bm_req, int64_t bn_req, int64_t splits_req,
                                 const c10::optional<at::Tensor>& sums, int64_t stages,
                                 const c10::optional<at::Tensor>& xf_sums, const c10::optional<at::Tensor>& xf_w,
                                 const c10::optional<at::Tensor>& xf_b, const c10::optional<at::Tensor>& xf_rm,
                                 const c10::optional<at::Tensor>& xf_rv, double xf_momentum, double xf_eps,
                                 const c10::optional<at::Tensor>& xf_out, const c10::optional<at::Tensor>& xf_stats) {
  HYP_CHECK_CUDA_TENSOR(x);
  TORCH_CHECK(x.dim() == 4 && w.dim() == 4, "conv_fwd: 4D tensors");
  TORCH_CHECK(x.is_contiguous(at::MemoryFormat::ChannelsLast) && w.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv_fwd: channels-last input and weight required");
  TORCH_CHECK(x.scalar_type() == w.scalar_type() && (x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kHalf),
              "conv_fwd: bf16/f16 input and weight of one dtype");
  const int N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int K = w.size(0), R = w.size(2), S = w.size(3);
  TORCH_CHECK(w.size(1) == C, "conv_fwd: channel mismatch");
  TORCH_CHECK(hyp::conv_fwd_supported(C, K), "conv_fwd: needs C % 64 == 0 and K % 8 == 0");
  const int P = (H + 2 * ph - R) / sh + 1, Q = (W + 2 * pw - S) / sw + 1;
  TORCH_CHECK(P > 0 && Q > 0, "conv_fwd: empty output");
  const at::DeviceGuard guard(x.device());
  auto y = at::empty({N, K, P, Q}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  const int M = N * P * Q;
  int bm = 128, bn = 128;
  hyp::conv_fwd_tile(M, K, &bm, &bn);
  if (bm_req > 0) bm = (int)bm_req;  // tuning sweeps
  if (bn_req > 0) bn = (int)bn_req;
  TORCH_CHECK((bm == 64 || bm == 128) && (bn == 64 || bn == 128) && !(bm == 64 && bn == 128),
              "conv_fwd: tiles 64x64, 128x64 or 128x128");
  // split-K below ~2 workgroups per CU (the stats then come from the reduce)
  const int splits = plan_splits(M, K, R * S * (C / 64), bm, bn, splits_req);
  at::Tensor acc, slabs;
  if (stats) acc = stats_sums(sums, K, x);
  if (splits > 1) slabs = at::empty({splits, M, K}, x.options().dtype(at::kFloat));
  // xf_sums: x is the RAW output of a conv whose training BN (+ ReLU) this conv applies to its input
  // as it reads it (hyp_kernels.h ConvInXform); xf_stats [2, C] fp32 receives save_mean / invstd,
  // xf_out (optional, x's shape) the transformed activation
  hyp::ConvInXform xf;
  const bool has_xf = xf_sums.has_value() && xf_sums->defined();
  if (has_xf) {
    TORCH_CHECK(xf_sums->scalar_type() == at::kDouble && xf_sums->is_contiguous() &&
                    xf_sums->numel() == 2 * C * hyp::kStatSlots && xf_sums->device() == x.device(),
                "conv_fwd: xf_sums must be a contiguous fp64 [kStatSlots * 2 * C] tensor on x's device");
    TORCH_CHECK(xf_stats.has_value() && xf_stats->scalar_type() == at::kFloat && xf_stats->is_contiguous() &&
                    xf_stats->numel() == 2 * C,
                "conv_fwd: xf_stats must be a contiguous fp32 [2, C] tensor");
    TORCH_CHECK(C <= hyp::kXfMaxC, "conv_fwd: input transform supports at most ", hyp::kXfMaxC, " channels");
    auto chk = [&](const c10::optional<at::Tensor>& t, const char* nm) -> float* {
      if (!t.has_value() || !t->defined()) return nullptr;
      TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous() && t->numel() == C, "conv_fwd: ", nm,
                  " must be a contiguous fp32 [C] tensor");
      return t->data_ptr<float>();
    };
    xf.sums = xf_sums->data_ptr<double>();
    xf.weight = chk(xf_w, "xf_w");
    xf.bias = chk(xf_b, "xf_b");
    xf.running_mean = chk(xf_rm, "xf_rm");
    xf.running_var = chk(xf_rv, "xf_rv");
    TORCH_CHECK((xf.running_mean == nullptr) == (xf.running_var == nullptr), "conv_fwd: xf_rm and xf_rv together");
    xf.momentum = (float)xf_momentum;
    xf.eps = (float)xf_eps;
    xf.save_mean = xf_stats->data_ptr<float>();
    xf.save_invstd = xf_stats->data_ptr<float>() + C;
    if (xf_out.has_value() && xf_out->defined()) {
      TORCH_CHECK(xf_out->sizes() == x.sizes() && xf_out->scalar_type() == x.scalar_type() &&
                      xf_out->is_contiguous(at::MemoryFormat::ChannelsLast) && !xf_out->is_same(x),
                  "conv_fwd: xf_out must be a separate channels-last tensor shaped like x");
      TORCH_CHECK(sh == 1 && sw == 1 && 2 * ph == R - 1 && 2 * pw == S - 1,
                  "conv_fwd: xf_out needs stride 1 and 'same' padding (the centre tap covers every pixel)");
      xf.out = xf_out->data_ptr();
    }
  }
  HYP_CHECK_HIP(hyp::conv_fwd(dtype_code(x), x.data_ptr(), w.data_ptr(), y.data_ptr(), device_zero_page(x.device()),
                              stats ? acc.data_ptr<double>() : nullptr, stats ? acc.data_ptr<double>() + K : nullptr, N, H,
                              W, C, K, P, Q, R, S, (int)sh, (int)sw, (int)ph, (int)pw, bm, bn, 0, splits,
                              splits > 1 ? slabs.data_ptr<float>() : nullptr, cur_stream(), 1.f, nullptr, nullptr,
                              nullptr, 0, 1, 0, 0, (int)stages, has_xf ? &xf : nullptr));
  if (!stats) return {y, at::Tensor(), at::Tensor()};
  return {y, acc.select(1, 0), acc.select(1, 1)};  // [kStatSlots, K] each: .sum(0) = per-channel totals
}

// Eval-mode conv -> BN -> (+ residual) -> (ReLU) in one launch: y = act(conv(x, w) * scale[k] +
// shift[k] (+ residual)), scale / shift the BN's running-stat affine (fp32 [K]).
at::Tensor conv_fwd_affine(const at::Tensor& x, const at::Tensor& w, int64_t sh, int64_t sw, int64_t ph, int64_t pw,
                           const at::Tensor& scale, const at::Tensor& shift, const c10::optional<at::Tensor>& residual,
                           bool act) {
  HYP_CHECK_CUDA_TENSOR(x);
  TORCH_CHECK(x.dim() == 4 && w.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                  w.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv_fwd_affine: channels-last 4D input and weight");
  TORCH_CHECK(x.scalar_type() == w.scalar_type() && (x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kHalf),
              "conv_fwd_affine: bf16/f16 input and weight of one dtype");
  const int N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int K = w.size(0), R = w.size(2), S = w.size(3);
  TORCH_CHECK(w.size(1) == C && hyp::conv_fwd_supported(C, K), "conv_fwd_affine: needs C % 64 == 0, K % 8 == 0");
  TORCH_CHECK(scale.scalar_type() == at::kFloat && shift.scalar_type() == at::kFloat && scale.numel() == K &&
                  shift.numel() == K && scale.is_contiguous() && shift.is_contiguous(),
              "conv_fwd_affine: fp32 [K] scale / shift");
  const int P = (H + 2 * ph - R) / sh + 1, Q = (W + 2 * pw - S) / sw + 1;
  TORCH_CHECK(P > 0 && Q > 0, "conv_fwd_affine: empty output");
  const at::DeviceGuard guard(x.device());
  auto y = at::empty({N, K, P, Q}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  const bool has_res = residual.has_value() && residual->defined();
  if (has_res)
    TORCH_CHECK(residual->sizes() == y.sizes() && residual->scalar_type() == y.scalar_type() &&
                    residual->is_contiguous(at::MemoryFormat::ChannelsLast),
                "conv_fwd_affine: residual must match the output (shape, dtype, channels-last)");
  const int M = N * P * Q;
  int bm = 128, bn = 128;
  hyp::conv_fwd_tile(M, K, &bm, &bn);
  const int splits = plan_splits(M, K, R * S * (C / 64), bm, bn, -1);
  at::Tensor slabs;
  if (splits > 1) slabs = at::empty({splits, M, K}, x.options().dtype(at::kFloat));
  hyp::SplitkEpilogue ep;
  ep.N = K;
  ep.scale = scale.data_ptr<float>();
  ep.shift = shift.data_ptr<float>();
  ep.residual = has_res ? residual->data_ptr() : nullptr;
  ep.act = act ? 1 : 0;
  HYP_CHECK_HIP(hyp::conv_fwd(dtype_code(x), x.data_ptr(), w.data_ptr(), y.data_ptr(), device_zero_page(x.device()),
                              nullptr, nullptr, N, H, W, C, K, P, Q, R, S, (int)sh, (int)sw, (int)ph, (int)pw, bm, bn,
                              0, splits, splits > 1 ? slabs.data_ptr<float>() : nullptr, cur_stream(), 1.f, &ep));
  return y;
}

// ---- fused linear + cross-entropy (ops/cross_entropy.py) ----------------------------------------
namespace {
hyp::CeEpilogue ce_args(const c10::optional<at::Tensor>& bias, const at::Tensor& target, int64_t ignore, int64_t M,
                        int64_t V, const at::Tensor& x) {
  TORCH_CHECK(target.is_contiguous() && target.scalar_type() == at::kLong && target.numel() == M &&
                  target.device() == x.device(),
              "linear_ce: target must be a contiguous int64 [M] tensor on the input's device");
  hyp::CeEpilogue ce;
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->is_contiguous() && bias->numel() == V,
                "linear_ce: bias must be a contiguous fp32 [V] tensor");
    ce.bias = bias->data_ptr<float>();
  }
  ce.target = target.data_ptr<int64_t>();
  ce.ignore = ignore;
  return ce;
}

void check_ce_operands(const at::Tensor& x, const at::Tensor& w) {
  HYP_CHECK_CUDA_TENSOR(x);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && x.is_contiguous() && w.is_contiguous() && x.size(1) == w.size(1),
              "linear_ce: contiguous x [M, E], w [V, E]");
  TORCH_CHECK(x.scalar_type() == w.scalar_type() && (x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kHalf),
              "linear_ce: bf16/f16 x and w of one dtype");
  TORCH_CHECK(x.size(1) % 64 == 0, "linear_ce: E % 64 == 0");
}
}  // namespace

// Pass 1: (lse [M], loss_rows [M]) of z = x wᵀ (+ b) over all V classes without storing z.
std::vector<at::Tensor> linear_ce_lse(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& bias,
                                      const at::Tensor& target, int64_t ignore, int64_t bn) {
  check_ce_operands(x, w);
  const int64_t M = x.size(0), E = x.size(1), V = w.size(0);
  TORCH_CHECK(M < INT32_MAX && V < INT32_MAX, "linear_ce: sizes");
  const at::DeviceGuard guard(x.device());
  hyp::CeEpilogue ce = ce_args(bias, target, ignore, M, V, x);
  TORCH_CHECK(bn == 64 || bn == 128, "linear_ce_lse: bn 64 or 128");
  const int kcols = (int)((V + 7) / 8 * 8);
  const int tiles = (kcols + (int)bn - 1) / (int)bn;
  auto fopt = x.options().dtype(at::kFloat);
  auto part = at::empty({(int64_t)tiles * M * 2}, fopt);
  auto zt = at::zeros({M}, fopt);
  auto lse = at::empty({M}, fopt);
  auto loss_rows = at::empty({M}, fopt);
  ce.part = reinterpret_cast<float2*>(part.data_ptr<float>());
  ce.zt = zt.data_ptr<float>();
  HYP_CHECK_HIP(hyp::linear_ce(dtype_code(x), 1, x.data_ptr(), w.data_ptr(), nullptr, device_zero_page(x.device()),
                               (int)M, (int)E, kcols, (int)V, ce, cur_stream(), (int)bn));
  HYP_CHECK_HIP(hyp::ce_lse_combine(ce.part, tiles, (int)M, ce.zt, ce.target, ignore, lse.data_ptr<float>(),
                                    loss_rows.data_ptr<float>(), cur_stream()));
  return {lse, loss_rows};
}

// Pass 2: dz [M, ceil8(n)] of classes [c0, c0 + n) (columns >= n are zero): the softmax gradient
// (exp(z - lse) - onehot) * scale straight from the recomputed GEMM accumulators.
at::Tensor linear_ce_grad(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& bias,
                          const at::Tensor& target, int64_t ignore, const at::Tensor& lse, const at::Tensor& scale,
                          int64_t c0, int64_t n, int64_t bn) {
  check_ce_operands(x, w);
  const int64_t M = x.size(0), E = x.size(1), V = w.size(0);
  TORCH_CHECK(c0 >= 0 && n >= 1 && c0 + n <= V, "linear_ce_grad: class range");
  TORCH_CHECK(lse.scalar_type() == at::kFloat && lse.numel() == M && scale.scalar_type() == at::kFloat &&
                  scale.numel() == 1 && lse.device() == x.device() && scale.device() == x.device(),
              "linear_ce_grad: fp32 lse [M] and device scalar scale");
  const at::DeviceGuard guard(x.device());
  hyp::CeEpilogue ce = ce_args(bias, target, ignore, M, V, x);
  ce.col_off = (int)c0;
  ce.lse = lse.data_ptr<float>();
  ce.scale = scale.data_ptr<float>();
  const int kcols = (int)((n + 7) / 8 * 8);
  auto dz = at::empty({M, kcols}, x.options());
  const char* wrow = static_cast<const char*>(w.data_ptr()) + c0 * E * w.element_size();
  TORCH_CHECK(bn == 64 || bn == 128, "linear_ce_grad: bn 64 or 128");
  HYP_CHECK_HIP(hyp::linear_ce(dtype_code(x), 2, x.data_ptr(), wrow, dz.data_ptr(), device_zero_page(x.device()),
                               (int)M, (int)E, kcols, (int)n, ce, cur_stream(), (int)bn));
  return dz;
}

// Deferred weight-gradient reduce (per device): the split-K reduce of the last conv_wgrad(defer=True)
// waits here and rides on the next conv_wgrad launch as extra workgroups; conv_wgrad_flush() runs
// it standalone.  The partials tensor and the OUTPUT's storage are held until the kernel that uses
// them is queued (stream order protects the reuse of their memory after that).  The output is held
// by storage, not as a tensor: an extra tensor reference would stop AccumulateGrad from stealing
// the gradient (it would clone the not-yet-reduced values instead).
struct PendingWgrad {
  at::Tensor part;
  c10::Storage out_storage;
  void* out = nullptr;
  int out_dtype = 0;
  int64_t n = 0;
  int splits = 0;
  float alpha = 1.f;
  hipStream_t stream = nullptr;
};
// leaked on purpose: no tensor destructor may run after the HIP runtime is torn down at exit
PendingWgrad* const g_pending_wgrad = new PendingWgrad[64];

bool conv_wgrad_flush_dev(int dev) {
  PendingWgrad& p = g_pending_wgrad[dev];
  if (!p.part.defined()) return false;
  PendingWgrad q = std::move(p);
  p = PendingWgrad{};
  HYP_CHECK_HIP(hyp::splitk_reduce(q.out_dtype, q.part.data_ptr<float>(), q.out, q.n, q.splits, q.stream, q.alpha));
  return true;
}

bool conv_wgrad_flush() {
  bool any = false;
  for (int d = 0; d < 64; ++d) any |= conv_wgrad_flush_dev(d);
  return any;
}

// The pending reduce of this device's stream, taken out to ride on the next weight-gradient launch
// (another stream's pending reduce is flushed instead: no chaining across streams).
hyp::WgradPendingReduce take_pending_wgrad(int dev, hipStream_t stream, PendingWgrad& taken) {
  PendingWgrad& pend = g_pending_wgrad[dev];
  if (pend.part.defined() && pend.stream != stream) conv_wgrad_flush_dev(dev);
  hyp::WgradPendingReduce pr{};
  if (pend.part.defined()) {
    taken = std::move(pend);
    pend = PendingWgrad{};
    pr.part = taken.part.data_ptr<float>();
    pr.out = taken.out;
    pr.n = taken.n;
    pr.splits = taken.splits;
    pr.alpha = taken.alpha;
    pr.dtype = taken.out_dtype;
  }
  return pr;
}

void park_pending_wgrad(int dev, const at::Tensor& part, const at::Tensor& dw, int splits, float alpha,
                        hipStream_t stream) {
  PendingWgrad& pend = g_pending_wgrad[dev];
  pend.part = part;
  pend.out_storage = dw.storage();
  pend.out = dw.data_ptr();
  pend.out_dtype = dtype_code(dw);
  pend.n = dw.numel();
  pend.splits = splits;
  pend.alpha = alpha;
  pend.stream = stream;
}

// Stride-1 data gradient: dy [N,K,P,Q] channels-last, w [K,C,R,S] channels-last (the forward
// filter, NOT flipped) -> dx [N,C,H,W] channels-last with H = P + R - 1 - 2 ph.
// bn_mode >= 0: BN-backward epilogue for the BN layer whose OUTPUT is dx's tensor (hyp::BnBwdEpilogue):
// bn_x its input [N,C,H,W], bn_y its output (mode 2), bn_w/bn_b/bn_mean/bn_invstd (mode 1), bn_sums
// a zeroed fp64 [kStatSlots*2*C] accumulator; the result is then dz = dx · mask.
// The weight gradient that may ride in the data gradient's launch (conv_dual.hip)
struct WgradReq {
  const at::Tensor* x = nullptr;  // the conv's input [N, C, H, W] channels-last
  int64_t R = 1, S = 1, sh = 1, sw = 1, ph = 0, pw = 0;
  int64_t bm = 64, bn = 64;       // weight-gradient tile
  int64_t splits = -1;            // <= 0: conv_wgrad_plan's (64 x 64 tiles)
  bool defer = false;
  int64_t order = 0;
  at::Tensor dw;                  // out (given: written in place — a gradient handed to autograd earlier)
};

// Validate the request against dY [N, K, P, Q] and fill the kernel-side description (allocates dW and
// the split-K partials)
void fill_dual(hyp::DualWgrad& dual, WgradReq& wg, const at::Tensor& dy, at::Tensor& wpart, const char* who) {
  const int N = dy.size(0), K = dy.size(1), P = dy.size(2), Q = dy.size(3);
  const at::Tensor& x = *wg.x;
  TORCH_CHECK(x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast) && x.scalar_type() == dy.scalar_type() &&
                  x.size(0) == N && dy.is_contiguous(at::MemoryFormat::ChannelsLast),
              who, ": x and dY must be channels-last [N, C, H, W] / [N, K, P, Q] tensors of one dtype");
  const int Cx = x.size(1), Hi = x.size(2), Wi = x.size(3);
  TORCH_CHECK(P == (Hi + 2 * wg.ph - wg.R) / wg.sh + 1 && Q == (Wi + 2 * wg.pw - wg.S) / wg.sw + 1, who,
              ": dY spatial shape vs x");
  TORCH_CHECK(hyp::conv_wgrad_supported(Cx, K), who, ": needs C % 64 == 0 and K % 8 == 0");
  TORCH_CHECK((wg.bm == 64 || wg.bm == 128) && (wg.bn == 64 || wg.bn == 128) && Cx % wg.bn == 0, who,
              ": weight-gradient tile 64 / 128 each (bn | C)");
  int wbm, wbn, wsplits, per;
  hyp::conv_wgrad_plan(N * P * Q, K, Cx, (int)wg.R, (int)wg.S, &wbm, &wbn, &wsplits, &per);
  if (wg.splits > 0) {
    const int steps = (N * P * Q + 63) / 64;
    per = (steps + (int)wg.splits - 1) / (int)wg.splits;
    wsplits = (steps + per - 1) / per;
  }
  if (wg.dw.defined()) {
    TORCH_CHECK(wg.dw.dim() == 4 && wg.dw.size(0) == K && wg.dw.size(1) == Cx && wg.dw.size(2) == wg.R &&
                    wg.dw.size(3) == wg.S && wg.dw.scalar_type() == x.scalar_type() &&
                    wg.dw.is_contiguous(at::MemoryFormat::ChannelsLast) && wg.dw.device() == x.device(),
                who, ": out must be a channels-last [K, C, R, S] tensor of x's dtype");
  } else {
    wg.dw = at::empty({K, Cx, wg.R, wg.S}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  }
  if (wsplits > 1) wpart = at::empty({(int64_t)wsplits * K * wg.R * wg.S * Cx}, x.options().dtype(at::kFloat));
  dual.dy = dy.data_ptr();
  dual.x = x.data_ptr();
  dual.dw = wg.dw.data_ptr();
  dual.partials = wsplits > 1 ? wpart.data_ptr<float>() : nullptr;
  dual.N = N, dual.H = Hi, dual.W = Wi, dual.C = Cx, dual.K = K, dual.P = P, dual.Q = Q;
  dual.R = (int)wg.R, dual.S = (int)wg.S, dual.sh = (int)wg.sh, dual.sw = (int)wg.sw;
  dual.ph = (int)wg.ph, dual.pw = (int)wg.pw;
  dual.bm = (int)wg.bm, dual.bn = (int)wg.bn;
  dual.splits = wsplits, dual.steps_per_split = per;
  dual.defer_reduce = wg.defer && wsplits > 1;
  dual.order = (int)wg.order;
}

at::Tensor conv_dgrad_impl(const at::Tensor& dy, const at::Tensor& w, int64_t ph, int64_t pw, int64_t bm_req,
                           int64_t bn_req, int64_t splits_req, const c10::optional<at::Tensor>& addend,
                           const c10::optional<at::Tensor>& bn_x, const c10::optional<at::Tensor>& bn_y,
                           const c10::optional<at::Tensor>& bn_w, const c10::optional<at::Tensor>& bn_b,
                           const c10::optional<at::Tensor>& bn_mean, const c10::optional<at::Tensor>& bn_invstd,
                           int64_t bn_mode, const c10::optional<at::Tensor>& bn_sums, int64_t stride, int64_t Hx,
                           int64_t Wx, int64_t stages, WgradReq* wg) {
  HYP_CHECK_CUDA_TENSOR(dy);
  TORCH_CHECK(dy.dim() == 4 && w.dim() == 4, "conv_dgrad: 4D tensors");
  TORCH_CHECK(dy.is_contiguous(at::MemoryFormat::ChannelsLast) && w.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv_dgrad: channels-last dy and weight required");
  TORCH_CHECK(dy.scalar_type() == w.scalar_type() &&
                  (dy.scalar_type() == at::kBFloat16 || dy.scalar_type() == at::kHalf),
              "conv_dgrad: bf16/f16 dy and weight of one dtype");
  const int N = dy.size(0), K = dy.size(1), P = dy.size(2), Q = dy.size(3);
  const int C = w.size(1), R = w.size(2), S = w.size(3);
  TORCH_CHECK(w.size(0) == K, "conv_dgrad: channel mismatch");
  TORCH_CHECK(hyp::conv_fwd_supported(K, C), "conv_dgrad: needs K % 64 == 0 and C % 8 == 0");
  const int dph = R - 1 - (int)ph, dpw = S - 1 - (int)pw;
  TORCH_CHECK(dph >= 0 && dpw >= 0, "conv_dgrad: padding larger than the filter");
  TORCH_CHECK(stride == 1 || stride == 2, "conv_dgrad: stride 1 or 2");
  const bool s2 = stride == 2;
  // stride 2: dX [N, C, Hx, Wx] with Hx, Wx even and the forward's output size equal to dY's
  if (s2)
    TORCH_CHECK(Hx % 2 == 0 && Wx % 2 == 0 && Hx / 2 == P && Wx / 2 == Q && (Hx + 2 * ph - R) / 2 + 1 == P &&
                    (Wx + 2 * pw - S) / 2 + 1 == Q,
                "conv_dgrad: stride 2 needs an even dX size whose forward output is dY's (Hx = 2 P)");
  const int H = s2 ? (int)Hx : P + R - 1 - 2 * (int)ph, W = s2 ? (int)Wx : Q + S - 1 - 2 * (int)pw;
  TORCH_CHECK(H > 0 && W > 0, "conv_dgrad: empty output");
  const at::DeviceGuard guard(dy.device());
  auto dx = at::empty({N, C, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  int bm = 128, bn = 128;
  hyp::conv_fwd_tile(N * H * W, C, &bm, &bn);
  if (bn_mode >= 0) {
    // BN-backward epilogue: its store phase (x / y reads, masked stores, column sums) is memory
    // bound — 64-wide tiles keep 3-4 workgroups per CU on it (128x128: 264 VGPRs, one; 3x slower
    // on layer1, scripts/bnb_tiles.py); 64 rows for 1x1 (one MFMA k-step), 128 for 3x3
    bn = 64;
    bm = R * S == 1 ? 64 : 128;
  }
  if (bm_req > 0) bm = (int)bm_req;
  if (bn_req > 0) bn = (int)bn_req;
  TORCH_CHECK((bm == 64 || bm == 128) && (bn == 64 || bn == 128) && !(bm == 64 && bn == 128),
              "conv_dgrad: tiles 64x64, 128x64 or 128x128");
  const int splits = s2 ? 1 : plan_splits(N * H * W, C, R * S * (K / 64), bm, bn, splits_req);
  at::Tensor slabs;
  if (splits > 1) slabs = at::empty({splits, (int64_t)N * H * W, C}, dy.options().dtype(at::kFloat));
  const bool add = addend.has_value() && addend->defined();
  if (add)
    TORCH_CHECK(addend->sizes() == dx.sizes() && addend->scalar_type() == dx.scalar_type() &&
                    addend->is_contiguous(at::MemoryFormat::ChannelsLast) && addend->device() == dx.device(),
                "conv_dgrad: addend must match dx (shape, dtype, channels-last)");
  hyp::BnBwdEpilogue bnb;
  const bool fuse_bn = bn_mode >= 0;
  if (fuse_bn) {
    TORCH_CHECK(bn_mode <= 2 && bn_x.has_value() && bn_x->defined() && bn_sums.has_value() && bn_sums->defined(),
                "conv_dgrad: BN epilogue needs bn_x and bn_sums");
    TORCH_CHECK(bn_x->sizes() == dx.sizes() && bn_x->scalar_type() == dx.scalar_type() &&
                    bn_x->is_contiguous(at::MemoryFormat::ChannelsLast),
                "conv_dgrad: bn_x must match dx (shape, dtype, channels-last)");
    TORCH_CHECK(bn_sums->scalar_type() == at::kDouble && bn_sums->is_contiguous() &&
                    bn_sums->numel() == 2 * C * hyp::kStatSlots,
                "conv_dgrad: bn_sums must be a zeroed fp64 [kStatSlots * 2 * C] tensor");
    if (bn_mode == 2)
      TORCH_CHECK(bn_y.has_value() && bn_y->defined() && bn_y->sizes() == dx.sizes() &&
                      bn_y->scalar_type() == dx.scalar_type() && bn_y->is_contiguous(at::MemoryFormat::ChannelsLast),
                  "conv_dgrad: bn_y must match dx");
    if (bn_mode == 1)
      TORCH_CHECK(bn_mean.has_value() && bn_invstd.has_value() && bn_mean->numel() == C && bn_invstd->numel() == C,
                  "conv_dgrad: mode 1 needs bn_mean / bn_invstd");
    bnb.x = bn_x->data_ptr();
    bnb.y = bn_mode == 2 ? bn_y->data_ptr() : nullptr;
    bnb.w = ptr_or_null<float>(bn_w);
    bnb.b = ptr_or_null<float>(bn_b);
    bnb.mean = ptr_or_null<float>(bn_mean);
    bnb.invstd = ptr_or_null<float>(bn_invstd);
    bnb.mode = (int)bn_mode;
    bnb.sums = bn_sums->data_ptr<double>();
  }
  // the weight gradient of the same conv, from the same dY, in the same launch
  hyp::DualWgrad dual;
  PendingWgrad taken;  // (holds the taken pending reduce's partials until the launch is queued)
  at::Tensor wpart;
  const int dev = dy.device().index() < 0 ? 0 : dy.device().index();
  if (wg != nullptr) fill_dual(dual, *wg, dy, wpart, "conv_dgrad_wgrad");
  hyp::WgradPendingReduce pr{};
  if (wg != nullptr) {
    pr = take_pending_wgrad(dev, cur_stream(), taken);
    dual.pending = pr.part != nullptr ? &pr : nullptr;
  }
  HYP_CHECK_HIP(hyp::conv_fwd(dtype_code(dy), dy.data_ptr(), w.data_ptr(), dx.data_ptr(),
                              device_zero_page(dy.device()), nullptr, nullptr, N, P, Q, K, C, s2 ? H / 2 : H,
                              s2 ? W / 2 : W, R, S, 1, 1, s2 ? (int)ph : dph, s2 ? (int)pw : dpw, bm, bn, 1, splits,
                              splits > 1 ? slabs.data_ptr<float>() : nullptr, cur_stream(), 1.f, nullptr,
                              (add && (splits == 1 || fuse_bn)) ? addend->data_ptr() : nullptr,
                              fuse_bn ? &bnb : nullptr, 0, s2 ? 2 : 1, s2 ? H : 0, s2 ? W : 0, (int)stages, nullptr,
                              wg != nullptr ? &dual : nullptr));
  if (wg != nullptr && dual.defer_reduce) park_pending_wgrad(dev, wpart, wg->dw, dual.splits, 1.f, cur_stream());
  if (add && splits > 1 && !fuse_bn) dx.add_(*addend);  // the plain split-K reduce has no addend input
  return dx;
}

at::Tensor conv_dgrad(const at::Tensor& dy, const at::Tensor& w, int64_t ph, int64_t pw, int64_t bm_req,
                      int64_t bn_req, int64_t splits_req, const c10::optional<at::Tensor>& addend,
                      const c10::optional<at::Tensor>& bn_x, const c10::optional<at::Tensor>& bn_y,
                      const c10::optional<at::Tensor>& bn_w, const c10::optional<at::Tensor>& bn_b,
                      const c10::optional<at::Tensor>& bn_mean, const c10::optional<at::Tensor>& bn_invstd,
                      int64_t bn_mode, const c10::optional<at::Tensor>& bn_sums, int64_t stride, int64_t Hx,
                      int64_t Wx, int64_t stages) {
  return conv_dgrad_impl(dy, w, ph, pw, bm_req, bn_req, splits_req, addend, bn_x, bn_y, bn_w, bn_b, bn_mean,
                         bn_invstd, bn_mode, bn_sums, stride, Hx, Wx, stages, nullptr);
}

// conv_dgrad + the same conv's weight gradient dW = dYᵀ·X (x, R, S, stride, padding: the FORWARD conv's)
// in one launch (conv_dual.hip) -> [dx, dw].  wg_splits <= 0: conv_wgrad_plan's pixel split;
// wg_defer: leave dW's split-K reduce pending (conv_wgrad(defer=True) semantics).
std::vector<at::Tensor> conv_dgrad_wgrad(const at::Tensor& dy, const at::Tensor& w, int64_t ph, int64_t pw,
                                         int64_t bm_req, int64_t bn_req, int64_t splits_req,
                                         const c10::optional<at::Tensor>& addend, const c10::optional<at::Tensor>& bn_x,
                                         const c10::optional<at::Tensor>& bn_y, const c10::optional<at::Tensor>& bn_w,
                                         const c10::optional<at::Tensor>& bn_b,
                                         const c10::optional<at::Tensor>& bn_mean,
                                         const c10::optional<at::Tensor>& bn_invstd, int64_t bn_mode,
                                         const c10::optional<at::Tensor>& bn_sums, int64_t stride, int64_t Hx,
                                         int64_t Wx, int64_t stages, const at::Tensor& wg_x, int64_t wg_R, int64_t wg_S,
                                         int64_t wg_sh, int64_t wg_sw, int64_t wg_ph, int64_t wg_pw, int64_t wg_splits,
                                         bool wg_defer, int64_t order) {
  HYP_CHECK_CUDA_TENSOR(wg_x);
  WgradReq wg;
  wg.x = &wg_x;
  wg.R = wg_R, wg.S = wg_S, wg.sh = wg_sh, wg.sw = wg_sw, wg.ph = wg_ph, wg.pw = wg_pw;
  wg.splits = wg_splits, wg.defer = wg_defer, wg.order = order;
  at::Tensor dx = conv_dgrad_impl(dy, w, ph, pw, bm_req, bn_req, splits_req, addend, bn_x, bn_y, bn_w, bn_b, bn_mean,
                                  bn_invstd, bn_mode, bn_sums, stride, Hx, Wx, stages, &wg);
  return {dx, wg.dw};
}

// bn_bwd_dx (norm_ops.cpp) + the weight gradient of the conv ABOVE this BN layer (its dY wg_dy, input
// wg_x, forward geometry) in one launch (bn_wgrad.hip) -> [dx, dweight, dbias, dw].  wg_defer:
// leave dW's split-K reduce pending (conv_wgrad(defer=True) semantics); an earlier pending reduce
// rides on this launch.
std::vector<at::Tensor> bn_bwd_dx_wgrad(const at::Tensor& dz, const at::Tensor& x,
                                        const c10::optional<at::Tensor>& weight, const at::Tensor& save_mean,
                                        const at::Tensor& save_invstd, bool training, const at::Tensor& sums,
                                        const at::Tensor& wg_dy, const at::Tensor& wg_x, int64_t wg_R, int64_t wg_S,
                                        int64_t wg_sh, int64_t wg_sw, int64_t wg_ph, int64_t wg_pw, int64_t wg_bm,
                                        int64_t wg_bn, int64_t wg_splits, bool wg_defer,
                                        const c10::optional<at::Tensor>& wg_out) {
  HYP_CHECK_CUDA_TENSOR(x);
  HYP_CHECK_CUDA_TENSOR(wg_x);
  HYP_CHECK_CUDA_TENSOR(wg_dy);
  const int64_t C = x.size(1);
  const int64_t M = x.numel() / C;
  TORCH_CHECK(x.dim() == 4 && dz.sizes() == x.sizes() && dz.scalar_type() == x.scalar_type() &&
                  dz.is_contiguous(at::MemoryFormat::ChannelsLast) && x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "bn_bwd_dx_wgrad: dz and x of one shape / dtype, channels-last");
  TORCH_CHECK(sums.scalar_type() == at::kDouble && sums.is_contiguous() && sums.numel() == 2 * C * hyp::kStatSlots,
              "bn_bwd_dx_wgrad: sums must be an fp64 [kStatSlots * 2 * C] tensor");
  TORCH_CHECK(save_mean.numel() == C && save_invstd.numel() == C, "bn_bwd_dx_wgrad: mean / invstd of C channels");
  const at::DeviceGuard guard(x.device());
  WgradReq wg;
  wg.x = &wg_x;
  wg.R = wg_R, wg.S = wg_S, wg.sh = wg_sh, wg.sw = wg_sw, wg.ph = wg_ph, wg.pw = wg_pw;
  wg.bm = wg_bm, wg.bn = wg_bn, wg.splits = wg_splits, wg.defer = wg_defer;
  if (wg_out.has_value() && wg_out->defined()) wg.dw = *wg_out;
  hyp::DualWgrad dual;
  at::Tensor wpart;
  fill_dual(dual, wg, wg_dy, wpart, "bn_bwd_dx_wgrad");
  auto dx = at::empty_like(x);
  auto dwb = at::empty({2, C}, x.options().dtype(at::kFloat));
  const int dev = x.device().index() < 0 ? 0 : x.device().index();
  PendingWgrad taken;
  hyp::WgradPendingReduce pr = take_pending_wgrad(dev, cur_stream(), taken);
  dual.pending = pr.part != nullptr ? &pr : nullptr;
  hipError_t e = hyp::bn_backward_dx_wgrad(dtype_code(x), dz.data_ptr(), x.data_ptr(), dx.data_ptr(), M, (int)C,
                                           ptr_or_null<float>(weight), save_mean.data_ptr<float>(),
                                           save_invstd.data_ptr<float>(), training ? 1 : 0, sums.data_ptr<double>(),
                                           dwb.data_ptr<float>(), dwb.data_ptr<float>() + C, dual,
                                           device_zero_page(x.device()), cur_stream());
  if (e == hipErrorNotSupported) {  // (f16) the two launches
    HYP_CHECK_HIP(hyp::bn_backward_dx(dtype_code(x), dz.data_ptr(), x.data_ptr(), dx.data_ptr(), M, (int)C,
                                      ptr_or_null<float>(weight), save_mean.data_ptr<float>(),
                                      save_invstd.data_ptr<float>(), training ? 1 : 0, sums.data_ptr<double>(),
                                      dwb.data_ptr<float>(), dwb.data_ptr<float>() + C, cur_stream()));
    e = hyp::conv_wgrad(dtype_code(x), dual.dy, dual.x, dual.dw, dual.partials, device_zero_page(x.device()), dual.N,
                        dual.H, dual.W, dual.C, dual.K, dual.P, dual.Q, dual.R, dual.S, dual.sh, dual.sw, dual.ph,
                        dual.pw, dual.bm, dual.bn, dual.splits, dual.steps_per_split, cur_stream(), 1.f,
                        dual.pending, dual.defer_reduce);
  }
  HYP_CHECK_HIP(e);
  if (dual.defer_reduce) park_pending_wgrad(dev, wpart, wg.dw, dual.splits, 1.f, cur_stream());
  return {dx, dwb[0], dwb[1], wg.dw};
}

// ---- skinny GEMMs (weight-streaming regime: few hundred tokens x large frozen weights) ----------
// The same implicit-GEMM kernel with R = S = 1 and split-K over the reduction: at M = 128 tokens a
// 4096 x 4096 projection is only 64 output tiles, so the reduction is split until ~600 workgroups
// stream disjoint weight slices (the vendor GEMM launched 64 workgroups: 0.6 TB/s of weight reads).
// Plan from scripts/skinny_sweep.py on MI355X (profiles/llama_r01/skinny_sweep.json): 64-wide
// tiles, 2 LDS stages, splits = ceil(600 / tiles) — 512-700 workgroups won at every Llama-2-7B
// projection shape, forward and data gradient.
namespace {
int skinny_splits(int M, int N, int Kred, int bm, int bn, int64_t splits_req) {
  if (splits_req > 0) return (int)splits_req;
  const int tiles = ((M + bm - 1) / bm) * ((N + bn - 1) / bn);
  const int nk = Kred / 64;
  int sp = (600 + tiles - 1) / tiles;
  return std::max(1, std::min(sp, nk / 4));
}
}  // namespace

// Rank-r epilogue arguments: U [M, r]; V [r, N] (v_nr = false) or [N, r] (v_nr = true); mask [M, N].
hyp::SplitkEpilogue make_epilogue(const c10::optional<at::Tensor>& U, const c10::optional<at::Tensor>& V, bool v_nr,
                                  const c10::optional<at::Tensor>& mask, double beta, int64_t M, int64_t N,
                                  const at::Tensor& like) {
  hyp::SplitkEpilogue ep;
  if (!(U.has_value() && U->defined())) return ep;
  TORCH_CHECK(V.has_value() && V->defined(), "low-rank epilogue: V required with U");
  const int64_t r = U->size(1);
  TORCH_CHECK(U->dim() == 2 && U->size(0) == M && U->is_contiguous() && U->scalar_type() == like.scalar_type(),
              "low-rank epilogue: U must be a contiguous [M, r] tensor of the output dtype");
  TORCH_CHECK(V->dim() == 2 && V->is_contiguous() && V->scalar_type() == like.scalar_type(),
              "low-rank epilogue: V must be contiguous, output dtype");
  TORCH_CHECK(v_nr ? (V->size(0) == N && V->size(1) == r) : (V->size(0) == r && V->size(1) == N),
              "low-rank epilogue: V must be [N, r] (v_nr) or [r, N]");
  TORCH_CHECK(N % 4 == 0 && r % 8 == 0 && r <= 64, "low-rank epilogue: N % 4 == 0, r % 8 == 0, r <= 64");
  ep.U = U->data_ptr();
  ep.V = V->data_ptr();
  ep.sv_j = v_nr ? 1 : N;
  ep.sv_n = v_nr ? r : 1;
  ep.N = (int)N;
  ep.r = (int)r;
  ep.beta = (float)beta;
  if (mask.has_value() && mask->defined()) {
    TORCH_CHECK(mask->numel() == M * N && mask->is_contiguous() && mask->scalar_type() == like.scalar_type(),
                "low-rank epilogue: mask must be a contiguous [M, N] tensor of the output dtype");
    ep.mask = mask->data_ptr();
  }
  return ep;
}

// y[M, N] = x[M, K] · w[N, K]ᵀ  (nn.Linear layout; K % 64 == 0, N % 8 == 0)
// alpha scales x·wᵀ; U/V/mask/beta add the rank-r epilogue (forces a split-K launch: it runs in the reduce).
at::Tensor linear_nt(const at::Tensor& x, const at::Tensor& w, int64_t splits_req, int64_t bn_req, double alpha,
                     const c10::optional<at::Tensor>& U, const c10::optional<at::Tensor>& V, bool v_nr,
                     const c10::optional<at::Tensor>& mask, double beta) {
  HYP_CHECK_CUDA_TENSOR(x);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && x.is_contiguous() && w.is_contiguous(), "linear_nt: contiguous 2D");
  TORCH_CHECK(x.scalar_type() == w.scalar_type() && (x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kHalf),
              "linear_nt: bf16/f16 of one dtype");
  const int M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K && hyp::conv_fwd_supported(K, N), "linear_nt: needs K % 64 == 0, N % 8 == 0");
  const at::DeviceGuard guard(x.device());
  auto y = at::empty({M, N}, x.options());
  const int bm = M <= 64 ? 64 : 128, bn = bn_req == 128 && bm == 128 ? 128 : 64;
  const hyp::SplitkEpilogue ep = make_epilogue(U, V, v_nr, mask, beta, M, N, x);
  int sp = skinny_splits(M, N, K, bm, bn, splits_req);
  if ((ep.U != nullptr || alpha != 1.0) && sp < 2) sp = std::min(2, K / 64);
  TORCH_CHECK(sp >= 2 || (ep.U == nullptr && alpha == 1.0), "linear_nt: epilogue needs K >= 128");
  at::Tensor part;
  if (sp > 1) part = at::empty({(int64_t)sp * M * N}, x.options().dtype(at::kFloat));
  HYP_CHECK_HIP(hyp::conv_fwd(dtype_code(x), x.data_ptr(), w.data_ptr(), y.data_ptr(), device_zero_page(x.device()),
                              nullptr, nullptr, M, 1, 1, K, N, 1, 1, 1, 1, 1, 1, 0, 0, bm, bn, 0, sp,
                              sp > 1 ? part.data_ptr<float>() : nullptr, cur_stream(), (float)alpha, &ep));
  return y;
}

// dx[M, K] = dy[M, N] · w[N, K]  (the data gradient of linear_nt; N % 64 == 0, K % 8 == 0)
at::Tensor linear_nn(const at::Tensor& dy, const at::Tensor& w, int64_t splits_req, int64_t bn_req, double alpha,
                     const c10::optional<at::Tensor>& U, const c10::optional<at::Tensor>& V, bool v_nr,
                     const c10::optional<at::Tensor>& mask, double beta) {
  HYP_CHECK_CUDA_TENSOR(dy);
  TORCH_CHECK(dy.dim() == 2 && w.dim() == 2 && dy.is_contiguous() && w.is_contiguous(), "linear_nn: contiguous 2D");
  TORCH_CHECK(dy.scalar_type() == w.scalar_type() &&
                  (dy.scalar_type() == at::kBFloat16 || dy.scalar_type() == at::kHalf),
              "linear_nn: bf16/f16 of one dtype");
  const int M = dy.size(0), N = dy.size(1), K = w.size(1);
  TORCH_CHECK(w.size(0) == N && hyp::conv_fwd_supported(N, K), "linear_nn: needs N % 64 == 0, K % 8 == 0");
  const at::DeviceGuard guard(dy.device());
  auto dx = at::empty({M, K}, dy.options());
  const int bm = M <= 64 ? 64 : 128, bn = bn_req == 128 && bm == 128 ? 128 : 64;
  const hyp::SplitkEpilogue ep = make_epilogue(U, V, v_nr, mask, beta, M, K, dy);
  int sp = skinny_splits(M, K, N, bm, bn, splits_req);
  if ((ep.U != nullptr || alpha != 1.0) && sp < 2) sp = std::min(2, N / 64);
  TORCH_CHECK(sp >= 2 || (ep.U == nullptr && alpha == 1.0), "linear_nn: epilogue needs N >= 128");
  at::Tensor part;
  if (sp > 1) part = at::empty({(int64_t)sp * M * K}, dy.options().dtype(at::kFloat));
  HYP_CHECK_HIP(hyp::conv_fwd(dtype_code(dy), dy.data_ptr(), w.data_ptr(), dx.data_ptr(),
                              device_zero_page(dy.device()), nullptr, nullptr, M, 1, 1, N, K, 1, 1, 1, 1, 1, 1, 0,
                              0, bm, bn, 1, sp, sp > 1 ? part.data_ptr<float>() : nullptr, cur_stream(), (float)alpha,
                              &ep));
  return dx;
}

// dy [N,K,P,Q] channels-last, x [N,C,H,W] channels-last -> dW [K,C,R,S] channels-last (x's dtype)
// bm / bn / splits < 0: automatic plan (conv_wgrad_plan); explicit values are for tuning sweeps.
// defer: leave this gradient's split-K reduce pending (see PendingWgrad); the values of the
// returned tensor are final only after the next conv_wgrad launch or conv_wgrad_flush().
at::Tensor conv_wgrad(const at::Tensor& dy, const at::Tensor& x, int64_t R, int64_t S, int64_t sh, int64_t sw,
                      int64_t ph, int64_t pw, int64_t bm_, int64_t bn_, int64_t splits_, double alpha, bool defer,
                      const c10::optional<at::Tensor>& out) {
  HYP_CHECK_CUDA_TENSOR(x);
  HYP_CHECK_CUDA_TENSOR(dy);
  TORCH_CHECK(x.dim() == 4 && dy.dim() == 4, "conv_wgrad: 4D tensors");
  TORCH_CHECK(x.is_contiguous(at::MemoryFormat::ChannelsLast) && dy.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv_wgrad: channels-last x and dy required");
  TORCH_CHECK(x.scalar_type() == dy.scalar_type() && (x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kHalf),
              "conv_wgrad: bf16/f16 x and dy of one dtype");
  const int N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int K = dy.size(1), P = dy.size(2), Q = dy.size(3);
  TORCH_CHECK(dy.size(0) == N, "conv_wgrad: batch mismatch");
  TORCH_CHECK(P == (H + 2 * ph - R) / sh + 1 && Q == (W + 2 * pw - S) / sw + 1, "conv_wgrad: dy spatial shape");
  TORCH_CHECK(hyp::conv_wgrad_supported(C, K), "conv_wgrad: needs C % 64 == 0 and K % 8 == 0");
  const at::DeviceGuard guard(x.device());
  at::Tensor dw;
  if (out.has_value() && out->defined()) {  // (a gradient handed to autograd before it was computed)
    dw = *out;
    TORCH_CHECK(dw.dim() == 4 && dw.size(0) == K && dw.size(1) == C && dw.size(2) == R && dw.size(3) == S &&
                    dw.scalar_type() == x.scalar_type() && dw.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                    dw.device() == x.device(),
                "conv_wgrad: out must be a channels-last [K, C, R, S] tensor of x's dtype");
  } else {
    dw = at::empty({K, C, R, S}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  }
  int bm, bn, splits, per;
  hyp::conv_wgrad_plan(N * P * Q, K, C, (int)R, (int)S, &bm, &bn, &splits, &per);
  if (bm_ > 0) bm = (int)bm_;
  if (bn_ > 0) bn = (int)bn_;
  if (splits_ > 0) {
    const int steps = (N * P * Q + 63) / 64;
    per = (steps + (int)splits_ - 1) / (int)splits_;
    splits = (steps + per - 1) / per;
  }
  at::Tensor part;
  if (splits > 1) part = at::empty({(int64_t)splits * K * R * S * C}, x.options().dtype(at::kFloat));
  const int dev = x.device().index() < 0 ? 0 : x.device().index();
  hipStream_t stream = cur_stream();
  PendingWgrad taken;
  const hyp::WgradPendingReduce pr = take_pending_wgrad(dev, stream, taken);
  const bool defer_now = defer && splits > 1;
  HYP_CHECK_HIP(hyp::conv_wgrad(dtype_code(x), dy.data_ptr(), x.data_ptr(), dw.data_ptr(),
                                splits > 1 ? part.data_ptr<float>() : nullptr, device_zero_page(x.device()), N, H,
                                W, C, K, P, Q, (int)R, (int)S, (int)sh, (int)sw, (int)ph, (int)pw, bm, bn, splits, per,
                                stream, (float)alpha, pr.part != nullptr ? &pr : nullptr, defer_now));
  if (defer_now) park_pending_wgrad(dev, part, dw, splits, (float)alpha, stream);
  return dw;
}

// BN forward (training) given the statistics sums [2, C] of x (conv epilogue): (y, save_mean, save_invstd)
std::vector<at::Tensor> bn_fwd_sums(const at::Tensor& x, const c10::optional<at::Tensor>& residual,
                                    const at::Tensor& sums, const c10::optional<at::Tensor>& weight,
                                    const c10::optional<at::Tensor>& bias, const c10::optional<at::Tensor>& running_mean,
                                    const c10::optional<at::Tensor>& running_var, double momentum, double eps,
                                    bool act) {
  HYP_CHECK_CUDA_TENSOR(x);
  TORCH_CHECK(is_rows_by_channels(x), "bn_fwd_sums: x must be channels-last");
  const int64_t C = x.size(1), M = x.numel() / C;
  TORCH_CHECK(sums.scalar_type() == at::kDouble && sums.is_contiguous() && sums.numel() == 2 * C * hyp::kStatSlots,
              "bn_fwd_sums: sums must be a contiguous fp64 [kStatSlots * 2 * C] tensor");
  if (residual.has_value() && residual->defined())
    TORCH_CHECK(residual->sizes() == x.sizes() && residual->scalar_type() == x.scalar_type() &&
                    is_rows_by_channels(*residual),
                "bn_fwd_sums: residual shape/dtype/layout mismatch");
  const at::DeviceGuard guard(x.device());
  auto y = at::empty_like(x);
  auto stats = at::empty({2, C}, x.options().dtype(at::kFloat));
  HYP_CHECK_HIP(hyp::bn_forward_from_sums(
      dtype_code(x), x.data_ptr(), vptr_or_null(residual), y.data_ptr(), M, (int)C, ptr_or_null<float>(weight),
      ptr_or_null<float>(bias), ptr_or_null<float>(running_mean), ptr_or_null<float>(running_var), (float)momentum,
      (float)eps, act ? 1 : 0, sums.data_ptr<double>(), stats.data_ptr<float>(), stats.data_ptr<float>() + C,
      cur_stream()));
  return {y, stats[0], stats[1]};
}

// ---- ResNet stem (csrc/kernels/stem.hip) ----------------------------------------------------
// x [N, C <= 4, H, W] channels-last -> Xs [N, 16, P + 3, Q + 3] channels-last (space-to-depth)
at::Tensor stem_s2d(const at::Tensor& x) {
  HYP_CHECK_CUDA_TENSOR(x);
  TORCH_CHECK(x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast) && x.size(1) >= 1 && x.size(1) <= 4,
              "stem_s2d: channels-last [N, C <= 4, H, W]");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kHalf, "stem_s2d: bf16/f16");
  const int N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int P = (H - 1) / 2 + 1, Q = (W - 1) / 2 + 1;
  const at::DeviceGuard guard(x.device());
  auto out = at::empty({N, 16, P + 3, Q + 3}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  HYP_CHECK_HIP(hyp::stem_s2d(dtype_code(x), x.data_ptr(), out.data_ptr(), N, H, W, C, P + 3, Q + 3, cur_stream()));
  return out;
}

at::Tensor stem_weight4(const at::Tensor& w) {
  HYP_CHECK_CUDA_TENSOR(w);
  TORCH_CHECK(w.dim() == 4 && w.size(2) == 7 && w.size(3) == 7 && w.size(1) >= 1 && w.size(1) <= 4,
              "stem_weight4: W [K, C <= 4, 7, 7]");
  const int K = w.size(0), C = w.size(1);
  const at::DeviceGuard guard(w.device());
  auto w4 = at::empty({K, 64, 4, 1}, w.options().memory_format(at::MemoryFormat::ChannelsLast));
  HYP_CHECK_HIP(hyp::stem_weight4(dtype_code(w), w.data_ptr(), w4.data_ptr(), K, C, w.stride(0), w.stride(1),
                                  w.stride(2), w.stride(3), cur_stream()));
  return w4;
}

at::Tensor stem_weight4_grad(const at::Tensor& dw4, int64_t C, bool channels_last) {
  HYP_CHECK_CUDA_TENSOR(dw4);
  TORCH_CHECK(dw4.dim() == 4 && dw4.size(1) == 64 && dw4.size(2) == 4 && dw4.size(3) == 1 &&
                  dw4.is_contiguous(at::MemoryFormat::ChannelsLast),
              "stem_weight4_grad: channels-last dW4 [K, 64, 4, 1]");
  const int K = dw4.size(0);
  const at::DeviceGuard guard(dw4.device());
  auto dw = at::empty({K, C, 7, 7}, dw4.options().memory_format(channels_last ? at::MemoryFormat::ChannelsLast
                                                                              : at::MemoryFormat::Contiguous));
  HYP_CHECK_HIP(hyp::stem_weight4_grad(dtype_code(dw4), dw4.data_ptr(), dw.data_ptr(), K, (int)C, dw.stride(0),
                                       dw.stride(1), dw.stride(2), dw.stride(3), cur_stream()));
  return dw;
}

namespace {
void check_stem(const at::Tensor& xs, int64_t K) {
  HYP_CHECK_CUDA_TENSOR(xs);
  TORCH_CHECK(xs.dim() == 4 && xs.size(1) == 16 && xs.size(2) > 3 && xs.size(3) > 3 &&
                  xs.is_contiguous(at::MemoryFormat::ChannelsLast),
              "stem conv: Xs must be the channels-last [N, 16, P + 3, Q + 3] output of stem_s2d");
  TORCH_CHECK(K % 8 == 0, "stem conv: K % 8 == 0");
}
}  // namespace

// y [N, K, P, Q] = the stem conv from Xs and W4 [K, 64, 4, 1] (channels-last: memory [k][dr][64]),
// with the BN-statistics epilogue into `sums` (zeroed fp64 [kStatSlots * 2 * K]).
at::Tensor stem_conv_fwd(const at::Tensor& xs, const at::Tensor& w4, const at::Tensor& sums) {
  check_stem(xs, w4.size(0));
  TORCH_CHECK(w4.dim() == 4 && w4.size(1) == 64 && w4.size(2) == 4 && w4.size(3) == 1 &&
                  w4.is_contiguous(at::MemoryFormat::ChannelsLast) && w4.scalar_type() == xs.scalar_type(),
              "stem_conv_fwd: W4 must be a channels-last [K, 64, 4, 1] tensor of Xs's dtype");
  const int N = xs.size(0), Hs = xs.size(2), Ws = xs.size(3), K = w4.size(0), P = Hs - 3, Q = Ws - 3;
  const at::DeviceGuard guard(xs.device());
  auto y = at::empty({N, K, P, Q}, xs.options().memory_format(at::MemoryFormat::ChannelsLast));
  const int M = N * P * Q;
  int bm = 128, bn = 128;
  hyp::conv_fwd_tile(M, K, &bm, &bn);
  const int splits = plan_splits(M, K, 4, bm, bn, -1);
  at::Tensor slabs;
  if (splits > 1) slabs = at::empty({splits, M, K}, xs.options().dtype(at::kFloat));
  at::Tensor acc = stats_sums(sums, K, xs);
  HYP_CHECK_HIP(hyp::conv_fwd(dtype_code(xs), xs.data_ptr(), w4.data_ptr(), y.data_ptr(), device_zero_page(xs.device()),
                              acc.data_ptr<double>(), acc.data_ptr<double>() + K, N, Hs, Ws, 64, K, P, Q, 4, 1, 1, 1, 0,
                              0, bm, bn, 0, splits, splits > 1 ? slabs.data_ptr<float>() : nullptr, cur_stream(), 1.f,
                              nullptr, nullptr, nullptr, 16));
  return y;
}

// dW4 [K, 64, 4, 1] (channels-last) of the stem conv from dY [N, K, P, Q] and Xs.
at::Tensor stem_conv_wgrad(const at::Tensor& dy, const at::Tensor& xs, int64_t splits_req) {
  check_stem(xs, dy.size(1));
  TORCH_CHECK(dy.dim() == 4 && dy.is_contiguous(at::MemoryFormat::ChannelsLast) && dy.scalar_type() == xs.scalar_type() &&
                  dy.size(0) == xs.size(0) && dy.size(2) == xs.size(2) - 3 && dy.size(3) == xs.size(3) - 3,
              "stem_conv_wgrad: dY must be channels-last [N, K, P, Q] of Xs's dtype");
  const int N = xs.size(0), Hs = xs.size(2), Ws = xs.size(3), K = dy.size(1), P = Hs - 3, Q = Ws - 3;
  const at::DeviceGuard guard(xs.device());
  auto dw = at::empty({K, 64, 4, 1}, xs.options().memory_format(at::MemoryFormat::ChannelsLast));
  // a 4-tile output over a ~4e5-pixel reduction: split the pixels until ~1024 workgroups stream
  // (the generic plan's <= 64 splits leave 256 workgroups 98 k-steps deep: 68 us on MI355X)
  const int bm = 64, bn = 64, tiles = ((K + 63) / 64) * 4, steps = (N * P * Q + 63) / 64;
  int per = std::max(16, (steps * tiles + 1023) / 1024);
  if (splits_req > 0) per = (steps + (int)splits_req - 1) / (int)splits_req;
  const int splits = (steps + per - 1) / per;
  at::Tensor part;
  if (splits > 1) part = at::empty({(int64_t)splits * K * 4 * 64}, xs.options().dtype(at::kFloat));
  HYP_CHECK_HIP(hyp::conv_wgrad(dtype_code(xs), dy.data_ptr(), xs.data_ptr(), dw.data_ptr(),
                                splits > 1 ? part.data_ptr<float>() : nullptr, device_zero_page(xs.device()), N, Hs, Ws,
                                64, K, P, Q, 4, 1, 1, 1, 0, 0, bm, bn, splits, per, cur_stream(), 1.f, nullptr, false,
                                16));
  return dw;
}

// ---- pooling (NHWC) -------------------------------------------------------------------------
std::vector<at::Tensor> maxpool2d_fwd(const at::Tensor& x, int64_t k, int64_t s, int64_t pad) {
  HYP_CHECK_CUDA_TENSOR(x);
  TORCH_CHECK(x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast) && x.size(1) % 8 == 0,
              "maxpool2d_fwd: channels-last [N, C, H, W] with C % 8 == 0");
  const int N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int P = (H + 2 * pad - k) / s + 1, Q = (W + 2 * pad - k) / s + 1;
  TORCH_CHECK(P > 0 && Q > 0 && k * k <= 256 && pad < k, "maxpool2d_fwd: bad geometry");
  const at::DeviceGuard guard(x.device());
  auto y = at::empty({N, C, P, Q}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto idx = at::empty({N, P, Q, C}, x.options().dtype(at::kByte));
  HYP_CHECK_HIP(hyp::maxpool2d_forward(dtype_code(x), x.data_ptr(), y.data_ptr(), idx.data_ptr<uint8_t>(), N, H, W, C,
                                       (int)k, (int)s, (int)pad, cur_stream()));
  return {y, idx};
}

at::Tensor maxpool2d_bwd(const at::Tensor& dy, const at::Tensor& idx, int64_t H, int64_t W, int64_t k, int64_t s,
                         int64_t pad) {
  HYP_CHECK_CUDA_TENSOR(dy);
  TORCH_CHECK(dy.dim() == 4 && dy.is_contiguous(at::MemoryFormat::ChannelsLast), "maxpool2d_bwd: channels-last dy");
  const int N = dy.size(0), C = dy.size(1);
  TORCH_CHECK(dy.size(2) == (H + 2 * pad - k) / s + 1 && dy.size(3) == (W + 2 * pad - k) / s + 1 &&
                  idx.numel() == dy.numel() && idx.scalar_type() == at::kByte,
              "maxpool2d_bwd: shape mismatch");
  const at::DeviceGuard guard(dy.device());
  auto dx = at::empty({N, C, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  HYP_CHECK_HIP(hyp::maxpool2d_backward(dtype_code(dy), dy.data_ptr(), idx.data_ptr<uint8_t>(), dx.data_ptr(), N,
                                        (int)H, (int)W, C, (int)k, (int)s, (int)pad, cur_stream()));
  return dx;
}

// comp [N, C, P, Q] channels-last -> [N, C, H, W]: comp scattered to (p*sh, q*sw) (+ addend)
at::Tensor upsample_add(const at::Tensor& comp, const c10::optional<at::Tensor>& addend, int64_t H, int64_t W,
                        int64_t sh, int64_t sw) {
  HYP_CHECK_CUDA_TENSOR(comp);
  TORCH_CHECK(comp.dim() == 4 && comp.is_contiguous(at::MemoryFormat::ChannelsLast) && comp.size(1) % 8 == 0,
              "upsample_add: channels-last [N, C, P, Q] with C % 8 == 0");
  const int N = comp.size(0), C = comp.size(1), P = comp.size(2), Q = comp.size(3);
  TORCH_CHECK(sh >= 1 && sw >= 1 && (P - 1) * sh < H && (Q - 1) * sw < W, "upsample_add: bad geometry");
  const at::DeviceGuard guard(comp.device());
  auto out = at::empty({N, C, H, W}, comp.options().memory_format(at::MemoryFormat::ChannelsLast));
  const void* add = nullptr;
  if (addend.has_value() && addend->defined()) {
    const auto& a = *addend;
    TORCH_CHECK(a.sizes() == out.sizes() && a.scalar_type() == comp.scalar_type() &&
                    a.is_contiguous(at::MemoryFormat::ChannelsLast) && a.device() == comp.device(),
                "upsample_add: addend must match the output (shape, dtype, channels-last)");
    add = a.data_ptr();
  }
  HYP_CHECK_HIP(hyp::upsample_add(dtype_code(comp), comp.data_ptr(), add, out.data_ptr(), N, (int)H, (int)W, C, P, Q,
                                  (int)sh, (int)sw, cur_stream()));
  return out;
}

// x [N, C, H, W] channels-last -> [N, C]
at::Tensor global_avgpool_fwd(const at::Tensor& x) {
  HYP_CHECK_CUDA_TENSOR(x);
  TORCH_CHECK(x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast) && x.size(1) % 8 == 0,
              "global_avgpool_fwd: channels-last [N, C, H, W] with C % 8 == 0");
  const at::DeviceGuard guard(x.device());
  auto y = at::empty({x.size(0), x.size(1)}, x.options());
  HYP_CHECK_HIP(hyp::global_avgpool_forward(dtype_code(x), x.data_ptr(), y.data_ptr(), x.size(0),
                                            x.size(2) * x.size(3), x.size(1), cur_stream()));
  return y;
}

at::Tensor global_avgpool_bwd(const at::Tensor& dy, int64_t H, int64_t W) {
  HYP_CHECK_CUDA_TENSOR(dy);
  TORCH_CHECK(dy.dim() == 2 && dy.is_contiguous() && dy.size(1) % 8 == 0, "global_avgpool_bwd: [N, C] dy");
  const at::DeviceGuard guard(dy.device());
  auto dx = at::empty({dy.size(0), dy.size(1), H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  HYP_CHECK_HIP(hyp::global_avgpool_backward(dtype_code(dy), dy.data_ptr(), dx.data_ptr(), dy.size(0), H * W,
                                             dy.size(1), cur_stream()));
  return dx;
}

}  // namespace

void register_conv_ops(pybind11::module& m) {
  m.def("conv_fwd", &conv_fwd, "NHWC implicit-GEMM conv on MFMA (+ BN statistics partials)", pybind11::arg("x"),
        pybind11::arg("w"), pybind11::arg("sh"), pybind11::arg("sw"), pybind11::arg("ph"), pybind11::arg("pw"),
        pybind11::arg("stats"), pybind11::arg("bm") = -1, pybind11::arg("bn") = -1, pybind11::arg("splits") = -1,
        pybind11::arg("sums") = pybind11::none(), pybind11::arg("stages") = 0,
        pybind11::arg("xf_sums") = pybind11::none(), pybind11::arg("xf_w") = pybind11::none(),
        pybind11::arg("xf_b") = pybind11::none(), pybind11::arg("xf_rm") = pybind11::none(),
        pybind11::arg("xf_rv") = pybind11::none(), pybind11::arg("xf_momentum") = 0.1,
        pybind11::arg("xf_eps") = 1e-5, pybind11::arg("xf_out") = pybind11::none(),
        pybind11::arg("xf_stats") = pybind11::none());
  m.def("conv_set_xf_debug", [](int64_t bits) { hyp::conv_set_xf_debug((int)bits); },
        "diagnostic: disable parts of the fused input transform (1 transform, 2 finalize, 4 side store)");
  m.def("conv_fwd_affine", &conv_fwd_affine, "eval conv + folded BN affine (+ residual) (+ ReLU), one launch",
        pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("sh"), pybind11::arg("sw"), pybind11::arg("ph"),
        pybind11::arg("pw"), pybind11::arg("scale"), pybind11::arg("shift"),
        pybind11::arg("residual") = pybind11::none(), pybind11::arg("act") = false);
  m.def("linear_ce_lse", &linear_ce_lse, "fused linear+CE pass 1: (lse, loss_rows), logits never stored",
        pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("bias"), pybind11::arg("target"), pybind11::arg("ignore"),
        pybind11::arg("bn") = 128);
  m.def("linear_ce_grad", &linear_ce_grad, "fused linear+CE pass 2: softmax gradient of classes [c0, c0+n)",
        pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("bias"), pybind11::arg("target"), pybind11::arg("ignore"),
        pybind11::arg("lse"), pybind11::arg("scale"), pybind11::arg("c0"), pybind11::arg("n"), pybind11::arg("bn") = 128);
  m.def("conv_set_stages", [](int64_t fwd, int64_t wgrad) {
    hyp::conv_set_stages((int)fwd);
    hyp::conv_wgrad_set_stages((int)wgrad);
  }, "LDS pipeline depth of the conv kernels (2..4; 0 = automatic) — tuning sweeps only");
  m.def("linear_nt", &linear_nt, "skinny y = alpha x wᵀ [+ beta mask∘(U V)] (split-K MFMA, weight streaming)",
        pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("splits") = -1, pybind11::arg("bn") = -1,
        pybind11::arg("alpha") = 1.0, pybind11::arg("U") = pybind11::none(), pybind11::arg("V") = pybind11::none(),
        pybind11::arg("v_nr") = false, pybind11::arg("mask") = pybind11::none(), pybind11::arg("beta") = 1.0);
  m.def("linear_nn", &linear_nn, "skinny dx = alpha dy w [+ beta mask∘(U V)] (split-K MFMA, w read transposed)",
        pybind11::arg("dy"), pybind11::arg("w"), pybind11::arg("splits") = -1, pybind11::arg("bn") = -1,
        pybind11::arg("alpha") = 1.0, pybind11::arg("U") = pybind11::none(), pybind11::arg("V") = pybind11::none(),
        pybind11::arg("v_nr") = false, pybind11::arg("mask") = pybind11::none(), pybind11::arg("beta") = 1.0);
  m.def("conv_set_stamps", [](const c10::optional<at::Tensor>& buf) {
    hyp::conv_set_stamps(buf.has_value() && buf->defined() ? buf->data_ptr() : nullptr);
  }, "diagnostic: record a per-workgroup timeline (int64 [>= 6 * workgroups]) of the next conv_fwd launches",
        pybind11::arg("buf") = pybind11::none());
  m.def("stem_s2d", &stem_s2d, "ResNet 7x7/s2/p3 stem input as space-to-depth Xs [N, 16, P+3, Q+3]");
  m.def("stem_weight4", &stem_weight4, "stem W [K, C, 7, 7] -> W4 channels-last [K, 64, 4, 1] (one launch)");
  m.def("stem_weight4_grad", &stem_weight4_grad, "dW4 [K, 64, 4, 1] -> dW [K, C, 7, 7] (one launch)",
        pybind11::arg("dw4"), pybind11::arg("C"), pybind11::arg("channels_last") = false);
  m.def("stem_conv_fwd", &stem_conv_fwd, "the stem conv (R=4 x 64 over Xs, pixel stride 16) + BN statistics");
  m.def("stem_conv_wgrad", &stem_conv_wgrad, "dW4 [K, 64, 4, 1] of the stem conv", pybind11::arg("dy"),
        pybind11::arg("xs"), pybind11::arg("splits") = -1);
  m.def("maxpool2d_fwd", &maxpool2d_fwd, "NHWC max pool (+ window-tap index)");
  m.def("maxpool2d_bwd", &maxpool2d_bwd, "NHWC max pool backward (gather, deterministic)");
  m.def("global_avgpool_fwd", &global_avgpool_fwd, "NHWC global average pool");
  m.def("upsample_add", &upsample_add, "strided dgrad completion: comp scattered to every s-th pixel (+ addend)",
        pybind11::arg("comp"), pybind11::arg("addend"), pybind11::arg("H"), pybind11::arg("W"), pybind11::arg("sh"),
        pybind11::arg("sw"));
  m.def("global_avgpool_bwd", &global_avgpool_bwd, "NHWC global average pool backward");
  m.def("conv_dgrad", &conv_dgrad, "stride-1 conv data gradient on MFMA (filter read flipped/transposed)",
        pybind11::arg("dy"), pybind11::arg("w"), pybind11::arg("ph"), pybind11::arg("pw"), pybind11::arg("bm") = -1,
        pybind11::arg("bn") = -1, pybind11::arg("splits") = -1, pybind11::arg("addend") = pybind11::none(),
        pybind11::arg("bn_x") = pybind11::none(), pybind11::arg("bn_y") = pybind11::none(),
        pybind11::arg("bn_w") = pybind11::none(), pybind11::arg("bn_b") = pybind11::none(),
        pybind11::arg("bn_mean") = pybind11::none(), pybind11::arg("bn_invstd") = pybind11::none(),
        pybind11::arg("bn_mode") = -1, pybind11::arg("bn_sums") = pybind11::none(), pybind11::arg("stride") = 1,
        pybind11::arg("H") = 0, pybind11::arg("W") = 0, pybind11::arg("stages") = 0);
  m.def("conv_dgrad_wgrad", &conv_dgrad_wgrad,
        "conv_dgrad + the same conv's weight gradient in ONE launch (conv_dual.hip) -> [dx, dw]", pybind11::arg("dy"),
        pybind11::arg("w"), pybind11::arg("ph"), pybind11::arg("pw"), pybind11::arg("bm") = -1,
        pybind11::arg("bn") = -1, pybind11::arg("splits") = -1, pybind11::arg("addend") = pybind11::none(),
        pybind11::arg("bn_x") = pybind11::none(), pybind11::arg("bn_y") = pybind11::none(),
        pybind11::arg("bn_w") = pybind11::none(), pybind11::arg("bn_b") = pybind11::none(),
        pybind11::arg("bn_mean") = pybind11::none(), pybind11::arg("bn_invstd") = pybind11::none(),
        pybind11::arg("bn_mode") = -1, pybind11::arg("bn_sums") = pybind11::none(), pybind11::arg("stride") = 1,
        pybind11::arg("H") = 0, pybind11::arg("W") = 0, pybind11::arg("stages") = 0, pybind11::arg("wg_x"),
        pybind11::arg("wg_R"), pybind11::arg("wg_S"), pybind11::arg("wg_sh"), pybind11::arg("wg_sw"),
        pybind11::arg("wg_ph"), pybind11::arg("wg_pw"), pybind11::arg("wg_splits") = -1,
        pybind11::arg("wg_defer") = false, pybind11::arg("order") = 0);
  m.def("bn_bwd_dx_wgrad", &bn_bwd_dx_wgrad,
        "BN backward dx pass + the weight gradient of the conv above it in ONE launch (bn_wgrad.hip) -> "
        "[dx, dweight, dbias, dw]",
        pybind11::arg("dz"), pybind11::arg("x"), pybind11::arg("weight"), pybind11::arg("save_mean"),
        pybind11::arg("save_invstd"), pybind11::arg("training"), pybind11::arg("sums"), pybind11::arg("wg_dy"),
        pybind11::arg("wg_x"), pybind11::arg("wg_R"), pybind11::arg("wg_S"), pybind11::arg("wg_sh"),
        pybind11::arg("wg_sw"), pybind11::arg("wg_ph"), pybind11::arg("wg_pw"), pybind11::arg("wg_bm") = 64,
        pybind11::arg("wg_bn") = 64, pybind11::arg("wg_splits") = -1, pybind11::arg("wg_defer") = false,
        pybind11::arg("wg_out") = pybind11::none());
  m.def("conv_set_group", [](int64_t mode) { hyp::conv_set_group((int)mode); },
        "A/B: conv tile-order group (M-tiles per L2 group): 0 model, > 0 fixed, -1 x2, -2 x0.5");
  m.def("bn_set_geom", [](int64_t blocks, int64_t iters) { hyp::bn_set_geom((int)blocks, (int)iters); },
        "A/B: BN apply / dx pass grid — row-block cap (default 2048) and min row iterations per thread (4)");
  m.def("conv_set_persist", [](int64_t on) { hyp::conv_set_persist((int)on); },
        "persistent conv launches (conv_persist.h: next tile's loads behind the current epilogue): 0 off, 1 on");
  m.def("conv_dual_set_order", [](int64_t o) { hyp::conv_dual_set_order((int)o); },
        "A/B: grid order of conv_dgrad_wgrad launches (-1 per call, 0 interleaved, 1 data gradient first)");
  m.def("conv_wgrad", &conv_wgrad, "NHWC conv weight gradient on MFMA (split-K, transposed LDS reads)",
        pybind11::arg("dy"), pybind11::arg("x"), pybind11::arg("R"), pybind11::arg("S"), pybind11::arg("sh"),
        pybind11::arg("sw"), pybind11::arg("ph"), pybind11::arg("pw"), pybind11::arg("bm") = -1,
        pybind11::arg("bn") = -1, pybind11::arg("splits") = -1, pybind11::arg("alpha") = 1.0,
        pybind11::arg("defer") = false, pybind11::arg("out") = pybind11::none());
  m.def("conv_wgrad_flush", &conv_wgrad_flush,
        "run a deferred weight-gradient split-K reduce now (returns whether one was pending)");
  m.def("bn_fwd_sums", &bn_fwd_sums, "BN apply (inline finalize) from conv-epilogue statistics sums");
}

}  // namespace hypbind

// Torch bindings: fused BatchNorm(+res)(+ReLU), multi-tensor optimizer kernels, STREAM kernels.
#include <atomic>
#include "bindings/common.h"
#include "bindings/registry.h"

namespace hyp {
void adam_set_streaming(int on);  // adam.hip
void colsum_set_fin_lanes(int lanes);  // reduce.hip
}

namespace hypbind {
namespace {

// x: [N,C,H,W] channels-last or [M,C]; returns (y, save_mean, save_invstd).  sums: optional zeroed
// fp64 [2, C] statistics accumulator (training).
std::vector<at::Tensor> bn_fwd(const at::Tensor& x, const c10::optional<at::Tensor>& residual,
                               const c10::optional<at::Tensor>& weight, const c10::optional<at::Tensor>& bias,
                               const c10::optional<at::Tensor>& running_mean,
                               const c10::optional<at::Tensor>& running_var, double momentum, double eps, bool training,
                               bool act, const c10::optional<at::Tensor>& sums) {
  HYP_CHECK_CUDA_TENSOR(x);
  TORCH_CHECK(is_rows_by_channels(x), "bn_fwd: x must be channels-last 4D or contiguous 2D");
  const int64_t C = x.size(1);
  const int64_t M = x.numel() / C;
  TORCH_CHECK(C % 8 == 0, "bn_fwd: C must be a multiple of 8");
  if (residual.has_value() && residual->defined()) {
    TORCH_CHECK(residual->sizes() == x.sizes() && residual->scalar_type() == x.scalar_type(),
                "bn_fwd: residual shape/dtype mismatch");
    TORCH_CHECK(is_rows_by_channels(*residual), "bn_fwd: residual must be channels-last");
  }
  if (!training) TORCH_CHECK(running_mean.has_value() && running_var.has_value(), "eval BN needs running stats");
  const at::DeviceGuard guard(x.device());
  auto y = at::empty_like(x);
  auto fopt = x.options().dtype(at::kFloat);
  auto stats = at::empty({2, C}, fopt);
  at::Tensor acc, consts;
  if (training)
    acc = stats_sums(sums, C, x);
  else
    consts = at::empty({2, C}, fopt);
  HYP_CHECK_HIP(hyp::bn_forward(dtype_code(x), x.data_ptr(), vptr_or_null(residual), y.data_ptr(), M, (int)C,
                                ptr_or_null<float>(weight), ptr_or_null<float>(bias), ptr_or_null<float>(running_mean),
                                ptr_or_null<float>(running_var), (float)momentum, (float)eps, training ? 1 : 0,
                                act ? 1 : 0, training ? acc.data_ptr<double>() : nullptr, stats.data_ptr<float>(),
                                stats.data_ptr<float>() + C, training ? nullptr : consts.data_ptr<float>(),
                                training ? nullptr : consts.data_ptr<float>() + C, cur_stream()));
  return {y, stats[0], stats[1]};
}

// returns (dx, dres or undefined, dweight, dbias)
// y may be None with act (training, no residual): the ReLU mask is recomputed from x, weight, bias.
// sums: optional zeroed fp64 [2, C] accumulator for Σdz, Σdz·x.
std::vector<at::Tensor> bn_bwd(const at::Tensor& dy, const at::Tensor& x, const c10::optional<at::Tensor>& y,
                               const c10::optional<at::Tensor>& weight, const c10::optional<at::Tensor>& bias,
                               const at::Tensor& save_mean, const at::Tensor& save_invstd, bool training, bool act,
                               bool has_res, const c10::optional<at::Tensor>& sums) {
  HYP_CHECK_CUDA_TENSOR(x);
  const int64_t C = x.size(1);
  const int64_t M = x.numel() / C;
  TORCH_CHECK(dy.sizes() == x.sizes(), "bn_bwd: dy shape mismatch");
  at::Tensor dyc = is_rows_by_channels(dy) ? dy : (dy.dim() == 4 ? dy.contiguous(at::MemoryFormat::ChannelsLast) : dy.contiguous());
  const bool have_y = y.has_value() && y->defined();
  if (act && have_y) TORCH_CHECK(is_rows_by_channels(*y), "bn_bwd: y must be channels-last");
  if (act && !have_y)
    TORCH_CHECK(training && !has_res, "bn_bwd: the mask-from-x backward (y=None) is training-mode, non-residual");
  const at::DeviceGuard guard(x.device());
  auto dx = at::empty_like(x);
  at::Tensor dres;
  if (has_res) dres = at::empty_like(x);
  auto acc = stats_sums(sums, C, x);
  auto dwb = at::empty({2, C}, x.options().dtype(at::kFloat));
  HYP_CHECK_HIP(hyp::bn_backward(dtype_code(x), dyc.data_ptr(), x.data_ptr(), (act && have_y) ? y->data_ptr() : nullptr,
                                 dx.data_ptr(), has_res ? dres.data_ptr() : nullptr, M, (int)C,
                                 ptr_or_null<float>(weight), ptr_or_null<float>(bias), save_mean.data_ptr<float>(),
                                 save_invstd.data_ptr<float>(), training ? 1 : 0, act ? 1 : 0, acc.data_ptr<double>(),
                                 dwb.data_ptr<float>(), dwb.data_ptr<float>() + C, cur_stream()));
  return {dx, dres, dwb[0], dwb[1]};
}

// BN backward dx pass only: dz (already masked, e.g. by the dgrad BN epilogue) and its complete
// Σdz, Σdz·x sums -> (dx, dweight, dbias); the residual gradient is dz itself.
std::vector<at::Tensor> bn_bwd_dx(const at::Tensor& dz, const at::Tensor& x, const c10::optional<at::Tensor>& weight,
                                  const at::Tensor& save_mean, const at::Tensor& save_invstd, bool training,
                                  const at::Tensor& sums) {
  HYP_CHECK_CUDA_TENSOR(x);
  const int64_t C = x.size(1);
  const int64_t M = x.numel() / C;
  TORCH_CHECK(dz.sizes() == x.sizes() && dz.scalar_type() == x.scalar_type() && is_rows_by_channels(dz) &&
                  is_rows_by_channels(x),
              "bn_bwd_dx: dz and x of one shape / dtype, channels-last");
  TORCH_CHECK(sums.scalar_type() == at::kDouble && sums.is_contiguous() && sums.numel() == 2 * C * hyp::kStatSlots,
              "bn_bwd_dx: sums must be an fp64 [kStatSlots * 2 * C] tensor");
  const at::DeviceGuard guard(x.device());
  auto dx = at::empty_like(x);
  auto dwb = at::empty({2, C}, x.options().dtype(at::kFloat));
  HYP_CHECK_HIP(hyp::bn_backward_dx(dtype_code(x), dz.data_ptr(), x.data_ptr(), dx.data_ptr(), M, (int)C,
                                    ptr_or_null<float>(weight), save_mean.data_ptr<float>(),
                                    save_invstd.data_ptr<float>(), training ? 1 : 0, sums.data_ptr<double>(),
                                    dwb.data_ptr<float>(), dwb.data_ptr<float>() + C, cur_stream()));
  return {dx, dwb[0], dwb[1]};
}

// ---- column sums (bias gradients) ---------------------------------------------------------------
// ticket slots of the one-launch column sums: a ring over device_counters' second half (each call
// takes the next `n` slots; its kernel resets them) — launches 512 calls apart never overlap.  A
// captured launch keeps its slot on every replay while eager calls cycle the ring, so under stream
// capture the callers take the two-launch path instead (colsum_fused_ok).  (Unsigned 64-bit
// counter: never wraps negative)
int* colsum_tickets(const at::Device& dev, int n) {
  static std::atomic<uint64_t> next{0};
  constexpr uint64_t kBase = 8192, kSpan = 8192;
  const uint64_t step = (uint64_t)((n + 15) & ~15);
  uint64_t at = next.fetch_add(step) % kSpan;
  if (at + step > kSpan) at = 0;
  return device_counters(dev) + kBase + at;
}

bool colsum_fused_ok() {
  if (hyp::colsum_fused_max_p() <= 0) return false;
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(cur_stream(), &st) == hipSuccess && st == hipStreamCaptureStatusNone;
}
// x: [..., N] contiguous -> Σ over all leading dims, [N] in out_dtype (default x's dtype)
at::Tensor column_sum(const at::Tensor& x, c10::optional<at::ScalarType> out_dtype) {
  HYP_CHECK_CUDA_TENSOR(x);
  TORCH_CHECK(x.is_contiguous() && x.dim() >= 1, "column_sum: contiguous input");
  const int64_t N = x.size(-1), M = N > 0 ? x.numel() / N : 0;
  TORCH_CHECK(N % 8 == 0 && M >= 1, "column_sum: N % 8 == 0 and at least one row");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0, "column_sum: 16-byte aligned input");
  const at::DeviceGuard guard(x.device());
  const auto odt = out_dtype.value_or(x.scalar_type());
  auto out = at::empty({N}, x.options().dtype(odt));
  const bool fused = colsum_fused_ok();
  const int P = fused ? hyp::colsum_partials_fused(M, (int)N) : hyp::colsum_partials(M, (int)N);
  auto part = at::empty({(int64_t)P * N}, x.options().dtype(at::kFloat));
  HYP_CHECK_HIP(hyp::column_sum(dtype_code(x), x.data_ptr(), M, (int)N, out.data_ptr(), dtype_code(out),
                                part.data_ptr<float>(), P, cur_stream(),
                                fused ? colsum_tickets(x.device(), (int)((N + 511) / 512)) : nullptr));
  return out;
}

// (dy, db): the activation backward (act "relu": z = the saved output; "gelu": z = the pre-activation)
// with the bias gradient summed in the same pass
std::vector<at::Tensor> act_bwd_colsum(const at::Tensor& dh, const at::Tensor& z, int64_t act,
                                       c10::optional<at::ScalarType> db_dtype, double drop_p,
                                       const c10::optional<at::Tensor>& rng) {
  HYP_CHECK_CUDA_TENSOR(dh);
  TORCH_CHECK(dh.is_contiguous() && z.is_contiguous() && dh.sizes() == z.sizes() && dh.scalar_type() == z.scalar_type(),
              "act_bwd_colsum: dh / z contiguous, one shape and dtype");
  TORCH_CHECK(dh.scalar_type() == at::kBFloat16 || dh.scalar_type() == at::kHalf, "act_bwd_colsum: bf16/f16");
  const int64_t N = dh.size(-1), M = dh.numel() / N;
  TORCH_CHECK(N % 8 == 0 && M >= 1, "act_bwd_colsum: N % 8 == 0");
  const at::DeviceGuard guard(dh.device());
  auto dy = at::empty_like(dh);
  const auto odt = db_dtype.value_or(dh.scalar_type());
  auto db = at::empty({N}, dh.options().dtype(odt));
  const bool fused = colsum_fused_ok();
  const int P = fused ? hyp::colsum_partials_fused(M, (int)N) : hyp::act_colsum_partials(M, (int)N);
  auto part = at::empty({(int64_t)P * N}, dh.options().dtype(at::kFloat));
  hyp::RngState rs{};
  if (drop_p > 0.0) {
    TORCH_CHECK(drop_p < 1.0 && rng.has_value() && rng->defined(), "act_bwd_colsum: dropout needs p < 1 and the rng record");
    rs = unpack_rng(*rng);
  }
  HYP_CHECK_HIP(hyp::act_bwd_colsum(dtype_code(dh), (int)act, dh.data_ptr(), z.data_ptr(), dy.data_ptr(), M, (int)N,
                                    db.data_ptr(), dtype_code(db), part.data_ptr<float>(), P, cur_stream(),
                                    (float)drop_p, drop_p > 0.0 ? &rs : nullptr,
                                    fused ? colsum_tickets(dh.device(), (int)((N + 511) / 512)) : nullptr));
  return {dy, db};
}

// ---- multi-tensor optimizer ------------------------------------------------------------------
void adam_mt(const at::Tensor& ptrs, const at::Tensor& sizes, const at::Tensor& blocks, int64_t T, int64_t chunk,
             double lr, double b1, double b2, double eps, double wd, bool adamw, const c10::optional<at::Tensor>& lr_t,
             const at::Tensor& step_t, const c10::optional<at::Tensor>& inv_scale,
             const c10::optional<at::Tensor>& found_inf, int64_t grad_dtype, int64_t param_dtype, bool zero_grad) {
  const at::DeviceGuard guard(ptrs.device());
  HYP_CHECK_HIP(hyp::adam_multi_tensor((int)grad_dtype, (int)param_dtype, ptrs.data_ptr<int64_t>(), sizes.data_ptr<int64_t>(),
                                       blocks.data_ptr<int>(), (int)blocks.size(0), (int)T, (int)chunk, (float)lr,
                                       (float)b1, (float)b2, (float)eps, (float)wd, adamw ? 1 : 0,
                                       ptr_or_null<float>(lr_t), step_t.data_ptr<float>(),
                                       ptr_or_null<float>(inv_scale), ptr_or_null<float>(found_inf), cur_stream(),
                                       zero_grad ? 1 : 0));
}

void unscale_mt(const at::Tensor& ptrs, const at::Tensor& sizes, const at::Tensor& blocks, int64_t chunk,
                const at::Tensor& inv_scale, const at::Tensor& found_inf, int64_t grad_dtype) {
  const at::DeviceGuard guard(ptrs.device());
  HYP_CHECK_HIP(hyp::unscale_multi_tensor((int)grad_dtype, ptrs.data_ptr<int64_t>(), sizes.data_ptr<int64_t>(),
                                          blocks.data_ptr<int>(), (int)blocks.size(0), (int)chunk,
                                          inv_scale.data_ptr<float>(), found_inf.data_ptr<float>(), cur_stream()));
}

at::Tensor sumsq_mt(const at::Tensor& ptrs, const at::Tensor& sizes, const at::Tensor& blocks, int64_t chunk,
                    int64_t grad_dtype) {
  const at::DeviceGuard guard(ptrs.device());
  auto fopt = at::TensorOptions().device(ptrs.device()).dtype(at::kFloat);
  auto part = at::empty({std::max<int64_t>(1, blocks.size(0))}, fopt);
  auto out = at::empty({1}, fopt);
  HYP_CHECK_HIP(hyp::sumsq_multi_tensor((int)grad_dtype, ptrs.data_ptr<int64_t>(), sizes.data_ptr<int64_t>(),
                                        blocks.data_ptr<int>(), (int)blocks.size(0), (int)chunk, part.data_ptr<float>(),
                                        out.data_ptr<float>(), cur_stream()));
  return out;
}

void clip_mt(const at::Tensor& ptrs, const at::Tensor& sizes, const at::Tensor& blocks, int64_t chunk,
             const at::Tensor& total_sq, double max_norm, int64_t grad_dtype) {
  const at::DeviceGuard guard(ptrs.device());
  HYP_CHECK_HIP(hyp::clip_multi_tensor((int)grad_dtype, ptrs.data_ptr<int64_t>(), sizes.data_ptr<int64_t>(),
                                       blocks.data_ptr<int>(), (int)blocks.size(0), (int)chunk,
                                       total_sq.data_ptr<float>(), (float)max_norm, cur_stream()));
}

void copy_mt(const at::Tensor& ptrs, const at::Tensor& sizes, const at::Tensor& blocks, int64_t T, int64_t chunk,
             int64_t src_dtype, int64_t dst_dtype) {
  TORCH_CHECK(ptrs.numel() == 2 * T && sizes.numel() == T, "copy_mt: table of 2 x T pointers and T sizes");
  const at::DeviceGuard guard(ptrs.device());
  HYP_CHECK_HIP(hyp::copy_multi_tensor((int)src_dtype, (int)dst_dtype, ptrs.data_ptr<int64_t>(),
                                       sizes.data_ptr<int64_t>(), blocks.data_ptr<int>(), (int)blocks.size(0), (int)T,
                                       (int)chunk, cur_stream()));
}

// ---- STREAM ----------------------------------------------------------------------------------
void stream(int64_t op, const at::Tensor& a, const c10::optional<at::Tensor>& b, at::Tensor& c, double s,
            bool nontemporal, int64_t blocks) {
  TORCH_CHECK(a.scalar_type() == at::kFloat && c.scalar_type() == at::kFloat, "stream: fp32 only");
  const at::DeviceGuard guard(a.device());
  HYP_CHECK_HIP(hyp::stream_op((int)op, a.data_ptr<float>(), ptr_or_null<float>(b), c.data_ptr<float>(), (float)s,
                               a.numel(), nontemporal ? 1 : 0, (int)blocks, cur_stream()));
}

}  // namespace

void register_norm_ops(pybind11::module& m) {
  m.def("bn_fwd", &bn_fwd, "fused NHWC batch-norm (+residual)(+relu) forward", pybind11::arg("x"),
        pybind11::arg("residual"), pybind11::arg("weight"), pybind11::arg("bias"), pybind11::arg("running_mean"),
        pybind11::arg("running_var"), pybind11::arg("momentum"), pybind11::arg("eps"), pybind11::arg("training"),
        pybind11::arg("act"), pybind11::arg("sums") = pybind11::none());
  m.def("bn_set_small_paths", [](bool on) { hyp::bn_set_small_paths(on ? 1 : 0); },
        "small-M BN one-launch backward (default on)");
  m.def("bn_bwd", &bn_bwd, "fused NHWC batch-norm (+residual)(+relu) backward", pybind11::arg("dy"), pybind11::arg("x"),
        pybind11::arg("y"), pybind11::arg("weight"), pybind11::arg("bias"), pybind11::arg("save_mean"),
        pybind11::arg("save_invstd"), pybind11::arg("training"), pybind11::arg("act"), pybind11::arg("has_res"),
        pybind11::arg("sums") = pybind11::none());
  m.def("bn_bwd_dx", &bn_bwd_dx, "BN backward dx pass from a pre-masked dz and its complete sums");
  m.def("adam_mt", &adam_mt, "multi-tensor fused Adam/AdamW");
  m.def("adam_set_streaming", [](int64_t on) { hyp::adam_set_streaming((int)on); },
        "A/B: non-temporal loads / stores of the fp32 optimizer state in adam_mt");
  m.def("mse_fwd_bwd", [](const at::Tensor& x, const at::Tensor& t) {
    HYP_CHECK_CUDA_TENSOR(x);
    TORCH_CHECK(x.is_contiguous() && t.is_contiguous() && t.scalar_type() == at::kFloat && x.numel() == t.numel() &&
                    t.device() == x.device(), "mse_fwd_bwd: contiguous x and fp32 target of the same size");
    const at::DeviceGuard guard(x.device());
    auto loss = at::empty({}, x.options().dtype(at::kFloat));
    auto g = at::empty_like(x);
    HYP_CHECK_HIP(hyp::mse_fwd_bwd(dtype_code(x), x.data_ptr(), t.data_ptr<float>(), x.numel(), loss.data_ptr<float>(),
                                   g.data_ptr(), cur_stream()));
    return std::vector<at::Tensor>{loss, g};
  }, "mean-squared error and its gradient 2(x - t)/n in one pass", pybind11::arg("x"), pybind11::arg("target"));
  m.def("colsum_set_fused", [](int64_t max_p) { hyp::colsum_set_fused((int)max_p); },
        "column sums: partial-row cap of the one-launch last-arriver combine (0 = two launches, the default)");
  m.def("colsum_set_fin_lanes", [](int64_t lanes) { hyp::colsum_set_fin_lanes((int)lanes); },
        "A/B: row lanes of the final column-sum combine (64 = 1024 threads, default; 16 = 256 threads)");
  m.def("colsum_set_act_wgs", [](int64_t wgs) { hyp::colsum_set_act_wgs((int)wgs); },
        "act_bwd_colsum: target workgroup count of the partial pass (A/B; default 1024)");
  m.def("column_sum", &column_sum, "column sums of a [.., N] matrix (bias gradients)", pybind11::arg("x"),
        pybind11::arg("out_dtype") = pybind11::none());
  m.def("act_bwd_colsum", &act_bwd_colsum, "activation backward + bias gradient in one pass (act 1 relu, 2 gelu)",
        pybind11::arg("dh"), pybind11::arg("z"), pybind11::arg("act"), pybind11::arg("db_dtype") = pybind11::none(),
        pybind11::arg("drop_p") = 0.0, pybind11::arg("rng") = pybind11::none());
  m.def("unscale_mt", &unscale_mt, "multi-tensor unscale + non-finite check");
  m.def("sumsq_mt", &sumsq_mt, "multi-tensor sum of squares");
  m.def("clip_mt", &clip_mt, "multi-tensor clip by global norm (device scalar)");
  m.def("copy_mt", &copy_mt, "multi-tensor copy with dtype conversion (ptrs [2][T]: sources, destinations)");
  m.def("stream", &stream, "STREAM copy/scale/add/triad");
}

}  // namespace hypbind

// Torch bindings: graph-safe RNG state (torch's default HIP generator, philox seed/offset) and the
// dropout kernels that consume it.
#include <ATen/core/Generator.h>
#include <ATen/hip/HIPGeneratorImpl.h>

#include <map>
#include <mutex>
#include <utility>

#include "bindings/common.h"
#include "bindings/registry.h"

namespace hypbind {

// Under capture the generator hands out POINTERS to its extragraph (seed, offset) tensors, which
// every CUDAGraph::replay() rewrites in its prologue.  A record taken in graph 1 (forward) but
// consumed in graph 2 (a split backward, train/step.py) would therefore read graph 2's offset and
// regenerate a DIFFERENT mask.  So the first rng_state() of each capture snapshots (seed, offset)
// into a 16-byte device buffer with two captured D2D copies at that point of the graph, and every
// record of that capture points at the snapshot: replay N of graph 1 writes it, graph 2's backward
// of the same step reads it (one pair of 8-byte copies per captured graph, not per dropout site).
namespace {
const int64_t* capture_snapshot(int64_t device, const at::PhiloxCudaState& st) {
  static std::mutex mu;
  static std::map<std::pair<int64_t, unsigned long long>, at::Tensor> snaps;
  hipStream_t stream = c10::hip::getCurrentHIPStream((c10::DeviceIndex)device).stream();
  hipStreamCaptureStatus status = hipStreamCaptureStatusNone;
  unsigned long long id = 0;
  HYP_CHECK_HIP(hipStreamGetCaptureInfo(stream, &status, &id));
  TORCH_CHECK(status == hipStreamCaptureStatusActive, "rng_state: captured philox state outside an active capture");
  std::lock_guard<std::mutex> g(mu);
  auto key = std::make_pair(device, id);
  auto it = snaps.find(key);
  if (it == snaps.end()) {
    auto snap = at::empty({2}, at::TensorOptions().device(at::Device(at::kCUDA, (c10::DeviceIndex)device)).dtype(at::kLong));
    int64_t* d = snap.data_ptr<int64_t>();
    HYP_CHECK_HIP(hipMemcpyAsync(d, st.seed_.ptr, sizeof(int64_t), hipMemcpyDeviceToDevice, stream));
    HYP_CHECK_HIP(hipMemcpyAsync(d + 1, st.offset_.ptr, sizeof(int64_t), hipMemcpyDeviceToDevice, stream));
    it = snaps.emplace(key, snap).first;  // kept for the process lifetime (16 B per capture)
  }
  return it->second.data_ptr<int64_t>();
}
}  // namespace

// The generator's (seed, offset) for `increment` random draws per element-thread, advancing it —
// the call torch's own dropout makes.  Returned as a CPU int64 [6] record (seed, offset,
// seed_ptr, offset_ptr, offset_intragraph, captured) that forward and backward share.
at::Tensor rng_state(int64_t device, int64_t increment) {
  auto gen = at::cuda::detail::getDefaultCUDAGenerator((c10::DeviceIndex)device);
  at::PhiloxCudaState st;
  {
    std::lock_guard<std::mutex> lock(gen.mutex());
    st = at::check_generator<at::CUDAGeneratorImpl>(gen)->philox_cuda_state((uint64_t)increment);
  }
  auto t = at::empty({6}, at::TensorOptions().dtype(at::kLong));
  int64_t* p = t.data_ptr<int64_t>();
  if (st.captured_) {
    const int64_t* snap = capture_snapshot(device, st);
    p[0] = 0;
    p[1] = 0;
    p[2] = reinterpret_cast<int64_t>(snap);
    p[3] = reinterpret_cast<int64_t>(snap + 1);
    p[4] = (int64_t)st.offset_intragraph_;
    p[5] = 1;
  } else {
    p[0] = (int64_t)st.seed_.val;
    p[1] = (int64_t)st.offset_.val;
    p[2] = p[3] = p[4] = 0;
    p[5] = 0;
  }
  return t;
}

hyp::RngState unpack_rng(const at::Tensor& t) {
  TORCH_CHECK(t.device().is_cpu() && t.scalar_type() == at::kLong && t.numel() == 6, "rng state: CPU int64 [6]");
  const int64_t* p = t.data_ptr<int64_t>();
  hyp::RngState s;
  s.seed = (uint64_t)p[0];
  s.offset = (uint64_t)p[1];
  s.seed_ptr = reinterpret_cast<const int64_t*>(p[2]);
  s.offset_ptr = reinterpret_cast<const int64_t*>(p[3]);
  s.intra = (uint64_t)p[4];
  s.captured = (int)p[5];
  return s;
}

namespace {

// out = dropout(x) with the state's mask (mode 0), or the scaled keep mask keep/(1-p) shaped like x
at::Tensor dropout_apply(const at::Tensor& x, double p, const c10::optional<at::Tensor>& state, bool mask,
                         int64_t act) {
  HYP_CHECK_CUDA_TENSOR(x);
  TORCH_CHECK(x.is_contiguous(), "dropout: contiguous input");
  TORCH_CHECK(p >= 0.0 && p < 1.0, "dropout: 0 <= p < 1");
  TORCH_CHECK(act == 0 || (act == 2 && !mask), "dropout: act is 0 (none) or 2 (exact GELU before the dropout)");
  TORCH_CHECK(p == 0.0 || (state.has_value() && state->defined()), "dropout: p > 0 needs an rng state");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0, "dropout: 16-byte aligned input");
  const at::DeviceGuard guard(x.device());
  auto out = at::empty_like(x);
  const hyp::RngState rs = (state.has_value() && state->defined()) ? unpack_rng(*state) : hyp::RngState{};
  HYP_CHECK_HIP(hyp::dropout_apply(dtype_code(x), mask ? 1 : (act == 2 ? 2 : 0), x.data_ptr(), out.data_ptr(),
                                   x.numel(), (float)p, rs, cur_stream()));
  return out;
}

}  // namespace

void register_rng_ops(pybind11::module& m) {
  m.def("rng_state", &rng_state, "graph-safe philox (seed, offset) record from torch's default HIP generator",
        pybind11::arg("device"), pybind11::arg("increment"));
  m.def("dropout", &dropout_apply, "counter-based dropout (mask regenerated from the rng state; mask=True: keep/(1-p))",
        pybind11::arg("x"), pybind11::arg("p"), pybind11::arg("state"), pybind11::arg("mask") = false,
        pybind11::arg("act") = 0);
}

}  // namespace hypbind

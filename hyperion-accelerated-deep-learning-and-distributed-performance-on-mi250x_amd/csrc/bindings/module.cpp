// hyperion._C module definition.
#include <torch/extension.h>

#include "bindings/registry.h"
#include "hyp_kernels.h"

#ifndef HYP_MODULE_NAME
#define HYP_MODULE_NAME _C
#endif

PYBIND11_MODULE(HYP_MODULE_NAME, m) {
  m.doc() = "Hyperion-MI355X native kernels (gfx950 HIP) and RCCL communicator";
  m.attr("arch") = "gfx950";
  m.attr("STAT_SLOTS") = hyp::kStatSlots;
#ifdef HYP_DEBUG
  m.attr("debug_build") = true;
#else
  m.attr("debug_build") = false;
#endif
  hypbind::register_norm_ops(m);
  hypbind::register_attn_ops(m);
  hypbind::register_loss_ops(m);
  hypbind::register_llama_ops(m);
  hypbind::register_gemm_ops(m);
  hypbind::register_comm(m);
  hypbind::register_conv_ops(m);
  hypbind::register_rng_ops(m);
  hypbind::register_ws_ops(m);
  // segmented hipGraph capture (train/segments.py): has the capture on `stream` recorded any work
  // yet?  An open capture with no leaf node is still empty — a hole right after it merges into the
  // previous hole instead of leaving an empty graph segment to end and replay
  m.def("capture_is_empty", [](int64_t stream) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    unsigned long long id = 0;
    hipGraph_t g = nullptr;
    const hipGraphNode_t* deps = nullptr;
    size_t ndeps = 0;
    const hipError_t e = hipStreamGetCaptureInfo_v2(reinterpret_cast<hipStream_t>(stream), &st, &id, &g, &deps, &ndeps);
    TORCH_CHECK(e == hipSuccess, "capture_is_empty: ", hipGetErrorString(e));
    TORCH_CHECK(st == hipStreamCaptureStatusActive, "capture_is_empty: the stream is not capturing");
    return ndeps == 0;
  }, "segmented capture: no work recorded yet on the capturing stream", pybind11::arg("stream"));
}

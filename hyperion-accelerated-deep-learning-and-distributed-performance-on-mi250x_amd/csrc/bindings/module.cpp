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
}

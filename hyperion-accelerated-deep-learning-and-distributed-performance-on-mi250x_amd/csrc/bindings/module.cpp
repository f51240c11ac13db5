// hyperion._C module definition.
#include <torch/extension.h>

#include "bindings/registry.h"

PYBIND11_MODULE(_C, m) {
  m.doc() = "Hyperion-MI355X native kernels (gfx950 HIP) and RCCL communicator";
  m.attr("arch") = "gfx950";
  hypbind::register_norm_ops(m);
  hypbind::register_attn_ops(m);
  hypbind::register_loss_ops(m);
  hypbind::register_llama_ops(m);
  hypbind::register_gemm_ops(m);
  hypbind::register_comm(m);
  hypbind::register_conv_ops(m);
  hypbind::register_rng_ops(m);
}

// Registration hooks: each binding translation unit contributes its functions to hyperion._C.
#pragma once
#include <pybind11/pybind11.h>

namespace hypbind {
void register_norm_ops(pybind11::module& m);
void register_attn_ops(pybind11::module& m);
void register_loss_ops(pybind11::module& m);
void register_llama_ops(pybind11::module& m);
void register_gemm_ops(pybind11::module& m);
void register_comm(pybind11::module& m);
void register_conv_ops(pybind11::module& m);
void register_rng_ops(pybind11::module& m);
void register_ws_ops(pybind11::module& m);
}  // namespace hypbind

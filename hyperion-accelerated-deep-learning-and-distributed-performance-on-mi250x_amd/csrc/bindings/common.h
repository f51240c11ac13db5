// Helpers shared by the torch-facing binding translation units.
#pragma once
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <c10/core/DeviceGuard.h>

#include "hyp_common.h"
#include "hyp_kernels.h"

namespace hypbind {

// rng_ops.cpp: a CPU int64 [6] rng-state record -> the kernels' RngState
hyp::RngState unpack_rng(const at::Tensor& t);

inline hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

inline int dtype_code(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat:
      return hyp::kF32;
    case at::kBFloat16:
      return hyp::kBF16;
    case at::kHalf:
      return hyp::kF16;
    default:
      TORCH_CHECK(false, "hyperion: unsupported dtype ", t.scalar_type());
  }
}

#define HYP_CHECK_HIP(expr)                                                                          \
  do {                                                                                               \
    hipError_t _e = (expr);                                                                          \
    TORCH_CHECK(_e == hipSuccess, "hyperion HIP error: ", hipGetErrorString(_e), " at ", __FILE__, \
                ":", __LINE__);                                                                      \
  } while (0)

#define HYP_CHECK_CUDA_TENSOR(t) TORCH_CHECK((t).is_cuda(), #t " must be a GPU tensor")

template <typename T>
inline T* ptr_or_null(const c10::optional<at::Tensor>& t) {
  return (t.has_value() && t->defined()) ? t->data_ptr<T>() : nullptr;
}

inline const void* vptr_or_null(const c10::optional<at::Tensor>& t) {
  return (t.has_value() && t->defined()) ? t->data_ptr() : nullptr;
}

// [M, C] row-major view check for channels-last activations or plain 2D tensors
inline bool is_rows_by_channels(const at::Tensor& x) {
  if (x.dim() == 4) return x.is_contiguous(at::MemoryFormat::ChannelsLast);
  if (x.dim() == 2) return x.is_contiguous();
  return false;
}

// A zeroed fp64 [kStatSlots, 2, C] statistics accumulator (the BN kernels ADD into it with
// atomics): the caller's (a slice of a pre-zeroed arena, ops/_native.py) or a fresh zeroed one.
inline at::Tensor stats_sums(const c10::optional<at::Tensor>& sums, int64_t C, const at::Tensor& like) {
  if (sums.has_value() && sums->defined()) {
    TORCH_CHECK(sums->scalar_type() == at::kDouble && sums->is_contiguous() &&
                    sums->numel() == 2 * C * hyp::kStatSlots && sums->device() == like.device(),
                "stats sums: a contiguous fp64 [kStatSlots * 2 * C] tensor on the input's device (zeroed)");
    return sums->view({hyp::kStatSlots, 2, C});
  }
  return at::zeros({hyp::kStatSlots, 2, C}, like.options().dtype(at::kDouble));
}

}  // namespace hypbind

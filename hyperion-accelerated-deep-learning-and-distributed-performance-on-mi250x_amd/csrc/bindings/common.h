// Helpers shared by the torch-facing binding translation units.
#pragma once
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <c10/core/DeviceGuard.h>

#include "hyp_common.h"
#include "hyp_kernels.h"

namespace hypbind {

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

}  // namespace hypbind

// Helpers shared by the torch-facing binding translation units.
#pragma once
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <c10/core/DeviceGuard.h>

#include <mutex>

#include "hyp_common.h"
#include "hyp_kernels.h"

namespace hypbind {

// rng_ops.cpp: a CPU int64 [6] rng-state record -> the kernels' RngState
hyp::RngState unpack_rng(const at::Tensor& t);

inline hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

inline int dtype_code(at::ScalarType t) {
  switch (t) {
    case at::kFloat:
      return hyp::kF32;
    case at::kBFloat16:
      return hyp::kBF16;
    case at::kHalf:
      return hyp::kF16;
    default:
      TORCH_CHECK(false, "hyperion: unsupported dtype ", t);
  }
}

inline int dtype_code(const at::Tensor& t) { return dtype_code(t.scalar_type()); }

inline at::ScalarType scalar_of_code(int64_t code) {
  TORCH_CHECK(code == hyp::kF32 || code == hyp::kBF16 || code == hyp::kF16, "hyperion: bad dtype code ", code);
  return code == hyp::kF32 ? at::kFloat : (code == hyp::kBF16 ? at::kBFloat16 : at::kHalf);
}

#define HYP_CHECK_HIP(expr)                                                                          \
  do {                                                                                               \
    hipError_t _e = (expr);                                                                          \
    TORCH_CHECK(_e == hipSuccess, "hyperion HIP error: ", hipGetErrorString(_e), " at ", __FILE__, \
                ":", __LINE__);                                                                      \
  } while (0)

// 4 KiB of zeros per device that the tiled GEMM / implicit-GEMM conv kernels read for out-of-range
// operand rows and padding taps.  Allocated
// with hipMalloc outside torch's caching allocator and never freed (no destructor runs after HIP
// teardown at exit), and zeroed SYNCHRONOUSLY on a private stream: a first call under hipGraph
// capture would otherwise take the buffer from the graph's pool with the zero-fill merely
// recorded, so eager GEMMs before the first replay would read garbage.  The calls run
// in relaxed capture mode, so they are legal (and not captured) while another stream captures.
// kind 0: the 4 KiB zero page; kind 1: 64 KiB of int32 work counters (see device_counters)
inline void* device_zeroed_block(const at::Device& dev, int kind) {
  static void* z[2][64] = {{nullptr}};
  static std::mutex mu;
  const int i = dev.index() < 0 ? 0 : dev.index();
  TORCH_CHECK(i < 64 && kind >= 0 && kind < 2, "device_zeroed_block: bad device index / kind");
  const size_t bytes = kind == 0 ? 4096 : 65536;
  std::lock_guard<std::mutex> g(mu);
  if (z[kind][i] == nullptr) {
    hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
    HYP_CHECK_HIP(hipThreadExchangeStreamCaptureMode(&mode));
    void* p = nullptr;
    hipStream_t s = nullptr;
    hipError_t e = hipMalloc(&p, bytes);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMemsetAsync(p, 0, bytes, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (s) (void)hipStreamDestroy(s);
    HYP_CHECK_HIP(hipThreadExchangeStreamCaptureMode(&mode));  // restore the caller's mode
    HYP_CHECK_HIP(e);
    z[kind][i] = p;
  }
  return z[kind][i];
}

inline const void* device_zero_page(const at::Device& dev) { return device_zeroed_block(dev, 0); }

// 16K int32 counters per device for last-arriver reductions (a kernel's workgroups count in on a
// slot; the last one reduces and RESETS the slot to zero, so every launch — eager or a graph
// replay — finds its slots zeroed).  Users must be stream-ordered: two kernels sharing slots must
// never run concurrently.
inline int* device_counters(const at::Device& dev) { return static_cast<int*>(device_zeroed_block(dev, 1)); }

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

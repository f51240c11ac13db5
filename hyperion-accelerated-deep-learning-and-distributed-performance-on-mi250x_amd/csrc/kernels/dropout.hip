// Graph-safe dropout for gfx950: y = keep ? x / (1 - p) : 0 with keep regenerated (never stored)
// from a counter-based hash of (generator seed/offset, element index).
//
// Reference: nn.TransformerEncoderLayer's three dropouts (p = 0.1) and PEFT's LoRA dropout
// (p = 0.05) run as torch's philox fused_dropout (+ masked_scale in backward) with a stored
// mask (SURVEY §2.4 "Dropout").  On the Llama-2-7B LoRA step the 128 per-projection bernoulli
// masks alone took ~4.5 ms of 44 (profiles/r02: distribution_elementwise_grid_stride_kernel).
// Here one vectorized pass forward (8 elements / thread, 16-byte IO) and one backward, the mask
// recomputed — and the seed/offset come from torch's generator so hipGraph replays draw fresh
// masks (hyp_common.h RngState).
#include "hyp_common.h"
#include "hyp_kernels.h"

namespace hyp {
namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ float gelu_erf(float v) { return 0.5f * v * (1.f + erff(v * 0.70710678118654752f)); }

// MODE 0: y = keep ? x*scale : 0 ; MODE 1: y = keep ? scale : 0 (the scaled mask in T, x unused);
// MODE 2: y = keep ? gelu(x)*scale : 0 (exact erf GELU: the activation + dropout of an FFN whose
// GEMM ran on the vendor library with a bias epilogue — one pass over the pre-activation instead
// of torch's GELU kernel and a separate dropout pass)
template <typename T, int MODE>
__device__ __forceinline__ void dropout_body(const T* __restrict__ x, T* __restrict__ y, int64_t n, uint32_t thr,
                                             float scale, const RngState& rs) {
  const uint64_t key = rng_key(rs);
  const int64_t i0 = ((int64_t)blockIdx.x * kThreads + threadIdx.x) * 8;
  const int64_t stride = (int64_t)gridDim.x * kThreads * 8;
  for (int64_t i = i0; i < n; i += stride) {
    if (i + 8 <= n) {
      float v[8];
      if (MODE != 1) Vec8<T>::load(x + i, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const bool keep = thr == 0u || rng_u32(key, (uint64_t)(i + e)) >= thr;
        if (MODE == 2) v[e] = gelu_erf(v[e]);
        v[e] = MODE != 1 ? (keep ? v[e] * scale : 0.f) : (keep ? scale : 0.f);
      }
      Vec8<T>::store(y + i, v);
    } else {
      for (int64_t j = i; j < n; ++j) {
        const bool keep = thr == 0u || rng_u32(key, (uint64_t)j) >= thr;
        float xv = MODE != 1 ? ld1<T>(x + j) : 0.f;
        if (MODE == 2) xv = gelu_erf(xv);
        st1<T>(y + j, MODE != 1 ? (keep ? xv * scale : 0.f) : (keep ? scale : 0.f));
      }
    }
  }
}

template <typename T, int MODE>
__global__ __launch_bounds__(kThreads) void dropout_k(const T* __restrict__ x, T* __restrict__ y, int64_t n,
                                                      uint32_t thr, float scale, RngState rs) {
  dropout_body<T, MODE>(x, y, n, thr, scale, rs);
}

// mode 2 under its own name: an FFN's activation (+ its dropout), not a standalone dropout pass
template <typename T>
__global__ __launch_bounds__(kThreads) void gelu_dropout_k(const T* __restrict__ x, T* __restrict__ y, int64_t n,
                                                           uint32_t thr, float scale, RngState rs) {
  dropout_body<T, 2>(x, y, n, thr, scale, rs);
}

template <typename T, int MODE>
hipError_t launch(const void* x, void* y, int64_t n, float p, const RngState& rs, hipStream_t st) {
  const uint32_t thr = (uint32_t)fminf(p * 4294967296.f, 4294967295.f);
  const float scale = p < 1.f ? 1.f / (1.f - p) : 0.f;
  int64_t blocks = (n + kThreads * 8 - 1) / (kThreads * 8);
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) blocks = 1;
  if (MODE == 2)
    hipLaunchKernelGGL((gelu_dropout_k<T>), dim3((unsigned)blocks), dim3(kThreads), 0, st, static_cast<const T*>(x),
                       static_cast<T*>(y), n, thr, scale, rs);
  else
    hipLaunchKernelGGL((dropout_k<T, MODE>), dim3((unsigned)blocks), dim3(kThreads), 0, st, static_cast<const T*>(x),
                       static_cast<T*>(y), n, thr, scale, rs);
  return hipGetLastError();
}

}  // namespace

// mode 0: out = dropout(x) (the same call with the same state is its own backward on dy);
// mode 1: out = the scaled keep mask (keep / (1 - p)); mode 2: out = dropout(gelu(x)) (p may be 0).
// x / out contiguous (16-byte aligned for the vector body).
hipError_t dropout_apply(int dtype, int mode, const void* x, void* out, int64_t n, float p, const RngState& rs,
                         hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (mode < 0 || mode > 2) return hipErrorInvalidValue;
  HYP_DISPATCH_FLOAT(dtype, T, {
    return mode == 0 ? launch<T, 0>(x, out, n, p, rs, st)
                     : mode == 1 ? launch<T, 1>(x, out, n, p, rs, st) : launch<T, 2>(x, out, n, p, rs, st);
  });
  return hipErrorInvalidValue;
}

}  // namespace hyp

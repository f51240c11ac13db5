// Llama's per-layer elementwise work as two fused gfx950 kernels: rotary embeddings (q and k in
// one launch) and SwiGLU (silu(gate) * up), forward and backward.
//
// Reference: HF LlamaForCausalLM runs RoPE as ~10 eager kernels per layer (cos/sin gather,
// rotate_half slices + cat, 2 muls + add for q and again for k) and SwiGLU as silu + mul
// (SURVEY §2.4 row "RMSNorm / RoPE / SwiGLU", C26).
//
// RoPE (HF rotate_half convention): for pair i < D/2 with angle a = pos * theta^(-2i/D)
//   out[i]       = x[i] cos a - x[i + D/2] sin a
//   out[i + D/2] = x[i + D/2] cos a + x[i] sin a
// The backward is the same rotation by -a.  One 256-thread workgroup per token; each lane owns
// 8 consecutive pairs (two 16-byte loads), angles in fp32 with accurate sincosf (positions reach
// thousands of radians).
#include "hyp_common.h"
#include "hyp_kernels.h"

namespace hyp {
namespace {

constexpr int kRopeThreads = 256;

template <typename T>
__global__ __launch_bounds__(kRopeThreads) void rope_k(const T* __restrict__ q, const T* __restrict__ k,
                                                       T* __restrict__ qo, T* __restrict__ ko, int S, int Hq,
                                                       int Hk, int D, int64_t q_tok, int64_t k_tok, int64_t q_head,
                                                       int64_t k_head, const int64_t* __restrict__ pos,
                                                       float log2_theta, float sign) {
  const int64_t tok = blockIdx.x;  // b * S + s
  const int half = D >> 1;
  const int vec_per_head = half >> 3;  // 8 pairs per lane-task
  const float p = pos ? (float)pos[tok] : (float)(tok % S);
  const int tasks_q = Hq * vec_per_head, tasks = tasks_q + Hk * vec_per_head;
  for (int task = threadIdx.x; task < tasks; task += kRopeThreads) {
    const bool isq = task < tasks_q;
    const int tt = isq ? task : task - tasks_q;
    const int h = tt / vec_per_head, i0 = (tt - h * vec_per_head) * 8;
    const T* src = isq ? q + tok * q_tok + h * q_head : k + tok * k_tok + h * k_head;
    T* dst = isq ? qo + tok * q_tok + h * q_head : ko + tok * k_tok + h * k_head;
    float a[8], b[8];
    Vec8<T>::load(src + i0, a);
    Vec8<T>::load(src + i0 + half, b);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      // inv_freq = theta^(-2i/D) = exp2(-(2i/D) log2 theta)
      const float inv_freq = exp2f(-(float)(2 * (i0 + j)) / (float)D * log2_theta);
      float sn, cs;
      sincosf(p * inv_freq, &sn, &cs);
      sn *= sign;
      const float x0 = a[j], x1 = b[j];
      a[j] = x0 * cs - x1 * sn;
      b[j] = x1 * cs + x0 * sn;
    }
    Vec8<T>::store(dst + i0, a);
    Vec8<T>::store(dst + i0 + half, b);
  }
}

constexpr int kEwThreads = 256;

__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }

template <typename T>
__global__ __launch_bounds__(kEwThreads) void swiglu_fwd_k(const T* __restrict__ g, const T* __restrict__ u,
                                                           T* __restrict__ h, int64_t n8) {
  for (int64_t i = (int64_t)blockIdx.x * kEwThreads + threadIdx.x; i < n8; i += (int64_t)gridDim.x * kEwThreads) {
    float gv[8], uv[8];
    Vec8<T>::load(g + i * 8, gv);
    Vec8<T>::load(u + i * 8, uv);
#pragma unroll
    for (int j = 0; j < 8; ++j) gv[j] = gv[j] * sigmoidf_(gv[j]) * uv[j];
    Vec8<T>::store(h + i * 8, gv);
  }
}

template <typename T>
__global__ __launch_bounds__(kEwThreads) void swiglu_bwd_k(const T* __restrict__ dh, const T* __restrict__ g,
                                                           const T* __restrict__ u, T* __restrict__ dg,
                                                           T* __restrict__ du, int64_t n8) {
  for (int64_t i = (int64_t)blockIdx.x * kEwThreads + threadIdx.x; i < n8; i += (int64_t)gridDim.x * kEwThreads) {
    float d[8], gv[8], uv[8];
    Vec8<T>::load(dh + i * 8, d);
    Vec8<T>::load(g + i * 8, gv);
    Vec8<T>::load(u + i * 8, uv);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float s = sigmoidf_(gv[j]);
      const float silu = gv[j] * s;
      const float dsilu = s * (1.f + gv[j] * (1.f - s));
      const float dd = d[j];
      gv[j] = dd * uv[j] * dsilu;
      uv[j] = dd * silu;
    }
    Vec8<T>::store(dg + i * 8, gv);
    Vec8<T>::store(du + i * 8, uv);
  }
}

inline int ew_grid(int64_t n8) {
  int64_t b = (n8 + kEwThreads - 1) / kEwThreads;
  const int64_t cap = 256 * 16;  // 16 workgroups per CU is plenty for a streaming kernel
  if (b > cap) b = cap;
  return (int)(b < 1 ? 1 : b);
}

}  // namespace

hipError_t rope_apply(int dtype, const void* q, const void* k, void* qo, void* ko, int64_t tokens, int S, int Hq,
                      int Hk, int D, int64_t q_tok, int64_t k_tok, int64_t q_head, int64_t k_head, const int64_t* pos,
                      float theta, int inverse, hipStream_t st) {
  if (tokens == 0) return hipSuccess;
  if (D % 16 != 0) return hipErrorInvalidValue;
  const float l2t = log2f(theta);
  const float sign = inverse ? -1.f : 1.f;
  HYP_DISPATCH_FLOAT(dtype, T, {
    hipLaunchKernelGGL(rope_k<T>, dim3((unsigned)tokens), dim3(kRopeThreads), 0, st, static_cast<const T*>(q),
                       static_cast<const T*>(k), static_cast<T*>(qo), static_cast<T*>(ko), S, Hq, Hk, D, q_tok, k_tok,
                       q_head, k_head, pos, l2t, sign);
  });
  return hipGetLastError();
}

hipError_t swiglu_forward(int dtype, const void* g, const void* u, void* h, int64_t n, hipStream_t st) {
  if (n == 0) return hipSuccess;
  if (n % 8 != 0) return hipErrorInvalidValue;
  HYP_DISPATCH_FLOAT(dtype, T, {
    hipLaunchKernelGGL(swiglu_fwd_k<T>, dim3(ew_grid(n / 8)), dim3(kEwThreads), 0, st, static_cast<const T*>(g),
                       static_cast<const T*>(u), static_cast<T*>(h), n / 8);
  });
  return hipGetLastError();
}

hipError_t swiglu_backward(int dtype, const void* dh, const void* g, const void* u, void* dg, void* du, int64_t n,
                           hipStream_t st) {
  if (n == 0) return hipSuccess;
  if (n % 8 != 0) return hipErrorInvalidValue;
  HYP_DISPATCH_FLOAT(dtype, T, {
    hipLaunchKernelGGL(swiglu_bwd_k<T>, dim3(ew_grid(n / 8)), dim3(kEwThreads), 0, st, static_cast<const T*>(dh),
                       static_cast<const T*>(g), static_cast<const T*>(u), static_cast<T*>(dg), static_cast<T*>(du),
                       n / 8);
  });
  return hipGetLastError();
}

}  // namespace hyp

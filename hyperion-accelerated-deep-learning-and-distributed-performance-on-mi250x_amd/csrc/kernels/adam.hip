// Multi-tensor fused Adam / AdamW (+ GradScaler unscale + skip-on-inf) and multi-tensor
// unscale/inf-check + L2-norm kernels for gfx950.
//
// Replaces torch's `_foreach_*` Adam/AdamW and `_amp_foreach_non_finite_check_and_unscale_`
// (reference: AdamW everywhere in distributed_utils.py, Adam in baseline_performance.ipynb:282,
// GradScaler in distributed_utils.py:163-180; SURVEY §2.4 rows Optimizers / GradScaler / Grad-norm).
//
// One launch updates every parameter: the host builds (once) a device table of tensor pointers
// and a block table (tensor id, chunk id).  All scalars that change during training (step count,
// inverse loss scale, found-inf flag, optional lr) are read from device memory, so the whole
// optimizer step is capturable in a hipGraph.
#include "hyp_common.h"
#include "hyp_kernels.h"

namespace hyp {
namespace {

constexpr int kThreads = 256;

template <typename G>
__device__ __forceinline__ void load4(const G* p, float (&v)[4]);
template <>
__device__ __forceinline__ void load4<float>(const float* p, float (&v)[4]) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
}
template <>
__device__ __forceinline__ void load4<bf16_t>(const bf16_t* p, float (&v)[4]) {
  const uint2 a = *reinterpret_cast<const uint2*>(p);
  v[0] = __uint_as_float(a.x << 16); v[1] = __uint_as_float(a.x & 0xffff0000u);
  v[2] = __uint_as_float(a.y << 16); v[3] = __uint_as_float(a.y & 0xffff0000u);
}
template <>
__device__ __forceinline__ void load4<f16_t>(const f16_t* p, float (&v)[4]) {
  const uint2 a = *reinterpret_cast<const uint2*>(p);
  v[0] = f16_lo(a.x); v[1] = f16_hi(a.x); v[2] = f16_lo(a.y); v[3] = f16_hi(a.y);
}

struct AdamArgs {
  float lr, b1, b2, eps, wd;
  int adamw;
  int zero_grad;  // write zeros over the gradient once read (replaces a separate zero_grad pass)
  int nt;         // streaming (non-temporal) loads / stores of the fp32 state (adam_set_streaming)
};

typedef float f32x4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ld_state(const float* p, int nt) {
  if (nt) {
    const f32x4v v = __builtin_nontemporal_load(reinterpret_cast<const f32x4v*>(p));
    return make_float4(v[0], v[1], v[2], v[3]);
  }
  return *reinterpret_cast<const float4*>(p);
}
__device__ __forceinline__ void st_state(float* p, const float4& v, int nt) {
  if (nt) __builtin_nontemporal_store(f32x4v{v.x, v.y, v.z, v.w}, reinterpret_cast<f32x4v*>(p));
  else *reinterpret_cast<float4*>(p) = v;
}

__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, const AdamArgs& a, float lr,
                                          float bc1, float bc2_sqrt) {
  if (a.adamw) {
    p *= (1.f - lr * a.wd);
  } else if (a.wd != 0.f) {
    g = fmaf(a.wd, p, g);
  }
  m = fmaf(a.b1, m, (1.f - a.b1) * g);
  v = fmaf(a.b2, v, (1.f - a.b2) * g * g);
  const float denom = sqrtf(v) / bc2_sqrt + a.eps;
  p -= (lr / bc1) * (m / denom);
}

template <typename PL>
__device__ __forceinline__ void store4(PL* p, const float4& v);
template <>
__device__ __forceinline__ void store4<bf16_t>(bf16_t* p, const float4& v) {
  *reinterpret_cast<uint2*>(p) = make_uint2(pack_bf16x2(v.x, v.y), pack_bf16x2(v.z, v.w));
}
template <>
__device__ __forceinline__ void store4<f16_t>(f16_t* p, const float4& v) {
  *reinterpret_cast<uint2*>(p) = make_uint2(pack_f16x2(v.x, v.y), pack_f16x2(v.z, v.w));
}

template <typename G>
__device__ __forceinline__ void store4z(G* p) {
  if (sizeof(G) == 4) *reinterpret_cast<float4*>(p) = make_float4(0.f, 0.f, 0.f, 0.f);
  else *reinterpret_cast<uint2*>(p) = make_uint2(0u, 0u);
}

// ptrs: [4][T] int64 addresses (param f32, grad G, exp_avg f32, exp_avg_sq f32)
// MASTER: [5][T] (param PL (bf16/f16 compute copy), grad G, exp_avg, exp_avg_sq, fp32 master);
// the fp32 master is updated and the low-precision compute copy rewritten in the same pass.
template <typename G, typename PL, bool MASTER>
__global__ __launch_bounds__(kThreads) void adam_mt_k(const int64_t* __restrict__ ptrs, const int64_t* __restrict__ sizes,
                                                      const int* __restrict__ blocks, int T, int chunk, AdamArgs a,
                                                      const float* __restrict__ lr_t, const float* __restrict__ step_t,
                                                      const float* __restrict__ inv_scale,
                                                      const float* __restrict__ found_inf) {
  const int t = blocks[2 * blockIdx.x];
  const int ck = blocks[2 * blockIdx.x + 1];
  if (found_inf != nullptr && *found_inf != 0.f) {  // GradScaler: skip the step on inf/nan
    if (a.zero_grad) {
      G* gz = reinterpret_cast<G*>(ptrs[T + t]);
      const int64_t n = sizes[t], s0 = (int64_t)ck * chunk, s1 = min(n, s0 + chunk);
      for (int64_t i = s0 + threadIdx.x; i < s1; i += kThreads) st1<G>(gz + i, 0.f);
    }
    return;
  }
  float* __restrict__ p = reinterpret_cast<float*>(MASTER ? ptrs[4 * T + t] : ptrs[t]);
  PL* __restrict__ pl = reinterpret_cast<PL*>(ptrs[t]);
  G* __restrict__ g = reinterpret_cast<G*>(ptrs[T + t]);
  float* __restrict__ m = reinterpret_cast<float*>(ptrs[2 * T + t]);
  float* __restrict__ v = reinterpret_cast<float*>(ptrs[3 * T + t]);
  const int64_t n = sizes[t];
  const int64_t start = (int64_t)ck * chunk;
  const int64_t end = min(n, start + chunk);
  const float step = *step_t;
  const float bc1 = 1.f - powf(a.b1, step);
  const float bc2_sqrt = sqrtf(1.f - powf(a.b2, step));
  const float lr = lr_t ? *lr_t : a.lr;
  const float gs = inv_scale ? *inv_scale : 1.f;
  // vector body: all of p/g/m/v are >=16B aligned at `start` (host checks base alignment; chunk % 4 == 0)
  const int64_t nvec_end = start + ((end - start) & ~int64_t(3));
  for (int64_t i = start + 4 * threadIdx.x; i < nvec_end; i += 4 * kThreads) {
    float4 pv = ld_state(p + i, a.nt);
    float4 mv = ld_state(m + i, a.nt);
    float4 vv = ld_state(v + i, a.nt);
    float gv[4];
    load4<G>(g + i, gv);
    if (a.zero_grad) store4z<G>(g + i);
    adam_elem(pv.x, gv[0] * gs, mv.x, vv.x, a, lr, bc1, bc2_sqrt);
    adam_elem(pv.y, gv[1] * gs, mv.y, vv.y, a, lr, bc1, bc2_sqrt);
    adam_elem(pv.z, gv[2] * gs, mv.z, vv.z, a, lr, bc1, bc2_sqrt);
    adam_elem(pv.w, gv[3] * gs, mv.w, vv.w, a, lr, bc1, bc2_sqrt);
    st_state(p + i, pv, a.nt);
    st_state(m + i, mv, a.nt);
    st_state(v + i, vv, a.nt);
    if (MASTER) store4<PL>(pl + i, pv);
  }
  for (int64_t i = nvec_end + threadIdx.x; i < end; i += kThreads) {
    float pp = p[i], mm = m[i], vv = v[i];
    adam_elem(pp, ld1<G>(g + i) * gs, mm, vv, a, lr, bc1, bc2_sqrt);
    if (a.zero_grad) st1<G>(g + i, 0.f);
    p[i] = pp;
    m[i] = mm;
    v[i] = vv;
    if (MASTER) st1<PL>(pl + i, pp);
  }
}

// Multi-tensor non-finite check + in-place unscale (grads of dtype G). ptrs: [T] grad addresses.
template <typename G>
__global__ __launch_bounds__(kThreads) void unscale_mt_k(const int64_t* __restrict__ ptrs, const int64_t* __restrict__ sizes,
                                                         const int* __restrict__ blocks, int chunk,
                                                         const float* __restrict__ inv_scale, float* __restrict__ found_inf) {
  const int t = blocks[2 * blockIdx.x];
  const int ck = blocks[2 * blockIdx.x + 1];
  G* __restrict__ g = reinterpret_cast<G*>(ptrs[t]);
  const int64_t n = sizes[t];
  const int64_t start = (int64_t)ck * chunk;
  const int64_t end = min(n, start + chunk);
  const float s = *inv_scale;
  bool bad = false;
  for (int64_t i = start + threadIdx.x; i < end; i += kThreads) {
    const float x = ld1<G>(g + i);
    bad |= !isfinite(x);
    st1<G>(g + i, x * s);
  }
  if (__any(bad) && (threadIdx.x & 63) == 0) *found_inf = 1.f;
}

// Multi-tensor sum of squares: one partial per block -> out[blockIdx.x]
template <typename G>
__global__ __launch_bounds__(kThreads) void sumsq_mt_k(const int64_t* __restrict__ ptrs, const int64_t* __restrict__ sizes,
                                                       const int* __restrict__ blocks, int chunk, float* __restrict__ out) {
  __shared__ float scratch[kThreads / 64];
  const int t = blocks[2 * blockIdx.x];
  const int ck = blocks[2 * blockIdx.x + 1];
  const G* __restrict__ g = reinterpret_cast<const G*>(ptrs[t]);
  const int64_t n = sizes[t];
  const int64_t start = (int64_t)ck * chunk;
  const int64_t end = min(n, start + chunk);
  float acc = 0.f;
  for (int64_t i = start + threadIdx.x; i < end; i += kThreads) {
    const float x = ld1<G>(g + i);
    acc = fmaf(x, x, acc);
  }
  acc = block_sum(acc, scratch);
  if (threadIdx.x == 0) out[blockIdx.x] = acc;
}

// Multi-tensor scale in place by a device scalar computed from a norm: g *= min(1, max_norm/(norm+1e-6))
template <typename G>
__global__ __launch_bounds__(kThreads) void clip_mt_k(const int64_t* __restrict__ ptrs, const int64_t* __restrict__ sizes,
                                                      const int* __restrict__ blocks, int chunk,
                                                      const float* __restrict__ total_sq, float max_norm) {
  const float norm = sqrtf(*total_sq);
  const float coef = max_norm / (norm + 1e-6f);
  if (coef >= 1.f) return;
  const int t = blocks[2 * blockIdx.x];
  const int ck = blocks[2 * blockIdx.x + 1];
  G* __restrict__ g = reinterpret_cast<G*>(ptrs[t]);
  const int64_t n = sizes[t];
  const int64_t start = (int64_t)ck * chunk;
  const int64_t end = min(n, start + chunk);
  for (int64_t i = start + threadIdx.x; i < end; i += kThreads) st1<G>(g + i, ld1<G>(g + i) * coef);
}

// Multi-tensor copy with conversion: ptrs [2][T] = (source S, destination D), same element order.
// DDP packs a whole gradient bucket with ONE launch (one copy kernel per parameter was ~160 launches
// and ~0.8 ms of a ResNet-50 step, profiles/r05/ddp_schedule_ab.json).
template <typename S, typename D>
__global__ __launch_bounds__(kThreads) void copy_mt_k(const int64_t* __restrict__ ptrs, const int64_t* __restrict__ sizes,
                                                      const int* __restrict__ blocks, int T, int chunk) {
  const int t = blocks[2 * blockIdx.x];
  const int ck = blocks[2 * blockIdx.x + 1];
  const S* __restrict__ src = reinterpret_cast<const S*>(ptrs[t]);
  D* __restrict__ dst = reinterpret_cast<D*>(ptrs[T + t]);
  const int64_t n = sizes[t];
  const int64_t start = (int64_t)ck * chunk;
  const int64_t end = min(n, start + chunk);
  int64_t i = start + threadIdx.x * 4;
  for (; i + 4 <= end; i += kThreads * 4) {  // chunk % 4 == 0 and 16-byte aligned bases: aligned quads
    float v[4];
    load4<S>(src + i, v);
#pragma unroll
    for (int q = 0; q < 4; ++q) st1<D>(dst + i + q, v[q]);
  }
  for (; i < end; ++i) st1<D>(dst + i, ld1<S>(src + i));  // the tensor's ragged tail (< 4, one thread)
}

__global__ void sum_partials_k(const float* __restrict__ part, int n, float* __restrict__ out) {
  __shared__ float scratch[1024 / 64];
  float acc = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) acc += part[i];
  acc = block_sum(acc, scratch);
  if (threadIdx.x == 0) *out = acc;
}

}  // namespace

int g_adam_nt = 0;
void adam_set_streaming(int on) { g_adam_nt = on; }

hipError_t adam_multi_tensor(int grad_dtype, int param_dtype, const int64_t* ptrs, const int64_t* sizes,
                             const int* blocks, int nblocks, int T, int chunk, float lr, float b1, float b2, float eps,
                             float wd, int adamw, const float* lr_t, const float* step_t, const float* inv_scale,
                             const float* found_inf, hipStream_t stream, int zero_grad) {
  if (nblocks == 0) return hipSuccess;
  AdamArgs a{lr, b1, b2, eps, wd, adamw, zero_grad, g_adam_nt};
  HYP_DISPATCH_FLOAT(grad_dtype, G, {
    if (param_dtype == kF32)
      hipLaunchKernelGGL((adam_mt_k<G, float, false>), dim3(nblocks), dim3(kThreads), 0, stream, ptrs, sizes, blocks,
                         T, chunk, a, lr_t, step_t, inv_scale, found_inf);
    else if (param_dtype == kBF16)
      hipLaunchKernelGGL((adam_mt_k<G, bf16_t, true>), dim3(nblocks), dim3(kThreads), 0, stream, ptrs, sizes, blocks,
                         T, chunk, a, lr_t, step_t, inv_scale, found_inf);
    else
      hipLaunchKernelGGL((adam_mt_k<G, f16_t, true>), dim3(nblocks), dim3(kThreads), 0, stream, ptrs, sizes, blocks,
                         T, chunk, a, lr_t, step_t, inv_scale, found_inf);
  });
  return hipGetLastError();
}

hipError_t unscale_multi_tensor(int grad_dtype, const int64_t* ptrs, const int64_t* sizes, const int* blocks,
                                int nblocks, int chunk, const float* inv_scale, float* found_inf, hipStream_t stream) {
  if (nblocks == 0) return hipSuccess;
  HYP_DISPATCH_FLOAT(grad_dtype, G, {
    hipLaunchKernelGGL(unscale_mt_k<G>, dim3(nblocks), dim3(kThreads), 0, stream, ptrs, sizes, blocks, chunk, inv_scale,
                       found_inf);
  });
  return hipGetLastError();
}

hipError_t sumsq_multi_tensor(int grad_dtype, const int64_t* ptrs, const int64_t* sizes, const int* blocks, int nblocks,
                              int chunk, float* partials, float* out, hipStream_t stream) {
  if (nblocks == 0) return hipMemsetAsync(out, 0, sizeof(float), stream);
  HYP_DISPATCH_FLOAT(grad_dtype, G, {
    hipLaunchKernelGGL(sumsq_mt_k<G>, dim3(nblocks), dim3(kThreads), 0, stream, ptrs, sizes, blocks, chunk, partials);
  });
  hipLaunchKernelGGL(sum_partials_k, dim3(1), dim3(1024), 0, stream, partials, nblocks, out);
  return hipGetLastError();
}

hipError_t copy_multi_tensor(int src_dtype, int dst_dtype, const int64_t* ptrs, const int64_t* sizes, const int* blocks,
                             int nblocks, int T, int chunk, hipStream_t stream) {
  if (nblocks == 0) return hipSuccess;
  if (chunk % (4 * kThreads) != 0) return hipErrorInvalidValue;
  HYP_DISPATCH_FLOAT(src_dtype, S, {
    HYP_DISPATCH_FLOAT(dst_dtype, D, {
      hipLaunchKernelGGL((copy_mt_k<S, D>), dim3(nblocks), dim3(kThreads), 0, stream, ptrs, sizes, blocks, T, chunk);
    });
  });
  return hipGetLastError();
}

hipError_t clip_multi_tensor(int grad_dtype, const int64_t* ptrs, const int64_t* sizes, const int* blocks, int nblocks,
                             int chunk, const float* total_sq, float max_norm, hipStream_t stream) {
  if (nblocks == 0) return hipSuccess;
  HYP_DISPATCH_FLOAT(grad_dtype, G, {
    hipLaunchKernelGGL(clip_mt_k<G>, dim3(nblocks), dim3(kThreads), 0, stream, ptrs, sizes, blocks, chunk, total_sq,
                       max_norm);
  });
  return hipGetLastError();
}

}  // namespace hyp

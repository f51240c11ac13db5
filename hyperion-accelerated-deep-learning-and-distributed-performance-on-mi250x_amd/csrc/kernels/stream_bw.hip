// STREAM-style HBM3E bandwidth kernels (copy / scale / add / triad) for gfx950.
//
// Replaces the reference's bandwidth microbenchmark, which timed one un-warmed `z = x + y` torch
// launch (`Phase 1/01_hardware_exploration.ipynb:263-301`, C4; 12 bytes per element).
//
// 16 B per lane (float4), grid-stride, grid capped at 8 blocks/CU × 256 CUs (Guideline 11); the
// stores optionally use the non-temporal path so the 256 MiB Infinity Cache does not flatter the
// result for arrays that fit in it.
#include "hyp_common.h"
#include "hyp_kernels.h"

namespace hyp {
namespace {

template <int OP, bool NT>
__device__ __forceinline__ float4 stream_apply(float4 x, float4 y, float s) {
  if (OP == 0) return x;                                                             // copy
  if (OP == 1) return make_float4(s * x.x, s * x.y, s * x.z, s * x.w);               // scale
  if (OP == 2) return make_float4(x.x + y.x, x.y + y.y, x.z + y.z, x.w + y.w);       // add
  return make_float4(fmaf(s, y.x, x.x), fmaf(s, y.y, x.y), fmaf(s, y.z, x.z), fmaf(s, y.w, x.w));  // triad
}

template <bool NT>
__device__ __forceinline__ void stream_store(float4* p, float4 r) {
  if (NT) {
    typedef float f4v __attribute__((ext_vector_type(4)));
    f4v rv = {r.x, r.y, r.z, r.w};
    __builtin_nontemporal_store(rv, reinterpret_cast<f4v*>(p));
  } else {
    *p = r;
  }
}

// Each thread moves kUnroll float4 per trip with all loads issued before any store (≥ U × 16 B per
// operand in flight per lane: HBM latency is hidden by memory-level parallelism, not occupancy).
template <int OP, bool NT, int kUnroll>
__global__ __launch_bounds__(256) void stream_k(const float4* __restrict__ a, const float4* __restrict__ b,
                                                float4* __restrict__ c, float s, int64_t n4) {
  const int64_t tile = (int64_t)blockDim.x * kUnroll;
  const int64_t stride = (int64_t)gridDim.x * tile;
  int64_t base = (int64_t)blockIdx.x * tile + threadIdx.x;
  for (; base + (kUnroll - 1) * blockDim.x < n4; base += stride) {
    float4 x[kUnroll], y[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) x[u] = a[base + u * blockDim.x];
    if (OP >= 2) {
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) y[u] = b[base + u * blockDim.x];
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u)
      stream_store<NT>(c + base + u * blockDim.x, stream_apply<OP, NT>(x[u], OP >= 2 ? y[u] : x[u], s));
  }
  for (int64_t i = base; i < n4; i += blockDim.x)  // ragged end of this thread's last tile
    stream_store<NT>(c + i, stream_apply<OP, NT>(a[i], OP >= 2 ? b[i] : a[i], s));
}

}  // namespace

hipError_t stream_op(int op, const float* a, const float* b, float* c, float s, int64_t n, int nontemporal,
                     int blocks, hipStream_t stream) {
  if (n % 4 != 0) return hipErrorInvalidValue;
  const int64_t n4 = n / 4;
  // blocks > 0: grid-stride over that many workgroups (4 float4 per lane per trip);
  // blocks = -U (U in 1, 2, 4, 8): one tile of U float4 per lane per workgroup (a full grid, every
  // workgroup exits after its tile); 0: the default — full grid, U = 1, measured best on MI355X
  // (add, 500M fp32: 6175 GB/s with non-temporal stores vs 6109 for torch's add, 5944 for the
  // grid-stride form; profiles/hardware_r02/stream_sweep.json)
  if (blocks == 0) blocks = -1;
  const int U = blocks < 0 ? -blocks : 4;
  if (U != 1 && U != 2 && U != 4 && U != 8) return hipErrorInvalidValue;
  const int64_t need = (n4 + 256 * U - 1) / (256 * U);
  int64_t grid = blocks > 0 ? blocks : need;
  if (need < grid) grid = need;
  if (grid > INT32_MAX) return hipErrorInvalidValue;
  if (grid < 1) grid = 1;
  auto A = reinterpret_cast<const float4*>(a);
  auto B = reinterpret_cast<const float4*>(b);
  auto C = reinterpret_cast<float4*>(c);
#define HYP_STREAM_U(OPV, UV)                                                                                      \
  if (U == UV) {                                                                                                   \
    if (nontemporal)                                                                                               \
      hipLaunchKernelGGL((stream_k<OPV, true, UV>), dim3((unsigned)grid), dim3(256), 0, stream, A, B, C, s, n4);   \
    else                                                                                                           \
      hipLaunchKernelGGL((stream_k<OPV, false, UV>), dim3((unsigned)grid), dim3(256), 0, stream, A, B, C, s, n4);  \
  }
#define HYP_STREAM_CASE(OPV) \
  case OPV:                  \
    HYP_STREAM_U(OPV, 1)     \
    HYP_STREAM_U(OPV, 2)     \
    HYP_STREAM_U(OPV, 4)     \
    HYP_STREAM_U(OPV, 8)     \
    break;
  switch (op) {
    HYP_STREAM_CASE(0)
    HYP_STREAM_CASE(1)
    HYP_STREAM_CASE(2)
    HYP_STREAM_CASE(3)
    default:
      return hipErrorInvalidValue;
  }
#undef HYP_STREAM_CASE
#undef HYP_STREAM_U
  return hipGetLastError();
}

}  // namespace hyp

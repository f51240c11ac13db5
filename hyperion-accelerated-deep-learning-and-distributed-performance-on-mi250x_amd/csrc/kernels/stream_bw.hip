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
__global__ __launch_bounds__(256) void stream_k(const float4* __restrict__ a, const float4* __restrict__ b,
                                                float4* __restrict__ c, float s, int64_t n4) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 r;
    const float4 x = a[i];
    if (OP == 0) {  // copy
      r = x;
    } else if (OP == 1) {  // scale
      r = make_float4(s * x.x, s * x.y, s * x.z, s * x.w);
    } else {
      const float4 y = b[i];
      if (OP == 2)  // add
        r = make_float4(x.x + y.x, x.y + y.y, x.z + y.z, x.w + y.w);
      else  // triad
        r = make_float4(fmaf(s, y.x, x.x), fmaf(s, y.y, x.y), fmaf(s, y.z, x.z), fmaf(s, y.w, x.w));
    }
    if (NT) {
      typedef float f4v __attribute__((ext_vector_type(4)));
      f4v rv = {r.x, r.y, r.z, r.w};
      __builtin_nontemporal_store(rv, reinterpret_cast<f4v*>(c + i));
    } else {
      c[i] = r;
    }
  }
}

}  // namespace

hipError_t stream_op(int op, const float* a, const float* b, float* c, float s, int64_t n, int nontemporal,
                     int blocks, hipStream_t stream) {
  if (n % 4 != 0) return hipErrorInvalidValue;
  const int64_t n4 = n / 4;
  int grid = blocks > 0 ? blocks : 2048;
  const int64_t need = (n4 + 255) / 256;
  if (need < grid) grid = (int)need;
  if (grid < 1) grid = 1;
  auto A = reinterpret_cast<const float4*>(a);
  auto B = reinterpret_cast<const float4*>(b);
  auto C = reinterpret_cast<float4*>(c);
#define HYP_STREAM_CASE(OPV)                                                                                     \
  case OPV:                                                                                                      \
    if (nontemporal)                                                                                             \
      hipLaunchKernelGGL((stream_k<OPV, true>), dim3(grid), dim3(256), 0, stream, A, B, C, s, n4);               \
    else                                                                                                         \
      hipLaunchKernelGGL((stream_k<OPV, false>), dim3(grid), dim3(256), 0, stream, A, B, C, s, n4);              \
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
  return hipGetLastError();
}

}  // namespace hyp

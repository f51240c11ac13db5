// Inline finalize of the BatchNorm forward statistics, shared by every kernel that consumes the
// fp64 sums (bn_act.hip's apply kernels and conv_igemm.hip's fused input transform): identical
// arithmetic in both, so a BN output produced by either is bit-identical.
#pragma once
#include "hyp_common.h"
#include "hyp_kernels.h"

namespace hyp {

// ---------------------------------------------------------------- inline finalize
struct FwdFin {
  const double* sums;  // [kStatSlots][2][C]: Σx, Σx²
  const float* weight;
  const float* bias;
  float* running_mean;
  float* running_var;
  float momentum, eps;
  float* save_mean;
  float* save_invstd;
  double invM;    // 1 / M
  double unbias;  // M / (M - 1): the running variance is unbiased
};

// scale / shift of channel c from its kStatSlots (Σx, Σx²) pairs, the weight w and bias b (the
// arithmetic the backward's ReluMask repeats bit for bit: invstd and mean rounded to float,
// scale = w*invstd, shift = b - mean*scale).  `writer`: also store save_mean / save_invstd and
// update the running statistics.
__device__ __forceinline__ void fwd_const_from(const FwdFin& f, int c, const double (&sa)[kStatSlots],
                                               const double (&sq)[kStatSlots], float w, float b, bool writer,
                                               float& sc, float& sh) {
  double a = 0.0, b2 = 0.0;
#pragma unroll
  for (int k = 0; k < kStatSlots; ++k) {  // fixed order
    a += sa[k];
    b2 += sq[k];
  }
  const double mean = a * f.invM;
  double var = b2 * f.invM - mean * mean;
  if (var < 0.0) var = 0.0;
  const float invstd = (float)(1.0 / sqrt(var + (double)f.eps));
  const float s = w * invstd;
  sc = s;
  sh = b - (float)mean * s;
  if (writer) {
    f.save_mean[c] = (float)mean;
    f.save_invstd[c] = invstd;
    if (f.running_mean != nullptr) {
      f.running_mean[c] = (float)((1.0 - f.momentum) * f.running_mean[c] + f.momentum * mean);
      f.running_var[c] = (float)((1.0 - f.momentum) * f.running_var[c] + f.momentum * var * f.unbias);
    }
  }
}

// the loads of channel c's inputs (split from the arithmetic so a kernel can issue them early)
__device__ __forceinline__ void fwd_const_load(const FwdFin& f, int C, int c, double (&sa)[kStatSlots],
                                               double (&sq)[kStatSlots], float& w, float& b) {
#pragma unroll
  for (int k = 0; k < kStatSlots; ++k) {
    sa[k] = f.sums[(int64_t)k * 2 * C + c];
    sq[k] = f.sums[(int64_t)k * 2 * C + C + c];
  }
  w = f.weight ? f.weight[c] : 1.f;
  b = f.bias ? f.bias[c] : 0.f;
}

__device__ __forceinline__ void fwd_const1(const FwdFin& f, int C, int c, bool writer, float& sc, float& sh) {
  double sa[kStatSlots], sq[kStatSlots];
  float w, b;
  fwd_const_load(f, C, c, sa, sq, w, b);
  fwd_const_from(f, c, sa, sq, w, b, writer, sc, sh);
}

}  // namespace hyp

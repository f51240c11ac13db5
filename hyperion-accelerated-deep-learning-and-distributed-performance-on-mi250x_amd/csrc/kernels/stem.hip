// The ResNet stem (7x7, stride 2, padding 3, C <= 4 input channels) as a 64-channel stride-1
// convolution the MFMA implicit-GEMM kernels already run.
//
// Reference: torchvision ResNet's ``conv1 = Conv2d(3, 64, 7, 2, 3)`` ran on MIOpen (forward
// ``igemm_fwd_gtcx35`` 55 us, weight gradient ``igemm_wrw_gtcx35`` 56 us plus its zero-fill per
// ResNet-50 bf16 batch-32 step on MI355X; profiles/r03/resnet50_kernels_graph_5.22ms.txt) —
// ``Phase 1/baseline_performance.ipynb:203-205``, SURVEY §2.4 conv row.
//
// Rewrite (space-to-depth):
//   r = 2·dr + a, s = 2·ds + b  (dr, ds ∈ [0, 4); a, b ∈ {0, 1}; taps r or s == 7 have zero weight)
//   Xs[n, i, j, (2a + b)·C + c] = x[n, 2i + a - 3, 2j + b - 3, c]      (0 outside; channels 4C..15 zero)
//   W4[k, dr, ds·16 + (2a + b)·C + c] = W[k, c, 2dr + a, 2ds + b]      (0 outside)
//   out[n, p, q, k] = Σ_{dr} Σ_{e < 64} Xs16[n, p + dr, q·16 + e] · W4[k, dr, e]
// where Xs16 reads Xs's pixels (p + dr, q), (p + dr, q + 1), ... as one 64-element run: the 4 taps
// ds of 16 channels each are 4 ADJACENT pixels of Xs [N, P + 3, Q + 3, 16].  So the stem is a
// conv with R = 4, S = 1, a 64-element reduction slice and stride 1 whose input pixel stride is 16
// elements instead of 64 — the `pix` argument of conv_fwd / conv_wgrad; consecutive output pixels'
// runs overlap by 48 elements (L2/L1 absorb the re-reads, HBM sees the 13.5 MB Xs once).  The 7x7
// filter's (3 x 49 = 147)-long reduction becomes 4 full 64-wide MFMA k-steps (256, 43 % zero taps
// — the price of a C = 3 input on a 64-wide reduction).
#include "hyp_common.h"
#include "hyp_kernels.h"

namespace hyp {
namespace {

template <typename T>
__global__ __launch_bounds__(256) void stem_s2d_k(const T* __restrict__ x, T* __restrict__ out, int N, int H, int W,
                                                  int C, int Hs, int Ws) {
  // one thread = one Xs pixel (16 channels = two 16-byte stores) from a 2 x 2 input block
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)N * Hs * Ws;
  if (t >= total) return;
  const int j = (int)(t % Ws);
  const int64_t ni = t / Ws;
  const int i = (int)(ni % Hs);
  const int n = (int)(ni / Hs);
  float v[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) v[e] = 0.f;
#pragma unroll
  for (int ab = 0; ab < 4; ++ab) {
    const int h = 2 * i + (ab >> 1) - 3, w = 2 * j + (ab & 1) - 3;
    if ((unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W) {
      const T* px = x + (((int64_t)n * H + h) * W + w) * C;
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (c < C) v[ab * C + c] = ld1<T>(px + c);
    }
  }
  float lo[8], hi[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    lo[e] = v[e];
    hi[e] = v[8 + e];
  }
  Vec8<T>::store(out + t * 16, lo);
  Vec8<T>::store(out + t * 16 + 8, hi);
}

// W [K, C, 7, 7] (any strides, in elements) -> W4 channels-last [K, 64, 4, 1], memory
// [k][dr][ds*16 + (2a+b)*C + c] = W[k, c, 2dr+a, 2ds+b] (zero past tap 6 and past 4C): one launch
// in place of pad + index_select + layout copy (3-4 torch kernels per step)
template <typename T>
__global__ __launch_bounds__(256) void stem_w4_k(const T* __restrict__ w, T* __restrict__ w4, int K, int C,
                                                 int64_t sk, int64_t sc, int64_t sr, int64_t sq) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= K * 256) return;
  const int k = i >> 8, col = i & 255, dr = col >> 6, e = col & 63, ds = e >> 4, ch = e & 15;
  const int ab = ch / C, c = ch - ab * C, r = 2 * dr + (ab >> 1), q = 2 * ds + (ab & 1);
  T v = T(0.f);
  if (ab < 4 && r < 7 && q < 7) v = w[k * sk + c * sc + r * sr + q * sq];
  w4[i] = v;
}

// dW4 (the same [k][dr][64] memory order) -> dW [K, C, 7, 7] contiguous: every W element feeds
// exactly one W4 column
template <typename T>
__global__ __launch_bounds__(256) void stem_w4_grad_k(const T* __restrict__ dw4, T* __restrict__ dw, int K, int C,
                                                      int64_t sk, int64_t sc, int64_t sr, int64_t sq) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= K * C * 49) return;
  const int k = i / (C * 49), rem = i - k * C * 49, c = rem / 49, rq = rem - c * 49, r = rq / 7, q = rq - r * 7;
  const int col = (r >> 1) * 64 + (q >> 1) * 16 + ((r & 1) * 2 + (q & 1)) * C + c;
  dw[k * sk + c * sc + r * sr + q * sq] = dw4[k * 256 + col];
}

}  // namespace

hipError_t stem_weight4(int dtype, const void* w, void* w4, int K, int C, int64_t sk, int64_t sc, int64_t sr,
                        int64_t sq, hipStream_t st) {
  if (C < 1 || C > 4 || K < 1 || (dtype != kBF16 && dtype != kF16)) return hipErrorInvalidValue;
  const unsigned blocks = (unsigned)((K * 256 + 255) / 256);
  if (dtype == kBF16)
    hipLaunchKernelGGL(stem_w4_k<bf16_t>, dim3(blocks), dim3(256), 0, st, static_cast<const bf16_t*>(w),
                       static_cast<bf16_t*>(w4), K, C, sk, sc, sr, sq);
  else
    hipLaunchKernelGGL(stem_w4_k<f16_t>, dim3(blocks), dim3(256), 0, st, static_cast<const f16_t*>(w),
                       static_cast<f16_t*>(w4), K, C, sk, sc, sr, sq);
  return hipGetLastError();
}

hipError_t stem_weight4_grad(int dtype, const void* dw4, void* dw, int K, int C, int64_t sk, int64_t sc, int64_t sr,
                             int64_t sq, hipStream_t st) {
  if (C < 1 || C > 4 || K < 1 || (dtype != kBF16 && dtype != kF16)) return hipErrorInvalidValue;
  const unsigned blocks = (unsigned)((K * C * 49 + 255) / 256);
  if (dtype == kBF16)
    hipLaunchKernelGGL(stem_w4_grad_k<bf16_t>, dim3(blocks), dim3(256), 0, st, static_cast<const bf16_t*>(dw4),
                       static_cast<bf16_t*>(dw), K, C, sk, sc, sr, sq);
  else
    hipLaunchKernelGGL(stem_w4_grad_k<f16_t>, dim3(blocks), dim3(256), 0, st, static_cast<const f16_t*>(dw4),
                       static_cast<f16_t*>(dw), K, C, sk, sc, sr, sq);
  return hipGetLastError();
}

hipError_t stem_s2d(int dtype, const void* x, void* out, int N, int H, int W, int C, int Hs, int Ws,
                    hipStream_t st) {
  if (C < 1 || C > 4 || (dtype != kBF16 && dtype != kF16)) return hipErrorInvalidValue;
  const int64_t total = (int64_t)N * Hs * Ws;
  const int64_t blocks = (total + 255) / 256;
  if (blocks <= 0 || blocks > INT32_MAX) return hipErrorInvalidValue;
  if (dtype == kBF16)
    hipLaunchKernelGGL(stem_s2d_k<bf16_t>, dim3((unsigned)blocks), dim3(256), 0, st, static_cast<const bf16_t*>(x),
                       static_cast<bf16_t*>(out), N, H, W, C, Hs, Ws);
  else
    hipLaunchKernelGGL(stem_s2d_k<f16_t>, dim3((unsigned)blocks), dim3(256), 0, st, static_cast<const f16_t*>(x),
                       static_cast<f16_t*>(out), N, H, W, C, Hs, Ws);
  return hipGetLastError();
}

}  // namespace hyp

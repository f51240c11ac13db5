// NHWC pooling for gfx950: max-pool forward (with a per-element window index for backward),
// max-pool backward as a GATHER (no atomics, deterministic), global average pool fwd/bwd.
//
// Reference: the ResNet stem's ``nn.MaxPool2d(3, 2, 1)`` and the head's
// ``nn.AdaptiveAvgPool2d((1, 1))`` ran as PyTorch/MIOpen kernels (SURVEY §2.4 "Pooling"); on
// MI355X the NHWC max-pool backward alone took 85 µs per ResNet-50 step (profiles/resnet50_r01).
//
// Every thread owns 8 consecutive channels of one pixel (one 16-byte vector).  Max-pool forward
// scans the k x k window and records the winning tap (uint8, taps < 256) per element; backward
// walks, for each INPUT pixel, the <= ceil(k/s)^2 output windows that cover it and sums the
// gradients of those whose recorded tap is this pixel — a gather, so no atomics and no zero-fill.
#include "hyp_common.h"
#include "hyp_kernels.h"

namespace hyp {
namespace {

struct PoolGeom {
  int N, H, W, C, P, Q, k, s, pad;
};

template <typename T>
__global__ __launch_bounds__(256) void maxpool_fwd_k(const T* __restrict__ x, T* __restrict__ y,
                                                     uint8_t* __restrict__ idx, PoolGeom g) {
  const int cv = g.C / 8;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)g.N * g.P * g.Q * cv;
  if (t >= total) return;
  const int c0 = (int)(t % cv) * 8;
  int64_t pix = t / cv;
  const int q = (int)(pix % g.Q);
  pix /= g.Q;
  const int p = (int)(pix % g.P);
  const int n = (int)(pix / g.P);
  float best[8];
  uint8_t arg[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    best[j] = -INFINITY;
    arg[j] = 0;
  }
  for (int r = 0; r < g.k; ++r) {
    const int h = p * g.s - g.pad + r;
    if ((unsigned)h >= (unsigned)g.H) continue;
    for (int c = 0; c < g.k; ++c) {
      const int w = q * g.s - g.pad + c;
      if ((unsigned)w >= (unsigned)g.W) continue;
      float v[8];
      Vec8<T>::load(x + (((int64_t)n * g.H + h) * g.W + w) * g.C + c0, v);
      const uint8_t tap = (uint8_t)(r * g.k + c);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (v[j] > best[j] || (v[j] != v[j] && best[j] == best[j])) {  // NaN propagates like PyTorch
          best[j] = v[j];
          arg[j] = tap;
        }
    }
  }
  const int64_t o = (((int64_t)n * g.P + p) * g.Q + q) * g.C + c0;
  Vec8<T>::store(y + o, best);
  uint2 packed;
  packed.x = arg[0] | (arg[1] << 8) | (arg[2] << 16) | ((uint32_t)arg[3] << 24);
  packed.y = arg[4] | (arg[5] << 8) | (arg[6] << 16) | ((uint32_t)arg[7] << 24);
  *reinterpret_cast<uint2*>(idx + o) = packed;
}

// The ResNet stem's 3x3 / stride-2 window at compile time: the 9 taps' loads are issued together
// (the runtime-k loop above waits one memory round trip per tap: 25 us per ResNet-50 step) —
// same tap order and NaN rule, so the values and recorded taps are identical.
template <typename T, int K, int S>
__global__ __launch_bounds__(256) void maxpool_fwd_fixed_k(const T* __restrict__ x, T* __restrict__ y,
                                                           uint8_t* __restrict__ idx, PoolGeom g) {
  const int cv = g.C / 8;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)g.N * g.P * g.Q * cv;
  if (t >= total) return;
  const int c0 = (int)(t % cv) * 8;
  int64_t pix = t / cv;
  const int q = (int)(pix % g.Q);
  pix /= g.Q;
  const int p = (int)(pix % g.P);
  const int n = (int)(pix / g.P);
  const int h0 = p * S - g.pad, w0 = q * S - g.pad;
  float v[K * K][8];
#pragma unroll
  for (int r = 0; r < K; ++r)
#pragma unroll
    for (int c = 0; c < K; ++c) {
      const int h = min(max(h0 + r, 0), g.H - 1), w = min(max(w0 + c, 0), g.W - 1);  // clamped (masked below)
      Vec8<T>::load(x + (((int64_t)n * g.H + h) * g.W + w) * g.C + c0, v[r * K + c]);
    }
  float best[8];
  uint8_t arg[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    best[j] = -INFINITY;
    arg[j] = 0;
  }
#pragma unroll
  for (int r = 0; r < K; ++r)
#pragma unroll
    for (int c = 0; c < K; ++c) {
      if ((unsigned)(h0 + r) >= (unsigned)g.H || (unsigned)(w0 + c) >= (unsigned)g.W) continue;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float vv = v[r * K + c][j];
        if (vv > best[j] || (vv != vv && best[j] == best[j])) {
          best[j] = vv;
          arg[j] = (uint8_t)(r * K + c);
        }
      }
    }
  const int64_t o = (((int64_t)n * g.P + p) * g.Q + q) * g.C + c0;
  Vec8<T>::store(y + o, best);
  uint2 packed;
  packed.x = arg[0] | (arg[1] << 8) | (arg[2] << 16) | ((uint32_t)arg[3] << 24);
  packed.y = arg[4] | (arg[5] << 8) | (arg[6] << 16) | ((uint32_t)arg[7] << 24);
  *reinterpret_cast<uint2*>(idx + o) = packed;
}

// backward gather with K < 2 S: at most two covering windows per axis (p_hi - 1, p_hi), all four
// candidates' loads in flight at once, summed in the generic kernel's (p, q) ascending order
template <typename T, int K, int S>
__global__ __launch_bounds__(256) void maxpool_bwd_fixed_k(const T* __restrict__ dy, const uint8_t* __restrict__ idx,
                                                           T* __restrict__ dx, PoolGeom g) {
  static_assert(K < 2 * S + 1 && K > S, "two candidate windows per axis");
  const int cv = g.C / 8;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)g.N * g.H * g.W * cv;
  if (t >= total) return;
  const int c0 = (int)(t % cv) * 8;
  int64_t pix = t / cv;
  const int w = (int)(pix % g.W);
  pix /= g.W;
  const int h = (int)(pix % g.H);
  const int n = (int)(pix / g.H);
  const int ph = (h + g.pad) / S, qh = (w + g.pad) / S;
  uint2 pk[2][2];
  float gv[2][2][8];
  bool ok[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int p = ph - 1 + a, q = qh - 1 + b;
      const int r = h + g.pad - p * S, c = w + g.pad - q * S;
      ok[a][b] = p >= 0 && p < g.P && q >= 0 && q < g.Q && r >= 0 && r < K && c >= 0 && c < K;
      const int pc = min(max(p, 0), g.P - 1), qc = min(max(q, 0), g.Q - 1);
      const int64_t o = (((int64_t)n * g.P + pc) * g.Q + qc) * g.C + c0;
      pk[a][b] = *reinterpret_cast<const uint2*>(idx + o);
      Vec8<T>::load(dy + o, gv[a][b]);
    }
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      if (!ok[a][b]) continue;
      const int r = h + g.pad - (ph - 1 + a) * S, c = w + g.pad - (qh - 1 + b) * S;
      const uint32_t tap = (uint32_t)(r * K + c);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t word = j < 4 ? pk[a][b].x : pk[a][b].y;
        if (((word >> (8 * (j & 3))) & 0xff) == tap) acc[j] += gv[a][b][j];
      }
    }
  Vec8<T>::store(dx + (((int64_t)n * g.H + h) * g.W + w) * g.C + c0, acc);
}

template <typename T>
__global__ __launch_bounds__(256) void maxpool_bwd_k(const T* __restrict__ dy, const uint8_t* __restrict__ idx,
                                                     T* __restrict__ dx, PoolGeom g) {
  const int cv = g.C / 8;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)g.N * g.H * g.W * cv;
  if (t >= total) return;
  const int c0 = (int)(t % cv) * 8;
  int64_t pix = t / cv;
  const int w = (int)(pix % g.W);
  pix /= g.W;
  const int h = (int)(pix % g.H);
  const int n = (int)(pix / g.H);
  // output rows p with p*s - pad <= h <= p*s - pad + k - 1
  const int p_lo = max(0, (h + g.pad - g.k + g.s) / g.s), p_hi = min(g.P - 1, (h + g.pad) / g.s);
  const int q_lo = max(0, (w + g.pad - g.k + g.s) / g.s), q_hi = min(g.Q - 1, (w + g.pad) / g.s);
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  for (int p = p_lo; p <= p_hi; ++p) {
    const int r = h + g.pad - p * g.s;
    if (r < 0 || r >= g.k) continue;
    for (int q = q_lo; q <= q_hi; ++q) {
      const int c = w + g.pad - q * g.s;
      if (c < 0 || c >= g.k) continue;
      const uint8_t tap = (uint8_t)(r * g.k + c);
      const int64_t o = (((int64_t)n * g.P + p) * g.Q + q) * g.C + c0;
      const uint2 packed = *reinterpret_cast<const uint2*>(idx + o);
      float gv[8];
      Vec8<T>::load(dy + o, gv);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t word = j < 4 ? packed.x : packed.y;
        if (((word >> (8 * (j & 3))) & 0xff) == tap) acc[j] += gv[j];
      }
    }
  }
  Vec8<T>::store(dx + (((int64_t)n * g.H + h) * g.W + w) * g.C + c0, acc);
}

// y[n, c] = mean over HW of x[n, hw, c]: one block per (image, 512-channel slab), 4 row groups.
template <typename T>
__global__ __launch_bounds__(256) void gap_fwd_k(const T* __restrict__ x, T* __restrict__ y, int HW, int C) {
  __shared__ float red[4][512];
  const int ct = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int c0 = (blockIdx.y * 64 + ct) * 8;
  const int n = blockIdx.x;
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  if (c0 < C) {
    for (int i = rg; i < HW; i += 4) {
      float v[8];
      Vec8<T>::load(x + ((int64_t)n * HW + i) * C + c0, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += v[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[rg][ct * 8 + j] = acc[j];
  __syncthreads();
  for (int i = threadIdx.x; i < 512; i += 256) {
    const int c = blockIdx.y * 512 + i;
    if (c < C) st1<T>(y + (int64_t)n * C + c, (red[0][i] + red[1][i] + red[2][i] + red[3][i]) / (float)HW);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void gap_bwd_k(const T* __restrict__ dy, T* __restrict__ dx, int64_t N, int HW,
                                                 int C) {
  const int cv = C / 8;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= N * HW * cv) return;
  const int c0 = (int)(t % cv) * 8;
  const int64_t n = t / cv / HW;
  float g[8];
  Vec8<T>::load(dy + n * C + c0, g);
  const float inv = 1.f / (float)HW;
#pragma unroll
  for (int j = 0; j < 8; ++j) g[j] *= inv;
  Vec8<T>::store(dx + (t / cv) * C + c0, g);
}

// Strided-conv data gradient completion: out[n, h, w] = addend[n, h, w] + (h % sh == 0 && w % sw == 0 ?
// comp[n, h / sh, w / sw] : 0).  A 1x1 stride-s convolution's dX is dY·W on the output grid
// scattered to every s-th input pixel (zeros elsewhere); `comp` is that GEMM (conv_igemm.hip,
// DGRAD, stride-1 geometry) and this one pass writes the zero-upsampled result — plus, when given,
// the other branch's gradient of the same block input (ResNet downsample + conv1), so neither the
// vendor kernel's zero fill nor autograd's separate add runs.  Sum rounded once, like the add.
template <typename T, bool ADD>
__global__ __launch_bounds__(256) void upsample_add_k(const T* __restrict__ comp, const T* __restrict__ addend,
                                                      T* __restrict__ out, int N, int H, int W, int C, int P, int Q,
                                                      int sh, int sw) {
  const int cv = C / 8;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= (int64_t)N * H * W * cv) return;
  const int c0 = (int)(t % cv) * 8;
  int64_t pix = t / cv;
  const int w = (int)(pix % W);
  pix /= W;
  const int h = (int)(pix % H);
  const int n = (int)(pix / H);
  float v[8];
  const int p = h / sh, q = w / sw;
  if (p * sh == h && q * sw == w && p < P && q < Q) {
    Vec8<T>::load(comp + (((int64_t)n * P + p) * Q + q) * C + c0, v);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = 0.f;
  }
  if (ADD) {
    float a[8];
    Vec8<T>::load(addend + t * 8, a);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] += a[j];
  }
  Vec8<T>::store(out + t * 8, v);
}

inline int blocks_for(int64_t n) { return (int)((n + 255) / 256); }

}  // namespace

hipError_t maxpool2d_forward(int dtype, const void* x, void* y, uint8_t* idx, int N, int H, int W, int C, int k,
                             int s, int pad, hipStream_t st) {
  if (C % 8 != 0 || k * k > 256 || k < 1 || s < 1) return hipErrorInvalidValue;
  const PoolGeom g{N, H, W, C, (H + 2 * pad - k) / s + 1, (W + 2 * pad - k) / s + 1, k, s, pad};
  const int64_t total = (int64_t)N * g.P * g.Q * (C / 8);
  HYP_DISPATCH_FLOAT(dtype, T, {
    if (k == 3 && s == 2)
      hipLaunchKernelGGL((maxpool_fwd_fixed_k<T, 3, 2>), dim3(blocks_for(total)), dim3(256), 0, st, (const T*)x, (T*)y,
                         idx, g);
    else
      hipLaunchKernelGGL(maxpool_fwd_k<T>, dim3(blocks_for(total)), dim3(256), 0, st, (const T*)x, (T*)y, idx, g);
  });
  return hipGetLastError();
}

hipError_t maxpool2d_backward(int dtype, const void* dy, const uint8_t* idx, void* dx, int N, int H, int W, int C,
                              int k, int s, int pad, hipStream_t st) {
  if (C % 8 != 0 || k * k > 256 || k < 1 || s < 1) return hipErrorInvalidValue;
  const PoolGeom g{N, H, W, C, (H + 2 * pad - k) / s + 1, (W + 2 * pad - k) / s + 1, k, s, pad};
  const int64_t total = (int64_t)N * H * W * (C / 8);
  HYP_DISPATCH_FLOAT(dtype, T, {
    if (k == 3 && s == 2)
      hipLaunchKernelGGL((maxpool_bwd_fixed_k<T, 3, 2>), dim3(blocks_for(total)), dim3(256), 0, st, (const T*)dy, idx,
                         (T*)dx, g);
    else
      hipLaunchKernelGGL(maxpool_bwd_k<T>, dim3(blocks_for(total)), dim3(256), 0, st, (const T*)dy, idx, (T*)dx, g);
  });
  return hipGetLastError();
}

hipError_t upsample_add(int dtype, const void* comp, const void* addend, void* out, int N, int H, int W, int C, int P,
                        int Q, int sh, int sw, hipStream_t st) {
  if (C % 8 != 0 || sh < 1 || sw < 1 || P < 1 || Q < 1) return hipErrorInvalidValue;
  const int64_t total = (int64_t)N * H * W * (C / 8);
  HYP_DISPATCH_FLOAT(dtype, T, {
    if (addend)
      hipLaunchKernelGGL((upsample_add_k<T, true>), dim3(blocks_for(total)), dim3(256), 0, st, (const T*)comp,
                         (const T*)addend, (T*)out, N, H, W, C, P, Q, sh, sw);
    else
      hipLaunchKernelGGL((upsample_add_k<T, false>), dim3(blocks_for(total)), dim3(256), 0, st, (const T*)comp,
                         (const T*)addend, (T*)out, N, H, W, C, P, Q, sh, sw);
  });
  return hipGetLastError();
}

hipError_t global_avgpool_forward(int dtype, const void* x, void* y, int N, int HW, int C, hipStream_t st) {
  if (C % 8 != 0) return hipErrorInvalidValue;
  const dim3 grid(N, (C + 511) / 512);
  HYP_DISPATCH_FLOAT(dtype, T, {
    hipLaunchKernelGGL(gap_fwd_k<T>, grid, dim3(256), 0, st, (const T*)x, (T*)y, HW, C);
  });
  return hipGetLastError();
}

hipError_t global_avgpool_backward(int dtype, const void* dy, void* dx, int N, int HW, int C, hipStream_t st) {
  if (C % 8 != 0) return hipErrorInvalidValue;
  const int64_t total = (int64_t)N * HW * (C / 8);
  HYP_DISPATCH_FLOAT(dtype, T, {
    hipLaunchKernelGGL(gap_bwd_k<T>, dim3(blocks_for(total)), dim3(256), 0, st, (const T*)dy, (T*)dx, (int64_t)N, HW,
                       C);
  });
  return hipGetLastError();
}

}  // namespace hyp

// Classifier head + mean-squared error: z = X W^T + b, loss = mean((z - y)^2), in two launches.
//
// Reference: the step benchmark's ``model.fc`` (2048 -> 1000) followed by ``nn.MSELoss()`` against
// random (32, 1000) targets (``Phase 1/baseline_performance.ipynb:252-358``).  On MI355X the torch
// path is 11 launch-bound kernels per step (~77 us: a hipBLASLt forward GEMM, a cast, the MSE
// forward, a mean, two fills, the MSE backward, a cast, the dX and dW GEMMs, the bias-gradient
// reduce) for only 0.4 GFLOP.  Here:
//
// * linear_mse_fwd_k: grid = (N / 16 column tiles, 4 K slices) — ~250 workgroups for the ResNet
//   head; X and the tile's 16 weight rows staged through LDS as fp32 in 128-deep K chunks (the
//   next chunk's loads in flight during this chunk's FMAs), 4 rows x 1 column per thread, fp32
//   slice partials.  linear_mse_epi_k sums a tile's slices in order, rounds z to the compute dtype
//   (the bf16 logits of the torch path), writes dz = 2 (z - y) / (M N) in fp32 and the tile's
//   squared-error partial; linear_mse_loss_k sums those in order — deterministic.
// * linear_mse_bwd_k: ONE launch for all three gradients, scaled by the incoming loss gradient
//   (a device scalar, so a captured step replays with whatever the loss scaler holds):
//   workgroups [0, N / 8) own 8 columns each and write dW (8 x K, 8 k per thread, 8 rows' loads
//   in flight) and db directly; the other (K / 64) x (N / 112) workgroups each stage 112 weight
//   rows x 64 columns and the matching dz block in LDS and write an fp32 dX partial, which
//   linear_mse_dx_k sums in slice order.
// The combines are separate launches on purpose: an in-kernel last-arriver combine needs an
// agent-scope release fence per workgroup (an L2 write-back on gfx950) and measured ~50 us slower
// per step (fwd 72 + bwd 70 us vs 21 + 15 us + three ~5 us combines; profiles/r06/linear_mse/).
#include "hyp_common.h"
#include "hyp_kernels.h"

namespace hyp {
namespace {

constexpr int kLmT = 256;        // threads per workgroup
constexpr int kLmN = 16;         // output columns per forward workgroup
constexpr int kLmKC = 128;       // forward K chunk
constexpr int kLmKS = 4;         // forward K slices (grid.y): ~4 x N/16 workgroups fill the chip
constexpr int kLmMaxM = 64;      // rows (batch) handled by one workgroup
constexpr int kLmNW = 8;         // dW columns per backward workgroup
constexpr int kLmDxK = 64;       // dX columns per backward workgroup
constexpr int kLmNC = 112;       // dX: weight rows (dz columns) per N slice, staged in LDS
constexpr int kLmMaxNS = 16;     // dX: N slices cap

template <typename T>
__device__ __forceinline__ float round_to(float v) {
  T t;
  st1<T>(&t, v);
  return ld1<T>(&t);
}

template <typename T>
__global__ __launch_bounds__(kLmT) void linear_mse_fwd_k(const T* __restrict__ X, const T* __restrict__ W,
                                                         const T* __restrict__ b, const float* __restrict__ y, int M,
                                                         int N, int K, float* __restrict__ zp) {
  __shared__ float xs[kLmMaxM][kLmKC + 4];
  __shared__ float ws[kLmN][kLmKC + 4];
  const int t = threadIdx.x, nl = t & (kLmN - 1), mg = t >> 4;
  const int n0 = blockIdx.x * kLmN;
  const int kper = (K + kLmKS * 8 - 1) / (kLmKS * 8) * 8;
  const int kbeg = blockIdx.y * kper, kend = min(K, kbeg + kper);
  float acc[kLmMaxM / 16] = {0.f, 0.f, 0.f, 0.f};
  // one chunk's global loads all in flight at once (<= 4 X vectors + 1 weight vector per thread),
  // and the next chunk's issued before this chunk's FMAs: one exposed memory round trip per slice
  float xr[kLmMaxM * kLmKC / 8 / kLmT][8], wr[8];
  auto gload = [&](int k0) {
    const int kv = min(kLmKC, kend - k0) / 8;
#pragma unroll
    for (int i = 0; i < kLmMaxM * kLmKC / 8 / kLmT; ++i) {
      const int v = t + i * kLmT;
      if (v < M * kv) {
        const int m = v / kv, kk = (v - m * kv) * 8;
        Vec8<T>::load(X + (int64_t)m * K + k0 + kk, xr[i]);
      }
    }
    if (t < kLmN * kv) {
      const int r = t / kv, kk = (t - r * kv) * 8;
      if (n0 + r < N) Vec8<T>::load(W + (int64_t)(n0 + r) * K + k0 + kk, wr);
      else
#pragma unroll
        for (int e = 0; e < 8; ++e) wr[e] = 0.f;
    }
  };
  auto lstore = [&](int kv) {
#pragma unroll
    for (int i = 0; i < kLmMaxM * kLmKC / 8 / kLmT; ++i) {
      const int v = t + i * kLmT;
      if (v < M * kv) {
        const int m = v / kv, kk = (v - m * kv) * 8;
        *reinterpret_cast<float4*>(&xs[m][kk]) = make_float4(xr[i][0], xr[i][1], xr[i][2], xr[i][3]);
        *reinterpret_cast<float4*>(&xs[m][kk + 4]) = make_float4(xr[i][4], xr[i][5], xr[i][6], xr[i][7]);
      }
    }
    if (t < kLmN * kv) {
      const int r = t / kv, kk = (t - r * kv) * 8;
      *reinterpret_cast<float4*>(&ws[r][kk]) = make_float4(wr[0], wr[1], wr[2], wr[3]);
      *reinterpret_cast<float4*>(&ws[r][kk + 4]) = make_float4(wr[4], wr[5], wr[6], wr[7]);
    }
  };
  if (kbeg < kend) gload(kbeg);
  for (int k0 = kbeg; k0 < kend; k0 += kLmKC) {
    const int kv = min(kLmKC, kend - k0) / 8;  // 8-element vectors in this chunk (K % 8 == 0)
    __syncthreads();
    lstore(kv);
    __syncthreads();
    if (k0 + kLmKC < kend) gload(k0 + kLmKC);
    const int kc = kv * 8;
#pragma unroll 4
    for (int kk = 0; kk < kc; kk += 4) {
      const float4 w4 = *reinterpret_cast<const float4*>(&ws[nl][kk]);
#pragma unroll
      for (int j = 0; j < kLmMaxM / 16; ++j) {
        // rows past M re-read row M - 1 (results dropped): no branch, so the LDS reads batch
        const int m = min(mg + 16 * j, M - 1);
        const float4 x4 = *reinterpret_cast<const float4*>(&xs[m][kk]);
        acc[j] = fmaf(x4.x, w4.x, fmaf(x4.y, w4.y, fmaf(x4.z, w4.z, fmaf(x4.w, w4.w, acc[j]))));
      }
    }
  }
  const int n = n0 + nl;
  // K-slice partials [slice][M][N]; the tile's last slice sums them in slice order (deterministic)
#pragma unroll
  for (int j = 0; j < kLmMaxM / 16; ++j) {
    const int m = mg + 16 * j;
    if (m < M && n < N) zp[((int64_t)blockIdx.y * M + m) * N + n] = acc[j];
  }
}

// the tile's K slices summed in order, bias, compute-dtype rounding, dz and the squared-error partial
template <typename T>
__global__ __launch_bounds__(kLmT) void linear_mse_epi_k(const float* __restrict__ zp, const T* __restrict__ b,
                                                         const float* __restrict__ y, int M, int N,
                                                         float* __restrict__ dz, float* __restrict__ part) {
  __shared__ float red[kLmT / 64];
  const int t = threadIdx.x, nl = t & (kLmN - 1), mg = t >> 4;
  const int tile = blockIdx.x, n = tile * kLmN + nl;
  const float inv = 1.f / ((float)M * (float)N);
  const float bv = (b != nullptr && n < N) ? ld1<T>(b + n) : 0.f;
  float lp = 0.f;
#pragma unroll
  for (int j = 0; j < kLmMaxM / 16; ++j) {
    const int m = mg + 16 * j;
    if (m < M && n < N) {
      float zs = 0.f;
#pragma unroll
      for (int s = 0; s < kLmKS; ++s) zs += zp[((int64_t)s * M + m) * N + n];
      const float z = round_to<T>(zs + bv);  // the compute-dtype logits of the unfused head
      const float d = z - y[(int64_t)m * N + n];
      lp = fmaf(d, d, lp);
      dz[(int64_t)m * N + n] = 2.f * d * inv;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) lp += __shfl_xor(lp, o, 64);
  if ((t & 63) == 0) red[t >> 6] = lp;
  __syncthreads();
  if (t == 0) part[tile] = (red[0] + red[1]) + (red[2] + red[3]);
}

// loss = sum of the tile partials (fixed order) / (M N); one wave
__global__ __launch_bounds__(64) void linear_mse_loss_k(const float* __restrict__ part, int nb, float inv,
                                                        float* __restrict__ loss) {
  float s = 0.f;
  for (int p = threadIdx.x; p < nb; p += 64) s += part[p];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (threadIdx.x == 0) *loss = s * inv;
}

template <typename T>
__global__ __launch_bounds__(kLmT) void linear_mse_bwd_k(const float* __restrict__ dz, const float* __restrict__ go,
                                                         const T* __restrict__ X, const T* __restrict__ W, int M,
                                                         int N, int K, int NBW, int NS, float* __restrict__ dxp,
                                                         T* __restrict__ dW, T* __restrict__ db) {
  __shared__ float dzs[kLmMaxM][kLmNC + 1];
  __shared__ float ws[kLmNC][kLmDxK + 4];
  const int t = threadIdx.x;
  const float g = *go;
  if ((int)blockIdx.x < NBW) {
    // ---- dW / db for columns [n0, n0 + 8): dW[n, k] = sum_m dz[m, n] X[m, k]
    const int n0 = blockIdx.x * kLmNW;
    for (int v = t; v < kLmMaxM * kLmNW; v += kLmT) {  // rows past M zeroed: they meet x = 0
      const int m = v / kLmNW, c = v % kLmNW;
      dzs[m][c] = (m < M && n0 + c < N) ? dz[(int64_t)m * N + n0 + c] * g : 0.f;
    }
    __syncthreads();
    if (db != nullptr && t < kLmNW && n0 + t < N) {
      float s = 0.f;
      for (int m = 0; m < M; ++m) s += dzs[m][t];
      st1<T>(db + n0 + t, s);
    }
    for (int kb = t * 8; kb < K; kb += kLmT * 8) {
      float acc[kLmNW][8];
#pragma unroll
      for (int c = 0; c < kLmNW; ++c)
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[c][e] = 0.f;
      for (int m0 = 0; m0 < M; m0 += 8) {
        float x[8][8];  // 8 rows' vectors in flight at once
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          if (m0 + i < M) Vec8<T>::load(X + (int64_t)(m0 + i) * K + kb, x[i]);
          else
#pragma unroll
            for (int e = 0; e < 8; ++e) x[i][e] = 0.f;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int m = min(m0 + i, kLmMaxM - 1);  // rows past M carry x = 0
#pragma unroll
          for (int c = 0; c < kLmNW; ++c) {
            const float d = dzs[m][c];
#pragma unroll
            for (int e = 0; e < 8; ++e) acc[c][e] = fmaf(d, x[i][e], acc[c][e]);
          }
        }
      }
#pragma unroll
      for (int c = 0; c < kLmNW; ++c)
        if (n0 + c < N) Vec8<T>::store(dW + (int64_t)(n0 + c) * K + kb, acc[c]);
    }
    return;
  }
  // ---- dX partial for columns [k0, k0 + 64) over weight rows [nbeg, nend): one N slice
  const int idx = blockIdx.x - NBW, kt = idx / NS, ns = idx - kt * NS;
  const int k0 = kt * kLmDxK;
  const int nbeg = ns * kLmNC, nc = min(kLmNC, N - nbeg);
  const int kg = (t & 7) * 8, mg = t >> 3;  // 8 column vectors x 32 rows (x 2 for M > 32)
  const bool kin = k0 + kg < K;
  for (int v = t; v < M * kLmNC; v += kLmT) {
    const int m = v / kLmNC, j = v - m * kLmNC;
    dzs[m][j] = j < nc ? dz[(int64_t)m * N + nbeg + j] * g : 0.f;
  }
  for (int v = t; v < kLmNC * (kLmDxK / 8); v += kLmT) {
    const int j = v >> 3, kk = (v & 7) * 8;
    float f[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (j < nc && k0 + kk < K) Vec8<T>::load(W + (int64_t)(nbeg + j) * K + k0 + kk, f);
    *reinterpret_cast<float4*>(&ws[j][kk]) = make_float4(f[0], f[1], f[2], f[3]);
    *reinterpret_cast<float4*>(&ws[j][kk + 4]) = make_float4(f[4], f[5], f[6], f[7]);
  }
  __syncthreads();
  float acc[2][8];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[r][e] = 0.f;
#pragma unroll 4
  for (int j = 0; j < nc; ++j) {
    const float4 wa = *reinterpret_cast<const float4*>(&ws[j][kg]);
    const float4 wb = *reinterpret_cast<const float4*>(&ws[j][kg + 4]);
    const float w[8] = {wa.x, wa.y, wa.z, wa.w, wb.x, wb.y, wb.z, wb.w};
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const float d = dzs[min(mg + 32 * r, kLmMaxM - 1)][j];
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[r][e] = fmaf(d, w[e], acc[r][e]);
    }
  }
  if (kin) {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int m = mg + 32 * r;
      if (m < M) Vec8<float>::store(dxp + ((int64_t)ns * M + m) * K + k0 + kg, acc[r]);
    }
  }
}

// dX[m, k] = sum of the N-slice partials in slice order (deterministic)
template <typename T>
__global__ __launch_bounds__(kLmT) void linear_mse_dx_k(const float* __restrict__ dxp, int M, int K, int NS,
                                                        T* __restrict__ dX) {
  const int t = threadIdx.x, kg = (t & 7) * 8, mg = t >> 3;
  const int k0 = blockIdx.x * kLmDxK;
  if (k0 + kg >= K) return;
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int m = mg + 32 * r;
    if (m >= M) continue;
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int q = 0; q < NS; ++q) {
      float v[8];
      Vec8<float>::load(dxp + ((int64_t)q * M + m) * K + k0 + kg, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) s[e] += v[e];
    }
    Vec8<T>::store(dX + (int64_t)m * K + k0 + kg, s);
  }
}

}  // namespace

int linear_mse_partials(int N) { return (N + kLmN - 1) / kLmN; }

// workspace floats: forward kLmKS*M*N (+ nb partials), backward NS*M*K
int64_t linear_mse_workspace(int M, int N, int K) {
  const int ns = (N + kLmNC - 1) / kLmNC;
  const int64_t f = (int64_t)kLmKS * M * N + linear_mse_partials(N), bw = (int64_t)ns * M * K;
  return f > bw ? f : bw;
}

hipError_t linear_mse_fwd(int dtype, const void* X, const void* W, const void* b, const float* y, int M, int N, int K,
                          float* dz, float* ws, float* loss, hipStream_t st) {
  const int nb = linear_mse_partials(N);
  if (M < 1 || M > kLmMaxM || N < 1 || K < 8 || K % 8 != 0) return hipErrorInvalidValue;
  float* part = ws + (int64_t)kLmKS * M * N;
  HYP_DISPATCH_FLOAT(dtype, T, {
    hipLaunchKernelGGL(linear_mse_fwd_k<T>, dim3(nb, kLmKS), dim3(kLmT), 0, st, static_cast<const T*>(X),
                       static_cast<const T*>(W), static_cast<const T*>(b), y, M, N, K, ws);
    hipLaunchKernelGGL(linear_mse_epi_k<T>, dim3(nb), dim3(kLmT), 0, st, ws, static_cast<const T*>(b), y, M, N, dz,
                       part);
  });
  hipLaunchKernelGGL(linear_mse_loss_k, dim3(1), dim3(64), 0, st, part, nb, 1.f / ((float)M * (float)N), loss);
  return hipGetLastError();
}

hipError_t linear_mse_bwd(int dtype, const float* dz, const float* go, const void* X, const void* W, int M, int N,
                          int K, void* dX, void* dW, void* db, float* ws, hipStream_t st) {
  const int nbw = (N + kLmNW - 1) / kLmNW, kt = (K + kLmDxK - 1) / kLmDxK, ns = (N + kLmNC - 1) / kLmNC;
  if (M < 1 || M > kLmMaxM || N < 1 || K < 8 || K % 8 != 0 || ns > kLmMaxNS)
    return hipErrorInvalidValue;
  HYP_DISPATCH_FLOAT(dtype, T, {
    hipLaunchKernelGGL(linear_mse_bwd_k<T>, dim3(nbw + kt * ns), dim3(kLmT), 0, st, dz, go, static_cast<const T*>(X),
                       static_cast<const T*>(W), M, N, K, nbw, ns, ws, static_cast<T*>(dW), static_cast<T*>(db));
    hipLaunchKernelGGL(linear_mse_dx_k<T>, dim3(kt), dim3(kLmT), 0, st, ws, M, K, ns, static_cast<T*>(dX));
  });
  return hipGetLastError();
}

}  // namespace hyp

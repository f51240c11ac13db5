// The rank-r halves of the fused LoRA projections (ops/llama_fused.py), around the weight-streaming
// GEMMs of kernels/wstream.hip.
//
// Reference: PEFT lora.Linear — dropout(x) -> lora_A -> lora_B -> * scaling -> add, per target
// module q/k/v/o (02_development/distributed_utils.py:463-476; SURVEY §2.4 "LoRA"), 4-5 kernels and a
// stored dropout mask per projection.  Here, for the P projections that read the same input x
// (q, k, v: P = 3; o: P = 1), with c' = scaling / (1 - p) and keep_p the regenerated dropout mask
// (lora_keep in hyp_common.h; never stored):
//   lora_down   t'[m, p r + j] = Σ_k keep_p(m, k) x[m, k] A_p[j, k]          (fp32, MFMA, atomics)
//   lora_bwd_t  du'[m, p r + j] = c' Σ_n dy_p[m, n] B_p[n, j]   (atomics),  dB_p = c' dy_pᵀ t'_p
//   lora_bwd_a  dA_p[j, k] = Σ_m du'[m, p r + j] keep_p(m, k) x[m, k]
// and the up term c' t' Bᵀ / the data-gradient term keep ∘ (du' A) ride in ws_epilogue.
#include "hyp_common.h"
#include "hyp_kernels.h"
#include "mfma_lds.h"

namespace hyp {
namespace {

using mfl::f32x4;
using mfl::u16x8;

struct LoraPtrs {
  const void* p[4];
};

// block = 16 rows x 256 k; wave p (< P) computes the 16 x r tile of projection p with 16x16x32
// MFMAs (A = masked x fragment from LDS, B = A_p rows from global), atomically added into t.
template <typename T>
__global__ __launch_bounds__(256) void lora_down_k(const T* __restrict__ x, int64_t ldx, LoraPtrs A, float* t, int ldt,
                                                   int M, int K, int P, int r, RngState rs, uint32_t thr, int drop) {
  __shared__ __attribute__((aligned(16))) uint16_t xs[4][16][256 + 8];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m0 = blockIdx.y * 16, k0 = blockIdx.x * 256;
  const uint64_t key = drop ? rng_key(rs) : 0ull;
  // 16 x 256 tile: thread -> row tid / 16, 16 consecutive k
  {
    const int rl = tid >> 4, kk = (tid & 15) * 16, m = m0 + rl;
    float v[16];
    if (m < M) {
      Vec8<T>::load(x + (int64_t)m * ldx + k0 + kk, *reinterpret_cast<float(*)[8]>(&v[0]));
      Vec8<T>::load(x + (int64_t)m * ldx + k0 + kk + 8, *reinterpret_cast<float(*)[8]>(&v[8]));
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = 0.f;
    }
    for (int p = 0; p < P; ++p) {
      float mv[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const bool keep = !drop || lora_keep(key, (uint32_t)(((int64_t)p * M + m) * K + k0 + kk + i), thr);
        mv[i] = keep ? v[i] : 0.f;
      }
      Vec8<T>::store(reinterpret_cast<T*>(&xs[p][rl][kk]), *reinterpret_cast<float(*)[8]>(&mv[0]));
      Vec8<T>::store(reinterpret_cast<T*>(&xs[p][rl][kk + 8]), *reinterpret_cast<float(*)[8]>(&mv[8]));
    }
  }
  __syncthreads();
  if (wave >= P) return;
  const int p = wave, l15 = lane & 15, g4 = lane >> 4;
  const T* Ap = static_cast<const T*>(A.p[p]);
  for (int j0 = 0; j0 < r; j0 += 16) {
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
    const bool jok = j0 + l15 < r;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      const u16x8 af = *reinterpret_cast<const u16x8*>(&xs[p][l15][ks * 32 + g4 * 8]);
      u16x8 bf = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if (jok) bf = *reinterpret_cast<const u16x8*>(Ap + (int64_t)(j0 + l15) * K + k0 + ks * 32 + g4 * 8);
      acc = mfl::mma16<T>(af, bf, acc);
    }
    // acc[e] = t[m0 + 4 g4 + e][j0 + l15]
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int m = m0 + 4 * g4 + e;
      if (m < M && jok) atomicAdd(t + (int64_t)m * ldt + p * r + j0 + l15, acc[e]);
    }
  }
}

// block (p, 64-column slice of dy_p): dB for those 64 rows of B_p (full reduction over M in-block)
// and the slice's contribution to du' (atomics).  LDS: dy slice [M<=256][64] fp32, t'_p, B rows.
template <typename T>
__global__ __launch_bounds__(256) void lora_bwd_t_k(const T* __restrict__ dy, int64_t ldy, int N, LoraPtrs B,
                                                    LoraPtrs dB, const float* __restrict__ t, int ldt, float* du,
                                                    int M, int r, float c) {
  __shared__ float ys[64][65];   // [n][m chunk of 64]
  __shared__ float ts[64][17];   // t'_p rows of the m chunk
  __shared__ float bs[64][17];   // B_p rows of the slice
  const int tid = threadIdx.x;
  const int p = blockIdx.y, n0 = blockIdx.x * 64;
  const T* Bp = static_cast<const T*>(B.p[p]);
  for (int i = tid; i < 64 * r; i += 256) {
    const int nn = i / r, j = i - nn * r;
    bs[nn][j] = ld1<T>(Bp + (int64_t)(n0 + nn) * r + j);
  }
  // dB accumulators: thread -> (n = tid / 4, j = (tid % 4) * 4 .. +3)
  const int dn = tid >> 2, dj = (tid & 3) * 4;
  float db[4] = {0.f, 0.f, 0.f, 0.f};
  for (int mc = 0; mc < M; mc += 64) {
    __syncthreads();
    for (int i = tid; i < 64 * 64; i += 256) {
      const int mm = i >> 6, nn = i & 63, m = mc + mm;
      ys[nn][mm] = m < M ? ld1<T>(dy + (int64_t)m * ldy + (int64_t)p * N + n0 + nn) : 0.f;
    }
    for (int i = tid; i < 64 * r; i += 256) {
      const int mm = i / r, j = i - mm * r, m = mc + mm;
      ts[mm][j] = m < M ? t[(int64_t)m * ldt + p * r + j] : 0.f;
    }
    __syncthreads();
    // dB[n][j] += Σ_m dy[m][n] t[m][j]
#pragma unroll 4
    for (int mm = 0; mm < 64; ++mm) {
      const float yv = ys[dn][mm];
#pragma unroll
      for (int q = 0; q < 4; ++q) db[q] += yv * ts[mm][dj + q];
    }
    // du'[m][j] += c Σ_{n in slice} dy[m][n] B[n][j]: thread -> (m = tid / 4, 4 ranks)
    {
      const int mm = tid >> 2, m = mc + mm;
      float s[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
      for (int nn = 0; nn < 64; ++nn) {
        const float yv = ys[nn][mm];
#pragma unroll
        for (int q = 0; q < 4; ++q) s[q] += yv * bs[nn][dj + q];
      }
      if (m < M) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (dj + q < r) atomicAdd(du + (int64_t)m * ldt + p * r + dj + q, c * s[q]);
      }
    }
  }
  T* dBp = static_cast<T*>(const_cast<void*>(dB.p[p]));
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (dj + q < r) st1<T>(dBp + (int64_t)(n0 + dn) * r + dj + q, c * db[q]);
}

// block (p, 64-column slice of x): dA_p[:, slice] = Σ_m du'[m, p r + j] keep_p(m, k) x[m, k]
template <typename T>
__global__ __launch_bounds__(256) void lora_bwd_a_k(const T* __restrict__ x, int64_t ldx, int K, LoraPtrs dA,
                                                    const float* __restrict__ du, int ldt, int M, int r, RngState rs,
                                                    uint32_t thr, int drop) {
  __shared__ float xs[64][65];  // [m chunk][k]
  __shared__ float us[64][17];
  const int tid = threadIdx.x;
  const int p = blockIdx.y, k0 = blockIdx.x * 64;
  const uint64_t key = drop ? rng_key(rs) : 0ull;
  // thread -> (k = tid % 64, ranks (tid / 64) * 4 .. +3)
  const int kk = tid & 63, j0 = (tid >> 6) * 4;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int mc = 0; mc < M; mc += 64) {
    __syncthreads();
    for (int i = tid; i < 64 * 64; i += 256) {
      const int mm = i >> 6, c = i & 63, m = mc + mm;
      float v = 0.f;
      if (m < M) {
        v = ld1<T>(x + (int64_t)m * ldx + k0 + c);
        if (drop && !lora_keep(key, (uint32_t)(((int64_t)p * M + m) * K + k0 + c), thr)) v = 0.f;
      }
      xs[mm][c] = v;
    }
    for (int i = tid; i < 64 * r; i += 256) {
      const int mm = i / r, j = i - mm * r, m = mc + mm;
      us[mm][j] = m < M ? du[(int64_t)m * ldt + p * r + j] : 0.f;
    }
    __syncthreads();
#pragma unroll 4
    for (int mm = 0; mm < 64; ++mm) {
      const float xv = xs[mm][kk];
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] += us[mm][j0 + q] * xv;
    }
  }
  T* dAp = static_cast<T*>(const_cast<void*>(dA.p[p]));
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (j0 + q < r) st1<T>(dAp + (int64_t)(j0 + q) * K + k0 + kk, acc[q]);
}

LoraPtrs pack(const void* const* v, int P) {
  LoraPtrs o{};
  for (int i = 0; i < 4; ++i) o.p[i] = i < P ? v[i] : nullptr;
  return o;
}

}  // namespace

hipError_t lora_down(int dtype, const void* x, int64_t ldx, const void* const* A, int P, int r, float* t, int ldt, int M,
                     int K, const RngState* rng, float p_drop, hipStream_t st) {
  if ((dtype != kBF16 && dtype != kF16) || P < 1 || P > 4 || r < 1 || r > 16 || K % 256 != 0 || M < 1)
    return hipErrorInvalidValue;
  const int drop = (rng != nullptr && p_drop > 0.f) ? 1 : 0;
  const RngState rs = drop ? *rng : RngState{};
  const uint32_t thr = (uint32_t)fminf(p_drop * 4294967296.f, 4294967295.f);
  dim3 grid(K / 256, (M + 15) / 16);
  if (dtype == kBF16)
    hipLaunchKernelGGL(lora_down_k<bf16_t>, grid, dim3(256), 0, st, static_cast<const bf16_t*>(x), ldx, pack(A, P), t,
                       ldt, M, K, P, r, rs, thr, drop);
  else
    hipLaunchKernelGGL(lora_down_k<f16_t>, grid, dim3(256), 0, st, static_cast<const f16_t*>(x), ldx, pack(A, P), t,
                       ldt, M, K, P, r, rs, thr, drop);
  return hipGetLastError();
}

hipError_t lora_bwd_t(int dtype, const void* dy, int64_t ldy, int N, const void* const* B, void* const* dB, int P,
                      int r, const float* t, int ldt, float* du, int M, float c, hipStream_t st) {
  if ((dtype != kBF16 && dtype != kF16) || P < 1 || P > 4 || r < 1 || r > 16 || N % 64 != 0 || M < 1)
    return hipErrorInvalidValue;
  dim3 grid(N / 64, P);
  LoraPtrs bp = pack(B, P), dbp = pack(const_cast<const void* const*>(reinterpret_cast<void* const*>(dB)), P);
  if (dtype == kBF16)
    hipLaunchKernelGGL(lora_bwd_t_k<bf16_t>, grid, dim3(256), 0, st, static_cast<const bf16_t*>(dy), ldy, N, bp, dbp,
                       t, ldt, du, M, r, c);
  else
    hipLaunchKernelGGL(lora_bwd_t_k<f16_t>, grid, dim3(256), 0, st, static_cast<const f16_t*>(dy), ldy, N, bp, dbp, t,
                       ldt, du, M, r, c);
  return hipGetLastError();
}

hipError_t lora_bwd_a(int dtype, const void* x, int64_t ldx, int K, void* const* dA, int P, int r, const float* du,
                      int ldt, int M, const RngState* rng, float p_drop, hipStream_t st) {
  if ((dtype != kBF16 && dtype != kF16) || P < 1 || P > 4 || r < 1 || r > 16 || K % 64 != 0 || M < 1)
    return hipErrorInvalidValue;
  const int drop = (rng != nullptr && p_drop > 0.f) ? 1 : 0;
  const RngState rs = drop ? *rng : RngState{};
  const uint32_t thr = (uint32_t)fminf(p_drop * 4294967296.f, 4294967295.f);
  dim3 grid(K / 64, P);
  LoraPtrs dap = pack(const_cast<const void* const*>(reinterpret_cast<void* const*>(dA)), P);
  if (dtype == kBF16)
    hipLaunchKernelGGL(lora_bwd_a_k<bf16_t>, grid, dim3(256), 0, st, static_cast<const bf16_t*>(x), ldx, K, dap, du,
                       ldt, M, r, rs, thr, drop);
  else
    hipLaunchKernelGGL(lora_bwd_a_k<f16_t>, grid, dim3(256), 0, st, static_cast<const f16_t*>(x), ldx, K, dap, du, ldt,
                       M, r, rs, thr, drop);
  return hipGetLastError();
}

}  // namespace hyp

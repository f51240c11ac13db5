// The rank-r halves of the fused LoRA projections (ops/llama_fused.py), around the weight-streaming
// GEMMs of kernels/wstream.hip.
//
// Reference: PEFT lora.Linear — dropout(x) -> lora_A -> lora_B -> * scaling -> add, per target
// module q/k/v/o (02_development/distributed_utils.py:463-476; SURVEY §2.4 "LoRA"), 4-5 kernels and a
// stored dropout mask per projection.  Here, for the P projections that read the same input x
// (q, k, v: P = 3; o: P = 1), with c' = scaling / (1 - p) and keep_p the regenerated dropout mask
// (lora_keep in hyp_common.h; never stored):
//   lora_down   t'[m, p r + j] = Σ_k keep_p(m, k) x[m, k] A_p[j, k]          (fp32, MFMA, written)
//   lora_bwd_t  du'[m, p r + j] += c' Σ_n dy_p[m, n] B_p[n, j]   (atomics),  dB_p = c' dy_pᵀ t'_p
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

// lora_down: block (p, 16-row m-tile, k-split q < KS), 4 waves splitting the block's K range; A
// fragments are the (masked) x rows and B fragments the rows of A_p, both straight from global
// memory (16 contiguous bytes per lane).  Each block leaves its 16 x 16 partial tile (summed over
// its waves through LDS) in `part`; the LAST block of the (p, m-tile) to count in on its counter
// slot sums the KS partials in fixed order and WRITES t (deterministic; no atomics on t and no
// zero-fill launch), then resets the slot.  The launch also zeroes z[0, nz) — the du buffer the
// backward's lora_bwd_t accumulates into.
template <typename T>
__global__ __launch_bounds__(256) void lora_down_k(const T* __restrict__ x, int64_t ldx, LoraPtrs A, float* t, int ldt,
                                                   int M, int K, int P, int r, RngState rs, uint32_t thr, int drop,
                                                   float* z, int nz, float* part, int* cnt, int KS) {
  __shared__ f32x4 red[4][64];
  __shared__ int is_last;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  {
    const int nb = gridDim.x * gridDim.y * gridDim.z;
    const int b = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
    for (int i = b * 256 + tid; i < nz; i += nb * 256) z[i] = 0.f;
  }
  const int p = blockIdx.x, mt = blockIdx.y, q = blockIdx.z, m0 = mt * 16;
  const uint64_t key = drop ? rng_key(rs) : 0ull;
  const int l15 = lane & 15, g4 = lane >> 4;
  const int m = m0 + l15;
  const bool mok = m < M, jok = l15 < r;
  const T* xr = x + (int64_t)(mok ? m : 0) * ldx;
  const T* ar = static_cast<const T*>(A.p[p]) + (int64_t)(jok ? l15 : 0) * K;
  const int kw = K / (KS * 4);  // % 32 == 0 (host check)
  const int kb = (q * 4 + wave) * kw, ke = kb + kw;
  const uint32_t ibase = (uint32_t)(((int64_t)p * M + m) * K);
  f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int k = kb; k < ke; k += 128) {
    u16x8 a[4], b[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {  // all loads of the group in flight together
      const int kk = min(k + 32 * u, ke - 32) + g4 * 8;
      a[u] = *reinterpret_cast<const u16x8*>(xr + kk);
      b[u] = *reinterpret_cast<const u16x8*>(ar + kk);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (k + 32 * u >= ke) break;
      u16x8 av = a[u], bv = b[u];
      if (!mok) av = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if (!jok) bv = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if (drop) {
        const int kk = k + 32 * u + g4 * 8;
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (!lora_keep(key, ibase + (uint32_t)(kk + e), thr)) av[e] = 0;
      }
      acc = mfl::mma16<T>(av, bv, acc);
    }
  }
  red[wave][lane] = acc;
  __syncthreads();
  const int tile = p * gridDim.y + mt;
  f32x4* tp = reinterpret_cast<f32x4*>(part) + (int64_t)tile * KS * 64;
  if (wave == 0) {
    f32x4 s = red[0][lane];
#pragma unroll
    for (int w = 1; w < 4; ++w) s += red[w][lane];
    tp[q * 64 + lane] = s;
  }
  __threadfence();  // release: this block's partial is visible device-wide before it counts in
  __syncthreads();
  if (tid == 0) {
    const int old = atomicAdd(cnt + tile, 1);
    is_last = old == KS - 1;
    if (is_last) cnt[tile] = 0;  // every block of the tile has counted: reset for the next launch
  }
  __syncthreads();
  if (!is_last || wave != 0) return;
  __threadfence();  // acquire: the other blocks' partials
  f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int i = 0; i < KS; ++i) s += __builtin_nontemporal_load(tp + i * 64 + lane);
  // s[e] = t[m0 + 4 g4 + e][p r + l15]
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int mm = m0 + 4 * g4 + e;
    if (mm < M && jok) t[(int64_t)mm * ldt + p * r + l15] = s[e];
  }
}

// lora_bwd_t: block (p, 256-column slice of dy_p), 512 threads.  The dy tile (128 rows per pass)
// is staged in LDS with 16-byte loads all in flight at once; then, with every LDS read a 16-byte
// vector feeding 8-16 FMAs:
//   dB rows of the slice, reduced over all M in the block (thread = (column, 8 ranks));
//   the slice's share of du' (thread = (row, 4 ranks)), added atomically — 16-way per element at
//   N = 4096 (du zeroed by the forward's lora_down).
constexpr int kBtN = 256, kBtM = 128;
template <typename T>
__global__ __launch_bounds__(512) void lora_bwd_t_k(const T* __restrict__ dy, int64_t ldy, int N, LoraPtrs B,
                                                    LoraPtrs dB, const float* __restrict__ t, int ldt, float* du,
                                                    int M, int r, float c) {
  __shared__ __attribute__((aligned(16))) uint16_t ys[kBtM][kBtN + 8];
  __shared__ __attribute__((aligned(16))) float ts[kBtM][16];
  __shared__ __attribute__((aligned(16))) float bs[kBtN][16];
  const int tid = threadIdx.x;
  const int p = blockIdx.y, n0 = blockIdx.x * kBtN;
  const T* Bp = static_cast<const T*>(B.p[p]);
  for (int i = tid; i < kBtN * 16; i += 512) {
    const int nn = i >> 4, j = i & 15;
    bs[nn][j] = j < r ? ld1<T>(Bp + (int64_t)(n0 + nn) * r + j) : 0.f;
  }
  const int dn = tid & 255, djh = (tid >> 8) * 8;  // dB: column dn, ranks djh .. djh+7
  float db[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) db[j] = 0.f;
  const T* dyp = dy + (int64_t)p * N + n0;
  for (int mc = 0; mc < M; mc += kBtM) {
    const int rows = min(kBtM, M - mc);
    __syncthreads();
    uint4 v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int idx = tid + 512 * i, row = idx >> 5, ch = idx & 31;
      v[i] = row < rows ? *reinterpret_cast<const uint4*>(dyp + (int64_t)(mc + row) * ldy + ch * 8)
                        : uint4{0u, 0u, 0u, 0u};
    }
    for (int i = tid; i < kBtM * 16; i += 512) {
      const int row = i >> 4, j = i & 15;
      ts[row][j] = (row < rows && j < r) ? t[(int64_t)(mc + row) * ldt + p * r + j] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int idx = tid + 512 * i, row = idx >> 5, ch = idx & 31;
      *reinterpret_cast<uint4*>(&ys[row][ch * 8]) = v[i];
    }
    __syncthreads();
    // dB[n][j] += Σ_m dy[m][n] t[m][j]
    for (int mm = 0; mm < rows; ++mm) {
      const float yv = ld1<T>(reinterpret_cast<const T*>(&ys[mm][dn]));
      const float4 t0 = *reinterpret_cast<const float4*>(&ts[mm][djh]);
      const float4 t1 = *reinterpret_cast<const float4*>(&ts[mm][djh + 4]);
      db[0] += yv * t0.x; db[1] += yv * t0.y; db[2] += yv * t0.z; db[3] += yv * t0.w;
      db[4] += yv * t1.x; db[5] += yv * t1.y; db[6] += yv * t1.z; db[7] += yv * t1.w;
    }
    // du'[m][j] += c Σ_{n in slice} dy[m][n] B[n][j]   (thread = row mm, ranks jq .. jq+3)
    const int mm = tid >> 2, jq = (tid & 3) * 4;
    if (mm < rows) {
      float s[4] = {0.f, 0.f, 0.f, 0.f};
      for (int n = 0; n < kBtN; n += 8) {
        float yv[8];
        Vec8<T>::load(reinterpret_cast<const T*>(&ys[mm][n]), yv);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float4 bv = *reinterpret_cast<const float4*>(&bs[n + e][jq]);
          s[0] += yv[e] * bv.x; s[1] += yv[e] * bv.y; s[2] += yv[e] * bv.z; s[3] += yv[e] * bv.w;
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (jq + j < r) atomicAdd(du + (int64_t)(mc + mm) * ldt + p * r + jq + j, c * s[j]);
    }
  }
  T* dBp = static_cast<T*>(const_cast<void*>(dB.p[p]));
#pragma unroll
  for (int j = 0; j < 8; ++j)
    if (djh + j < r) st1<T>(dBp + (int64_t)(n0 + dn) * r + djh + j, c * db[j]);
}

// lora_bwd_a: block (p, 64-column slice of x): dA_p[:, slice] = Σ_m du'[m, p r + j] keep_p(m, k) x[m, k];
// up to 128 rows per pass, the x tile arriving with four 16-byte loads per thread issued together.
template <typename T>
__global__ __launch_bounds__(256) void lora_bwd_a_k(const T* __restrict__ x, int64_t ldx, int K, LoraPtrs dA,
                                                    const float* __restrict__ du, int ldt, int M, int r, RngState rs,
                                                    uint32_t thr, int drop) {
  __shared__ float xs[128][65];  // [m chunk][k]
  __shared__ __attribute__((aligned(16))) float us[128][16];
  const int tid = threadIdx.x;
  const int p = blockIdx.y, k0 = blockIdx.x * 64;
  const uint64_t key = drop ? rng_key(rs) : 0ull;
  const int kk = tid & 63, j0 = (tid >> 6) * 4;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int mc = 0; mc < M; mc += 128) {
    __syncthreads();
    uint4 v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = tid + 256 * i, row = idx >> 3, ch = idx & 7, m = mc + row;
      v[i] = m < M ? *reinterpret_cast<const uint4*>(x + (int64_t)m * ldx + k0 + ch * 8) : uint4{0u, 0u, 0u, 0u};
    }
    float uv[8];
    {
      const int row = tid >> 1, q = (tid & 1) * 8, m = mc + row;
#pragma unroll
      for (int e = 0; e < 8; ++e) uv[e] = (m < M && q + e < r) ? du[(int64_t)m * ldt + p * r + q + e] : 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) us[row][q + e] = uv[e];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = tid + 256 * i, row = idx >> 3, ch = idx & 7, m = mc + row;
      float f[8];
      Vec8<T>::load(reinterpret_cast<const T*>(&v[i]), f);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = k0 + ch * 8 + e;
        if (drop && !lora_keep(key, (uint32_t)(((int64_t)p * M + m) * K + k), thr)) f[e] = 0.f;
        xs[row][ch * 8 + e] = f[e];
      }
    }
    __syncthreads();
    const int rows = min(128, M - mc);
#pragma unroll 8
    for (int mm = 0; mm < rows; ++mm) {
      const float xv = xs[mm][kk];
      const float4 u = *reinterpret_cast<const float4*>(&us[mm][j0]);
      acc[0] += u.x * xv; acc[1] += u.y * xv; acc[2] += u.z * xv; acc[3] += u.w * xv;
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
                     int K, const RngState* rng, float p_drop, float* zero, int nzero, float* part, int* counters,
                     int ksplit, hipStream_t st) {
  if ((dtype != kBF16 && dtype != kF16) || P < 1 || P > 4 || r < 1 || r > 16 || M < 1 || ksplit < 1 ||
      K % (128 * ksplit) != 0 || ldx % 8 != 0 || (nzero > 0 && zero == nullptr) || part == nullptr ||
      counters == nullptr || P * ((M + 15) / 16) > 4096)
    return hipErrorInvalidValue;
  const int drop = (rng != nullptr && p_drop > 0.f) ? 1 : 0;
  const RngState rs = drop ? *rng : RngState{};
  const uint32_t thr = (uint32_t)fminf(p_drop * 4294967296.f, 4294967295.f);
  dim3 grid(P, (M + 15) / 16, ksplit);
  if (dtype == kBF16)
    hipLaunchKernelGGL(lora_down_k<bf16_t>, grid, dim3(256), 0, st, static_cast<const bf16_t*>(x), ldx, pack(A, P), t,
                       ldt, M, K, P, r, rs, thr, drop, zero, nzero, part, counters, ksplit);
  else
    hipLaunchKernelGGL(lora_down_k<f16_t>, grid, dim3(256), 0, st, static_cast<const f16_t*>(x), ldx, pack(A, P), t,
                       ldt, M, K, P, r, rs, thr, drop, zero, nzero, part, counters, ksplit);
  return hipGetLastError();
}

hipError_t lora_bwd_t(int dtype, const void* dy, int64_t ldy, int N, const void* const* B, void* const* dB, int P,
                      int r, const float* t, int ldt, float* du, int M, float c, hipStream_t st) {
  if ((dtype != kBF16 && dtype != kF16) || P < 1 || P > 4 || r < 1 || r > 16 || N % kBtN != 0 || M < 1 || ldy % 8 != 0)
    return hipErrorInvalidValue;
  dim3 grid(N / kBtN, P);
  LoraPtrs bp = pack(B, P), dbp = pack(const_cast<const void* const*>(reinterpret_cast<void* const*>(dB)), P);
  if (dtype == kBF16)
    hipLaunchKernelGGL(lora_bwd_t_k<bf16_t>, grid, dim3(512), 0, st, static_cast<const bf16_t*>(dy), ldy, N, bp, dbp,
                       t, ldt, du, M, r, c);
  else
    hipLaunchKernelGGL(lora_bwd_t_k<f16_t>, grid, dim3(512), 0, st, static_cast<const f16_t*>(dy), ldy, N, bp, dbp, t,
                       ldt, du, M, r, c);
  return hipGetLastError();
}

hipError_t lora_bwd_a(int dtype, const void* x, int64_t ldx, int K, void* const* dA, int P, int r, const float* du,
                      int ldt, int M, const RngState* rng, float p_drop, hipStream_t st) {
  if ((dtype != kBF16 && dtype != kF16) || P < 1 || P > 4 || r < 1 || r > 16 || K % 64 != 0 || M < 1 || ldx % 8 != 0)
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

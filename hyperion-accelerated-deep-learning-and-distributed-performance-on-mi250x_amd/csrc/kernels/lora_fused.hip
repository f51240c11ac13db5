// The rank-r halves of the fused LoRA projections (ops/llama_fused.py), around the weight-streaming
// GEMMs of kernels/wstream.hip.
//
// Reference: PEFT lora.Linear — dropout(x) -> lora_A -> lora_B -> * scaling -> add, per target
// module q/k/v/o (02_development/distributed_utils.py:463-476; SURVEY §2.4 "LoRA"), 4-5 kernels and a
// stored dropout mask per projection.  Here, for the P projections that read the same input x
// (q, k, v: P = 3; o: P = 1), with c' = scaling / (1 - p) and keep_p the regenerated dropout mask
// (lora_keep in hyp_common.h; never stored):
//   lora_down   t'[m, p r + j] = Σ_k keep_p(m, k) x[m, k] A_p[j, k]          (fp32, MFMA, k-split partials)
//   lora_bwd_t  du'[m, p r + j] = c' Σ_n dy_p[m, n] B_p[n, j]   (n-split partials),  dB_p = c' dy_pᵀ t'_p
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

// Rank-r buffers (t', du') are fp32 [S][M][ld] split-partial stacks: the producer writes split q
// into slice q (no atomics, no zero-fill, no cross-workgroup synchronisation — workgroup fences
// cost microseconds per workgroup on the 8-XCD part), every consumer sums the S slices as it
// stages the rows it needs (ws_epilogue's LoRA terms, lora_bwd_t, lora_bwd_a).
struct RankR {
  float* p;
  int ld;            // row stride
  int64_t sstride;   // slice stride
  int S;             // slices
};

// Stage rows [row0, row0 + 128) x ranks [col0, col0 + 16) of a stack (its slices summed; zeros past
// `rows` and past r) into dst[128][16]: each of the 256 threads owns two float4 cells and issues all
// of its slice loads before summing (a per-element loop would wait a memory round trip per slice).
// Needs ld, col0 and sstride % 4 == 0 (host-checked).
__device__ __forceinline__ void stage_rank_rows(const RankR& u, int row0, int rows, int col0, int r, float (*dst)[16],
                                                int tid) {
  float4 acc[2] = {float4{0.f, 0.f, 0.f, 0.f}, float4{0.f, 0.f, 0.f, 0.f}};
  for (int q0 = 0; q0 < u.S; q0 += 4) {
    float4 v[2][4];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int cell = tid + 256 * c, row = cell >> 2, j4 = (cell & 3) * 4;
      const bool ok = row < rows;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int q = min(q0 + i, u.S - 1);
        v[c][i] = ok ? *reinterpret_cast<const float4*>(u.p + q * u.sstride + (int64_t)(row0 + row) * u.ld + col0 + j4)
                     : float4{0.f, 0.f, 0.f, 0.f};
      }
    }
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (q0 + i < u.S) {
          acc[c].x += v[c][i].x; acc[c].y += v[c][i].y; acc[c].z += v[c][i].z; acc[c].w += v[c][i].w;
        }
  }
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int cell = tid + 256 * c, row = cell >> 2, j4 = (cell & 3) * 4;
    float4 o = acc[c];
    if (j4 + 0 >= r) o.x = 0.f;
    if (j4 + 1 >= r) o.y = 0.f;
    if (j4 + 2 >= r) o.z = 0.f;
    if (j4 + 3 >= r) o.w = 0.f;
    *reinterpret_cast<float4*>(&dst[row][j4]) = o;
  }
}

// lora_down: block (p, 16-row m-tile, k-split q), 4 waves over the block's K range; A fragments =
// (masked) x rows, B fragments = rows of A_p, both straight from global memory (16 contiguous bytes
// per lane, every load of a wave in flight at once); the 4 wave tiles are summed through LDS and the
// block's 16 x 16 partial is written to slice q of t'.
template <typename T>
__global__ __launch_bounds__(256) void lora_down_k(const T* __restrict__ x, int64_t ldx, LoraPtrs A, RankR t, int M,
                                                   int K, int P, int r, RngState rs, uint32_t thr, int drop) {
  __shared__ f32x4 red[4][64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int p = blockIdx.x, m0 = blockIdx.y * 16, q = blockIdx.z;
  const uint64_t key = drop ? rng_key(rs) : 0ull;
  const int l15 = lane & 15, g4 = lane >> 4;
  const int m = m0 + l15;
  const bool mok = m < M, jok = l15 < r;
  const T* xr = x + (int64_t)(mok ? m : 0) * ldx;
  const T* ar = static_cast<const T*>(A.p[p]) + (int64_t)(jok ? l15 : 0) * K;
  // 32-wide k-steps of this split, round-robin over the 4 waves
  const int nks = K >> 5, per = (nks + t.S - 1) / t.S;
  const int ks0 = q * per, ks1 = min(nks, ks0 + per);
  const uint32_t ibase = (uint32_t)(((int64_t)p * M + m) * K);
  f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int k0 = ks0 + wave; k0 < ks1; k0 += 32) {  // up to 8 k-steps (16 loads) in flight
    u16x8 a[8], b[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int kk = min(k0 + 4 * u, ks1 - 1) * 32 + g4 * 8;
      a[u] = *reinterpret_cast<const u16x8*>(xr + kk);
      b[u] = *reinterpret_cast<const u16x8*>(ar + kk);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (k0 + 4 * u >= ks1) break;
      u16x8 av = a[u], bv = b[u];
      if (!mok) av = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if (!jok) bv = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if (drop) {
        const int kk = (k0 + 4 * u) * 32 + g4 * 8;
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (!lora_keep(key, ibase + (uint32_t)(kk + e), thr)) av[e] = 0;
      }
      acc = mfl::mma16<T>(av, bv, acc);
    }
  }
  red[wave][lane] = acc;
  __syncthreads();
  if (wave == 0) {
    const f32x4 sum = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
    // sum[e] = t'_q[m0 + 4 g4 + e][p r + l15]
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int mm = m0 + 4 * g4 + e;
      if (mm < M && jok) t.p[q * t.sstride + (int64_t)mm * t.ld + p * r + l15] = sum[e];
    }
  }
}

// lora_bwd_t: ONE launch, two workgroup roles (256 threads each).
//  du role, block (p, 16-row m-tile, n-split q): slice q of du'[m, p r + j] = c Σ_{n in split} dy_p[m, n] B_p[n, j]
//    on MFMA — A fragments = dy rows from global (16 B per lane), B fragments = 8 rows of B_p (2-byte
//    loads: 16 lanes cover one 32-byte row); 4 waves round-robin over the split's 32-wide steps.
//  dB role, block (p, 64-column slice): dB_p[n, j] = c Σ_m dy[m, n] t'[m, j] — the dy tile staged in LDS
//    (four 16-byte loads per thread, all in flight), t' (its slices summed) beside it; thread =
//    (column, 4 ranks), every LDS read a broadcast or a 16-byte vector.
constexpr int kBtN = 64, kBtM = 128;
template <typename T>
__global__ __launch_bounds__(256) void lora_bwd_t_k(const T* __restrict__ dy, int64_t ldy, int N, LoraPtrs B,
                                                    LoraPtrs dB, RankR t, RankR du, int M, int r, float c,
                                                    int n_du_blocks, int mtiles) {
  __shared__ __attribute__((aligned(16))) uint16_t ys[kBtM][kBtN + 8];
  __shared__ __attribute__((aligned(16))) float ts[kBtM][16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if ((int)blockIdx.x < n_du_blocks) {
    f32x4* red = reinterpret_cast<f32x4*>(&ts[0][0]);  // [4][64] f32x4 = 4 KB
    const int l15 = lane & 15, g4 = lane >> 4;
    const int per_p = mtiles * du.S;
    const int p = blockIdx.x / per_p, rem = blockIdx.x - p * per_p;
    const int mt = rem / du.S, q = rem - mt * du.S, m0 = mt * 16;
    const int m = m0 + l15;
    const bool mok = m < M, jok = l15 < r;
    const T* yr = dy + (int64_t)(mok ? m : 0) * ldy + (int64_t)p * N;
    const uint16_t* Bp = static_cast<const uint16_t*>(B.p[p]) + (jok ? l15 : 0);
    const int nks = N >> 5, per = (nks + du.S - 1) / du.S;
    const int ks0 = q * per, ks1 = min(nks, ks0 + per);
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int k0 = ks0 + wave; k0 < ks1; k0 += 16) {  // 4 k-steps: 4 row loads + 32 B-element loads in flight
      u16x8 av4[4], bv4[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int nn = min(k0 + 4 * u, ks1 - 1) * 32 + g4 * 8;
        av4[u] = *reinterpret_cast<const u16x8*>(yr + nn);
#pragma unroll
        for (int e = 0; e < 8; ++e) bv4[u][e] = Bp[(int64_t)(nn + e) * r];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (k0 + 4 * u >= ks1) break;
        u16x8 av = av4[u], bv = bv4[u];
        if (!mok) av = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
        if (!jok) bv = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
        acc = mfl::mma16<T>(av, bv, acc);
      }
    }
    red[wave * 64 + lane] = acc;
    __syncthreads();
    if (wave == 0) {
      const f32x4 sum = red[lane] + red[64 + lane] + red[128 + lane] + red[192 + lane];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int mm = m0 + 4 * g4 + e;
        if (mm < M && jok) du.p[q * du.sstride + (int64_t)mm * du.ld + p * r + l15] = c * sum[e];
      }
    }
    return;
  }
  // ---- dB role
  const int nsl = N / kBtN;
  const int idx = blockIdx.x - n_du_blocks, p = idx / nsl, n0 = (idx - p * nsl) * kBtN;
  const int dn = tid & 63, j0 = (tid >> 6) * 4;
  float db[4] = {0.f, 0.f, 0.f, 0.f};
  const T* dyp = dy + (int64_t)p * N + n0;
  for (int mc = 0; mc < M; mc += kBtM) {
    const int rows = min(kBtM, M - mc);
    __syncthreads();
    uint4 v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // [128 rows][64 cols]: 8 chunks per row
      const int id = tid + 256 * i, row = id >> 3, ch = id & 7;
      v[i] = row < rows ? *reinterpret_cast<const uint4*>(dyp + (int64_t)(mc + row) * ldy + ch * 8)
                        : uint4{0u, 0u, 0u, 0u};
    }
    stage_rank_rows(t, mc, rows, p * r, r, ts, tid);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int id = tid + 256 * i, row = id >> 3, ch = id & 7;
      *reinterpret_cast<uint4*>(&ys[row][ch * 8]) = v[i];
    }
    __syncthreads();
#pragma unroll 8
    for (int mm = 0; mm < rows; ++mm) {
      const float yv = ld1<T>(reinterpret_cast<const T*>(&ys[mm][dn]));
      const float4 tv = *reinterpret_cast<const float4*>(&ts[mm][j0]);
      db[0] += yv * tv.x; db[1] += yv * tv.y; db[2] += yv * tv.z; db[3] += yv * tv.w;
    }
  }
  T* dBp = static_cast<T*>(const_cast<void*>(dB.p[p]));
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (j0 + j < r) st1<T>(dBp + (int64_t)(n0 + dn) * r + j0 + j, c * db[j]);
}

// lora_bwd_a: block (p, 64-column slice of x): dA_p[:, slice] = Σ_m du'[m, p r + j] keep_p(m, k) x[m, k];
// up to 128 rows per pass, the x tile arriving with four 16-byte loads per thread issued together,
// du' (its slices summed) staged beside it.
template <typename T>
__global__ __launch_bounds__(256) void lora_bwd_a_k(const T* __restrict__ x, int64_t ldx, int K, LoraPtrs dA, RankR du,
                                                    int M, int r, RngState rs, uint32_t thr, int drop) {
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
      const int id = tid + 256 * i, row = id >> 3, ch = id & 7, m = mc + row;
      v[i] = m < M ? *reinterpret_cast<const uint4*>(x + (int64_t)m * ldx + k0 + ch * 8) : uint4{0u, 0u, 0u, 0u};
    }
    stage_rank_rows(du, mc, min(128, M - mc), p * r, r, us, tid);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int id = tid + 256 * i, row = id >> 3, ch = id & 7, m = mc + row;
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

static RankR rank_r(float* p, int ld, int64_t sstride, int S) {
  RankR u;
  u.p = p;
  u.ld = ld;
  u.sstride = sstride;
  u.S = S;
  return u;
}

hipError_t lora_down(int dtype, const void* x, int64_t ldx, const void* const* A, int P, int r, float* t, int ldt,
                     int64_t t_sstride, int t_splits, int M, int K, const RngState* rng, float p_drop, hipStream_t st) {
  if ((dtype != kBF16 && dtype != kF16) || P < 1 || P > 4 || r < 1 || r > 16 || M < 1 || K % 32 != 0 ||
      ldx % 8 != 0 || t_splits < 1 || t_splits > K / 32)
    return hipErrorInvalidValue;
  const int drop = (rng != nullptr && p_drop > 0.f) ? 1 : 0;
  const RngState rs = drop ? *rng : RngState{};
  const uint32_t thr = (uint32_t)fminf(p_drop * 4294967296.f, 4294967295.f);
  dim3 grid(P, (M + 15) / 16, t_splits);
  const RankR tt = rank_r(t, ldt, t_sstride, t_splits);
  if (dtype == kBF16)
    hipLaunchKernelGGL(lora_down_k<bf16_t>, grid, dim3(256), 0, st, static_cast<const bf16_t*>(x), ldx, pack(A, P), tt,
                       M, K, P, r, rs, thr, drop);
  else
    hipLaunchKernelGGL(lora_down_k<f16_t>, grid, dim3(256), 0, st, static_cast<const f16_t*>(x), ldx, pack(A, P), tt,
                       M, K, P, r, rs, thr, drop);
  return hipGetLastError();
}

hipError_t lora_bwd_t(int dtype, const void* dy, int64_t ldy, int N, const void* const* B, void* const* dB, int P,
                      int r, const float* t, int ldt, int64_t t_sstride, int t_splits, float* du, int ldu,
                      int64_t du_sstride, int du_splits, int M, float c, hipStream_t st) {
  if ((dtype != kBF16 && dtype != kF16) || P < 1 || P > 4 || r < 1 || r > 16 || N % kBtN != 0 || M < 1 ||
      ldy % 8 != 0 || t_splits < 1 || du_splits < 1 || du_splits > N / 32 || ldt % 4 != 0 || t_sstride % 4 != 0 ||
      (P > 1 && r % 4 != 0) || reinterpret_cast<uintptr_t>(t) % 16 != 0)
    return hipErrorInvalidValue;
  const int mtiles = (M + 15) / 16, n_du = P * mtiles * du_splits, n_db = P * (N / kBtN);
  LoraPtrs bp = pack(B, P), dbp = pack(const_cast<const void* const*>(reinterpret_cast<void* const*>(dB)), P);
  const RankR tt = rank_r(const_cast<float*>(t), ldt, t_sstride, t_splits), uu = rank_r(du, ldu, du_sstride, du_splits);
  if (dtype == kBF16)
    hipLaunchKernelGGL(lora_bwd_t_k<bf16_t>, dim3(n_du + n_db), dim3(256), 0, st, static_cast<const bf16_t*>(dy), ldy,
                       N, bp, dbp, tt, uu, M, r, c, n_du, mtiles);
  else
    hipLaunchKernelGGL(lora_bwd_t_k<f16_t>, dim3(n_du + n_db), dim3(256), 0, st, static_cast<const f16_t*>(dy), ldy,
                       N, bp, dbp, tt, uu, M, r, c, n_du, mtiles);
  return hipGetLastError();
}

hipError_t lora_bwd_a(int dtype, const void* x, int64_t ldx, int K, void* const* dA, int P, int r, const float* du,
                      int ldu, int64_t du_sstride, int du_splits, int M, const RngState* rng, float p_drop,
                      hipStream_t st) {
  if ((dtype != kBF16 && dtype != kF16) || P < 1 || P > 4 || r < 1 || r > 16 || K % 64 != 0 || M < 1 || ldx % 8 != 0 ||
      du_splits < 1 || ldu % 4 != 0 || du_sstride % 4 != 0 || (P > 1 && r % 4 != 0) ||
      reinterpret_cast<uintptr_t>(du) % 16 != 0)
    return hipErrorInvalidValue;
  const int drop = (rng != nullptr && p_drop > 0.f) ? 1 : 0;
  const RngState rs = drop ? *rng : RngState{};
  const uint32_t thr = (uint32_t)fminf(p_drop * 4294967296.f, 4294967295.f);
  dim3 grid(K / 64, P);
  LoraPtrs dap = pack(const_cast<const void* const*>(reinterpret_cast<void* const*>(dA)), P);
  const RankR uu = rank_r(const_cast<float*>(du), ldu, du_sstride, du_splits);
  if (dtype == kBF16)
    hipLaunchKernelGGL(lora_bwd_a_k<bf16_t>, grid, dim3(256), 0, st, static_cast<const bf16_t*>(x), ldx, K, dap, uu, M,
                       r, rs, thr, drop);
  else
    hipLaunchKernelGGL(lora_bwd_a_k<f16_t>, grid, dim3(256), 0, st, static_cast<const f16_t*>(x), ldx, K, dap, uu, M,
                       r, rs, thr, drop);
  return hipGetLastError();
}

}  // namespace hyp

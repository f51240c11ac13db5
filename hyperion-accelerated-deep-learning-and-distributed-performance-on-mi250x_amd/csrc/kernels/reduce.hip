// Column sums of a row-major [M, N] activation matrix: bias gradients (db = Σ_rows dY) and the
// final combine of per-block partial rows (LayerNorm dγ/dβ).
//
// Reference: autograd's AddmmBackward / LinearBackward computes db with ``grad.sum(0)`` — on
// MI355X the generic reduce kernel ran a [6304, 768] bf16 sum at 0.4 TB/s (ViT-B/16 batch 32:
// 51 launches, 1 ms per step; profiles/vit_r01).  Here:
//
// * colsum_partial_k: each thread owns 8 consecutive columns (one 16-byte vector per row) and
//   strides over a slab of rows with 4 independent accumulators in flight; the block's 4 row
//   groups combine through LDS into one fp32 partial row.  grid = (column slabs, P row slabs)
//   with P chosen so the launch has ~2 workgroups per CU.
// * colsum_final_k: out[c] = Σ_p part[p][c] with 16 row lanes x 8 independent 16-byte loads in
//   flight per column quad (see the kernel).
#include "hyp_common.h"
#include "hyp_kernels.h"

namespace hyp {
namespace {

constexpr int kThreads = 256;
constexpr int kColThreads = 64;  // threads across columns (x 8 columns each = 512 columns per block)
constexpr int kRowGroups = kThreads / kColThreads;

// Last-arriver combine (no second launch): every block of column slab blockIdx.y publishes its
// partial row (agent-scope release: the L2 write-back that makes it visible to the other XCDs),
// counts in on the slab's ticket, and the LAST block (acquire) sums the slab's P partial rows in a
// fixed order — 2 row lanes x 4 independent accumulators per column quad, then lane 0 + lane 1 —
// so the result does not depend on which block arrived last (deterministic), writes out[] and
// resets the ticket for the next launch / graph replay.  The partial count is capped
// (colsum_partials_fused) so that one block reads at most 64 x 512 floats.
__device__ __forceinline__ void colsum_last_block(const float* part, int N, int* ticket, void* out, int odt,
                                                  float* red /* >= 2 * 512 floats of LDS */) {
  __shared__ int s_last;
  __threadfence();
  __syncthreads();
  if (threadIdx.x == 0) s_last = atomicAdd(ticket, 1) == (int)gridDim.x - 1;
  __syncthreads();
  if (!s_last) return;
  __threadfence();
  const int P = gridDim.x;
  const int q = threadIdx.x & 127, lane = threadIdx.x >> 7;
  const int c = blockIdx.y * kColThreads * 8 + q * 4;
  float4 a[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) a[u] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c < N) {  // N % 8 == 0: a quad never straddles the edge
    int p = lane;
    for (; p + 6 < P; p += 8) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float4 v = *reinterpret_cast<const float4*>(part + (int64_t)(p + 2 * u) * N + c);
        a[u].x += v.x; a[u].y += v.y; a[u].z += v.z; a[u].w += v.w;
      }
    }
    for (; p < P; p += 2) {
      const float4 v = *reinterpret_cast<const float4*>(part + (int64_t)p * N + c);
      a[0].x += v.x; a[0].y += v.y; a[0].z += v.z; a[0].w += v.w;
    }
  }
  const float4 s = make_float4((a[0].x + a[1].x) + (a[2].x + a[3].x), (a[0].y + a[1].y) + (a[2].y + a[3].y),
                               (a[0].z + a[1].z) + (a[2].z + a[3].z), (a[0].w + a[1].w) + (a[2].w + a[3].w));
  __syncthreads();  // red is the caller's partial-row scratch
  reinterpret_cast<float4*>(red)[lane * 128 + q] = s;
  __syncthreads();
  if (lane == 0 && c < N) {
    const float4 o = reinterpret_cast<const float4*>(red)[q];
    const float4 t = reinterpret_cast<const float4*>(red)[128 + q];
    const float r[4] = {o.x + t.x, o.y + t.y, o.z + t.z, o.w + t.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (odt == kF32) static_cast<float*>(out)[c + e] = r[e];
      else if (odt == kBF16) st1<bf16_t>(static_cast<bf16_t*>(out) + c + e, r[e]);
      else st1<f16_t>(static_cast<f16_t*>(out) + c + e, r[e]);
    }
  }
  if (threadIdx.x == 0) *ticket = 0;
}

template <typename T>
__global__ __launch_bounds__(kThreads) void colsum_partial_k(const T* __restrict__ x, int64_t M, int N,
                                                             int64_t rows_per_block, float* __restrict__ part,
                                                             int* tickets, void* out, int odt) {
  __shared__ float red[kRowGroups][kColThreads * 8];
  const int ct = threadIdx.x % kColThreads, rg = threadIdx.x / kColThreads;
  const int c0 = (blockIdx.y * kColThreads + ct) * 8;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(M, r0 + rows_per_block);
  float acc[4][8];
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[u][j] = 0.f;
  if (c0 < N) {
    int64_t r = r0 + rg;
    for (; r + 3 * kRowGroups < r1; r += 4 * kRowGroups) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float v[8];
        Vec8<T>::load(x + (r + u * kRowGroups) * N + c0, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[u][j] += v[j];
      }
    }
    for (; r < r1; r += kRowGroups) {
      float v[8];
      Vec8<T>::load(x + r * N + c0, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[0][j] += v[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[rg][ct * 8 + j] = (acc[0][j] + acc[1][j]) + (acc[2][j] + acc[3][j]);
  __syncthreads();
  for (int i = threadIdx.x; i < kColThreads * 8; i += kThreads) {
    const int c = blockIdx.y * kColThreads * 8 + i;
    if (c < N) part[(int64_t)blockIdx.x * N + c] = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
  }
  if (tickets != nullptr) colsum_last_block(part, N, tickets + blockIdx.y, out, odt, &red[0][0]);
}

// out[c] = Σ_p part[p][c].  One block = 64 columns (16 float4 column quads) x 16 row lanes, every
// lane with 8 independent 16-byte loads in flight: the P partial rows are read in ~P/128 memory
// round trips instead of P/8 (a thread-per-column combine over P = 256 partials was 11.5 us — 1.3 ms
// per ViT-B/16 step over its ~100 bias / LayerNorm-parameter gradients), then a fixed-order LDS
// sum over the 16 lanes (deterministic).
// row lanes of the final combine: 64 (1024 threads: four times the loads in flight of the original
// 16, for combines whose N / 64 column blocks leave most CUs idle — a LayerNorm's dγ | dβ at
// d = 768 is 24 workgroups); colsum_set_fin_lanes(16) restores the 256-thread kernel (A/B)
int g_fin_lanes = 64;

// Activation backward + bias-gradient partials in one pass (the FFN's first linear): dy = dh·act'(z)
// is written once and its column sums are accumulated from registers — autograd ran the
// activation backward, then read dy again for the bias gradient (two kernels more per layer).
// ACT 1: ReLU with z = the saved output h (dy = h > 0 ? dh : 0); ACT 2: exact-erf GELU with z =
// the saved pre-activation.
template <typename T, int ACT>
__global__ __launch_bounds__(kThreads) void act_bwd_colsum_k(const T* __restrict__ dh, const T* __restrict__ z,
                                                             T* __restrict__ dy, int64_t M, int N,
                                                             int64_t rows_per_block, float* __restrict__ part,
                                                             uint32_t dthr, float dscale, RngState drs,
                                                             int* tickets, void* out, int odt) {
  // dscale != 0: dh is the gradient of dropout(act(z)); the keep mask (dropout.hip's hash) is
  // regenerated per element and dh scaled in T first, as a separate dropout backward would store it
  const uint64_t dkey = dscale != 0.f ? rng_key(drs) : 0;
  __shared__ float red[kRowGroups][kColThreads * 8];
  const int ct = threadIdx.x % kColThreads, rg = threadIdx.x / kColThreads;
  const int c0 = (blockIdx.y * kColThreads + ct) * 8;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(M, r0 + rows_per_block);
  float acc[2][8];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[u][j] = 0.f;
  auto one = [&](int64_t r, float (&a)[8], const float (&g0)[8], const float (&zz)[8]) {
    float o[8], g[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
      g[j] = dscale == 0.f ? g0[j]
                           : (rng_u32(dkey, (uint64_t)(r * N + c0 + j)) >= dthr ? rnd<T>(g0[j] * dscale) : 0.f);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float d;
      if (ACT == 1) {
        d = zz[j] > 0.f ? g[j] : 0.f;
      } else {
        // Φ(x) + x·φ(x) with ONE exp: erf(u), u = |x|/√2, by Abramowitz-Stegun 7.1.26
        // (|error| <= 1.5e-7, far below the bf16 / f16 rounding of dy) reuses φ's exp(-x²/2) =
        // exp(-u²); erff's own polynomial made this pass VALU-bound (40 us for ViT-B/16's
        // [6304, 3072] at 2.9 TB/s)
        const float x = zz[j];
        const float e = __expf(-0.5f * x * x);
        const float t = __builtin_amdgcn_rcpf(fmaf(0.23164189f, fabsf(x), 1.f));  // 1 / (1 + p·u), p/√2
        const float poly = t * fmaf(t, fmaf(t, fmaf(t, fmaf(t, 1.061405429f, -1.453152027f), 1.421413741f),
                                         -0.284496736f), 0.254829592f);
        const float erf_abs = fmaf(-poly, e, 1.f);
        const float cdf = 0.5f + 0.5f * copysignf(erf_abs, x);
        d = g[j] * fmaf(x * 0.39894228040143268f, e, cdf);
      }
      o[j] = rnd<T>(d);  // the column sums see what is stored (the vendor bias grad reads dy)
      a[j] += o[j];
    }
    Vec8<T>::store(dy + r * N + c0, o);
  };
  if (c0 < N) {
    int64_t r = r0 + rg;
    for (; r + kRowGroups < r1; r += 2 * kRowGroups) {  // two rows' loads in flight
      float g0[8], z0[8], g1[8], z1[8];
      Vec8<T>::load(dh + r * N + c0, g0);
      Vec8<T>::load(z + r * N + c0, z0);
      Vec8<T>::load(dh + (r + kRowGroups) * N + c0, g1);
      Vec8<T>::load(z + (r + kRowGroups) * N + c0, z1);
      one(r, acc[0], g0, z0);
      one(r + kRowGroups, acc[1], g1, z1);
    }
    if (r < r1) {
      float g0[8], z0[8];
      Vec8<T>::load(dh + r * N + c0, g0);
      Vec8<T>::load(z + r * N + c0, z0);
      one(r, acc[0], g0, z0);
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[rg][ct * 8 + j] = acc[0][j] + acc[1][j];
  __syncthreads();
  for (int i = threadIdx.x; i < kColThreads * 8; i += kThreads) {
    const int c = blockIdx.y * kColThreads * 8 + i;
    if (c < N) part[(int64_t)blockIdx.x * N + c] = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
  }
  if (tickets != nullptr) colsum_last_block(part, N, tickets + blockIdx.y, out, odt, &red[0][0]);
}

// columns [0, split) go to out, [split, N) to out2 (its own dtype): a norm's dγ | dβ and the
// producing linear's bias gradient (the linear's dtype) from one combine, no cast kernel after it
template <typename O, typename O2 = O, int kFinLanes = 64>
__global__ __launch_bounds__(16 * kFinLanes) void colsum_final_k(const float* __restrict__ part, int P, int N,
                                                                 O* __restrict__ out, int split = 1 << 30,
                                                                 O2* __restrict__ out2 = nullptr) {
  __shared__ float red[kFinLanes][64];
  const int tx = threadIdx.x % 16, ty = threadIdx.x / 16;
  const int c = blockIdx.x * 64 + tx * 4;
  float4 s[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) s[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c < N) {  // N % 4 == 0: a quad never straddles the edge
    int p = ty;
    for (; p + 7 * kFinLanes < P; p += 8 * kFinLanes) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float4 v = *reinterpret_cast<const float4*>(part + (int64_t)(p + i * kFinLanes) * N + c);
        s[i].x += v.x; s[i].y += v.y; s[i].z += v.z; s[i].w += v.w;
      }
    }
    for (; p < P; p += kFinLanes) {
      const float4 v = *reinterpret_cast<const float4*>(part + (int64_t)p * N + c);
      s[0].x += v.x; s[0].y += v.y; s[0].z += v.z; s[0].w += v.w;
    }
  }
#pragma unroll
  for (int i = 1; i < 8; ++i) {
    s[0].x += s[i].x; s[0].y += s[i].y; s[0].z += s[i].z; s[0].w += s[i].w;
  }
  red[ty][tx * 4 + 0] = s[0].x;
  red[ty][tx * 4 + 1] = s[0].y;
  red[ty][tx * 4 + 2] = s[0].z;
  red[ty][tx * 4 + 3] = s[0].w;
  __syncthreads();
  if (threadIdx.x < 64) {
    const int cc = blockIdx.x * 64 + threadIdx.x;
    if (cc < N) {
      float a = 0.f;
#pragma unroll
      for (int l = 0; l < kFinLanes; ++l) a += red[l][threadIdx.x];
      if (cc < split) st1<O>(out + cc, a);
      else st1<O2>(out2 + (cc - split), a);
    }
  }
}

}  // namespace

int colsum_partials(int64_t M, int N) {
  const int slabs = (N + kColThreads * 8 - 1) / (kColThreads * 8);
  int64_t P = (512 + slabs - 1) / slabs;               // ~2 workgroups per CU in total
  const int64_t max_p = (M + 4 * kRowGroups - 1) / (4 * kRowGroups);  // >= 16 rows per slab
  if (P > max_p) P = max_p;
  if (P < 1) P = 1;
  return (int)P;
}

// the activation backward (act_bwd_colsum_k) computes per element and stores a second stream:
// more resident waves than the plain column sum's ~2 workgroups per CU (colsum_set_act_wgs: A/B)
int g_act_colsum_wgs = 1024;

int act_colsum_partials(int64_t M, int N) {
  const int slabs = (N + kColThreads * 8 - 1) / (kColThreads * 8);
  int64_t P = (g_act_colsum_wgs + slabs - 1) / slabs;
  const int64_t max_p = (M + 4 * kRowGroups - 1) / (4 * kRowGroups);  // >= 16 rows per slab
  if (P > max_p) P = max_p;
  if (P < 1) P = 1;
  return (int)P;
}

void colsum_set_act_wgs(int wgs) { g_act_colsum_wgs = wgs < 64 ? 64 : (wgs > 8192 ? 8192 : wgs); }

int g_colsum_fused_max_p = 0;  // colsum_set_fused (0: the two-launch path — measured faster, see README)

int colsum_partials_fused(int64_t M, int N) {
  const int P = colsum_partials(M, N);
  return g_colsum_fused_max_p > 0 && P > g_colsum_fused_max_p ? g_colsum_fused_max_p : P;
}

void colsum_set_fused(int max_p) { g_colsum_fused_max_p = max_p < 0 ? 0 : (max_p > 256 ? 256 : max_p); }

int colsum_fused_max_p() { return g_colsum_fused_max_p; }

void colsum_set_fin_lanes(int lanes) { g_fin_lanes = lanes == 16 ? 16 : 64; }

template <typename O, typename O2>
static void launch_final(const float* part, int P, int N, O* out, int split, O2* out2, hipStream_t st) {
  const dim3 grid((N + 63) / 64);
  if (g_fin_lanes == 16)
    hipLaunchKernelGGL((colsum_final_k<O, O2, 16>), grid, dim3(256), 0, st, part, P, N, out, split, out2);
  else
    hipLaunchKernelGGL((colsum_final_k<O, O2, 64>), grid, dim3(1024), 0, st, part, P, N, out, split, out2);
}

hipError_t colsum_combine(const float* part, int P, int N, void* out, int out_dtype, hipStream_t st) {
  if (N % 4 != 0 || P < 1) return hipErrorInvalidValue;
  if (out_dtype == kF32)
    launch_final<float, float>(part, P, N, static_cast<float*>(out), 1 << 30, nullptr, st);
  else if (out_dtype == kBF16)
    launch_final<bf16_t, bf16_t>(part, P, N, static_cast<bf16_t*>(out), 1 << 30, nullptr, st);
  else if (out_dtype == kF16)
    launch_final<f16_t, f16_t>(part, P, N, static_cast<f16_t*>(out), 1 << 30, nullptr, st);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

template <typename O>
static hipError_t combine_split_to(const float* part, int P, int N, O* out, int split, void* out2, int dt2,
                                   hipStream_t st) {
  if (dt2 == kF32)
    launch_final<O, float>(part, P, N, out, split, static_cast<float*>(out2), st);
  else if (dt2 == kBF16)
    launch_final<O, bf16_t>(part, P, N, out, split, static_cast<bf16_t*>(out2), st);
  else if (dt2 == kF16)
    launch_final<O, f16_t>(part, P, N, out, split, static_cast<f16_t*>(out2), st);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t colsum_combine_split(const float* part, int P, int N, void* out, int out_dtype, int split, void* out2,
                                int out2_dtype, hipStream_t st) {
  if (N % 4 != 0 || P < 1 || split % 4 != 0 || split < 0 || split > N) return hipErrorInvalidValue;
  if (out_dtype == kF32) return combine_split_to(part, P, N, static_cast<float*>(out), split, out2, out2_dtype, st);
  if (out_dtype == kBF16) return combine_split_to(part, P, N, static_cast<bf16_t*>(out), split, out2, out2_dtype, st);
  if (out_dtype == kF16) return combine_split_to(part, P, N, static_cast<f16_t*>(out), split, out2, out2_dtype, st);
  return hipErrorInvalidValue;
}

hipError_t column_sum(int dtype, const void* x, int64_t M, int N, void* out, int out_dtype, float* part, int P,
                      hipStream_t st, int* tickets) {
  if (N % 8 != 0 || M < 1 || P < 1) return hipErrorInvalidValue;
  if (tickets != nullptr && out_dtype != kF32 && out_dtype != kBF16 && out_dtype != kF16) return hipErrorInvalidValue;
  const int64_t rpb = (M + P - 1) / P;
  const int Pe = (int)((M + rpb - 1) / rpb);  // blocks that own rows (= the partial rows written)
  const dim3 grid(Pe, (N + kColThreads * 8 - 1) / (kColThreads * 8));
  if (dtype == kBF16)
    hipLaunchKernelGGL(colsum_partial_k<bf16_t>, grid, dim3(kThreads), 0, st, static_cast<const bf16_t*>(x), M, N,
                       rpb, part, tickets, out, out_dtype);
  else if (dtype == kF16)
    hipLaunchKernelGGL(colsum_partial_k<f16_t>, grid, dim3(kThreads), 0, st, static_cast<const f16_t*>(x), M, N, rpb,
                       part, tickets, out, out_dtype);
  else if (dtype == kF32)
    hipLaunchKernelGGL(colsum_partial_k<float>, grid, dim3(kThreads), 0, st, static_cast<const float*>(x), M, N, rpb,
                       part, tickets, out, out_dtype);
  else
    return hipErrorInvalidValue;
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess || tickets != nullptr) return e;
  return colsum_combine(part, Pe, N, out, out_dtype, st);
}

// dy = dh·act'(z) and db = Σ_rows dy (out_dtype) in two launches (act: 1 ReLU on the output, 2 GELU
// on the pre-activation).  part: [P, N] fp32 workspace, P = colsum_partials(M, N).
hipError_t act_bwd_colsum(int dtype, int act, const void* dh, const void* z, void* dy, int64_t M, int N, void* db,
                          int out_dtype, float* part, int P, hipStream_t st, float drop_p,
                          const RngState* rs, int* tickets) {
  if (N % 8 != 0 || M < 1 || P < 1 || (act != 1 && act != 2) || (dtype != kBF16 && dtype != kF16))
    return hipErrorInvalidValue;
  if (db == nullptr) tickets = nullptr;
  if (tickets != nullptr && out_dtype != kF32 && out_dtype != kBF16 && out_dtype != kF16) return hipErrorInvalidValue;
  const int64_t rpb = (M + P - 1) / P;
  const int Pe = (int)((M + rpb - 1) / rpb);
  const dim3 grid(Pe, (N + kColThreads * 8 - 1) / (kColThreads * 8));
  if (drop_p > 0.f && (rs == nullptr || drop_p >= 1.f)) return hipErrorInvalidValue;
  const uint32_t dthr = drop_p > 0.f ? (uint32_t)fminf(drop_p * 4294967296.f, 4294967295.f) : 0u;
  const float dscale = drop_p > 0.f ? 1.f / (1.f - drop_p) : 0.f;
  const RngState drs = rs != nullptr ? *rs : RngState{};
#define HYP_ACT_COLSUM(TT, A)                                                                                   \
  hipLaunchKernelGGL((act_bwd_colsum_k<TT, A>), grid, dim3(kThreads), 0, st, static_cast<const TT*>(dh),        \
                     static_cast<const TT*>(z), static_cast<TT*>(dy), M, N, rpb, part, dthr, dscale, drs, tickets, \
                     db, out_dtype)
  if (dtype == kBF16) {
    if (act == 1) HYP_ACT_COLSUM(bf16_t, 1);
    else HYP_ACT_COLSUM(bf16_t, 2);
  } else {
    if (act == 1) HYP_ACT_COLSUM(f16_t, 1);
    else HYP_ACT_COLSUM(f16_t, 2);
  }
#undef HYP_ACT_COLSUM
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess || db == nullptr || tickets != nullptr) return e;
  return colsum_combine(part, Pe, N, db, out_dtype, st);
}

// ---- mean-squared error, forward + gradient in one pass ------------------------------------
// loss = mean((x - t)^2) and g = 2 (x - t) / n (x's dtype), one 1024-thread block (the ResNet
// benchmark's [32, 1000] bf16 logits against fp32 targets: torch ran a cast, a sub, a pow, a mean
// and three backward elementwise kernels).  Fixed-order reduction: deterministic.
namespace {
constexpr int kMseThreads = 1024;

template <typename T>
__global__ __launch_bounds__(kMseThreads) void mse_fwd_bwd_k(const T* __restrict__ x, const float* __restrict__ t,
                                                             int64_t n, float* __restrict__ loss, T* __restrict__ g) {
  __shared__ float red[kMseThreads / 64];
  const float inv = 1.f / (float)n;
  float acc = 0.f;
  // 32 elements per thread per round, every load of the round issued before any use: one memory
  // round trip for up to 32K elements (4 per round still cost 8 round trips, 21 us for 32 x 1000)
  constexpr int U = 32;
  for (int64_t base = 0; base < n; base += U * kMseThreads) {
    float xv[U], tv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = base + u * kMseThreads + threadIdx.x;
      xv[u] = i < n ? ld1<T>(x + i) : 0.f;
      tv[u] = i < n ? t[i] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = base + u * kMseThreads + threadIdx.x;
      const float d = xv[u] - tv[u];
      acc = fmaf(d, d, acc);
      if (i < n) st1<T>(g + i, 2.f * d * inv);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < kMseThreads / 64; ++w) s += red[w];
    *loss = s * inv;
  }
}
}  // namespace

hipError_t mse_fwd_bwd(int dtype, const void* x, const float* t, int64_t n, float* loss, void* g, hipStream_t st) {
  if (n < 1) return hipErrorInvalidValue;
  HYP_DISPATCH_FLOAT(dtype, T, {
    hipLaunchKernelGGL(mse_fwd_bwd_k<T>, dim3(1), dim3(kMseThreads), 0, st, static_cast<const T*>(x), t, n, loss,
                       static_cast<T*>(g));
  });
  return hipGetLastError();
}

}  // namespace hyp

// NHWC convolution WEIGHT gradient on gfx950 MFMA (split-K implicit GEMM).
//
// Reference: ResNet-50/18 weight gradients ran through MIOpen's `igemm_wrw` / CK batched-GEMM
// solvers plus their zero-fill and cast kernels (3-4 launches per conv; SURVEY §2.4
// "Convolution + BatchNorm + ReLU" backward, §2.5 ResNet rows).  Here
//
//   dW[k, r, s, c] = Σ_{m = (n,p,q)} dY[m, k] · X[n, p*sh + r - ph, q*sw + s - pw, c]
//
// is a GEMM with rows = output channels k, columns = (r, s, c) in the channels-last filter's own
// order, and a reduction over the N·P·Q output pixels.  BOTH operands have the reduction (pixel)
// dimension strided in memory — dY rows and input pixels are channel-contiguous — so tiles are
// staged pixel-major straight from HBM with 16-byte global_load_lds (a pixel's BM/BN-channel run
// is one contiguous row), and the MFMA operands are read back TRANSPOSED with gfx950's
// ds_read_b64_tr_b16 (guide T10): no register transpose, no ds_permute.
//
// LDS image per operand: [64 pixels][W channels] with W*2-byte rows and an XOR swizzle of the
// 16-byte chunks chosen so every 32-lane half of a transposed read touches 64 distinct banks
// (rows 0..7 of a read half land on disjoint chunk pairs).  The pixel <-> MFMA k-slot mapping is
// free (both operands sum over the same pixels), so each 16-lane group reads 4 consecutive rows.
//
// Work split: tiles BM x BN (k x c) of one filter tap, 4 waves as 2 x 2, 16x16x32 bf16/f16 MFMA;
// the pixel reduction is split over `splits` workgroups (the outputs of a ResNet wgrad are small —
// 64 x 576 for a layer1 3x3 — while the reduction is up to 10^5 pixels long).  splits == 1 stores
// the result in the parameter dtype; otherwise fp32 partials [splits][K][R·S·C] are summed (in a
// fixed order: deterministic) and cast by conv_wgrad_reduce_k.
#include "conv_wgrad_impl.h"

namespace hyp {
namespace {

using namespace mfl;

// out = alpha * Σ_s part[s] (fixed order: deterministic), cast to T; 4 elements per thread
// (16-byte loads).  Optional rank-r epilogue (the LoRA update fused into the base GEMM's reduce):
//   out[m, n] += beta * (mask ? mask[m, n] : 1) * Σ_j U[m, j] · V[j * sv_j + n * sv_n]
// with U [M, r] and V any 2D view (B of y += t·Bᵀ is V = Bᵀ: sv_j = 1, sv_n = r).
// 64-thread blocks (a wgrad output can be only 37K floats: 256-thread blocks left ~36 workgroups
// on 256 CUs) and 4 independent accumulators, so 4 slab loads are in flight per thread.
constexpr int kRedThreads = 64;

template <typename T, bool LOWRANK, bool AFF>
__global__ __launch_bounds__(kRedThreads) void splitk_reduce_k(const float* __restrict__ part, T* __restrict__ out,
                                                               int64_t n, int splits, float alpha, SplitkEpilogue ep) {
  const int64_t i4 = ((int64_t)blockIdx.x * kRedThreads + threadIdx.x) * 4;
  if (i4 >= n) return;
  const f32x4* src = reinterpret_cast<const f32x4*>(part + i4);
  const int64_t sn = n / 4;  // slab stride in f32x4
  f32x4 a0 = __builtin_nontemporal_load(src), a1 = {0.f, 0.f, 0.f, 0.f}, a2 = a1, a3 = a1;
  int s = 1;
  for (; s + 3 < splits; s += 4) {
    a0 += __builtin_nontemporal_load(src + (int64_t)s * sn);
    a1 += __builtin_nontemporal_load(src + (int64_t)(s + 1) * sn);
    a2 += __builtin_nontemporal_load(src + (int64_t)(s + 2) * sn);
    a3 += __builtin_nontemporal_load(src + (int64_t)(s + 3) * sn);
  }
  for (; s < splits; ++s) a0 += __builtin_nontemporal_load(src + (int64_t)s * sn);
  f32x4 acc = (a0 + a1) + (a2 + a3);
  acc *= alpha;
  if (LOWRANK) {
    // r % 8 == 0, r <= 64: U's row and V's rows / columns are read as 16- / 8-byte vectors
    const int64_t m = i4 / ep.N, n0 = i4 - m * ep.N;  // N % 4 == 0: the 4 elements share a row
    const T* u = reinterpret_cast<const T*>(ep.U) + m * ep.r;
    const T* v = reinterpret_cast<const T*>(ep.V);
    f32x4 lr = {0.f, 0.f, 0.f, 0.f};
    for (int j0 = 0; j0 < ep.r; j0 += 8) {
      float uj[8];
      Vec8<T>::load(u + j0, uj);
      if (ep.sv_n != 1) {  // V = [N, r] (row n holds the r coefficients of output column n)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float vv[8];
          Vec8<T>::load(v + (n0 + e) * ep.sv_n + j0, vv);
#pragma unroll
          for (int q = 0; q < 8; ++q) lr[e] += uj[q] * vv[q];
        }
      } else {  // V = [r, N]: 4 consecutive outputs = one 8-byte run per coefficient row
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const uint2 raw = *reinterpret_cast<const uint2*>(v + (int64_t)(j0 + q) * ep.sv_j + n0);
          const T* h = reinterpret_cast<const T*>(&raw);
#pragma unroll
          for (int e = 0; e < 4; ++e) lr[e] += uj[q] * ld1<T>(h + e);
        }
      }
    }
    if (ep.mask != nullptr) {
      const uint2 raw = *reinterpret_cast<const uint2*>(reinterpret_cast<const T*>(ep.mask) + i4);
      const T* mk = reinterpret_cast<const T*>(&raw);
#pragma unroll
      for (int e = 0; e < 4; ++e) lr[e] *= ld1<T>(mk + e);
    }
    acc += ep.beta * lr;
  }
  if (AFF) {  // eval BN folded in: act(round(acc) * scale + shift (+ residual)), N % 4 == 0
    const int64_t n0 = i4 % ep.N;
    const T* res = static_cast<const T*>(ep.residual);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float v = fmaf(rnd<T>(acc[e]), ep.scale[n0 + e], ep.shift[n0 + e]);
      if (res != nullptr) v += ld1<T>(res + i4 + e);
      acc[e] = ep.act ? fmaxf(v, 0.f) : v;
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) st1<T>(out + i4 + e, acc[e]);
}

// Small outputs with many splits (weight gradients: 37K-262K elements, 8-256 splits): 4 split
// lanes per output quad (split s goes to lane s % 4, summed in increasing s), combined in lane
// order through LDS — still a fixed order, 4x the loads in flight of splitk_reduce_k.
template <typename T>
__global__ __launch_bounds__(256) void splitk_reduce4_k(const float* __restrict__ part, T* __restrict__ out,
                                                        int64_t n, int splits, float alpha) {
  __shared__ f32x4 red[3][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int64_t i4 = ((int64_t)blockIdx.x * 64 + tx) * 4;
  const bool ok = i4 < n;
  f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0;
  if (ok) {
    const f32x4* src = reinterpret_cast<const f32x4*>(part + i4);
    const int64_t sn = n / 4;
    int s = ty;
    for (; s + 4 < splits; s += 8) {
      a0 += __builtin_nontemporal_load(src + (int64_t)s * sn);
      a1 += __builtin_nontemporal_load(src + (int64_t)(s + 4) * sn);
    }
    if (s < splits) a0 += __builtin_nontemporal_load(src + (int64_t)s * sn);
  }
  f32x4 acc = a0 + a1;
  if (ty > 0) red[ty - 1][tx] = acc;
  __syncthreads();
  if (ty == 0 && ok) {
    acc = ((acc + red[0][tx]) + red[1][tx]) + red[2][tx];
    acc *= alpha;
#pragma unroll
    for (int e = 0; e < 4; ++e) st1<T>(out + i4 + e, acc[e]);
  }
}

template <typename T>
hipError_t reduce_launch(const float* part, T* out, int64_t n, int splits, float alpha, const SplitkEpilogue* ep,
                         hipStream_t st) {
  const int blocks = (int)((n / 4 + kRedThreads - 1) / kRedThreads);
  if (ep != nullptr && ep->U != nullptr)
    hipLaunchKernelGGL((splitk_reduce_k<T, true, false>), dim3(blocks), dim3(kRedThreads), 0, st, part, out, n, splits,
                       alpha, *ep);
  else if (ep != nullptr && ep->scale != nullptr)
    hipLaunchKernelGGL((splitk_reduce_k<T, false, true>), dim3(blocks), dim3(kRedThreads), 0, st, part, out, n, splits,
                       alpha, *ep);
  else if (splits >= 8 && n / 4 <= (1 << 16))
    hipLaunchKernelGGL((splitk_reduce4_k<T>), dim3((int)((n / 4 + 63) / 64)), dim3(256), 0, st, part, out, n, splits,
                       alpha);
  else
    hipLaunchKernelGGL((splitk_reduce_k<T, false, false>), dim3(blocks), dim3(kRedThreads), 0, st, part, out, n,
                       splits, alpha, SplitkEpilogue{});
  return hipGetLastError();
}

}  // namespace

namespace {
// Split-K reduce of a convolution's [splits, M, K] fp32 partials with the BN-statistics epilogue
// of conv_fwd_k: out = Σ_s part[s] rounded to T, and per-channel Σy, Σy² of the ROUNDED outputs
// over kStatRows-row blocks, added atomically into psum[K] / psq[K] (the sums the BN apply
// finalizes inline).  Used when a forward conv has too few output tiles to fill 256 CUs
// (ResNet-50 layer3/4: 200-392 tiles, 55 us at 0.8 workgroups per CU).  Block = 64 column quads
// (256 channels, 16-byte loads) x 4 row lanes.
template <typename T>
__global__ __launch_bounds__(256) void splitk_reduce_stats_k(const float* __restrict__ part, T* __restrict__ out,
                                                             int M, int K, int splits, int rows,
                                                             double* __restrict__ psum, double* __restrict__ psq) {
  __shared__ float red[2][4][256];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = blockIdx.y * 256 + tx * 4;
  const int r0 = blockIdx.x * rows;
  const int r1 = min(M, r0 + rows);
  const int64_t slab = (int64_t)M * K;
  f32x4 cs = {0.f, 0.f, 0.f, 0.f}, cq = cs;
  if (c < K) {
    for (int r = r0 + ty; r < r1; r += 4) {
      const float* src = part + (int64_t)r * K + c;
      f32x4 a0 = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(src)), a1 = {0.f, 0.f, 0.f, 0.f};
      int s = 1;
      for (; s + 1 < splits; s += 2) {
        a0 += __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(src + (int64_t)s * slab));
        a1 += __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(src + (int64_t)(s + 1) * slab));
      }
      if (s < splits) a0 += __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(src + (int64_t)s * slab));
      const f32x4 acc = a0 + a1;
      T* o = out + (int64_t)r * K + c;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float v = rnd<T>(acc[e]);
        st1<T>(o + e, v);
        cs[e] += v;
        cq[e] += v * v;
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    red[0][ty][tx * 4 + e] = cs[e];
    red[1][ty][tx * 4 + e] = cq[e];
  }
  __syncthreads();
  // one atomic per channel per block: 64 consecutive channels per wave instruction (256-byte runs)
  if (threadIdx.x < 256) {
    const int j = threadIdx.x, ch = blockIdx.y * 256 + j;
    if (ch < K) {
      const int64_t slot = (int64_t)(blockIdx.x % kStatSlots) * 2 * K;
      unsafeAtomicAdd(psum + slot + ch, (double)((red[0][0][j] + red[0][1][j]) + (red[0][2][j] + red[0][3][j])));
      unsafeAtomicAdd(psq + slot + ch, (double)((red[1][0][j] + red[1][1][j]) + (red[1][2][j] + red[1][3][j])));
    }
  }
}
}  // namespace

hipError_t splitk_reduce_stats(int dtype, const float* part, void* out, int M, int K, int splits, double* psum,
                               double* psq, hipStream_t st) {
  if (K % 4 != 0 || splits < 1 || M < 1) return hipErrorInvalidValue;
  // kStatRows-row blocks (fewer atomic adders per channel) unless that leaves < 512 blocks
  const int cb = (K + 255) / 256;
  const int rows = (int64_t)((M + kStatRows - 1) / kStatRows) * cb >= 512 ? kStatRows : 16;
  const dim3 grid((M + rows - 1) / rows, cb);
  if (dtype == kBF16)
    hipLaunchKernelGGL(splitk_reduce_stats_k<bf16_t>, grid, dim3(256), 0, st, part, static_cast<bf16_t*>(out), M, K,
                       splits, rows, psum, psq);
  else if (dtype == kF16)
    hipLaunchKernelGGL(splitk_reduce_stats_k<f16_t>, grid, dim3(256), 0, st, part, static_cast<f16_t*>(out), M, K,
                       splits, rows, psum, psq);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

namespace {
// Split-K reduce of a stride-1 data gradient with the BN-backward epilogue (conv_igemm.hip's BNB
// epilogue for the split case): out = dz = round(round(Σ_s part[s]) + addend) · mask and Σdz,
// Σdz·x per channel into slot blockIdx.x % kStatSlots of bnb.sums.  Same block shape as
// splitk_reduce_stats_k (64 column quads x 4 row lanes, `rows` rows per block).
template <typename T>
__global__ __launch_bounds__(256) void splitk_reduce_bnb_k(const float* __restrict__ part, T* __restrict__ out,
                                                           const T* __restrict__ addend, int M, int K, int splits,
                                                           int rows, BnBwdEpilogue bnb) {
  __shared__ float red[2][4][256];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = blockIdx.y * 256 + tx * 4;
  const int r0 = blockIdx.x * rows;
  const int r1 = min(M, r0 + rows);
  const int64_t slab = (int64_t)M * K;
  const T* xb = static_cast<const T*>(bnb.x);
  const T* yb = static_cast<const T*>(bnb.y);
  float msc[4] = {0.f, 0.f, 0.f, 0.f}, msh[4] = {0.f, 0.f, 0.f, 0.f};
  if (bnb.mode == 1 && c < K) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float sc = (bnb.w ? bnb.w[c + e] : 1.f) * bnb.invstd[c + e];
      msc[e] = sc;
      msh[e] = (bnb.b ? bnb.b[c + e] : 0.f) - bnb.mean[c + e] * sc;
    }
  }
  f32x4 cs = {0.f, 0.f, 0.f, 0.f}, cq = cs;
  if (c < K) {
    for (int r = r0 + ty; r < r1; r += 4) {
      const int64_t off = (int64_t)r * K + c;
      const float* src = part + off;
      f32x4 a0 = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(src)), a1 = {0.f, 0.f, 0.f, 0.f};
      int s = 1;
      for (; s + 1 < splits; s += 2) {
        a0 += __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(src + (int64_t)s * slab));
        a1 += __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(src + (int64_t)(s + 1) * slab));
      }
      if (s < splits) a0 += __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(src + (int64_t)s * slab));
      const f32x4 acc = a0 + a1;
      // 4 channels = one 8-byte run of each 2-byte operand
      const uint2 rx = *reinterpret_cast<const uint2*>(xb + off);
      const uint2 ry = bnb.mode == 2 ? *reinterpret_cast<const uint2*>(yb + off) : uint2{0u, 0u};
      const uint2 rd = addend != nullptr ? *reinterpret_cast<const uint2*>(addend + off) : uint2{0u, 0u};
      const T* hx = reinterpret_cast<const T*>(&rx);
      const T* hy = reinterpret_cast<const T*>(&ry);
      const T* hd = reinterpret_cast<const T*>(&rd);
      T ov[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v = rnd<T>(acc[e]);
        if (addend != nullptr) v = rnd<T>(v + ld1<T>(hd + e));
        const float xv = ld1<T>(hx + e);
        const bool keep = bnb.mode == 0 || (bnb.mode == 1 ? fmaf(xv, msc[e], msh[e]) > 0.f : ld1<T>(hy + e) > 0.f);
        v = keep ? v : 0.f;
        st1<T>(ov + e, v);
        cs[e] += v;
        cq[e] += v * xv;
      }
      *reinterpret_cast<uint2*>(out + off) = *reinterpret_cast<const uint2*>(ov);
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    red[0][ty][tx * 4 + e] = cs[e];
    red[1][ty][tx * 4 + e] = cq[e];
  }
  __syncthreads();
  const int j = threadIdx.x, ch = blockIdx.y * 256 + j;
  if (ch < K) {
    double* slot = bnb.sums + (int64_t)(blockIdx.x % kStatSlots) * 2 * K;
    unsafeAtomicAdd(slot + ch, (double)((red[0][0][j] + red[0][1][j]) + (red[0][2][j] + red[0][3][j])));
    unsafeAtomicAdd(slot + K + ch, (double)((red[1][0][j] + red[1][1][j]) + (red[1][2][j] + red[1][3][j])));
  }
}
}  // namespace

hipError_t splitk_reduce_bnb(int dtype, const float* part, void* out, const void* addend, int M, int K, int splits,
                             const BnBwdEpilogue& bnb, hipStream_t st) {
  if (K % 4 != 0 || splits < 1 || M < 1) return hipErrorInvalidValue;
  const int cb = (K + 255) / 256;
  const int rows = (int64_t)((M + kStatRows - 1) / kStatRows) * cb >= 512 ? kStatRows : 16;
  const dim3 grid((M + rows - 1) / rows, cb);
  if (dtype == kBF16)
    hipLaunchKernelGGL(splitk_reduce_bnb_k<bf16_t>, grid, dim3(256), 0, st, part, static_cast<bf16_t*>(out),
                       static_cast<const bf16_t*>(addend), M, K, splits, rows, bnb);
  else if (dtype == kF16)
    hipLaunchKernelGGL(splitk_reduce_bnb_k<f16_t>, grid, dim3(256), 0, st, part, static_cast<f16_t*>(out),
                       static_cast<const f16_t*>(addend), M, K, splits, rows, bnb);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t splitk_reduce(int dtype, const float* part, void* out, int64_t n, int splits, hipStream_t st, float alpha,
                         const SplitkEpilogue* ep) {
  if (n % 4 != 0 || splits < 1) return hipErrorInvalidValue;
  if (ep != nullptr && ep->U != nullptr && (ep->N % 4 != 0 || ep->r < 8 || ep->r % 8 != 0 || n % ep->N != 0))
    return hipErrorInvalidValue;
  if (ep != nullptr && ep->scale != nullptr && (ep->N % 4 != 0 || n % ep->N != 0 || ep->shift == nullptr))
    return hipErrorInvalidValue;
  if (dtype == kBF16) return reduce_launch<bf16_t>(part, static_cast<bf16_t*>(out), n, splits, alpha, ep, st);
  if (dtype == kF16) return reduce_launch<f16_t>(part, static_cast<f16_t*>(out), n, splits, alpha, ep, st);
  return hipErrorInvalidValue;
}

namespace {

uint64_t magic36(int d) { return ((1ull << 36) + (uint64_t)d - 1) / (uint64_t)d; }

// tuning overrides (conv_wgrad_set_stages, for sweeps); 0 = the plan's choice
int g_wgrad_stages = 0;  // LDS ring depth
int g_wgrad_lean = 1;    // dense shapes on conv_wgrad_dense_k (0: the general kernel)
int g_wgrad_kp = 0;      // pixels per LDS stage of the dense kernel

template <typename T, int BM, int BN, bool DENSE>
hipError_t launch_d(const WgradArgs& a, hipStream_t st, int nb, int kp) {
  const int tiles = ((a.K + BM - 1) / BM) * (a.R * a.S * a.C / BN);
  const dim3 grid(tiles * a.splits + a.pr.blocks);
  if (DENSE && g_wgrad_lean) {
    if (kp == 128) {  // 3 stages of 128 pixels fit 160 KiB of LDS up to 128 x 64 tiles
      if constexpr (BM + BN <= 192) {
        if (nb >= 3) {
          hipLaunchKernelGGL((conv_wgrad_dense_k<T, BM, BN, 3, 128>), grid, dim3(kThreads), 0, st, a);
          return hipGetLastError();
        }
      }
      hipLaunchKernelGGL((conv_wgrad_dense_k<T, BM, BN, 2, 128>), grid, dim3(kThreads), 0, st, a);
    } else {
      if (nb == 2) hipLaunchKernelGGL((conv_wgrad_dense_k<T, BM, BN, 2, 64>), grid, dim3(kThreads), 0, st, a);
      else if (nb == 3) hipLaunchKernelGGL((conv_wgrad_dense_k<T, BM, BN, 3, 64>), grid, dim3(kThreads), 0, st, a);
      else hipLaunchKernelGGL((conv_wgrad_dense_k<T, BM, BN, 4, 64>), grid, dim3(kThreads), 0, st, a);
    }
  } else {
    if (nb == 2) hipLaunchKernelGGL((conv_wgrad_k<T, BM, BN, 2, DENSE>), grid, dim3(kThreads), 0, st, a);
    else if (nb == 3) hipLaunchKernelGGL((conv_wgrad_k<T, BM, BN, 3, DENSE>), grid, dim3(kThreads), 0, st, a);
    else hipLaunchKernelGGL((conv_wgrad_k<T, BM, BN, 4, DENSE>), grid, dim3(kThreads), 0, st, a);
  }
  return hipGetLastError();
}

// Ring depth / stage size: dense shapes with long reductions (ResNet layer1 1x1, M ~ 10^5) run
// 3 stages of 128 pixels (conv_wgrad_dense_k: 15.0 -> 12.2 us on MI355X, scripts/wgrad_probe.py);
// everything else 2 stages of 64 (deeper rings measured slower on the 3x3 shapes).
template <typename T, int BM, int BN>
hipError_t launch(const WgradArgs& a, hipStream_t st) {
  const bool dense = a.R == 1 && a.S == 1 && a.sh == 1 && a.sw == 1 && a.ph == 0 && a.pw == 0;
  const bool longk = dense && a.M >= 65536;
  const int nb = g_wgrad_stages > 0 ? g_wgrad_stages : (longk ? 3 : 2);
  const int kp = g_wgrad_kp > 0 ? g_wgrad_kp : (longk && g_wgrad_stages == 0 ? 128 : 64);
  return dense ? launch_d<T, BM, BN, true>(a, st, nb, kp) : launch_d<T, BM, BN, false>(a, st, nb, kp);
}

}  // namespace

bool conv_wgrad_supported(int C, int K) { return C % 64 == 0 && K % 8 == 0; }

void conv_wgrad_set_stages(int nb) {
  g_wgrad_stages = (nb & 7) >= 2 && (nb & 7) <= 4 ? (nb & 7) : 0;
  g_wgrad_lean = ((nb >> 4) & 1) ^ 1;  // tuning: bit 4 sends dense shapes to the general kernel
  g_wgrad_kp = (nb >> 5) & 1 ? 128 : 0;  // tuning: bit 5 stages 128 pixels (dense kernel)
}

// Plan (from the per-layer sweep of bench/conv_shapes.py over ResNet-50 at batch 32 on MI355X,
// profiles/conv_r01/conv_shapes_wgrad_sweep.json): 64 x 64 tiles win at every layer (more workgroups in flight;
// the kernel is latency- not MFMA-bound at these sizes), and the best pixel split keeps each
// workgroup at ~16-25 stages of 64 pixels — enough to amortize the prologue/epilogue, short enough
// that the grid fills the chip.  Fewer splits also bound the fp32 partial traffic (splits*K*RSC*8 B).
void conv_wgrad_plan(int M, int K, int C, int R, int S, int* bm, int* bn, int* splits, int* steps_per_split) {
  (void)K, (void)C, (void)R, (void)S;
  *bm = 64;
  *bn = 64;
  const int total_steps = (M + kBP - 1) / kBP;
  const int per = max(16, (total_steps + 63) / 64);
  *steps_per_split = per;
  *splits = (total_steps + per - 1) / per;
}

namespace {
// conv_wgrad's checks and argument block (shared with conv_wgrad_prepare)
hipError_t wgrad_fill(WgradArgs& a, int dtype, const void* dy, const void* x, void* dw, float* partials,
                      const void* zero, int N, int H, int W, int C, int K, int P, int Q, int R, int S, int sh, int sw,
                      int ph, int pw, int bm, int bn, int splits, int steps_per_split, float alpha,
                      const WgradPendingReduce* pending, int pix) {
  if (!conv_wgrad_supported(C, K) || dtype == kF32) return hipErrorInvalidValue;
  if (C % bn != 0 || (bm != 64 && bm != 128) || (bn != 64 && bn != 128) || splits < 1) return hipErrorInvalidValue;
  const int64_t M64 = (int64_t)N * P * Q;
  // fdiv's 36-bit magic is exact for numerators < 2^22 and divisors < 2^14
  if (M64 <= 0 || M64 >= (1ll << 22) || (int64_t)P * Q >= (1 << 14)) return hipErrorInvalidValue;
  if ((int64_t)splits * steps_per_split * kBP < M64) return hipErrorInvalidValue;
  if (splits > 1 && partials == nullptr) return hipErrorInvalidValue;
  if ((int64_t)N * H * W * C >= (1ll << 31)) return hipErrorInvalidValue;  // 32-bit gather offsets
  a = WgradArgs{static_cast<const uint16_t*>(dy), static_cast<const uint16_t*>(x),
                splits > 1 ? static_cast<void*>(partials) : dw, static_cast<const uint16_t*>(zero), N, H, W, C, K, P,
                Q, R, S, sh, sw, ph, pw, (int)M64, splits, steps_per_split, magic36(Q), magic36(P * Q), alpha,
                kBP / (P * Q), kBP % (P * Q)};
  a.pix = pix > 0 ? pix : C;
  if (pix > 0 && (pix % 8 != 0 || (R == 1 && S == 1 && sh == 1 && sw == 1 && ph == 0 && pw == 0)))
    return hipErrorInvalidValue;  // (the DENSE 1x1 path reads x as a plain [M, C] matrix)
  a.pr = WgradPendingReduce{};
  if (pending != nullptr && pending->part != nullptr) {
    if (pending->n % 4 != 0 || pending->splits < 1 || (pending->dtype != kBF16 && pending->dtype != kF16))
      return hipErrorInvalidValue;
    a.pr = *pending;
    // one extra workgroup per 64 output quads, at most 256 (they loop)
    const int64_t want = (pending->n / 4 + 63) / 64;
    a.pr.blocks = (int)(want < 256 ? want : 256);
  }
  a.nwg_main = ((K + bm - 1) / bm) * (R * S * C / bn) * splits;
  return hipSuccess;
}
}  // namespace

hipError_t conv_wgrad_prepare(WgradArgs* a, int dtype, const DualWgrad& d, const void* zero) {
  return wgrad_fill(*a, dtype, d.dy, d.x, d.dw, d.partials, zero, d.N, d.H, d.W, d.C, d.K, d.P, d.Q, d.R, d.S, d.sh,
                    d.sw, d.ph, d.pw, d.bm, d.bn, d.splits, d.steps_per_split, 1.f, d.pending, 0);
}

hipError_t conv_wgrad(int dtype, const void* dy, const void* x, void* dw, float* partials, const void* zero, int N,
                      int H, int W, int C, int K, int P, int Q, int R, int S, int sh, int sw, int ph, int pw, int bm,
                      int bn, int splits, int steps_per_split, hipStream_t st, float alpha,
                      const WgradPendingReduce* pending, bool defer_reduce, int pix) {
  WgradArgs a;
  {
    const hipError_t e0 = wgrad_fill(a, dtype, dy, x, dw, partials, zero, N, H, W, C, K, P, Q, R, S, sh, sw, ph, pw,
                                     bm, bn, splits, steps_per_split, alpha, pending, pix);
    if (e0 != hipSuccess) return e0;
  }
  hipError_t e;
  if (dtype == kBF16) {
    if (bm == 128 && bn == 128) e = launch<bf16_t, 128, 128>(a, st);
    else if (bm == 128) e = launch<bf16_t, 128, 64>(a, st);
    else if (bn == 128) e = launch<bf16_t, 64, 128>(a, st);
    else e = launch<bf16_t, 64, 64>(a, st);
  } else {
    if (bm == 128 && bn == 128) e = launch<f16_t, 128, 128>(a, st);
    else if (bm == 128) e = launch<f16_t, 128, 64>(a, st);
    else if (bn == 128) e = launch<f16_t, 64, 128>(a, st);
    else e = launch<f16_t, 64, 64>(a, st);
  }
  if (e != hipSuccess || splits == 1 || defer_reduce) return e;
  return splitk_reduce(dtype, partials, dw, (int64_t)K * R * S * C, splits, st, alpha);  // C % 64 == 0: n % 4 == 0
}

}  // namespace hyp

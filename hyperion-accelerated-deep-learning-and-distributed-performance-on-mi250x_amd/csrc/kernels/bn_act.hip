// Fused NHWC BatchNorm (+ residual add) (+ ReLU) for gfx950 — forward and backward.
//
// Replaces the reference's MIOpen batch-norm + separate ReLU + separate residual-add kernels in
// every ResNet block (SURVEY §2.4 row "Convolution + BatchNorm + ReLU", §2.5 ResNet rows).
//
// Layout: x is channels-last, i.e. a row-major [M = N*H*W, C] matrix.  Each thread owns 8
// consecutive channels (one 16-byte vector for bf16/f16, two for f32) and walks rows; a
// 256-thread block covers `tpr` channel-vectors × `rpi` rows per iteration, so the per-channel
// constants (scale/shift, or the backward coefficients) sit in registers for the whole loop.
//
// Statistics are per-channel fp64 SUMS [kStatSlots][2][C] of fp32 per-block partials, accumulated with no-return
// global f64 atomics (channel runs per wave instruction, executed at the memory side: coherent
// across the 8 XCD L2s) by whichever kernel produces them — the conv epilogue (conv_igemm.hip), the
// split-K reduce, or the stats kernels below.  Every CONSUMER finalizes inline: an apply thread
// turns the two sums of its 8 channels into mean / invstd / scale / shift in a few fp64 ops, and
// block 0 also writes save_mean / save_invstd / running stats.  There is no finalize launch (the
// partial-row + finalize design cost 75 latency-bound 5-7 us launches per ResNet-50 step).  The
// sums must be zero before the producer runs: the caller hands in slices of one pre-zeroed arena
// (one fill per forward, ops/_native.py ZeroArena).  Atomic arrival order varies, but fp32
// partials summed in fp64 are exact while their exponents span < ~19 binades (53-bit mantissa vs
// 24 + log2(adders)), so the finalized float mean / invstd are reproducible in practice — the
// deterministic partial-row design's property, without its launches.
//
// Forward (training):  stats (atomic Σx, Σx²)  ->  apply  y = act(x*scale + shift [+ res])
// Backward:            reduce (atomic Σdz, Σdz·x with dz = dy·[y>0])  ->  dx = A·dz + B·x + C ; dres = dz
//                      (M <= 2048: one register-resident launch does all of it)
#include "hyp_common.h"
#include "hyp_kernels.h"
#include "bn_fin.h"
#include "bn_bwd_impl.h"

namespace hyp {
namespace {

// Statistics / backward-reduce geometry: every row block adds one fp64 pair per channel, so the
// atomic traffic is P x C x 16 bytes — keep it near 512 KB (P = 32768 / C row blocks, 16..512)
// and get the parallelism from narrow 64-channel blocks instead (gy = C / 64; one 128-byte row
// segment per block row).  At P = 512 for every C, layer3's C = 1024 reduce moved 8 MB of
// atomics and ran 3.5-8 us slower than with plain partial-row stores.
constexpr int64_t kAtomicBudget = 32768;

bool stats_geom(int64_t M, int C, BnGeom& g) {
  if (C % 8 != 0) return false;
  const int cv = C / 8;
  g.tpr = cv % 8 == 0 ? 8 : (cv <= kBlock ? cv : 0);
  if (g.tpr == 0) return bn_geom(M, C, kStatsBlocks, g);
  g.gy = cv / g.tpr;
  g.rpi = kBlock / g.tpr;
  int64_t P = kAtomicBudget / C;
  P = P < 16 ? 16 : (P > kStatsBlocks ? kStatsBlocks : P);
  const int64_t by_rows = (M + (int64_t)g.rpi * 4 - 1) / ((int64_t)g.rpi * 4);  // >= 4 row iterations
  if (P > by_rows) P = by_rows;
  if (P < 1) P = 1;
  g.rows_per_block = (M + P - 1) / P;
  g.P = (int)((M + g.rows_per_block - 1) / g.rows_per_block);
  return true;
}

// Block-level column sums of s/q (8 per thread) -> one atomic per channel per block
__device__ __forceinline__ void block_atomic_sums(const float (&s)[8], const float (&q)[8], int tpr, int rpi, int C,
                                                  int cbase, double* __restrict__ sums) {
  __shared__ float ls[kBlock * 8];
  __shared__ float lq[kBlock * 8];
  const int tid = threadIdx.x;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    ls[tid * 8 + j] = s[j];
    lq[tid * 8 + j] = q[j];
  }
  __syncthreads();
  const int nch = tpr * 8;
  for (int ch = tid; ch < nch; ch += kBlock) {
    float a = 0.f, b = 0.f;
    for (int rr = 0; rr < rpi; ++rr) {
      a += ls[rr * nch + ch];
      b += lq[rr * nch + ch];
    }
    double* slot = sums + (int64_t)(blockIdx.x % kStatSlots) * 2 * C;
    unsafeAtomicAdd(slot + cbase + ch, (double)a);  // hardware global_atomic_add_f64 (no CAS loop)
    unsafeAtomicAdd(slot + C + cbase + ch, (double)b);
  }
}

// ---------------------------------------------------------------- forward stats
template <typename T>
__global__ __launch_bounds__(kBlock) void bn_stats_k(const T* __restrict__ x, int64_t M, int C, int tpr, int rpi,
                                                     int64_t rpb, double* __restrict__ sums) {
  const int tid = threadIdx.x;
  const int r = tid / tpr, c8 = tid - r * tpr;
  const int cbase = blockIdx.y * tpr * 8;
  const int64_t row0 = (int64_t)blockIdx.x * rpb;
  const int64_t row1 = min(M, row0 + rpb);
  float s[8], q[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = q[j] = 0.f;
  if (r < rpi) {
    const int64_t step = (int64_t)rpi * C;
    const T* p = x + (row0 + r) * C + cbase + c8 * 8;
    int64_t row = row0 + r;
    for (; row + 3 * rpi < row1; row += 4 * rpi, p += 4 * step) {
      float v0[8], v1[8], v2[8], v3[8];
      Vec8<T>::load(p, v0);
      Vec8<T>::load(p + step, v1);
      Vec8<T>::load(p + 2 * step, v2);
      Vec8<T>::load(p + 3 * step, v3);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s[j] += (v0[j] + v1[j]) + (v2[j] + v3[j]);
        q[j] += (v0[j] * v0[j] + v1[j] * v1[j]) + (v2[j] * v2[j] + v3[j] * v3[j]);
      }
    }
    for (; row < row1; row += rpi, p += step) {
      float v[8];
      Vec8<T>::load(p, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s[j] += v[j];
        q[j] += v[j] * v[j];
      }
    }
  }
  block_atomic_sums(s, q, tpr, rpi, C, cbase, sums);
}

// eval-mode constants from running stats
__global__ void bn_eval_consts_k(int C, const float* __restrict__ weight, const float* __restrict__ bias,
                                 const float* __restrict__ rm, const float* __restrict__ rv, float eps,
                                 float* __restrict__ save_mean, float* __restrict__ save_invstd,
                                 float* __restrict__ scale, float* __restrict__ shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float invstd = rsqrtf(rv[c] + eps);
  const float w = weight ? weight[c] : 1.f;
  const float b = bias ? bias[c] : 0.f;
  save_mean[c] = rm[c];
  save_invstd[c] = invstd;
  scale[c] = w * invstd;
  shift[c] = b - rm[c] * w * invstd;
}

// ---------------------------------------------------------------- forward apply
// FIN: training — scale/shift finalized inline from the statistics sums; else read from arrays.
template <typename T, bool ACT, bool RES, bool FIN>
__global__ __launch_bounds__(kBlock) void bn_apply_k(const T* __restrict__ x, const T* __restrict__ res,
                                                     T* __restrict__ y, const float* __restrict__ scale,
                                                     const float* __restrict__ shift, FwdFin fin, int64_t M, int C,
                                                     int tpr, int rpi, int64_t rpb) {
  __shared__ float kk[2][FIN ? kFinCh : 1];
  const int tid = threadIdx.x;
  const int r = tid / tpr, c8 = tid - r * tpr;
  const int c0 = blockIdx.y * tpr * 8 + c8 * 8;
  float sc[8], sh[8];
  if (FIN) {  // finalize this block's <= kFinCh channels, one per thread (block x == 0 also writes)
    const int nch = tpr * 8, cb = blockIdx.y * nch;
    if (tid < nch) fwd_const1(fin, C, cb + tid, blockIdx.x == 0, kk[0][tid], kk[1][tid]);
    __syncthreads();
    if (r >= rpi) return;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sc[j] = kk[0][c8 * 8 + j];
      sh[j] = kk[1][c8 * 8 + j];
    }
  } else {
    if (r >= rpi) return;
    const float4 a = reinterpret_cast<const float4*>(scale + c0)[0];
    const float4 b = reinterpret_cast<const float4*>(scale + c0)[1];
    const float4 d = reinterpret_cast<const float4*>(shift + c0)[0];
    const float4 e = reinterpret_cast<const float4*>(shift + c0)[1];
    sc[0] = a.x; sc[1] = a.y; sc[2] = a.z; sc[3] = a.w; sc[4] = b.x; sc[5] = b.y; sc[6] = b.z; sc[7] = b.w;
    sh[0] = d.x; sh[1] = d.y; sh[2] = d.z; sh[3] = d.w; sh[4] = e.x; sh[5] = e.y; sh[6] = e.z; sh[7] = e.w;
  }
  const int64_t row0 = (int64_t)blockIdx.x * rpb;
  const int64_t row1 = min(M, row0 + rpb);
  const int64_t step = (int64_t)rpi * C;
  int64_t off = (row0 + r) * C + c0;
  int64_t row = row0 + r;
  for (; row + rpi < row1; row += 2 * rpi, off += 2 * step) {
    float v0[8], v1[8], r0[8], r1[8];
    Vec8<T>::load(x + off, v0);
    Vec8<T>::load(x + off + step, v1);
    if (RES) {
      Vec8<T>::load(res + off, r0);
      Vec8<T>::load(res + off + step, r1);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float a = fmaf(v0[j], sc[j], sh[j]);
      float b = fmaf(v1[j], sc[j], sh[j]);
      if (RES) {
        a += r0[j];
        b += r1[j];
      }
      if (ACT) {
        a = fmaxf(a, 0.f);
        b = fmaxf(b, 0.f);
      }
      v0[j] = a;
      v1[j] = b;
    }
    Vec8<T>::store_wt(y + off, v0);
    Vec8<T>::store_wt(y + off + step, v1);
  }
  if (row < row1) {
    float v[8], rr[8];
    Vec8<T>::load(x + off, v);
    if (RES) Vec8<T>::load(res + off, rr);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float a = fmaf(v[j], sc[j], sh[j]);
      if (RES) a += rr[j];
      if (ACT) a = fmaxf(a, 0.f);
      v[j] = a;
    }
    Vec8<T>::store_wt(y + off, v);
  }
}

// ---------------------------------------------------------------- backward
template <typename T, bool ACT, bool MASKX>
__global__ __launch_bounds__(kBlock) void bn_bwd_reduce_k(const T* __restrict__ dy, const T* __restrict__ x,
                                                          const T* __restrict__ y, int64_t M, int C, int tpr, int rpi,
                                                          int64_t rpb, double* __restrict__ sums,
                                                          const float* __restrict__ w, const float* __restrict__ b,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ invstd) {
  const int tid = threadIdx.x;
  const int r = tid / tpr, c8 = tid - r * tpr;
  const int cbase = blockIdx.y * tpr * 8;
  const int64_t row0 = (int64_t)blockIdx.x * rpb;
  const int64_t row1 = min(M, row0 + rpb);
  float s[8], q[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = q[j] = 0.f;
  ReluMask<T, ACT, MASKX> mk;
  if (r < rpi) mk.init(w, b, mean, invstd, cbase + c8 * 8);
  if (r < rpi) {
    const int64_t step = (int64_t)rpi * C;
    int64_t off = (row0 + r) * C + cbase + c8 * 8;
    int64_t row = row0 + r;
    for (; row + rpi < row1; row += 2 * rpi, off += 2 * step) {
      float g0[8], g1[8], x0[8], x1[8], y0[8], y1[8];
      Vec8<T>::load(dy + off, g0);
      Vec8<T>::load(dy + off + step, g1);
      Vec8<T>::load(x + off, x0);
      Vec8<T>::load(x + off + step, x1);
      if (ACT && !MASKX) {
        Vec8<T>::load(y + off, y0);
        Vec8<T>::load(y + off + step, y1);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d0 = mk.keep(x0, y0, j) ? g0[j] : 0.f;
        const float d1 = mk.keep(x1, y1, j) ? g1[j] : 0.f;
        s[j] += d0 + d1;
        q[j] += d0 * x0[j] + d1 * x1[j];
      }
    }
    if (row < row1) {
      float g[8], xv[8], yv[8];
      Vec8<T>::load(dy + off, g);
      Vec8<T>::load(x + off, xv);
      if (ACT && !MASKX) Vec8<T>::load(y + off, yv);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = mk.keep(xv, yv, j) ? g[j] : 0.f;
        s[j] += d;
        q[j] += d * xv[j];
      }
    }
  }
  block_atomic_sums(s, q, tpr, rpi, C, cbase, sums);
}

// ---------------------------------------------------------------- small-M backward
// Below ~2K rows (ResNet-50 layer4 at batch 32: M = 1568) the reduce + dx pair is latency-bound,
// so one block owns 8 channels over ALL M rows: grid C/8, block 256.  Every thread loads its
// <= 8 rows of dy / x (/ y) ONCE, in one burst (all loads in flight), keeps them packed in
// registers across the block reduction and the in-block finalize, and writes dx from them: one
// memory round trip per tensor, no atomics, deterministic.
constexpr int kBwdRows = 8;

template <typename T>
__device__ __forceinline__ void unpack8(const uint4& raw, float (&v)[8]) {
  Vec8<T>::load(reinterpret_cast<const T*>(&raw), v);
}

template <typename T, bool ACT, bool RES, bool MASKX, int NT, int ROWS>
__global__ __launch_bounds__(NT) void bn_bwd_small_k(const T* __restrict__ dy, const T* __restrict__ x,
                                                         const T* __restrict__ y, T* __restrict__ dx,
                                                         T* __restrict__ dres, int64_t M, int C, BwdFin fin,
                                                         const float* __restrict__ bn_b) {
  static_assert(sizeof(T) == 2, "packed 16-bit rows");
  __shared__ float red[2][NT / 64][8];
  __shared__ float kk[3][8];
  __shared__ double ksum[2][8];
  const int tid = threadIdx.x;
  // XCD-aware slice order: blocks b, b+8, ... share an XCD (round-robin dispatch), so give them
  // ADJACENT 8-channel slices — 8 slices = one 128-byte row segment is then fetched into one
  // L2 once instead of into 8 (the 16-byte-per-row access otherwise moves 8x the bytes)
  const int G = gridDim.x;
  int slice = blockIdx.x;
  if ((G & 7) == 0) slice = (slice & 7) * (G >> 3) + (slice >> 3);
  const int c0 = slice * 8;
  ReluMask<T, ACT, MASKX> mk;
  mk.init(fin.weight, bn_b, fin.mean, fin.invstd, c0);
  uint4 rg[ROWS], rx[ROWS], ryv[ROWS];
#pragma unroll
  for (int i = 0; i < ROWS; ++i) {
    const int64_t row = tid + (int64_t)i * NT;
    if (row < M) {
      const int64_t off = row * C + c0;
      rg[i] = *reinterpret_cast<const uint4*>(dy + off);
      rx[i] = *reinterpret_cast<const uint4*>(x + off);
      if (ACT && !MASKX) ryv[i] = *reinterpret_cast<const uint4*>(y + off);
    }
  }
  float s[8], q[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = q[j] = 0.f;
#pragma unroll
  for (int i = 0; i < ROWS; ++i) {
    if (tid + (int64_t)i * NT < M) {
      float g[8], xv[8], yv[8];
      unpack8<T>(rg[i], g);
      unpack8<T>(rx[i], xv);
      if (ACT && !MASKX) unpack8<T>(ryv[i], yv);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = mk.keep(xv, yv, j) ? g[j] : 0.f;
        s[j] += d;
        q[j] += d * xv[j];
      }
    }
  }
  // 8 channels x {Σdz, Σdz·x}: wave tree sums, then the 4 waves in fixed order (deterministic)
  const int lane = tid & 63, wv = tid >> 6;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float ws = wave_sum(s[j]), wq = wave_sum(q[j]);
    if (lane == 0) {
      red[0][wv][j] = ws;
      red[1][wv][j] = wq;
    }
  }
  __syncthreads();
  if (tid < 16) {
    const int j = tid & 7, which = tid >> 3;
    double acc = 0.0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) acc += red[which][w][j];
    ksum[which][j] = acc;
  }
  __syncthreads();
  if (tid < 8) bwd_coeffs(fin, c0 + tid, ksum[0][tid], ksum[1][tid], true, kk[0][tid], kk[1][tid], kk[2][tid]);
  __syncthreads();
  float A[8], B[8], Cc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    A[j] = kk[0][j];
    B[j] = kk[1][j];
    Cc[j] = kk[2][j];
  }
#pragma unroll
  for (int i = 0; i < ROWS; ++i) {
    const int64_t row = tid + (int64_t)i * NT;
    if (row < M) {
      const int64_t off = row * C + c0;
      float g[8], xv[8], yv[8];
      unpack8<T>(rg[i], g);
      unpack8<T>(rx[i], xv);
      if (ACT && !MASKX) unpack8<T>(ryv[i], yv);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = mk.keep(xv, yv, j) ? g[j] : 0.f;
        g[j] = d;
        xv[j] = fmaf(A[j], d, fmaf(B[j], xv[j], Cc[j]));
      }
      Vec8<T>::store_wt(dx + off, xv);
      if (RES) Vec8<T>::store_wt(dres + off, g);
    }
  }
}

int g_bn_small = 1;  // small-M one-launch backward on (bn_set_small_paths: A/B and tests)

// small-M backward: reduce + finalize + dx in one launch (false when not covered)
bool launch_bwd_small(int dtype, bool maskx, bool act, const void* dy, const void* x, const void* y, void* dx,
                      void* dres, int64_t M, int C, const BwdFin& fin, const float* bias, hipStream_t stream) {
  if (g_bn_small == 0 || M > (int64_t)kBwdRows * kBlock || C % 8 != 0 || (dtype != kBF16 && dtype != kF16))
    return false;
  const dim3 grid(C / 8);
  // 256 threads x 8 register-resident rows (M <= 2048: layer4).  Wider blocks for layer3's 6272
  // rows (512 x 13, 1024 x 8) spill VGPRs: that case keeps the 2-kernel path.
#define HYP_BN_SMALL(ACTV, RESV, MX)                                                                               \
  hipLaunchKernelGGL((bn_bwd_small_k<T, ACTV, RESV, MX, kBlock, kBwdRows>), grid, dim3(kBlock), 0, stream, dyt, xt, \
                     yt, dxt, drt, M, C, fin, bias)
  auto go = [&](auto tag) {
    using T = decltype(tag);
    const T* dyt = static_cast<const T*>(dy);
    const T* xt = static_cast<const T*>(x);
    const T* yt = static_cast<const T*>(y);
    T* dxt = static_cast<T*>(dx);
    T* drt = static_cast<T*>(dres);
    if (maskx) {
      HYP_BN_SMALL(true, false, true);
    } else if (act && dres) {
      HYP_BN_SMALL(true, true, false);
    } else if (act) {
      HYP_BN_SMALL(true, false, false);
    } else if (dres) {
      HYP_BN_SMALL(false, true, false);
    } else {
      HYP_BN_SMALL(false, false, false);
    }
  };
  if (dtype == kBF16)
    go(bf16_t{});
  else
    go(f16_t{});
#undef HYP_BN_SMALL
  return true;
}

template <typename T, bool FIN>
void launch_apply(bool act, const void* res, dim3 grid, hipStream_t stream, const T* xt, T* yt, const float* scale,
                  const float* shift, const FwdFin& fin, int64_t M, int C, const BnGeom& ga) {
  const T* rt = static_cast<const T*>(res);
#define HYP_BN_APPLY(ACTV, RESV)                                                                                  \
  hipLaunchKernelGGL((bn_apply_k<T, ACTV, RESV, FIN>), grid, dim3(kBlock), 0, stream, xt, rt, yt, scale, shift, fin, \
                     M, C, ga.tpr, ga.rpi, ga.rows_per_block)
  if (act && res)
    HYP_BN_APPLY(true, true);
  else if (act)
    HYP_BN_APPLY(true, false);
  else if (res)
    HYP_BN_APPLY(false, true);
  else
    HYP_BN_APPLY(false, false);
#undef HYP_BN_APPLY
}

}  // namespace

// ======================================================================== host launchers
void bn_set_small_paths(int on) { g_bn_small = on ? 1 : 0; }

hipError_t bn_stats(int dtype, const void* x, int64_t M, int C, double* sums, hipStream_t stream) {
  BnGeom gs;
  if (!stats_geom(M, C, gs)) return hipErrorInvalidValue;
  HYP_DISPATCH_FLOAT(dtype, T, {
    hipLaunchKernelGGL(bn_stats_k<T>, dim3(gs.P, gs.gy), dim3(kBlock), 0, stream, static_cast<const T*>(x), M, C,
                       gs.tpr, gs.rpi, gs.rows_per_block, sums);
  });
  return hipGetLastError();
}

hipError_t bn_forward(int dtype, const void* x, const void* res, void* y, int64_t M, int C, const float* weight,
                      const float* bias, float* running_mean, float* running_var, float momentum, float eps,
                      int training, int act, double* sums, float* save_mean, float* save_invstd, float* scale,
                      float* shift, hipStream_t stream) {
  if (training) {
    const hipError_t e = bn_stats(dtype, x, M, C, sums, stream);
    if (e != hipSuccess) return e;
    return bn_forward_from_sums(dtype, x, res, y, M, C, weight, bias, running_mean, running_var, momentum, eps, act,
                                sums, save_mean, save_invstd, stream);
  }
  BnGeom ga;
  if (!apply_geom(M, C, ga)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(bn_eval_consts_k, dim3((C + 255) / 256), dim3(256), 0, stream, C, weight, bias, running_mean,
                     running_var, eps, save_mean, save_invstd, scale, shift);
  HYP_DISPATCH_FLOAT(dtype, T, {
    launch_apply<T, false>(act != 0, res, dim3(ga.P, ga.gy), stream, static_cast<const T*>(x), static_cast<T*>(y),
                           scale, shift, FwdFin{}, M, C, ga);
  });
  return hipGetLastError();
}

// Training-mode BN forward whose per-channel sums were produced elsewhere (the conv epilogue of
// conv_igemm.hip, the split-K reduce, or bn_stats): one apply launch, finalize inline.
hipError_t bn_forward_from_sums(int dtype, const void* x, const void* res, void* y, int64_t M, int C,
                                const float* weight, const float* bias, float* running_mean, float* running_var,
                                float momentum, float eps, int act, const double* sums, float* save_mean,
                                float* save_invstd, hipStream_t stream) {
  BnGeom ga;
  if (!apply_geom(M, C, ga)) return hipErrorInvalidValue;
  const FwdFin fin{sums,        weight,     bias, running_mean, running_var, momentum, eps, save_mean,
                   save_invstd, 1.0 / (double)M, M > 1 ? (double)M / (double)(M - 1) : 1.0};
  HYP_DISPATCH_FLOAT(dtype, T, {
    launch_apply<T, true>(act != 0, res, dim3(ga.P, ga.gy), stream, static_cast<const T*>(x), static_cast<T*>(y),
                          nullptr, nullptr, fin, M, C, ga);
  });
  return hipGetLastError();
}

template <typename T>
void launch_bn_dx(bool maskx, bool act, bool res, dim3 grid, hipStream_t stream, const T* dy, const T* x, const T* y,
                  T* dx, T* dres, const BwdFin& fin, int64_t M, int C, const BnGeom& ga, const float* b) {
#define HYP_BN_DX(ACTV, RESV, MX)                                                                                     \
  hipLaunchKernelGGL((bn_bwd_dx_k<T, ACTV, RESV, MX>), grid, dim3(kBlock), 0, stream, dy, x, y, dx, dres, fin, M, C, \
                     ga.tpr, ga.rpi, ga.rows_per_block, b)
  if (maskx)
    HYP_BN_DX(true, false, true);
  else if (act && res)
    HYP_BN_DX(true, true, false);
  else if (act)
    HYP_BN_DX(true, false, false);
  else if (res)
    HYP_BN_DX(false, true, false);
  else
    HYP_BN_DX(false, false, false);
#undef HYP_BN_DX
}

hipError_t bn_backward(int dtype, const void* dy, const void* x, const void* y, void* dx, void* dres, int64_t M, int C,
                       const float* weight, const float* bias, const float* save_mean, const float* save_invstd,
                       int training, int act, double* sums, float* dweight, float* dbias, hipStream_t stream) {
  BnGeom gs, ga;
  if (!stats_geom(M, C, gs) || !apply_geom(M, C, ga)) return hipErrorInvalidValue;
  // act with no forward output given: recompute the ReLU mask from x (training stats only: the
  // eval-mode constants are running stats, which the mask recomputation below does not model)
  const bool maskx = act && y == nullptr;
  if (maskx && (!training || dres != nullptr)) return hipErrorInvalidValue;
  const BwdFin fin{weight, save_mean, save_invstd, training, dweight, dbias, sums, 1.0 / (double)M};
  if (launch_bwd_small(dtype, maskx, act != 0, dy, x, y, dx, dres, M, C, fin, bias, stream)) return hipGetLastError();
  HYP_DISPATCH_FLOAT(dtype, T, {
    const T* dyt = static_cast<const T*>(dy);
    const T* xt = static_cast<const T*>(x);
    const T* yt = static_cast<const T*>(y);
    const dim3 grs(gs.P, gs.gy);
    if (maskx)
      hipLaunchKernelGGL((bn_bwd_reduce_k<T, true, true>), grs, dim3(kBlock), 0, stream, dyt, xt, yt, M, C, gs.tpr,
                         gs.rpi, gs.rows_per_block, sums, weight, bias, save_mean, save_invstd);
    else if (act)
      hipLaunchKernelGGL((bn_bwd_reduce_k<T, true, false>), grs, dim3(kBlock), 0, stream, dyt, xt, yt, M, C, gs.tpr,
                         gs.rpi, gs.rows_per_block, sums, weight, bias, save_mean, save_invstd);
    else
      hipLaunchKernelGGL((bn_bwd_reduce_k<T, false, false>), grs, dim3(kBlock), 0, stream, dyt, xt, yt, M, C, gs.tpr,
                         gs.rpi, gs.rows_per_block, sums, weight, bias, save_mean, save_invstd);
    launch_bn_dx<T>(maskx, act, dres != nullptr, dim3(ga.P, ga.gy), stream, dyt, xt, yt, static_cast<T*>(dx),
                    static_cast<T*>(dres), fin, M, C, ga, bias);
  });
  return hipGetLastError();
}

// dy is already dz (masked by its producer, e.g. the dgrad epilogue) and the Σdz, Σdz·x sums are
// complete: only the dx pass remains (the residual gradient is dz itself).
hipError_t bn_backward_dx(int dtype, const void* dz, const void* x, void* dx, int64_t M, int C, const float* weight,
                          const float* save_mean, const float* save_invstd, int training, const double* sums,
                          float* dweight, float* dbias, hipStream_t stream) {
  BnGeom ga;
  if (!apply_geom(M, C, ga)) return hipErrorInvalidValue;
  const BwdFin fin{weight, save_mean, save_invstd, training, dweight, dbias, sums, 1.0 / (double)M};
  HYP_DISPATCH_FLOAT(dtype, T, {
    launch_bn_dx<T>(false, false, false, dim3(ga.P, ga.gy), stream, static_cast<const T*>(dz),
                    static_cast<const T*>(x), nullptr, static_cast<T*>(dx), nullptr, fin, M, C, ga, nullptr);
  });
  return hipGetLastError();
}

int g_bn_apply_blocks = 2048, g_bn_min_iters = 4;
int bn_apply_blocks() { return g_bn_apply_blocks; }
int bn_min_iters() { return g_bn_min_iters; }
void bn_set_geom(int apply_blocks, int min_iters) {
  g_bn_apply_blocks = apply_blocks > 0 ? apply_blocks : 2048;
  g_bn_min_iters = min_iters > 0 ? min_iters : 4;
}

}  // namespace hyp

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
// Forward (training):  stats_partial (deterministic per-block partial Σx, Σx²)
//                      -> stats_finalize (fp64 combine, running-stat update, scale/shift)
//                      -> apply   y = act(x*scale + shift [+ res])
// Backward:            bwd_reduce (Σdz, Σdz·x with dz = dy·[y>0])
//                      -> bwd_finalize (dγ, dβ, and dx = A·dz + B·x + C coefficients)
//                      -> bwd_dx  dx = A·dz + B·x + C ; dres = dz
#include "hyp_common.h"
#include "hyp_kernels.h"

namespace hyp {
namespace {

constexpr int kBlock = 256;
constexpr int kStatsBlocks = 512;  // partial rows per reduction: keeps the combine pass short
constexpr int kFinCh = 8;          // finalize block: 8 channels x 32 partial-row groups
constexpr int kFinGr = 32;

typedef float f32x4 __attribute__((ext_vector_type(4)));

struct BwdFin {  // backward finalize inputs / outputs (bn_bwd_finalize_k's arguments)
  const float* weight;
  const float* mean;
  const float* invstd;
  int training;
  float* dweight;
  float* dbias;
};

struct BnGeom {
  int tpr;   // threads per row (each owns 8 channels)
  int rpi;   // rows per block-iteration
  int gy;    // channel chunks (grid.y)
  int P;     // row blocks (grid.x)
  int64_t rows_per_block;
};

bool bn_geom(int64_t M, int C, int max_blocks, BnGeom& g) {
  if (C % 8 != 0) return false;
  const int cv = C / 8;
  if (cv <= kBlock) {
    g.tpr = cv;
    g.gy = 1;
  } else {
    if (cv % kBlock != 0) return false;
    g.tpr = kBlock;
    g.gy = cv / kBlock;
  }
  g.rpi = kBlock / g.tpr;
  // >= 4 row iterations per thread, and >= 16K elements per block so partial rows stay a tiny
  // fraction of the data (the combine pass reads P*C partials)
  int64_t min_rows = (int64_t)g.rpi * 4;
  const int64_t by_size = (16384 + C - 1) / C;
  if (max_blocks <= kStatsBlocks && by_size > min_rows) min_rows = by_size;
  int64_t want = (M + min_rows - 1) / min_rows;
  int64_t cap = max_blocks / g.gy;
  if (cap < 1) cap = 1;
  int64_t P = want < cap ? want : cap;
  if (P < 1) P = 1;
  g.rows_per_block = (M + P - 1) / P;
  g.P = (int)((M + g.rows_per_block - 1) / g.rows_per_block);
  if (g.P < 1) g.P = 1;
  return true;
}

// ---------------------------------------------------------------- forward stats
template <typename T>
__global__ __launch_bounds__(kBlock) void bn_stats_partial_k(const T* __restrict__ x, int64_t M, int C, int tpr,
                                                             int rpi, int64_t rpb, float* __restrict__ psum,
                                                             float* __restrict__ psq) {
  __shared__ float ls[kBlock * 8];
  __shared__ float lq[kBlock * 8];
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
    psum[(int64_t)blockIdx.x * C + cbase + ch] = a;
    psq[(int64_t)blockIdx.x * C + cbase + ch] = b;
  }
}

// Sum partial rows p = threadIdx.y, +16, ... of column c with 8 independent loads in flight
// (the loop is latency-bound; a rolled loop waits one L2 round trip per partial).
__device__ __forceinline__ void combine_partials(const float* __restrict__ pa, const float* __restrict__ pb, int P,
                                                 int C, int c, float& a, float& b) {
  float sa[8], sb[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) sa[i] = sb[i] = 0.f;
  int p = threadIdx.y;
  for (; p + kFinGr * 7 < P; p += kFinGr * 8) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      sa[i] += pa[(int64_t)(p + kFinGr * i) * C + c];
      sb[i] += pb[(int64_t)(p + kFinGr * i) * C + c];
    }
  }
  for (; p < P; p += kFinGr) {
    sa[0] += pa[(int64_t)p * C + c];
    sb[0] += pb[(int64_t)p * C + c];
  }
  a = ((sa[0] + sa[1]) + (sa[2] + sa[3])) + ((sa[4] + sa[5]) + (sa[6] + sa[7]));
  b = ((sb[0] + sb[1]) + (sb[2] + sb[3])) + ((sb[4] + sb[5]) + (sb[6] + sb[7]));
}

// grid: ceil(C/8); block (8, 32)
__global__ __launch_bounds__(256) void bn_stats_finalize_k(const float* __restrict__ psum, const float* __restrict__ psq,
                                                            int P, int C, int64_t M, const float* __restrict__ weight,
                                                            const float* __restrict__ bias, float* running_mean,
                                                            float* running_var, float momentum, float eps,
                                                            float* __restrict__ save_mean, float* __restrict__ save_invstd,
                                                            float* __restrict__ scale, float* __restrict__ shift) {
  __shared__ float red_s[kFinGr][kFinCh];
  __shared__ float red_q[kFinGr][kFinCh];
  const int c = blockIdx.x * kFinCh + threadIdx.x;
  float a = 0.f, b = 0.f;
  if (c < C) combine_partials(psum, psq, P, C, c, a, b);
  red_s[threadIdx.y][threadIdx.x] = a;
  red_q[threadIdx.y][threadIdx.x] = b;
  __syncthreads();
  if (threadIdx.y == 0 && c < C) {
    double da = a, db = b;
    for (int i = 1; i < kFinGr; ++i) {
      da += red_s[i][threadIdx.x];
      db += red_q[i][threadIdx.x];
    }
    const double a = da, b = db;
    const double mean = a / (double)M;
    double var = b / (double)M - mean * mean;
    if (var < 0.0) var = 0.0;
    const float invstd = (float)(1.0 / sqrt(var + (double)eps));
    save_mean[c] = (float)mean;
    save_invstd[c] = invstd;
    if (running_mean != nullptr) {
      const double unbiased = M > 1 ? var * (double)M / (double)(M - 1) : var;
      running_mean[c] = (float)((1.0 - momentum) * running_mean[c] + momentum * mean);
      running_var[c] = (float)((1.0 - momentum) * running_var[c] + momentum * unbiased);
    }
    const float w = weight ? weight[c] : 1.f;
    const float bb = bias ? bias[c] : 0.f;
    const float sc = w * invstd;
    scale[c] = sc;
    shift[c] = bb - (float)mean * sc;
  }
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
template <typename T, bool ACT, bool RES>
__global__ __launch_bounds__(kBlock) void bn_apply_k(const T* __restrict__ x, const T* __restrict__ res,
                                                     T* __restrict__ y, const float* __restrict__ scale,
                                                     const float* __restrict__ shift, int64_t M, int C, int tpr,
                                                     int rpi, int64_t rpb) {
  const int tid = threadIdx.x;
  const int r = tid / tpr, c8 = tid - r * tpr;
  if (r >= rpi) return;
  const int c0 = blockIdx.y * tpr * 8 + c8 * 8;
  float sc[8], sh[8];
  {
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
    Vec8<T>::store(y + off, v0);
    Vec8<T>::store(y + off + step, v1);
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
    Vec8<T>::store(y + off, v);
  }
}

// ---------------------------------------------------------------- backward
// ReLU mask of the forward output.  MASKX: recomputed from x as x*scale + shift > 0 with the
// forward's exact float scale/shift (scale = w*invstd, shift = b - mean*scale, the finalize
// kernel's arithmetic), so the non-residual backward never reads y (one stream less).
template <typename T, bool ACT, bool MASKX>
struct ReluMask {
  float sc[8], sh[8];
  __device__ __forceinline__ void init(const float* w, const float* b, const float* mean, const float* invstd, int c0) {
    if (MASKX) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float s = (w ? w[c0 + j] : 1.f) * invstd[c0 + j];
        sc[j] = s;
        sh[j] = (b ? b[c0 + j] : 0.f) - mean[c0 + j] * s;
      }
    }
  }
  __device__ __forceinline__ bool keep(const float (&xv)[8], const float (&yv)[8], int j) const {
    if (!ACT) return true;
    if (MASKX) return fmaf(xv[j], sc[j], sh[j]) > 0.f;
    return yv[j] > 0.f;
  }
};

template <typename T, bool ACT, bool MASKX>
__global__ __launch_bounds__(kBlock) void bn_bwd_reduce_k(const T* __restrict__ dy, const T* __restrict__ x,
                                                          const T* __restrict__ y, int64_t M, int C, int tpr, int rpi,
                                                          int64_t rpb, float* __restrict__ pdz,
                                                          float* __restrict__ pdzx, const float* __restrict__ w,
                                                          const float* __restrict__ b, const float* __restrict__ mean,
                                                          const float* __restrict__ invstd) {
  __shared__ float ls[kBlock * 8];
  __shared__ float lq[kBlock * 8];
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
    pdz[(int64_t)blockIdx.x * C + cbase + ch] = a;
    pdzx[(int64_t)blockIdx.x * C + cbase + ch] = b;
  }
}

__global__ __launch_bounds__(256) void bn_bwd_finalize_k(const float* __restrict__ pdz, const float* __restrict__ pdzx,
                                                          int P, int C, int64_t M, const float* __restrict__ weight,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ invstd, int training,
                                                          float* __restrict__ dweight, float* __restrict__ dbias,
                                                          float* __restrict__ kA, float* __restrict__ kB,
                                                          float* __restrict__ kC) {
  __shared__ float red_s[kFinGr][kFinCh];
  __shared__ float red_q[kFinGr][kFinCh];
  const int c = blockIdx.x * kFinCh + threadIdx.x;
  float a = 0.f, b = 0.f;
  if (c < C) combine_partials(pdz, pdzx, P, C, c, a, b);
  red_s[threadIdx.y][threadIdx.x] = a;
  red_q[threadIdx.y][threadIdx.x] = b;
  __syncthreads();
  if (threadIdx.y == 0 && c < C) {
    double da = a, db = b;
    for (int i = 1; i < kFinGr; ++i) {
      da += red_s[i][threadIdx.x];
      db += red_q[i][threadIdx.x];
    }
    const double a = da, b = db;
    const double mu = mean[c], is = invstd[c];
    const double sum_dz_xhat = is * (b - mu * a);
    if (dweight) dweight[c] = (float)sum_dz_xhat;
    if (dbias) dbias[c] = (float)a;
    const double g = weight ? weight[c] : 1.0;
    const double A = g * is;
    if (training) {
      const double Bc = -A * is * sum_dz_xhat / (double)M;
      const double Cc = -A * a / (double)M - Bc * mu;
      kA[c] = (float)A;
      kB[c] = (float)Bc;
      kC[c] = (float)Cc;
    } else {
      kA[c] = (float)A;
      kB[c] = 0.f;
      kC[c] = 0.f;
    }
  }
}

// ---------------------------------------------------------------- wide finalize
// The conv epilogue (forward) and bn_bwd_reduce_k (backward) leave P partial rows [P, C] — up to
// 784 for ResNet-50 layer1.  The finalize kernels above give each of C/8 blocks P/32 scalar loads
// per thread, issued 8 at a time: three or four dependent memory round trips, a 5-7 us
// latency-bound launch (8 blocks at C = 64; 75 such launches per ResNet-50 step).  A ticketed
// two-level variant (last arriver combines) measured 10-14 us: the agent-scope release/acquire
// fences and the winner's serial second pass cost more than they save (MI355X_MICROARCH.md
// "splitk-seam").  Here one 1024-thread block owns 16 channels (4 float4 lanes) x 256 row lanes:
// every partial is read by ONE round of independent 16-byte loads (<= 4 per thread for P <= 1024),
// then a fixed-order LDS tree over the 256 row lanes (deterministic) and the fp64 finalize.
struct Fin2Fwd {  // forward: statistics -> mean / invstd / running stats / scale / shift
  const float* weight;
  const float* bias;
  float* running_mean;
  float* running_var;
  float momentum, eps;
  float* save_mean;
  float* save_invstd;
  float* scale;
  float* shift;
};

constexpr int kWideRows = 256;  // row lanes per block
constexpr int kWideUnroll = 4;  // partial rows per thread per round

template <bool BWD>
__global__ __launch_bounds__(1024) void bn_fin_wide_k(const float* __restrict__ pa, const float* __restrict__ pb,
                                                       int P, int C, int64_t M, Fin2Fwd ff, BwdFin bf,
                                                       float* __restrict__ kA, float* __restrict__ kB,
                                                       float* __restrict__ kC) {
  __shared__ f32x4 red[2][kWideRows][4];
  const int tid = threadIdx.x, q = tid & 3, ry = tid >> 2;
  const int c = blockIdx.x * 16 + q * 4;
  f32x4 sa = {0.f, 0.f, 0.f, 0.f}, sb = sa;
  for (int r0 = ry; r0 < P; r0 += kWideRows * kWideUnroll) {
    f32x4 va[kWideUnroll], vb[kWideUnroll];
#pragma unroll
    for (int u = 0; u < kWideUnroll; ++u) {  // all loads of the round in flight before any add
      const int r = r0 + u * kWideRows;
      const bool ok = r < P;
      va[u] = ok ? *reinterpret_cast<const f32x4*>(pa + (int64_t)r * C + c) : f32x4{0.f, 0.f, 0.f, 0.f};
      vb[u] = ok ? *reinterpret_cast<const f32x4*>(pb + (int64_t)r * C + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < kWideUnroll; ++u) {
      sa += va[u];
      sb += vb[u];
    }
  }
  red[0][ry][q] = sa;
  red[1][ry][q] = sb;
  __syncthreads();
  for (int h = kWideRows / 2; h >= 1; h >>= 1) {  // fixed pairing: deterministic
    if (ry < h) {
      red[0][ry][q] += red[0][ry + h][q];
      red[1][ry][q] += red[1][ry + h][q];
    }
    __syncthreads();
  }
  if (tid < 16) {
    const int ch = blockIdx.x * 16 + tid;
    if (ch < C) {
      const double a = red[0][0][tid >> 2][tid & 3], b = red[1][0][tid >> 2][tid & 3];
      if (!BWD) {
        const double mean = a / (double)M;
        double var = b / (double)M - mean * mean;
        if (var < 0.0) var = 0.0;
        const float invstd = (float)(1.0 / sqrt(var + (double)ff.eps));
        ff.save_mean[ch] = (float)mean;
        ff.save_invstd[ch] = invstd;
        if (ff.running_mean != nullptr) {
          const double unbiased = M > 1 ? var * (double)M / (double)(M - 1) : var;
          ff.running_mean[ch] = (float)((1.0 - ff.momentum) * ff.running_mean[ch] + ff.momentum * mean);
          ff.running_var[ch] = (float)((1.0 - ff.momentum) * ff.running_var[ch] + ff.momentum * unbiased);
        }
        const float w = ff.weight ? ff.weight[ch] : 1.f;
        const float bb = ff.bias ? ff.bias[ch] : 0.f;
        const float sc = w * invstd;
        ff.scale[ch] = sc;
        ff.shift[ch] = bb - (float)mean * sc;
      } else {
        const double mu = bf.mean[ch], is = bf.invstd[ch];
        const double sum_dz_xhat = is * (b - mu * a);
        if (bf.dweight) bf.dweight[ch] = (float)sum_dz_xhat;
        if (bf.dbias) bf.dbias[ch] = (float)a;
        const double gw = bf.weight ? bf.weight[ch] : 1.0;
        const double A = gw * is;
        const double Bc = bf.training ? -A * is * sum_dz_xhat / (double)M : 0.0;
        const double Cc = bf.training ? -A * a / (double)M - Bc * mu : 0.0;
        kA[ch] = (float)A;
        kB[ch] = (float)Bc;
        kC[ch] = (float)Cc;
      }
    }
  }
}

template <typename T, bool ACT, bool RES, bool MASKX>
__global__ __launch_bounds__(kBlock) void bn_bwd_dx_k(const T* __restrict__ dy, const T* __restrict__ x,
                                                      const T* __restrict__ y, T* __restrict__ dx,
                                                      T* __restrict__ dres, const float* __restrict__ kA,
                                                      const float* __restrict__ kB, const float* __restrict__ kC,
                                                      int64_t M, int C, int tpr, int rpi, int64_t rpb,
                                                      const float* __restrict__ w, const float* __restrict__ b,
                                                      const float* __restrict__ mean,
                                                      const float* __restrict__ invstd) {
  const int tid = threadIdx.x;
  const int r = tid / tpr, c8 = tid - r * tpr;
  if (r >= rpi) return;
  const int c0 = blockIdx.y * tpr * 8 + c8 * 8;
  ReluMask<T, ACT, MASKX> mk;
  mk.init(w, b, mean, invstd, c0);
  float A[8], B[8], Cc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    A[j] = kA[c0 + j];
    B[j] = kB[c0 + j];
    Cc[j] = kC[c0 + j];
  }
  const int64_t row0 = (int64_t)blockIdx.x * rpb;
  const int64_t row1 = min(M, row0 + rpb);
  const int64_t step = (int64_t)rpi * C;
  int64_t off = (row0 + r) * C + c0;
  for (int64_t row = row0 + r; row < row1; row += rpi, off += step) {
    float g[8], xv[8], yv[8];
    Vec8<T>::load(dy + off, g);
    Vec8<T>::load(x + off, xv);
    if (ACT && !MASKX) Vec8<T>::load(y + off, yv);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float d = mk.keep(xv, yv, j) ? g[j] : 0.f;
      g[j] = d;
      xv[j] = fmaf(A[j], d, fmaf(B[j], xv[j], Cc[j]));
    }
    Vec8<T>::store(dx + off, xv);
    if (RES) Vec8<T>::store(dres + off, g);
  }
}

// ---------------------------------------------------------------- small-M fused paths
// Below ~8K rows (ResNet-50 layer3/layer4 at batch 32: M = 6272 / 1568) every BN kernel is
// launch/latency-bound (~4-5 us each on MI355X whatever its size), so the separate finalize
// launches are folded away:
//  * forward: each apply block re-derives scale/shift for ITS 64 channels from the P partial rows
//    (P <= 128, L2-resident) — the same double-precision finalize arithmetic, blockIdx.y == 0
//    also writes save_mean / save_invstd / running stats — then applies;
//  * backward (M <= 2048: layer4): one block owns 8 channels over ALL M rows, register-resident:
//    Σdz, Σdz·x, in-block finalize, dx — reduce + finalize + dx in one launch.
int g_bn_small = 1;  // small-M fused paths on (bn_set_small_paths: A/B and tests)
constexpr int kSmallFinP = 128;
constexpr int64_t kSmallBwdM = 8192;

struct StatsFin {  // forward finalize inputs / outputs (bn_stats_finalize_k's arguments)
  const float* weight;
  const float* bias;
  float* running_mean;
  float* running_var;
  float momentum, eps;
  float* save_mean;
  float* save_invstd;
};

template <typename T, bool ACT, bool RES>
__global__ __launch_bounds__(kBlock) void bn_fin_apply_k(const T* __restrict__ x, const T* __restrict__ res,
                                                         T* __restrict__ y, const float* __restrict__ psum,
                                                         const float* __restrict__ psq, int P, int64_t M, int C,
                                                         int64_t rpb, StatsFin fin) {
  __shared__ double red[2][32][64];
  __shared__ float s_sc[64], s_sh[64];
  const int tid = threadIdx.x, cx = tid & 7, ry = tid >> 3;
  const int cb = blockIdx.x * 64, c0 = cb + cx * 8;
  // ---- finalize this block's 64 channels (fixed summation order: identical in every block)
  float a[8], b[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = b[j] = 0.f;
  for (int p = ry; p < P; p += 32) {
    const float4* ps = reinterpret_cast<const float4*>(psum + (int64_t)p * C + c0);
    const float4* pq = reinterpret_cast<const float4*>(psq + (int64_t)p * C + c0);
    const float4 s0 = ps[0], s1 = ps[1], q0 = pq[0], q1 = pq[1];
    a[0] += s0.x; a[1] += s0.y; a[2] += s0.z; a[3] += s0.w; a[4] += s1.x; a[5] += s1.y; a[6] += s1.z; a[7] += s1.w;
    b[0] += q0.x; b[1] += q0.y; b[2] += q0.z; b[3] += q0.w; b[4] += q1.x; b[5] += q1.y; b[6] += q1.z; b[7] += q1.w;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[0][ry][cx * 8 + j] = a[j];
    red[1][ry][cx * 8 + j] = b[j];
  }
  __syncthreads();
  if (tid < 64) {
    double sa = 0.0, sb = 0.0;
    for (int i = 0; i < 32; ++i) {
      sa += red[0][i][tid];
      sb += red[1][i][tid];
    }
    const int c = cb + tid;
    const double mean = sa / (double)M;
    double var = sb / (double)M - mean * mean;
    if (var < 0.0) var = 0.0;
    const float invstd = (float)(1.0 / sqrt(var + (double)fin.eps));
    const float w = fin.weight ? fin.weight[c] : 1.f;
    const float bb = fin.bias ? fin.bias[c] : 0.f;
    const float sc = w * invstd;
    s_sc[tid] = sc;
    s_sh[tid] = bb - (float)mean * sc;
    if (blockIdx.y == 0) {
      fin.save_mean[c] = (float)mean;
      fin.save_invstd[c] = invstd;
      if (fin.running_mean != nullptr) {
        const double unbiased = M > 1 ? var * (double)M / (double)(M - 1) : var;
        fin.running_mean[c] = (float)((1.0 - fin.momentum) * fin.running_mean[c] + fin.momentum * mean);
        fin.running_var[c] = (float)((1.0 - fin.momentum) * fin.running_var[c] + fin.momentum * unbiased);
      }
    }
  }
  __syncthreads();
  float sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = s_sc[cx * 8 + j];
    sh[j] = s_sh[cx * 8 + j];
  }
  // ---- apply rows [y*rpb, +rpb)
  const int64_t row1 = min(M, (int64_t)(blockIdx.y + 1) * rpb);
  for (int64_t row = (int64_t)blockIdx.y * rpb + ry; row < row1; row += 32) {
    const int64_t off = row * C + c0;
    float v[8], rr[8];
    Vec8<T>::load(x + off, v);
    if (RES) Vec8<T>::load(res + off, rr);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float t = fmaf(v[j], sc[j], sh[j]);
      if (RES) t += rr[j];
      if (ACT) t = fmaxf(t, 0.f);
      v[j] = t;
    }
    Vec8<T>::store(y + off, v);
  }
}

// grid C/8, block 256: 8 channels (one 16-byte vector per row) x all M <= 2048 rows.  Every
// thread loads its <= 8 rows of dy / x (/ y) ONCE, in one burst (all loads in flight), keeps
// them packed in registers across the block reduction and the in-block finalize, and writes
// dx from them: one memory round trip per tensor (a row loop re-reading the data was
// latency-bound: 47-100 us at M = 6272).
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
  if (tid < 8) {
    const int c = c0 + tid;
    const double a = ksum[0][tid], b = ksum[1][tid];
    const double mu = fin.mean[c], is = fin.invstd[c];
    const double sum_dz_xhat = is * (b - mu * a);
    if (fin.dweight) fin.dweight[c] = (float)sum_dz_xhat;
    if (fin.dbias) fin.dbias[c] = (float)a;
    const double g = fin.weight ? fin.weight[c] : 1.0;
    const double A = g * is;
    const double Bc = fin.training ? -A * is * sum_dz_xhat / (double)M : 0.0;
    const double Cc = fin.training ? -A * a / (double)M - Bc * mu : 0.0;
    kk[0][tid] = (float)A;
    kk[1][tid] = (float)Bc;
    kk[2][tid] = (float)Cc;
  }
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
      Vec8<T>::store(dx + off, xv);
      if (RES) Vec8<T>::store(dres + off, g);
    }
  }
}

int g_fin2 = 1;  // wide finalize on (bn_set_fin2: A/B against the one-level kernels)

// Wide finalize launch (false: not applicable — C % 16, or disabled)
template <bool BWD>
bool launch_fin_wide(const float* pa, const float* pb, int P, int C, int64_t M, const Fin2Fwd& ff, const BwdFin& bf,
                     float* kA, float* kB, float* kC, hipStream_t stream) {
  if (!g_fin2 || C % 16 != 0) return false;
  hipLaunchKernelGGL((bn_fin_wide_k<BWD>), dim3(C / 16), dim3(1024), 0, stream, pa, pb, P, C, M, ff, bf, kA, kB, kC);
  return true;
}

// small-M forward: finalize folded into the apply (returns false when the shape is not covered)
bool launch_fin_apply(int dtype, const void* x, const void* res, void* y, int64_t M, int C, const float* psum,
                      const float* psq, int P, const float* weight, const float* bias, float* running_mean,
                      float* running_var, float momentum, float eps, int act, float* save_mean, float* save_invstd,
                      hipStream_t stream) {
  if (g_bn_small == 0 || P > kSmallFinP || M > 2 * kSmallBwdM || C % 64 != 0 || (dtype != kBF16 && dtype != kF16))
    return false;
  const int groups = C / 64;
  int64_t R = (M + 127) / 128;  // >= 4 rows per thread-lane (32 lanes)
  const int64_t cap = 512 / groups > 0 ? 512 / groups : 1;
  if (R > cap) R = cap;
  if (R < 1) R = 1;
  const int64_t rpb = (M + R - 1) / R;
  R = (M + rpb - 1) / rpb;
  const StatsFin fin{weight, bias, running_mean, running_var, momentum, eps, save_mean, save_invstd};
  const dim3 grid(groups, (unsigned)R);
  HYP_DISPATCH_FLOAT(dtype, T, {
    const T* xt = static_cast<const T*>(x);
    const T* rt = static_cast<const T*>(res);
    T* yt = static_cast<T*>(y);
    if (act && res)
      hipLaunchKernelGGL((bn_fin_apply_k<T, true, true>), grid, dim3(kBlock), 0, stream, xt, rt, yt, psum, psq, P, M,
                         C, rpb, fin);
    else if (act)
      hipLaunchKernelGGL((bn_fin_apply_k<T, true, false>), grid, dim3(kBlock), 0, stream, xt, rt, yt, psum, psq, P, M,
                         C, rpb, fin);
    else if (res)
      hipLaunchKernelGGL((bn_fin_apply_k<T, false, true>), grid, dim3(kBlock), 0, stream, xt, rt, yt, psum, psq, P, M,
                         C, rpb, fin);
    else
      hipLaunchKernelGGL((bn_fin_apply_k<T, false, false>), grid, dim3(kBlock), 0, stream, xt, rt, yt, psum, psq, P,
                         M, C, rpb, fin);
  });
  return true;
}

// small-M backward: reduce + finalize + dx in one launch (false when not covered)
bool launch_bwd_small(int dtype, bool maskx, bool act, const void* dy, const void* x, const void* y, void* dx,
                      void* dres, int64_t M, int C, const BwdFin& fin, const float* bias, hipStream_t stream) {
  if (g_bn_small == 0 || M > (int64_t)kBwdRows * kBlock || C % 8 != 0 || (dtype != kBF16 && dtype != kF16))
    return false;
  const dim3 grid(C / 8);
  // 256 threads x 8 register-resident rows (M <= 2048: layer4).  Wider blocks for layer3's 6272
  // rows (512 x 13, 1024 x 8) spill VGPRs: that case keeps the 3-kernel path.
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

}  // namespace

// ======================================================================== host launchers
void bn_set_small_paths(int on) { g_bn_small = on ? 1 : 0; }

hipError_t bn_workspace_rows(int64_t M, int C, int* P_out) {
  BnGeom g;
  if (!bn_geom(M, C, kStatsBlocks, g)) return hipErrorInvalidValue;
  *P_out = g.P;
  return hipSuccess;
}

void bn_set_fin2(int on) { g_fin2 = on ? 1 : 0; }

hipError_t bn_forward(int dtype, const void* x, const void* res, void* y, int64_t M, int C, const float* weight,
                      const float* bias, float* running_mean, float* running_var, float momentum, float eps,
                      int training, int act, float* psum, float* psq, float* save_mean, float* save_invstd,
                      float* scale, float* shift, hipStream_t stream) {
  BnGeom gs, ga;
  if (!bn_geom(M, C, kStatsBlocks, gs) || !bn_geom(M, C, 2048, ga)) return hipErrorInvalidValue;
  HYP_DISPATCH_FLOAT(dtype, T, {
    const T* xt = static_cast<const T*>(x);
    if (training) {
      hipLaunchKernelGGL(bn_stats_partial_k<T>, dim3(gs.P, gs.gy), dim3(kBlock), 0, stream, xt, M, C, gs.tpr, gs.rpi,
                         gs.rows_per_block, psum, psq);
      if (launch_fin_apply(dtype, x, res, y, M, C, psum, psq, gs.P, weight, bias, running_mean, running_var, momentum,
                           eps, act, save_mean, save_invstd, stream))
        return hipGetLastError();
      const Fin2Fwd ff{weight, bias, running_mean, running_var, momentum, eps, save_mean, save_invstd, scale, shift};
      if (!launch_fin_wide<false>(psum, psq, gs.P, C, M, ff, BwdFin{}, nullptr, nullptr, nullptr, stream))
        hipLaunchKernelGGL(bn_stats_finalize_k, dim3((C + kFinCh - 1) / kFinCh), dim3(kFinCh, kFinGr), 0, stream, psum,
                           psq, gs.P, C, M, weight, bias, running_mean, running_var, momentum, eps, save_mean,
                           save_invstd, scale, shift);
    } else {
      hipLaunchKernelGGL(bn_eval_consts_k, dim3((C + 255) / 256), dim3(256), 0, stream, C, weight, bias, running_mean,
                         running_var, eps, save_mean, save_invstd, scale, shift);
    }
    const dim3 grid(ga.P, ga.gy);
    const T* rt = static_cast<const T*>(res);
    T* yt = static_cast<T*>(y);
    if (act && res)
      hipLaunchKernelGGL((bn_apply_k<T, true, true>), grid, dim3(kBlock), 0, stream, xt, rt, yt, scale, shift, M, C,
                         ga.tpr, ga.rpi, ga.rows_per_block);
    else if (act)
      hipLaunchKernelGGL((bn_apply_k<T, true, false>), grid, dim3(kBlock), 0, stream, xt, rt, yt, scale, shift, M, C,
                         ga.tpr, ga.rpi, ga.rows_per_block);
    else if (res)
      hipLaunchKernelGGL((bn_apply_k<T, false, true>), grid, dim3(kBlock), 0, stream, xt, rt, yt, scale, shift, M, C,
                         ga.tpr, ga.rpi, ga.rows_per_block);
    else
      hipLaunchKernelGGL((bn_apply_k<T, false, false>), grid, dim3(kBlock), 0, stream, xt, rt, yt, scale, shift, M, C,
                         ga.tpr, ga.rpi, ga.rows_per_block);
  });
  return hipGetLastError();
}

template <typename T>
void launch_bn_dx(bool maskx, bool act, bool res, dim3 grid, hipStream_t stream, const T* dy, const T* x, const T* y,
                  T* dx, T* dres, const float* kA, const float* kB, const float* kC, int64_t M, int C,
                  const BnGeom& ga, const float* w, const float* b, const float* mean, const float* invstd) {
#define HYP_BN_DX(ACTV, RESV, MX)                                                                                 \
  hipLaunchKernelGGL((bn_bwd_dx_k<T, ACTV, RESV, MX>), grid, dim3(kBlock), 0, stream, dy, x, y, dx, dres, kA, kB, \
                     kC, M, C, ga.tpr, ga.rpi, ga.rows_per_block, w, b, mean, invstd)
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
                       int training, int act, float* pdz, float* pdzx, float* dweight, float* dbias, float* kA,
                       float* kB, float* kC, hipStream_t stream) {
  BnGeom gs, ga;
  if (!bn_geom(M, C, kStatsBlocks, gs) || !bn_geom(M, C, 2048, ga)) return hipErrorInvalidValue;
  // act with no forward output given: recompute the ReLU mask from x (training stats only: the
  // eval-mode constants are running stats, which the mask recomputation below does not model)
  const bool maskx = act && y == nullptr;
  if (maskx && (!training || dres != nullptr)) return hipErrorInvalidValue;
  if (launch_bwd_small(dtype, maskx, act != 0, dy, x, y, dx, dres, M, C,
                       BwdFin{weight, save_mean, save_invstd, training, dweight, dbias}, bias, stream))
    return hipGetLastError();
  HYP_DISPATCH_FLOAT(dtype, T, {
    const T* dyt = static_cast<const T*>(dy);
    const T* xt = static_cast<const T*>(x);
    const T* yt = static_cast<const T*>(y);
    const dim3 grs(gs.P, gs.gy);
    if (maskx)
      hipLaunchKernelGGL((bn_bwd_reduce_k<T, true, true>), grs, dim3(kBlock), 0, stream, dyt, xt, yt, M, C, gs.tpr,
                         gs.rpi, gs.rows_per_block, pdz, pdzx, weight, bias, save_mean, save_invstd);
    else if (act)
      hipLaunchKernelGGL((bn_bwd_reduce_k<T, true, false>), grs, dim3(kBlock), 0, stream, dyt, xt, yt, M, C, gs.tpr,
                         gs.rpi, gs.rows_per_block, pdz, pdzx, weight, bias, save_mean, save_invstd);
    else
      hipLaunchKernelGGL((bn_bwd_reduce_k<T, false, false>), grs, dim3(kBlock), 0, stream, dyt, xt, yt, M, C, gs.tpr,
                         gs.rpi, gs.rows_per_block, pdz, pdzx, weight, bias, save_mean, save_invstd);
    const BwdFin bf{weight, save_mean, save_invstd, training, dweight, dbias};
    if (!launch_fin_wide<true>(pdz, pdzx, gs.P, C, M, Fin2Fwd{}, bf, kA, kB, kC, stream))
      hipLaunchKernelGGL(bn_bwd_finalize_k, dim3((C + kFinCh - 1) / kFinCh), dim3(kFinCh, kFinGr), 0, stream, pdz,
                         pdzx, gs.P, C, M, weight, save_mean, save_invstd, training, dweight, dbias, kA, kB, kC);
    launch_bn_dx<T>(maskx, act, dres != nullptr, dim3(ga.P, ga.gy), stream, dyt, xt, yt, static_cast<T*>(dx),
                    static_cast<T*>(dres), kA, kB, kC, M, C, ga, weight, bias, save_mean, save_invstd);
  });
  return hipGetLastError();
}

}  // namespace hyp

namespace hyp {
// Training-mode BN forward whose per-channel partial sums were produced elsewhere (the conv
// epilogue of conv_igemm.hip: one partial row per M-tile) — finalize + apply only, no statistics
// pass over x.
hipError_t bn_forward_from_partials(int dtype, const void* x, const void* res, void* y, int64_t M, int C,
                                    const float* weight, const float* bias, float* running_mean, float* running_var,
                                    float momentum, float eps, int act, const float* psum, const float* psq, int P,
                                    float* save_mean, float* save_invstd, float* scale, float* shift,
                                    hipStream_t stream) {
  BnGeom ga;
  if (!bn_geom(M, C, 2048, ga)) return hipErrorInvalidValue;
  if (launch_fin_apply(dtype, x, res, y, M, C, psum, psq, P, weight, bias, running_mean, running_var, momentum, eps,
                       act, save_mean, save_invstd, stream))
    return hipGetLastError();
  const Fin2Fwd ff{weight, bias, running_mean, running_var, momentum, eps, save_mean, save_invstd, scale, shift};
  if (!launch_fin_wide<false>(psum, psq, P, C, M, ff, BwdFin{}, nullptr, nullptr, nullptr, stream))
    hipLaunchKernelGGL(bn_stats_finalize_k, dim3((C + kFinCh - 1) / kFinCh), dim3(kFinCh, kFinGr), 0, stream, psum,
                       psq, P, C, M, weight, bias, running_mean, running_var, momentum, eps, save_mean, save_invstd,
                       scale, shift);
  HYP_DISPATCH_FLOAT(dtype, T, {
    const T* xt = static_cast<const T*>(x);
    const T* rt = static_cast<const T*>(res);
    T* yt = static_cast<T*>(y);
    const dim3 grid(ga.P, ga.gy);
    if (act && res)
      hipLaunchKernelGGL((bn_apply_k<T, true, true>), grid, dim3(kBlock), 0, stream, xt, rt, yt, scale, shift, M, C,
                         ga.tpr, ga.rpi, ga.rows_per_block);
    else if (act)
      hipLaunchKernelGGL((bn_apply_k<T, true, false>), grid, dim3(kBlock), 0, stream, xt, rt, yt, scale, shift, M, C,
                         ga.tpr, ga.rpi, ga.rows_per_block);
    else if (res)
      hipLaunchKernelGGL((bn_apply_k<T, false, true>), grid, dim3(kBlock), 0, stream, xt, rt, yt, scale, shift, M, C,
                         ga.tpr, ga.rpi, ga.rows_per_block);
    else
      hipLaunchKernelGGL((bn_apply_k<T, false, false>), grid, dim3(kBlock), 0, stream, xt, rt, yt, scale, shift, M, C,
                         ga.tpr, ga.rpi, ga.rows_per_block);
  });
  return hipGetLastError();
}
}  // namespace hyp

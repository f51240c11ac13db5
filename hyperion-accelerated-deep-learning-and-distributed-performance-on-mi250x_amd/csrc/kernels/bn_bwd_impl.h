// BatchNorm backward dx pass device code (the design is described in bn_act.hip): shared by
// bn_act.hip (the plain launches) and bn_wgrad.hip (the dx pass horizontally fused with the
// previous layer's weight gradient).  Anonymous namespace: each including TU instantiates what it
// launches.
#pragma once
#include "hyp_common.h"
#include "hyp_kernels.h"
#include "bn_fin.h"

namespace hyp {
namespace {

constexpr int kBlock = 256;
constexpr int kStatsBlocks = 512;  // row blocks of the statistics kernels (= atomic adders per channel)
constexpr int kFinCh = 256;        // channels per apply / dx block: one inline-finalized channel per thread
constexpr int kApplyBlocks = 2048;


struct BnGeom {
  int tpr;   // threads per row (each owns 8 channels)
  int rpi;   // rows per block-iteration
  int gy;    // channel chunks (grid.y)
  int P;     // row blocks (grid.x)
  int64_t rows_per_block;
};

// max_tpr: channel-vectors per block row (the apply / dx kernels cap a block at kFinCh channels,
// so their inline finalize is one channel per thread)
bool bn_geom(int64_t M, int C, int max_blocks, BnGeom& g, int max_tpr = kBlock, int min_iters = 4) {
  if (C % 8 != 0) return false;
  const int cv = C / 8;
  if (cv <= max_tpr) {
    g.tpr = cv;
    g.gy = 1;
  } else {
    if (cv % max_tpr != 0) return false;
    g.tpr = max_tpr;
    g.gy = cv / max_tpr;
  }
  g.rpi = kBlock / g.tpr;
  // >= 4 row iterations per thread, and >= 16K elements per block so each block's atomics are a
  // tiny fraction of its traffic
  int64_t min_rows = (int64_t)g.rpi * min_iters;
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

// the apply / dx passes' grid: <= bn_apply_blocks() row blocks, >= bn_min_iters() row iterations
// per thread (bn_set_geom: A/B sweeps; defaults kApplyBlocks and 4)
bool apply_geom(int64_t M, int C, BnGeom& g) { return bn_geom(M, C, bn_apply_blocks(), g, kFinCh / 8, bn_min_iters()); }

struct BwdFin {
  const float* weight;
  const float* mean;
  const float* invstd;
  int training;
  float* dweight;
  float* dbias;
  const double* sums;  // [kStatSlots][2][C]: Σdz, Σdz·x (the reduce + dx path)
  double invM;         // 1 / M
};

// dx = A·dz + B·x + C coefficients of channel c from a = Σdz, b = Σdz·x (fp64)
__device__ __forceinline__ void bwd_coeffs(const BwdFin& f, int c, double a, double b, bool writer, float& A,
                                           float& B, float& Cc) {
  const double mu = f.mean[c], is = f.invstd[c];
  const double sum_dz_xhat = is * (b - mu * a);
  if (writer) {
    if (f.dweight) f.dweight[c] = (float)sum_dz_xhat;
    if (f.dbias) f.dbias[c] = (float)a;
  }
  const double g = f.weight ? f.weight[c] : 1.0;
  const double Ad = g * is;
  const double Bd = f.training ? -Ad * is * sum_dz_xhat * f.invM : 0.0;
  const double Cd = f.training ? -Ad * a * f.invM - Bd * mu : 0.0;
  A = (float)Ad;
  B = (float)Bd;
  Cc = (float)Cd;
}

// ReLU mask of the forward output.  MASKX: recomputed from x as x*scale + shift > 0 with the
// forward's exact float scale/shift (fwd_const1's arithmetic), so the non-residual backward
// never reads y (one stream less).
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

// dx = A·dz + B·x + C with the coefficients finalized inline from the Σdz, Σdz·x sums (block 0
// writes dγ, dβ).  Without ACT, dy is already dz (masked — e.g. by the dgrad epilogue that
// produced it), and the residual gradient IS dy: RES only matters for the masking variants.
// The workgroup body: (bx, by) = its (row block, channel chunk) — blockIdx of a plain launch, a
// remapped id in bn_wgrad.hip's fused launch.
template <typename T, bool ACT, bool RES, bool MASKX>
__device__ __forceinline__ void bn_bwd_dx_body(const T* __restrict__ dy, const T* __restrict__ x,
                                               const T* __restrict__ y, T* __restrict__ dx, T* __restrict__ dres,
                                               const BwdFin& fin, int64_t M, int C, int tpr, int rpi, int64_t rpb,
                                               const float* __restrict__ bn_b, const int bx, const int by) {
  __shared__ float kk[3][kFinCh];
  const int tid = threadIdx.x;
  const int r = tid / tpr, c8 = tid - r * tpr;
  {  // this block's <= kFinCh channels, one per thread (block x == 0 also writes dγ, dβ)
    const int nch = tpr * 8, c = by * nch + tid;
    if (tid < nch) {
      double a = 0.0, b = 0.0;
#pragma unroll
      for (int k = 0; k < kStatSlots; ++k) {  // fixed order
        a += fin.sums[(int64_t)k * 2 * C + c];
        b += fin.sums[(int64_t)k * 2 * C + C + c];
      }
      bwd_coeffs(fin, c, a, b, bx == 0, kk[0][tid], kk[1][tid], kk[2][tid]);
    }
  }
  __syncthreads();
  if (r >= rpi) return;
  const int c0 = by * tpr * 8 + c8 * 8;
  ReluMask<T, ACT, MASKX> mk;
  mk.init(fin.weight, bn_b, fin.mean, fin.invstd, c0);
  float A[8], B[8], Cc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    A[j] = kk[0][c8 * 8 + j];
    B[j] = kk[1][c8 * 8 + j];
    Cc[j] = kk[2][c8 * 8 + j];
  }
  const int64_t row0 = (int64_t)bx * rpb;
  const int64_t row1 = min(M, row0 + rpb);
  const int64_t step = (int64_t)rpi * C;
  int64_t off = (row0 + r) * C + c0;
  int64_t row = row0 + r;
  auto one = [&](const float (&gi)[8], const float (&xi)[8], const float (&yi)[8], int64_t o) {
    float g[8], xo[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float d = mk.keep(xi, yi, j) ? gi[j] : 0.f;
      g[j] = d;
      xo[j] = fmaf(A[j], d, fmaf(B[j], xi[j], Cc[j]));
    }
    Vec8<T>::store_wt(dx + o, xo);
    if (RES) Vec8<T>::store_wt(dres + o, g);
  };
  for (; row + rpi < row1; row += 2 * rpi, off += 2 * step) {  // two rows' loads in flight
    float g0[8], x0[8], y0[8], g1[8], x1[8], y1[8];
    Vec8<T>::load(dy + off, g0);
    Vec8<T>::load(dy + off + step, g1);
    Vec8<T>::load(x + off, x0);
    Vec8<T>::load(x + off + step, x1);
    if (ACT && !MASKX) {
      Vec8<T>::load(y + off, y0);
      Vec8<T>::load(y + off + step, y1);
    }
    one(g0, x0, y0, off);
    one(g1, x1, y1, off + step);
  }
  if (row < row1) {
    float g[8], xv[8], yv[8];
    Vec8<T>::load(dy + off, g);
    Vec8<T>::load(x + off, xv);
    if (ACT && !MASKX) Vec8<T>::load(y + off, yv);
    one(g, xv, yv, off);
  }
}

template <typename T, bool ACT, bool RES, bool MASKX>
__global__ __launch_bounds__(kBlock) void bn_bwd_dx_k(const T* __restrict__ dy, const T* __restrict__ x,
                                                      const T* __restrict__ y, T* __restrict__ dx,
                                                      T* __restrict__ dres, BwdFin fin, int64_t M, int C, int tpr,
                                                      int rpi, int64_t rpb, const float* __restrict__ bn_b) {
  bn_bwd_dx_body<T, ACT, RES, MASKX>(dy, x, y, dx, dres, fin, M, C, tpr, rpi, rpb, bn_b, blockIdx.x, blockIdx.y);
}

}  // namespace
}  // namespace hyp

// LayerNorm / RMSNorm forward + backward (optionally fused with a residual add) for gfx950.
//
// Replaces PyTorch's layer_norm kernels inside every nn.TransformerEncoderLayer of the reference
// (post-norm, two per layer: SimpleTransformerLM C14/C15, CustomTransformer C5) and HF Llama's
// eager RMSNorm (C26) — SURVEY §2.4 rows LayerNorm, RMSNorm.
//
// One row per wave64 for d <= 2048 (each lane owns d/64 contiguous-in-chunks elements loaded as
// 16-byte vectors), row statistics by __shfl_xor reductions only (no LDS, no block barrier).
// Forward saves mean and rstd (fp32).  The fused form computes  s = x + r  and  y = LN(s),
// writing s as well (it is the next residual stream and the backward input).
// Backward: dx per row in the same wave; dγ/dβ as deterministic per-block partial sums followed
// by a column reduction kernel.
#include "hyp_common.h"
#include "hyp_kernels.h"

namespace hyp {
namespace {

constexpr int kWavesPerBlock = 4;
// wave-count target of the narrow-row forward / backward grids (0: the defaults of
// ln_fwd_dispatch / layernorm_bwd_geom; ln_set_waves: A/B sweeps)
int g_ln_waves = 0;

// Each lane handles VPL vectors of 8 elements: lane l, vector v covers [ (v*64 + l)*8, +8 ).
// Latency structure (the kernels are HBM-bound only when enough loads are in flight): the affine
// parameters are loaded ONCE per lane before the first row, and every wave walks `rpw` rows with
// the NEXT row's 16-byte vectors already in flight while the current row is reduced and written
// (register double buffering).  One row per wave with w/b fetched after the row statistics cost
// three dependent memory round trips per row: 26 us for a [6304, 768] bf16 LN on MI355X.
template <typename T, int VPL>
struct RowRegs {
  static constexpr int kQ = sizeof(T) / 2;  // 16-byte quads per 8-element vector (2-byte T: 1, fp32: 2)
  uint4 v[VPL][kQ];
  __device__ __forceinline__ void load(const T* base, int64_t row, int d, int lane) {
#pragma unroll
    for (int k = 0; k < VPL; ++k) {
      const int c = (k * 64 + lane) * 8;
#pragma unroll
      for (int q = 0; q < kQ; ++q)
        v[k][q] = c < d ? reinterpret_cast<const uint4*>(base + row * d + c)[q] : uint4{0u, 0u, 0u, 0u};
    }
  }
  __device__ __forceinline__ void unpack(int k, float (&o)[8]) const { Vec8<T>::load(reinterpret_cast<const T*>(&v[k][0]), o); }
};

// 8 affine values from p + c: fp32, or (wt) in the activation dtype T — a module cast wholesale to
// bf16 (FSDP mixed precision, HF-style Llama) hands over bf16 weights; reading them as such saves
// the two cast kernels per LayerNorm per direction the fp32-only interface cost
template <typename T>
__device__ __forceinline__ void affine8(const float* p, int wt, int c, float (&o)[8]) {
  if (wt) {
    Vec8<T>::load(reinterpret_cast<const T*>(p) + c, o);
  } else {
    const float4 a = reinterpret_cast<const float4*>(p + c)[0];
    const float4 b = reinterpret_cast<const float4*>(p + c)[1];
    o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w;
    o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
  }
}

template <typename T, int VPL>
__device__ __forceinline__ void load_affine(const float* p, int wt, int d, int lane, float (&o)[VPL][8], float dflt) {
#pragma unroll
  for (int k = 0; k < VPL; ++k) {
    const int c = (k * 64 + lane) * 8;
    if (p != nullptr && c < d) {
      affine8<T>(p, wt, c, o[k]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) o[k][j] = dflt;
    }
  }
}

// Dropout on the residual branch (DROP, post-norm transformer layers: s = r + dropout(x)): the keep
// mask is regenerated from the counter-based hash of dropout.hip (same key, element index row·d +
// col), so fwd, bwd and an unfused dropout kernel with the same state draw identical masks.
struct LnDrop {
  uint32_t thr;  // keep iff rng_u32(key, index) >= thr
  float scale;   // 1 / (1 - p)
  RngState rs;
};

template <typename T, int VPL, bool RMS, bool HAS_RES, bool DROP = false>
__global__ __launch_bounds__(64 * kWavesPerBlock) void ln_fwd_k(const T* __restrict__ x, const T* __restrict__ r,
                                                                  T* __restrict__ s_out, T* __restrict__ y,
                                                                  const float* __restrict__ w,
                                                                  const float* __restrict__ b, float* __restrict__ mean_out,
                                                                  float* __restrict__ rstd_out, int64_t rows, int d,
                                                                  float eps, int rpw, int wt, LnDrop dp = LnDrop{}) {
  const int lane = threadIdx.x & 63;
  const uint64_t dkey = DROP ? rng_key(dp.rs) : 0;
  const int64_t row0 = ((int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * rpw;
  if (row0 >= rows) return;
  float wv[VPL][8], bv[VPL][8];
  load_affine<T, VPL>(w, wt, d, lane, wv, 1.f);
  load_affine<T, VPL>(RMS ? nullptr : b, wt, d, lane, bv, 0.f);
  RowRegs<T, VPL> cx, cr, nx, nr;
  cx.load(x, row0, d, lane);
  if (HAS_RES) cr.load(r, row0, d, lane);
  for (int i = 0; i < rpw; ++i) {
    const int64_t row = row0 + i;
    if (row >= rows) break;
    const bool more = i + 1 < rpw && row + 1 < rows;
    if (more) {  // the next row's vectors in flight during this row's work
      nx.load(x, row + 1, d, lane);
      if (HAS_RES) nr.load(r, row + 1, d, lane);
    }
    float v[VPL][8];
    float sum = 0.f;
#pragma unroll
    for (int k = 0; k < VPL; ++k) {
      const int c = (k * 64 + lane) * 8;
      cx.unpack(k, v[k]);
      if (HAS_RES && c < d) {
        float rv[8];
        cr.unpack(k, rv);
        if (DROP) {  // the dropped branch in T, as a separate dropout kernel would have stored it
#pragma unroll
          for (int j = 0; j < 8; ++j)
            v[k][j] = rng_u32(dkey, (uint64_t)(row * d + c + j)) >= dp.thr ? rnd<T>(v[k][j] * dp.scale) : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) v[k][j] = rnd<T>(v[k][j] + rv[j]);  // stats of the stored stream
        Vec8<T>::store(s_out + row * d + c, v[k]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) sum += v[k][j];  // zero-filled past d
    }
    float mean = 0.f;
    if (!RMS) mean = wave_sum(sum) / d;
    float sq = 0.f;
#pragma unroll
    for (int k = 0; k < VPL; ++k) {
      const int c = (k * 64 + lane) * 8;
      if (c < d) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float t = v[k][j] - mean;
          sq += t * t;
        }
      }
    }
    const float rstd = rsqrtf(wave_sum(sq) / d + eps);
    if (lane == 0) {
      if (mean_out) mean_out[row] = mean;
      rstd_out[row] = rstd;
    }
#pragma unroll
    for (int k = 0; k < VPL; ++k) {
      const int c = (k * 64 + lane) * 8;
      if (c < d) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (v[k][j] - mean) * rstd * wv[k][j] + bv[k][j];
        Vec8<T>::store(y + row * d + c, o);
      }
    }
    if (more) {
      cx = nx;
      if (HAS_RES) cr = nr;
    }
  }
}

// dx and per-block partial dγ, dβ.  grid.x = ceil(rows / (kWavesPerBlock * rows_per_wave))
// DROP: also dxa = dropout(dx) with the forward's mask — the gradient of the dropped branch (the
// residual branch gets dx itself): the separate dropout-backward pass over dx disappears.
// BSUM: also the column sums of the branch gradient as stored (dxa, or dx) — the bias gradient of
// the linear layer whose output is this norm's input (ops/layernorm.py BiasGradLink): a third
// partial segment [P][.. | d] combined in the same launch as dγ / dβ (no column-sum passes).
template <typename T, int VPL, bool RMS, bool HAS_DRES, bool DROP = false, bool BSUM = false>
__global__ __launch_bounds__(64 * kWavesPerBlock) void ln_bwd_k(const T* __restrict__ dy, const T* __restrict__ xin,
                                                                  const float* __restrict__ w,
                                                                  const float* __restrict__ mean_in,
                                                                  const float* __restrict__ rstd_in,
                                                                  const T* __restrict__ dres, T* __restrict__ dx,
                                                                  float* __restrict__ pdw, float* __restrict__ pdb,
                                                                  int64_t rows, int d, int rows_per_wave, int wt,
                                                                  T* __restrict__ dxa = nullptr, LnDrop dp = LnDrop{},
                                                                  int bs_off = 0) {
  const int lane = threadIdx.x & 63;
  const uint64_t dkey = DROP ? rng_key(dp.rs) : 0;
  const int wid = threadIdx.x >> 6;
  float gw[VPL][8], gb[VPL][8], wv[VPL][8], gs[BSUM ? VPL : 1][8];
#pragma unroll
  for (int k = 0; k < VPL; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) gw[k][j] = gb[k][j] = 0.f;
  if constexpr (BSUM) {
#pragma unroll
    for (int k = 0; k < VPL; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) gs[k][j] = 0.f;
  }
  load_affine<T, VPL>(w, wt, d, lane, wv, 1.f);

  const int64_t row_begin = ((int64_t)blockIdx.x * kWavesPerBlock + wid) * rows_per_wave;
  RowRegs<T, VPL> cg, cxr, cd, ng, nxr, nd;
  if (row_begin < rows) {
    cg.load(dy, row_begin, d, lane);
    cxr.load(xin, row_begin, d, lane);
    if (HAS_DRES) cd.load(dres, row_begin, d, lane);
  }
  for (int rr = 0; rr < rows_per_wave; ++rr) {
    const int64_t row = row_begin + rr;
    if (row >= rows) break;
    const bool more = rr + 1 < rows_per_wave && row + 1 < rows;
    if (more) {  // next row in flight
      ng.load(dy, row + 1, d, lane);
      nxr.load(xin, row + 1, d, lane);
      if (HAS_DRES) nd.load(dres, row + 1, d, lane);
    }
    const float mean = RMS ? 0.f : mean_in[row];
    const float rstd = rstd_in[row];
    float g[VPL][8], xh[VPL][8];
    float s1 = 0.f, s2 = 0.f;  // Σ g·w, Σ g·w·xhat
#pragma unroll
    for (int k = 0; k < VPL; ++k) {
      const int c = (k * 64 + lane) * 8;
      cg.unpack(k, g[k]);
      if (c < d) {
        float xv[8];
        cxr.unpack(k, xv);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xh[k][j] = (xv[j] - mean) * rstd;
          const float gwv = g[k][j] * wv[k][j];
          s1 += gwv;
          s2 += gwv * xh[k][j];
          gw[k][j] += g[k][j] * xh[k][j];
          gb[k][j] += g[k][j];
        }
      }
    }
    s1 = wave_sum(s1) / d;
    s2 = wave_sum(s2) / d;
#pragma unroll
    for (int k = 0; k < VPL; ++k) {
      const int c = (k * 64 + lane) * 8;
      if (c < d) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = rstd * (g[k][j] * wv[k][j] - (RMS ? 0.f : s1) - xh[k][j] * s2);
        if (HAS_DRES) {
          float rv[8];
          cd.unpack(k, rv);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] += rv[j];
        }
        Vec8<T>::store(dx + row * d + c, o);
        if (DROP) {
          float oa[8];
#pragma unroll
          for (int j = 0; j < 8; ++j)
            oa[j] = rng_u32(dkey, (uint64_t)(row * d + c + j)) >= dp.thr ? rnd<T>(o[j]) * dp.scale : 0.f;
          Vec8<T>::store(dxa + row * d + c, oa);
          if constexpr (BSUM) {
#pragma unroll
            for (int j = 0; j < 8; ++j) gs[k][j] += rnd<T>(oa[j]);  // the stored (rounded) values
          }
        } else if constexpr (BSUM) {
#pragma unroll
          for (int j = 0; j < 8; ++j) gs[k][j] += rnd<T>(o[j]);
        }
      }
    }
    if (more) {
      cg = ng;
      cxr = nxr;
      if (HAS_DRES) cd = nd;
    }
  }
  // block partials of dγ/dβ through LDS: [wave][d]
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sw = smem;
  float* sb = smem + kWavesPerBlock * d;
  float* ss = smem + 2 * kWavesPerBlock * d;  // BSUM
#pragma unroll
  for (int k = 0; k < VPL; ++k) {
    const int c = (k * 64 + lane) * 8;
    if (c < d) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sw[wid * d + c + j] = gw[k][j];
        sb[wid * d + c + j] = gb[k][j];
        if constexpr (BSUM) ss[wid * d + c + j] = gs[k][j];
      }
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < d; c += 64 * kWavesPerBlock) {
    float a = 0.f, bb = 0.f, sa = 0.f;
#pragma unroll
    for (int q = 0; q < kWavesPerBlock; ++q) {
      a += sw[q * d + c];
      bb += sb[q * d + c];
      if constexpr (BSUM) sa += ss[q * d + c];
    }
    // partial rows [P][d] (dγ only) or [P][2d] (dγ | dβ: one combine pass for both), + d (BSUM:
    // the branch-gradient sums at column bs_off)
    const int64_t ps = (pdb ? 2 * (int64_t)d : d) + (BSUM ? d : 0);
    pdw[(int64_t)blockIdx.x * ps + c] = a;
    if (pdb) pdb[(int64_t)blockIdx.x * ps + c] = bb;
    if constexpr (BSUM) pdw[(int64_t)blockIdx.x * ps + bs_off + c] = sa;
  }
}

// ---- wide rows (2048 < d <= 4096: Llama-2-7B's 4096) ------------------------------------------
// One 256-thread block per row (4 waves x 64 lanes x VW vectors of 8): at one row per wave the
// backward's register image of a 4096-wide row (dy, x, dres, their prefetch, dγ/dβ and the affine:
// ~1 KB per lane) spilled 788 B/lane to scratch — 40-47 us per [128, 4096] RMSNorm backward on
// MI355X, 2.7 ms of a Llama-2-7B LoRA step.  Here a lane holds VW <= 2 vectors per tensor, the row
// statistics are a wave shuffle + a 4-wave LDS combine, and dγ/dβ partials are per-thread columns
// written straight to the block's partial row (no LDS transpose).
constexpr int kWideThreads = 256;

template <typename T, int VW>
__device__ __forceinline__ void wide_load(const T* base, int64_t row, int d, int tid, float (&o)[VW][8]) {
#pragma unroll
  for (int k = 0; k < VW; ++k) {
    const int c = (k * kWideThreads + tid) * 8;
    if (c < d) {
      Vec8<T>::load(base + row * d + c, o[k]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) o[k][j] = 0.f;
    }
  }
}

template <typename T, int VW>
__device__ __forceinline__ void wide_affine(const float* p, int wt, int d, int tid, float (&o)[VW][8], float dflt) {
#pragma unroll
  for (int k = 0; k < VW; ++k) {
    const int c = (k * kWideThreads + tid) * 8;
    if (p != nullptr && c < d) {
      affine8<T>(p, wt, c, o[k]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) o[k][j] = dflt;
    }
  }
}

// two block sums at once (one LDS round): red holds 2 x 4 floats
__device__ __forceinline__ float2 block_sum2(float a, float b, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  a = wave_sum(a);
  b = wave_sum(b);
  __syncthreads();  // the previous row's readers are done with red
  if (lane == 0) {
    red[wid] = a;
    red[4 + wid] = b;
  }
  __syncthreads();
  return make_float2((red[0] + red[1]) + (red[2] + red[3]), (red[4] + red[5]) + (red[6] + red[7]));
}

template <typename T, int VW, bool RMS, bool HAS_RES>
__global__ __launch_bounds__(kWideThreads) void ln_fwd_wide_k(const T* __restrict__ x, const T* __restrict__ r,
                                                              T* __restrict__ s_out, T* __restrict__ y,
                                                              const float* __restrict__ w, const float* __restrict__ b,
                                                              float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                              int64_t rows, int d, float eps, int rpb, int wt) {
  __shared__ float red[8];
  const int tid = threadIdx.x;
  float wv[VW][8], bv[VW][8];
  wide_affine<T, VW>(w, wt, d, tid, wv, 1.f);
  wide_affine<T, VW>(RMS ? nullptr : b, wt, d, tid, bv, 0.f);
  for (int i = 0; i < rpb; ++i) {
    const int64_t row = (int64_t)blockIdx.x * rpb + i;
    if (row >= rows) break;
    float v[VW][8];
    wide_load<T, VW>(x, row, d, tid, v);
    if (HAS_RES) {
      float rv[VW][8];
      wide_load<T, VW>(r, row, d, tid, rv);
#pragma unroll
      for (int k = 0; k < VW; ++k) {
        const int c = (k * kWideThreads + tid) * 8;
#pragma unroll
        for (int j = 0; j < 8; ++j) v[k][j] = rnd<T>(v[k][j] + rv[k][j]);  // stats of the stored stream
        if (c < d) Vec8<T>::store(s_out + row * d + c, v[k]);
      }
    }
    // two passes like the narrow kernel: the mean, then Σ(x - mean)² (zero-filled lanes past d
    // are excluded from the second)
    float mean = 0.f;
    if (!RMS) {
      float s1 = 0.f;
#pragma unroll
      for (int k = 0; k < VW; ++k)
#pragma unroll
        for (int j = 0; j < 8; ++j) s1 += v[k][j];
      mean = block_sum2(s1, 0.f, red).x / d;
    }
    float s2 = 0.f;
#pragma unroll
    for (int k = 0; k < VW; ++k) {
      if ((k * kWideThreads + tid) * 8 < d) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float tt = v[k][j] - mean;
          s2 += tt * tt;
        }
      }
    }
    const float rstd = rsqrtf(block_sum2(s2, 0.f, red).x / d + eps);
    if (tid == 0) {
      if (mean_out) mean_out[row] = mean;
      rstd_out[row] = rstd;
    }
#pragma unroll
    for (int k = 0; k < VW; ++k) {
      const int c = (k * kWideThreads + tid) * 8;
      if (c < d) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (v[k][j] - mean) * rstd * wv[k][j] + bv[k][j];
        Vec8<T>::store(y + row * d + c, o);
      }
    }
  }
}

template <typename T, int VW, bool RMS, bool HAS_DRES>
__global__ __launch_bounds__(kWideThreads) void ln_bwd_wide_k(const T* __restrict__ dy, const T* __restrict__ xin,
                                                              const float* __restrict__ w,
                                                              const float* __restrict__ mean_in,
                                                              const float* __restrict__ rstd_in,
                                                              const T* __restrict__ dres, T* __restrict__ dx,
                                                              float* __restrict__ pdw, float* __restrict__ pdb,
                                                              int64_t rows, int d, int rpb, int wt) {
  __shared__ float red[8];
  const int tid = threadIdx.x;
  float gw[VW][8], gb[VW][8], wv[VW][8];
#pragma unroll
  for (int k = 0; k < VW; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) gw[k][j] = gb[k][j] = 0.f;
  wide_affine<T, VW>(w, wt, d, tid, wv, 1.f);
  for (int i = 0; i < rpb; ++i) {
    const int64_t row = (int64_t)blockIdx.x * rpb + i;
    if (row >= rows) break;
    const float mean = RMS ? 0.f : mean_in[row];
    const float rstd = rstd_in[row];
    float g[VW][8], xh[VW][8];
    wide_load<T, VW>(dy, row, d, tid, g);
    wide_load<T, VW>(xin, row, d, tid, xh);
    float s1 = 0.f, s2 = 0.f;  // Σ g·w, Σ g·w·xhat
#pragma unroll
    for (int k = 0; k < VW; ++k) {
      const int c = (k * kWideThreads + tid) * 8;
      if (c < d) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xh[k][j] = (xh[k][j] - mean) * rstd;
          const float gwv = g[k][j] * wv[k][j];
          s1 += gwv;
          s2 += gwv * xh[k][j];
          gw[k][j] += g[k][j] * xh[k][j];
          gb[k][j] += g[k][j];
        }
      }
    }
    const float2 t = block_sum2(s1, s2, red);
    const float m1 = t.x / d, m2 = t.y / d;
#pragma unroll
    for (int k = 0; k < VW; ++k) {
      const int c = (k * kWideThreads + tid) * 8;
      if (c < d) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = rstd * (g[k][j] * wv[k][j] - (RMS ? 0.f : m1) - xh[k][j] * m2);
        if (HAS_DRES) {
          float rv[8];
          Vec8<T>::load(dres + row * d + c, rv);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] += rv[j];
        }
        Vec8<T>::store(dx + row * d + c, o);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < VW; ++k) {
    const int c = (k * kWideThreads + tid) * 8;
    if (c < d) {
      const int64_t ps = pdb ? 2 * (int64_t)d : d;  // [P][d] or [P][2d] (dγ | dβ)
      float4* pw = reinterpret_cast<float4*>(pdw + (int64_t)blockIdx.x * ps + c);
      pw[0] = make_float4(gw[k][0], gw[k][1], gw[k][2], gw[k][3]);
      pw[1] = make_float4(gw[k][4], gw[k][5], gw[k][6], gw[k][7]);
      if (pdb) {
        float4* pb = reinterpret_cast<float4*>(pdb + (int64_t)blockIdx.x * ps + c);
        pb[0] = make_float4(gb[k][0], gb[k][1], gb[k][2], gb[k][3]);
        pb[1] = make_float4(gb[k][4], gb[k][5], gb[k][6], gb[k][7]);
      }
    }
  }
}

// rows per block of the wide kernels: >= 1 block per row up to 1024 blocks
int wide_rows_per_block(int64_t rows) { return (int)((rows + 1023) / 1024); }

template <typename T, bool RMS>
hipError_t ln_fwd_dispatch(const T* x, const T* r, T* s, T* y, const float* w, const float* b, float* mean,
                           float* rstd, int64_t rows, int d, float eps, hipStream_t st, int wt, const LnDrop* drop) {
  if (drop != nullptr && (d > 2048 || r == nullptr)) return hipErrorInvalidValue;
  if (d > 2048) {
    const int rpb = wide_rows_per_block(rows);
    const dim3 grid((unsigned)((rows + rpb - 1) / rpb)), block(kWideThreads);
    if (r)
      hipLaunchKernelGGL((ln_fwd_wide_k<T, 2, RMS, true>), grid, block, 0, st, x, r, s, y, w, b, mean, rstd, rows, d,
                         eps, rpb, wt);
    else
      hipLaunchKernelGGL((ln_fwd_wide_k<T, 2, RMS, false>), grid, block, 0, st, x, r, s, y, w, b, mean, rstd, rows, d,
                         eps, rpb, wt);
    return hipGetLastError();
  }
  const int vpl = (d + 511) / 512;
  // rows per wave: 2+ once there are enough rows to keep ~2048 waves busy (the prefetch needs a next row)
  int rpw = 1;
  if (rows >= 4096) rpw = (int)((rows + 2047) / 2048 < 8 ? (rows + 2047) / 2048 : 8);
  if (g_ln_waves > 0) rpw = (int)std::min<int64_t>(8, std::max<int64_t>(1, (rows + g_ln_waves - 1) / g_ln_waves));
  const int64_t waves = (rows + rpw - 1) / rpw;
  const dim3 grid((unsigned)((waves + kWavesPerBlock - 1) / kWavesPerBlock)), block(64 * kWavesPerBlock);
#define HYP_LN_F(V)                                                                                          \
  case V:                                                                                                    \
    if (drop)                                                                                                \
      hipLaunchKernelGGL((ln_fwd_k<T, V, RMS, true, true>), grid, block, 0, st, x, r, s, y, w, b, mean, rstd, \
                         rows, d, eps, rpw, wt, *drop);                                                       \
    else if (r)                                                                                              \
      hipLaunchKernelGGL((ln_fwd_k<T, V, RMS, true>), grid, block, 0, st, x, r, s, y, w, b, mean, rstd, rows, \
                         d, eps, rpw, wt);                                                                       \
    else                                                                                                     \
      hipLaunchKernelGGL((ln_fwd_k<T, V, RMS, false>), grid, block, 0, st, x, r, s, y, w, b, mean, rstd, rows, \
                         d, eps, rpw, wt);                                                                       \
    break;
  switch (vpl) {
    HYP_LN_F(1)
    HYP_LN_F(2)
    HYP_LN_F(3)
    HYP_LN_F(4)
    HYP_LN_F(8)
    default:
      return hipErrorInvalidValue;
  }
#undef HYP_LN_F
  return hipGetLastError();
}

template <typename T, bool RMS>
hipError_t ln_bwd_dispatch(const T* dy, const T* xin, const float* w, const float* mean, const float* rstd,
                           const T* dres, T* dx, float* pdw, float* pdb, void* dw, void* db, int64_t rows, int d,
                           int P, int rows_per_wave, hipStream_t st, int wt, int wdt, T* dxa, const LnDrop* drop,
                           void* dbs, int dbs_dt) {
  if (drop != nullptr && (d > 2048 || dxa == nullptr)) return hipErrorInvalidValue;
  if (dbs != nullptr) {  // the branch-gradient sums follow dw (| db) in the combined output
    const size_t wb = wdt == kF32 ? 4 : 2;
    if (d > 2048 || dw == nullptr ||
        (dbs_dt < 0 &&
         static_cast<char*>(dbs) != static_cast<char*>(dw) + (size_t)(pdb != nullptr ? 2 : 1) * d * wb))
      return hipErrorInvalidValue;
    if (pdb != nullptr) pdb = pdw + d;
    const int bs_off = pdb != nullptr ? 2 * d : d;
    const int vpl = (d + 511) / 512;
    const dim3 grid(P), block(64 * kWavesPerBlock);
    const size_t lds = 3 * kWavesPerBlock * d * sizeof(float);
    const LnDrop dp0 = drop != nullptr ? *drop : LnDrop{};
#define HYP_LN_BS(V)                                                                                           \
  case V:                                                                                                      \
    if (drop && dres)                                                                                          \
      hipLaunchKernelGGL((ln_bwd_k<T, V, RMS, true, true, true>), grid, block, lds, st, dy, xin, w, mean, rstd, \
                         dres, dx, pdw, pdb, rows, d, rows_per_wave, wt, dxa, dp0, bs_off);                    \
    else if (drop)                                                                                             \
      hipLaunchKernelGGL((ln_bwd_k<T, V, RMS, false, true, true>), grid, block, lds, st, dy, xin, w, mean, rstd, \
                         dres, dx, pdw, pdb, rows, d, rows_per_wave, wt, dxa, dp0, bs_off);                    \
    else if (dres)                                                                                             \
      hipLaunchKernelGGL((ln_bwd_k<T, V, RMS, true, false, true>), grid, block, lds, st, dy, xin, w, mean, rstd, \
                         dres, dx, pdw, pdb, rows, d, rows_per_wave, wt, dxa, dp0, bs_off);                    \
    else                                                                                                       \
      hipLaunchKernelGGL((ln_bwd_k<T, V, RMS, false, false, true>), grid, block, lds, st, dy, xin, w, mean, rstd, \
                         dres, dx, pdw, pdb, rows, d, rows_per_wave, wt, dxa, dp0, bs_off);                    \
    break;
    switch (vpl) {
      HYP_LN_BS(1)
      HYP_LN_BS(2)
      HYP_LN_BS(3)
      HYP_LN_BS(4)
      HYP_LN_BS(8)
      default:
        return hipErrorInvalidValue;
    }
#undef HYP_LN_BS
    hipError_t e = hipGetLastError();
    if (e == hipSuccess)
      e = dbs_dt < 0 ? colsum_combine(pdw, P, bs_off + d, dw, wdt, st)
                     : colsum_combine_split(pdw, P, bs_off + d, dw, wdt, bs_off, dbs, dbs_dt, st);
    return e;
  }
  // with a bias: dγ and dβ partials interleave per block row ([P][2d]) and ONE combine writes
  // dw | db (the caller's db must directly follow dw)
  const size_t wbytes = wdt == kF32 ? 4 : 2;
  if (pdb != nullptr) {
    pdb = pdw + d;
    if (dw == nullptr || db == nullptr || static_cast<char*>(db) != static_cast<char*>(dw) + (size_t)d * wbytes)
      return hipErrorInvalidValue;
  }
  if (d > 2048) {  // P blocks of rows_per_wave rows (layernorm_bwd_geom)
    if (dres)
      hipLaunchKernelGGL((ln_bwd_wide_k<T, 2, RMS, true>), dim3(P), dim3(kWideThreads), 0, st, dy, xin, w, mean, rstd,
                         dres, dx, pdw, pdb, rows, d, rows_per_wave, wt);
    else
      hipLaunchKernelGGL((ln_bwd_wide_k<T, 2, RMS, false>), dim3(P), dim3(kWideThreads), 0, st, dy, xin, w, mean, rstd,
                         dres, dx, pdw, pdb, rows, d, rows_per_wave, wt);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess && dw) e = colsum_combine(pdw, P, pdb ? 2 * d : d, dw, wdt, st);
    return e;
  }
  const int vpl = (d + 511) / 512;
  const dim3 grid(P), block(64 * kWavesPerBlock);
  const size_t lds = 2 * kWavesPerBlock * d * sizeof(float);
#define HYP_LN_B(V)                                                                                          \
  case V:                                                                                                    \
    if (drop && dres)                                                                                        \
      hipLaunchKernelGGL((ln_bwd_k<T, V, RMS, true, true>), grid, block, lds, st, dy, xin, w, mean, rstd, dres, \
                         dx, pdw, pdb, rows, d, rows_per_wave, wt, dxa, *drop);                               \
    else if (drop)                                                                                           \
      hipLaunchKernelGGL((ln_bwd_k<T, V, RMS, false, true>), grid, block, lds, st, dy, xin, w, mean, rstd, dres, \
                         dx, pdw, pdb, rows, d, rows_per_wave, wt, dxa, *drop);                               \
    else if (dres)                                                                                           \
      hipLaunchKernelGGL((ln_bwd_k<T, V, RMS, true>), grid, block, lds, st, dy, xin, w, mean, rstd, dres, dx, \
                         pdw, pdb, rows, d, rows_per_wave, wt);                                              \
    else                                                                                                     \
      hipLaunchKernelGGL((ln_bwd_k<T, V, RMS, false>), grid, block, lds, st, dy, xin, w, mean, rstd, dres, dx, \
                         pdw, pdb, rows, d, rows_per_wave, wt);                                              \
    break;
  switch (vpl) {
    HYP_LN_B(1)
    HYP_LN_B(2)
    HYP_LN_B(3)
    HYP_LN_B(4)
    HYP_LN_B(8)
    default:
      return hipErrorInvalidValue;
  }
#undef HYP_LN_B
  hipError_t e = hipGetLastError();
  if (e == hipSuccess && dw) e = colsum_combine(pdw, P, pdb ? 2 * d : d, dw, wdt, st);
  return e;
}

}  // namespace

bool layernorm_supported(int d) {
  if (d % 8 != 0 || d > 4096) return false;
  if (d > 2048) return true;  // block-per-row kernels
  const int vpl = (d + 511) / 512;
  return vpl <= 4 || vpl == 8;
}

void ln_set_waves(int waves) { g_ln_waves = waves < 0 ? 0 : (waves > 16384 ? 16384 : waves); }

void layernorm_bwd_geom(int64_t rows, int d, int* P, int* rows_per_wave) {
  if (d > 2048) {  // wide rows: one 256-thread block per row group (ln_bwd_wide_k)
    const int rpb = wide_rows_per_block(rows);
    *rows_per_wave = rpb;
    *P = (int)((rows + rpb - 1) / rpb);
    if (*P < 1) *P = 1;
    return;
  }
  // enough waves to fill 256 CUs (>= min(rows, 2048) waves: a 128-token Llama step has only 128
  // rows of 4096 — at 8 rows per wave that was 4 workgroups, 136 us per RMSNorm backward), with
  // ~4 rows per wave so the row prefetch has work to hide behind; the partial rows (<= 1024
  // blocks) are combined by the wide colsum_combine (reduce.hip)
  int64_t waves = (rows + 3) / 4;  // ~4 rows per wave (the next row prefetched while one is reduced)
  const int64_t floor_waves = rows < 2048 ? rows : 2048;
  if (waves < floor_waves) waves = floor_waves;
  if (g_ln_waves > 0) waves = std::min<int64_t>(rows, g_ln_waves);
  if (waves > 4096) waves = 4096;
  if (waves < 1) waves = 1;
  int rpw = (int)((rows + waves - 1) / waves);
  int64_t nwaves = (rows + rpw - 1) / rpw;
  *rows_per_wave = rpw;
  *P = (int)((nwaves + kWavesPerBlock - 1) / kWavesPerBlock);
  if (*P < 1) *P = 1;
}

namespace {
LnDrop make_drop(float p, const RngState& rs) {
  LnDrop dp;
  dp.thr = (uint32_t)fminf(p * 4294967296.f, 4294967295.f);  // dropout.hip's threshold
  dp.scale = p < 1.f ? 1.f / (1.f - p) : 0.f;
  dp.rs = rs;
  return dp;
}
}  // namespace

hipError_t layernorm_forward(int dtype, int rms, const void* x, const void* r, void* s, void* y, const float* w,
                             const float* b, float* mean, float* rstd, int64_t rows, int d, float eps,
                             hipStream_t st, int wt, float drop_p, const RngState* rs) {
  if (!layernorm_supported(d)) return hipErrorInvalidValue;
  if (drop_p > 0.f && (rs == nullptr || drop_p >= 1.f)) return hipErrorInvalidValue;
  const LnDrop dp = drop_p > 0.f ? make_drop(drop_p, *rs) : LnDrop{};
  const LnDrop* dptr = drop_p > 0.f ? &dp : nullptr;
  HYP_DISPATCH_FLOAT(dtype, T, {
    if (rms)
      return ln_fwd_dispatch<T, true>((const T*)x, (const T*)r, (T*)s, (T*)y, w, b, mean, rstd, rows, d, eps, st, wt,
                                      dptr);
    return ln_fwd_dispatch<T, false>((const T*)x, (const T*)r, (T*)s, (T*)y, w, b, mean, rstd, rows, d, eps, st, wt,
                                     dptr);
  });
  return hipSuccess;
}

hipError_t layernorm_backward(int dtype, int rms, const void* dy, const void* xin, const float* w, const float* mean,
                              const float* rstd, const void* dres, void* dx, float* pdw, float* pdb, void* dw,
                              void* db, int64_t rows, int d, int P, int rows_per_wave, hipStream_t st, int wt,
                              void* dxa, float drop_p, const RngState* rs, void* dbs, int dbs_dtype) {
  const int wdt = wt ? dtype : kF32;  // dγ / dβ in the weight's dtype
  if (!layernorm_supported(d)) return hipErrorInvalidValue;
  if (drop_p > 0.f && (rs == nullptr || drop_p >= 1.f || dxa == nullptr)) return hipErrorInvalidValue;
  const LnDrop dp = drop_p > 0.f ? make_drop(drop_p, *rs) : LnDrop{};
  const LnDrop* dptr = drop_p > 0.f ? &dp : nullptr;
  HYP_DISPATCH_FLOAT(dtype, T, {
    if (rms)
      return ln_bwd_dispatch<T, true>((const T*)dy, (const T*)xin, w, mean, rstd, (const T*)dres, (T*)dx, pdw, pdb, dw,
                                      db, rows, d, P, rows_per_wave, st, wt, wdt, (T*)dxa, dptr, dbs, dbs_dtype);
    return ln_bwd_dispatch<T, false>((const T*)dy, (const T*)xin, w, mean, rstd, (const T*)dres, (T*)dx, pdw, pdb, dw,
                                     db, rows, d, P, rows_per_wave, st, wt, wdt, (T*)dxa, dptr, dbs, dbs_dtype);
  });
  return hipSuccess;
}

}  // namespace hyp

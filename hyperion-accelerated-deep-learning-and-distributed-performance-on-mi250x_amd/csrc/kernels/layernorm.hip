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

// Each lane handles VPL vectors of 8 elements: lane l, vector v covers [ (v*64 + l)*8, +8 ).
template <typename T, int VPL, bool RMS, bool HAS_RES>
__global__ __launch_bounds__(64 * kWavesPerBlock) void ln_fwd_k(const T* __restrict__ x, const T* __restrict__ r,
                                                                  T* __restrict__ s_out, T* __restrict__ y,
                                                                  const float* __restrict__ w,
                                                                  const float* __restrict__ b, float* __restrict__ mean_out,
                                                                  float* __restrict__ rstd_out, int64_t rows, int d,
                                                                  float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  if (row >= rows) return;
  const T* xr = x + row * d;
  float v[VPL][8];
  float sum = 0.f;
#pragma unroll
  for (int k = 0; k < VPL; ++k) {
    const int c = (k * 64 + lane) * 8;
    if (c < d) {
      Vec8<T>::load(xr + c, v[k]);
      if (HAS_RES) {
        float rv[8];
        Vec8<T>::load(r + row * d + c, rv);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[k][j] = rnd<T>(v[k][j] + rv[j]);  // stats of the stored stream
        Vec8<T>::store(s_out + row * d + c, v[k]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) sum += v[k][j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[k][j] = 0.f;
    }
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
      for (int j = 0; j < 8; ++j) {
        const float wj = w ? w[c + j] : 1.f;
        const float bj = (b && !RMS) ? b[c + j] : 0.f;
        o[j] = (v[k][j] - mean) * rstd * wj + bj;
      }
      Vec8<T>::store(y + row * d + c, o);
    }
  }
}

// dx and per-block partial dγ, dβ.  grid.x = ceil(rows / (kWavesPerBlock * rows_per_wave))
template <typename T, int VPL, bool RMS, bool HAS_DRES>
__global__ __launch_bounds__(64 * kWavesPerBlock) void ln_bwd_k(const T* __restrict__ dy, const T* __restrict__ xin,
                                                                  const float* __restrict__ w,
                                                                  const float* __restrict__ mean_in,
                                                                  const float* __restrict__ rstd_in,
                                                                  const T* __restrict__ dres, T* __restrict__ dx,
                                                                  float* __restrict__ pdw, float* __restrict__ pdb,
                                                                  int64_t rows, int d, int rows_per_wave) {
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  float gw[VPL][8], gb[VPL][8];
#pragma unroll
  for (int k = 0; k < VPL; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) gw[k][j] = gb[k][j] = 0.f;

  const int64_t row_begin = ((int64_t)blockIdx.x * kWavesPerBlock + wid) * rows_per_wave;
  for (int rr = 0; rr < rows_per_wave; ++rr) {
    const int64_t row = row_begin + rr;
    if (row >= rows) break;
    const float mean = RMS ? 0.f : mean_in[row];
    const float rstd = rstd_in[row];
    float g[VPL][8], xh[VPL][8];
    float s1 = 0.f, s2 = 0.f;  // Σ g·w, Σ g·w·xhat
#pragma unroll
    for (int k = 0; k < VPL; ++k) {
      const int c = (k * 64 + lane) * 8;
      if (c < d) {
        float xv[8];
        Vec8<T>::load(dy + row * d + c, g[k]);
        Vec8<T>::load(xin + row * d + c, xv);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xh[k][j] = (xv[j] - mean) * rstd;
          const float gwv = g[k][j] * (w ? w[c + j] : 1.f);
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
        for (int j = 0; j < 8; ++j) {
          const float gwv = g[k][j] * (w ? w[c + j] : 1.f);
          o[j] = rstd * (gwv - (RMS ? 0.f : s1) - xh[k][j] * s2);
        }
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
  // block partials of dγ/dβ through LDS: [wave][d]
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sw = smem;
  float* sb = smem + kWavesPerBlock * d;
#pragma unroll
  for (int k = 0; k < VPL; ++k) {
    const int c = (k * 64 + lane) * 8;
    if (c < d) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sw[wid * d + c + j] = gw[k][j];
        sb[wid * d + c + j] = gb[k][j];
      }
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < d; c += 64 * kWavesPerBlock) {
    float a = 0.f, bb = 0.f;
#pragma unroll
    for (int q = 0; q < kWavesPerBlock; ++q) {
      a += sw[q * d + c];
      bb += sb[q * d + c];
    }
    pdw[(int64_t)blockIdx.x * d + c] = a;
    if (pdb) pdb[(int64_t)blockIdx.x * d + c] = bb;
  }
}

template <typename T, bool RMS>
hipError_t ln_fwd_dispatch(const T* x, const T* r, T* s, T* y, const float* w, const float* b, float* mean,
                           float* rstd, int64_t rows, int d, float eps, hipStream_t st) {
  const int vpl = (d + 511) / 512;
  const dim3 grid((unsigned)((rows + kWavesPerBlock - 1) / kWavesPerBlock)), block(64 * kWavesPerBlock);
#define HYP_LN_F(V)                                                                                          \
  case V:                                                                                                    \
    if (r)                                                                                                   \
      hipLaunchKernelGGL((ln_fwd_k<T, V, RMS, true>), grid, block, 0, st, x, r, s, y, w, b, mean, rstd, rows, \
                         d, eps);                                                                            \
    else                                                                                                     \
      hipLaunchKernelGGL((ln_fwd_k<T, V, RMS, false>), grid, block, 0, st, x, r, s, y, w, b, mean, rstd, rows, \
                         d, eps);                                                                            \
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
                           const T* dres, T* dx, float* pdw, float* pdb, float* dw, float* db, int64_t rows, int d,
                           int P, int rows_per_wave, hipStream_t st) {
  const int vpl = (d + 511) / 512;
  const dim3 grid(P), block(64 * kWavesPerBlock);
  const size_t lds = 2 * kWavesPerBlock * d * sizeof(float);
#define HYP_LN_B(V)                                                                                          \
  case V:                                                                                                    \
    if (dres)                                                                                                \
      hipLaunchKernelGGL((ln_bwd_k<T, V, RMS, true>), grid, block, lds, st, dy, xin, w, mean, rstd, dres, dx, \
                         pdw, pdb, rows, d, rows_per_wave);                                                  \
    else                                                                                                     \
      hipLaunchKernelGGL((ln_bwd_k<T, V, RMS, false>), grid, block, lds, st, dy, xin, w, mean, rstd, dres, dx, \
                         pdw, pdb, rows, d, rows_per_wave);                                                  \
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
  if (e == hipSuccess && dw) e = colsum_combine(pdw, P, d, dw, kF32, st);
  if (e == hipSuccess && db && pdb) e = colsum_combine(pdb, P, d, db, kF32, st);
  return e;
}

}  // namespace

bool layernorm_supported(int d) {
  if (d % 8 != 0 || d > 4096) return false;
  const int vpl = (d + 511) / 512;
  return vpl <= 4 || vpl == 8;
}

void layernorm_bwd_geom(int64_t rows, int* P, int* rows_per_wave) {
  // enough waves to fill 256 CUs (>= min(rows, 1024) waves: a 128-token Llama step has only 128
  // rows of 4096 — at 8 rows per wave that was 4 workgroups, 136 us per RMSNorm backward), but
  // few partial rows for the column reduction (<= 2048 waves, >= 8 rows per wave when possible)
  int64_t waves = (rows + 7) / 8;
  const int64_t floor_waves = rows < 1024 ? rows : 1024;
  if (waves < floor_waves) waves = floor_waves;
  if (waves > 2048) waves = 2048;
  if (waves < 1) waves = 1;
  int rpw = (int)((rows + waves - 1) / waves);
  int64_t nwaves = (rows + rpw - 1) / rpw;
  *rows_per_wave = rpw;
  *P = (int)((nwaves + kWavesPerBlock - 1) / kWavesPerBlock);
  if (*P < 1) *P = 1;
}

hipError_t layernorm_forward(int dtype, int rms, const void* x, const void* r, void* s, void* y, const float* w,
                             const float* b, float* mean, float* rstd, int64_t rows, int d, float eps,
                             hipStream_t st) {
  if (!layernorm_supported(d)) return hipErrorInvalidValue;
  HYP_DISPATCH_FLOAT(dtype, T, {
    if (rms)
      return ln_fwd_dispatch<T, true>((const T*)x, (const T*)r, (T*)s, (T*)y, w, b, mean, rstd, rows, d, eps, st);
    return ln_fwd_dispatch<T, false>((const T*)x, (const T*)r, (T*)s, (T*)y, w, b, mean, rstd, rows, d, eps, st);
  });
  return hipSuccess;
}

hipError_t layernorm_backward(int dtype, int rms, const void* dy, const void* xin, const float* w, const float* mean,
                              const float* rstd, const void* dres, void* dx, float* pdw, float* pdb, float* dw,
                              float* db, int64_t rows, int d, int P, int rows_per_wave, hipStream_t st) {
  if (!layernorm_supported(d)) return hipErrorInvalidValue;
  HYP_DISPATCH_FLOAT(dtype, T, {
    if (rms)
      return ln_bwd_dispatch<T, true>((const T*)dy, (const T*)xin, w, mean, rstd, (const T*)dres, (T*)dx, pdw, pdb, dw,
                                      db, rows, d, P, rows_per_wave, st);
    return ln_bwd_dispatch<T, false>((const T*)dy, (const T*)xin, w, mean, rstd, (const T*)dres, (T*)dx, pdw, pdb, dw,
                                     db, rows, d, P, rows_per_wave, st);
  });
  return hipSuccess;
}

}  // namespace hyp

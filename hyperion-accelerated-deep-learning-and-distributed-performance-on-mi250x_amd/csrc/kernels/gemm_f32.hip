// FP32 GEMM on the gfx950 fp32-input matrix cores — the fp32 training path (linear layers and the
// im2col convolutions of the reference-methodology fp32 rows):
//
//   C[M, N] = epi( alpha · Σ_k A(m, k) · B(n, k) ),  epi: + beta·C_old, + bias[n], ReLU
//
// Reference: the fp32 rows of the matmul precision sweep (`Phase 1/01_hardware_exploration.ipynb:
// 208-242`) and the fp32 ResNet / ViT / CustomTransformer model benchmarks (`Phase 1/
// baseline_performance.ipynb:252-358`, `02_development/compilation_optimization.py:47-51`), which
// the reference runs on MIOpen / rocBLAS fp32 kernels (SURVEY C3 / C6 / §2.4 "GEMM").
//
// gfx950 has no xf32 (TF32-like) MFMA, but it has exact fp32-in / fp32-accumulate MFMA at the fp32
// VALU peak (cdna_hip_programming.md §3 "FP32-input MFMA"): v_mfma_f32_32x32x2_f32, 64 cycles per
// instruction, one float of A and of B per lane — a k-ordered fma chain per output, the numerics
// of a scalar fp32 GEMM.  At 64 MFMA cycles per 16 KiB of fragment data the kernel is MFMA-bound:
// LDS traffic and address arithmetic are noise, so one kernel serves every layout and raggedness.
//
// Operand forms (like gemm_tiles_impl.h): "row" X(i, k) at X + i·ld + k (nn.Linear weights, im2col
// matrices, activations in a forward) or "tr" X(i, k) at X + k·ld + i (the weight in a data gradient,
// both operands of a weight gradient) — forward (NT), data gradient (NN) and weight gradient (TN)
// without transposed copies.
//
// Structure:
//  * 128x128 output tile, 256 threads = 4 waves as 2 x 2, each wave 64 x 64 = 2 x 2 blocks of
//    32 x 32 (16 accumulators per block); two workgroups per CU (64 KiB of LDS each);
//  * K staged in 32-deep slices by global_load_lds_dwordx4 (LDS-DMA, no VGPR round trip),
//    double-buffered; out-of-range rows / columns / reduction indices read the zero page (ragged
//    M, N, K and split-K slice ends cost nothing but a select per staged chunk);
//  * row image [128][32] floats, 16-byte chunk XOR-swizzled by (row >> 1) & 7; per 4-wide k chunk
//    lane (row, half h) reads ONE ds_read_b64 (k = 4c + 2h, +1) feeding the two MFMA k-steps;
//  * tr image [32 k][128] floats, chunk swizzled by ((k >> 1) & 1) << 3 so the two half-waves
//    (k rows 4c + e and 4c + 2 + e) land in opposite bank halves; two ds_read_b32 per fragment;
//  * split-K: slices of one tile are adjacent workgroup ids (same XCD after the remap), each writes
//    an fp32 slab; gemm_f32_reduce_k sums the slabs in slice order (deterministic) and applies
//    the epilogue;
//  * XCD-aware remap + grouped tile order (T1).
// Requirements (host-checked): row-form operands K % 4 == 0; tr-form operands extent % 4 == 0;
// leading dimensions % 4 == 0; 16-byte aligned bases.
#include <algorithm>

#include "hyp_common.h"
#include "hyp_kernels.h"

namespace hyp {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int kBK = 32, kThreads = 256, kGroupM = 8;

struct F32Args {
  const float* A;
  const float* B;
  float* C;            // output (splits == 1) — row stride ldc
  float* part;         // split-K slabs [splits][M][N] (splits > 1)
  const float* bias;   // [N] or null
  const float* zero;   // >= 16 bytes of zeros
  int M, N, K, lda, ldb, ldc;
  int kper, splits;    // reduction indices per split (multiple of 32)
  float alpha, beta;
  int relu;
};

__device__ __forceinline__ int swz_row(int row) { return (row >> 1) & 7; }
__device__ __forceinline__ int swz_tr(int k) { return ((k >> 1) & 1) << 3; }

__device__ __forceinline__ void glds16(const float* src, float* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const void*)src, (void __attribute__((address_space(3)))*)lds_wave_base, 16, 0, 0);
}

// Row form: [ROWS rows][32 k] slice starting at (i0, k0).  One wave instruction = 8 rows.
template <int ROWS>
__device__ __forceinline__ void stage_row(const float* __restrict__ g, int ld, int i0, int rows, int k0, int kend,
                                          float* img, int wave, int lane, const float* zero) {
#pragma unroll
  for (int it = 0; it < ROWS / 32; ++it) {
    const int r0 = (it * 4 + wave) * 8;
    const int row = r0 + (lane >> 3);
    const int chunk = (lane & 7) ^ swz_row(row);
    const int gi = i0 + row, gk = k0 + chunk * 4;
    const float* src = (gi < rows && gk < kend) ? g + (int64_t)gi * ld + gk : zero;
    glds16(src, img + r0 * kBK);
  }
}

// Tr form: [32 k][ROWS i] slice.  One wave instruction = 256 / ROWS k-rows of ROWS / 4 chunks.
template <int ROWS>
__device__ __forceinline__ void stage_tr(const float* __restrict__ g, int ld, int i0, int rows, int k0, int kend,
                                         float* img, int wave, int lane, const float* zero) {
  constexpr int CPR = ROWS / 4, KPI = 64 / CPR;  // chunks per k-row, k-rows per instruction
#pragma unroll
  for (int it = 0; it < ROWS / 32; ++it) {
    const int kr0 = (it * 4 + wave) * KPI;
    const int kr = kr0 + lane / CPR;
    const int chunk = (lane % CPR) ^ swz_tr(kr);
    const int gk = k0 + kr, gi = i0 + chunk * 4;
    const float* src = (gk < kend && gi < rows) ? g + (int64_t)gk * ld + gi : zero;
    glds16(src, img + kr0 * ROWS);
  }
}

template <bool TR, int ROWS>
__device__ __forceinline__ f32x2 frag(const float* img, int row, int c, int h) {
  if constexpr (!TR) {
    return *reinterpret_cast<const f32x2*>(img + row * kBK + ((c ^ swz_row(row)) << 2) + 2 * h);
  } else {
    const int k = 4 * c + 2 * h;
    const int p0 = (((row >> 2) ^ swz_tr(k)) << 2) | (row & 3);  // k and k + 1 share the swizzle
    return f32x2{img[k * ROWS + p0], img[(k + 1) * ROWS + p0]};
  }
}

// WM x WN waves, each FM x FN blocks of 32 x 32 outputs: 128x128 (2x2 waves of 2x2), 256x64, 64x256,
// and the one-workgroup-per-CU 256x128 / 128x256 (2x2 waves of 4x2 / 2x4: twice the MFMA work per
// fragment read and per barrier, one wave per SIMD)
template <int WM, int WN, int FM, int FN, bool ATR, bool BTR>
__global__ __launch_bounds__(kThreads) void gemm_f32_k(const F32Args p) {
  static_assert(WM * WN == 4, "4 waves");
  constexpr int BM = 32 * FM * WM, BN = 32 * FN * WN, IA = BM * kBK, IB = BN * kBK;
  __shared__ __attribute__((aligned(16))) float smem[2 * (IA + IB)];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;

  const int tiles_m = (p.M + BM - 1) / BM, tiles_n = (p.N + BN - 1) / BN;
  const int nwg = tiles_m * tiles_n * p.splits;
  int bid = blockIdx.x;
  {  // XCD remap: consecutive logical ids on one XCD (split slices of a tile share its L2)
    const int q = nwg / 8, r = nwg % 8, xcd = bid % 8, idx = bid / 8;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
  }
  const int split = bid % p.splits;
  const int tile = bid / p.splits;
  const int group = kGroupM * tiles_n;
  const int first_m = (tile / group) * kGroupM;
  const int gsize = min(tiles_m - first_m, kGroupM);
  const int tm = first_m + (tile % group) % gsize;
  const int tn = (tile % group) / gsize;
  const int m0 = tm * BM, n0 = tn * BN;

  const int kbeg = split * p.kper;
  const int kend = min(p.K, kbeg + p.kper);
  const int nk = (kend - kbeg + kBK - 1) / kBK;

  f32x16 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[i][j][v] = 0.f;

  auto stage = [&](int t, float* buf) {
    const int k0 = kbeg + t * kBK;
    if constexpr (ATR) stage_tr<BM>(p.A, p.lda, m0, p.M, k0, kend, buf, wave, lane, p.zero);
    else stage_row<BM>(p.A, p.lda, m0, p.M, k0, kend, buf, wave, lane, p.zero);
    if constexpr (BTR) stage_tr<BN>(p.B, p.ldb, n0, p.N, k0, kend, buf + IA, wave, lane, p.zero);
    else stage_row<BN>(p.B, p.ldb, n0, p.N, k0, kend, buf + IA, wave, lane, p.zero);
  };

  if (nk > 0) {
    stage(0, smem);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
  }
  const int r32 = lane & 31, h = lane >> 5;
  const int wr = wm * 32 * FM, wc = wn * 32 * FN;
  for (int t = 0; t < nk; ++t) {
    const int cur = t & 1;
    if (t + 1 < nk) stage(t + 1, smem + (cur ^ 1) * (IA + IB));
    const float* as = smem + cur * (IA + IB);
    const float* bs = as + IA;
    // fragments double-buffered in registers: chunk c + 1's LDS reads are in flight while chunk
    // c's 2·FM·FN MFMAs (64 cycles each) run — one register set would serialize read latency and MFMAs
    f32x2 a[2][FM], b[2][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i) a[0][i] = frag<ATR, BM>(as, wr + i * 32 + r32, 0, h);
#pragma unroll
    for (int j = 0; j < FN; ++j) b[0][j] = frag<BTR, BN>(bs, wc + j * 32 + r32, 0, h);
#pragma unroll
    for (int c = 0; c < kBK / 4; ++c) {
      const int q = c & 1;
      if (c + 1 < kBK / 4) {
#pragma unroll
        for (int i = 0; i < FM; ++i) a[q ^ 1][i] = frag<ATR, BM>(as, wr + i * 32 + r32, c + 1, h);
#pragma unroll
        for (int j = 0; j < FN; ++j) b[q ^ 1][j] = frag<BTR, BN>(bs, wc + j * 32 + r32, c + 1, h);
      }
      // the .x k-step of every block, then the .y one: an accumulator's two MFMAs are FM·FN issues
      // apart (back-to-back dependent MFMAs wait out the 64-cycle result latency)
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[q][i].x, b[q][j].x, acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[q][i].y, b[q][j].y, acc[i][j], 0, 0, 0);
      // interleave the next chunk's LDS reads between this chunk's MFMAs (hipcc otherwise issues
      // them after the last MFMA and waits on them before the next chunk: ~10 % MFMA idle)
#pragma unroll
      for (int g = 0; g < FM + FN; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // up to 2 DS reads
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 2 * FM * FN - (FM + FN), 0);
    }
    __builtin_amdgcn_s_waitcnt(0);  // next slice's LDS-DMA (this wave)
    __syncthreads();                // ... every wave's; everyone done with `cur`
  }

  // acc[i][j][v] = C[m0 + wr + i*32 + 8 (v / 4) + 4 h + (v % 4)][n0 + wc + j*32 + r32]
  const bool slab = p.splits > 1;
  float* part = slab ? p.part + (int64_t)split * p.M * p.N : nullptr;
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int col = n0 + wc + j * 32 + r32;
    if (col >= p.N) continue;
    const float bv = (!slab && p.bias) ? p.bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int row = m0 + wr + i * 32 + 8 * (v >> 2) + 4 * h + (v & 3);
        if (row >= p.M) continue;
        if (slab) {
          part[(int64_t)row * p.N + col] = acc[i][j][v];
        } else {
          float* dst = p.C + (int64_t)row * p.ldc + col;
          float y = p.alpha * acc[i][j][v] + bv;
          if (p.beta != 0.f) y += p.beta * *dst;
          if (p.relu) y = fmaxf(y, 0.f);
          *dst = y;
        }
      }
  }
}

// Σ over the split slabs in slice order + epilogue; VEC = 4: four consecutive columns per thread
template <int VEC>
__global__ __launch_bounds__(256) void gemm_f32_reduce_k(const F32Args p) {
  const int64_t total = (int64_t)p.M * p.N / VEC, slab = (int64_t)p.M * p.N;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int64_t f = e * VEC;
    const int row = (int)(f / p.N), col = (int)(f % p.N);
    float s[VEC];
    if constexpr (VEC == 4) {
      float4 v = *reinterpret_cast<const float4*>(p.part + f);
      for (int q = 1; q < p.splits; ++q) {
        const float4 u = *reinterpret_cast<const float4*>(p.part + q * slab + f);
        v.x += u.x, v.y += u.y, v.z += u.z, v.w += u.w;
      }
      s[0] = v.x, s[1] = v.y, s[2] = v.z, s[3] = v.w;
    } else {
      s[0] = 0.f;
      for (int q = 0; q < p.splits; ++q) s[0] += p.part[q * slab + f];
    }
    float* dst = p.C + (int64_t)row * p.ldc + col;
#pragma unroll
    for (int u = 0; u < VEC; ++u) {
      float y = p.alpha * s[u] + (p.bias ? p.bias[col + u] : 0.f);
      if (p.beta != 0.f) y += p.beta * dst[u];
      if (p.relu) y = fmaxf(y, 0.f);
      s[u] = y;
    }
    if constexpr (VEC == 4) *reinterpret_cast<float4*>(dst) = make_float4(s[0], s[1], s[2], s[3]);
    else *dst = s[0];
  }
}

// ---- im2col / col2im (NHWC fp32) -----------------------------------------------------------------
// cols[(n, ho, wo), (r, s, c)] = x[n, ho·sh − ph + r, wo·sw − pw + s, c] (0 outside), row pitch Kp
// (>= R·S·C, the pad columns written as 0) — the operand of the forward and weight-gradient GEMMs.
template <int VEC>
__global__ __launch_bounds__(256) void im2col_k(const float* __restrict__ x, float* __restrict__ cols, int Nb, int H,
                                                int W, int C, int Ho, int Wo, int R, int S, int sh, int sw, int ph,
                                                int pw, int Kp) {
  const int cv = C / VEC, Kv = Kp / VEC;
  const int64_t total = (int64_t)Nb * Ho * Wo * Kv;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int kv = (int)(e % Kv);
    const int64_t m = e / Kv;
    const int wo = (int)(m % Wo), ho = (int)((m / Wo) % Ho), n = (int)(m / ((int64_t)Wo * Ho));
    const int tap = kv / cv, c = (kv % cv) * VEC;
    const int r = tap / S, s = tap % S;
    const int hi = ho * sh - ph + r, wi = wo * sw - pw + s;
    float* dst = cols + m * Kp + (int64_t)kv * VEC;
    if (tap < R * S && hi >= 0 && hi < H && wi >= 0 && wi < W) {
      const float* src = x + (((int64_t)n * H + hi) * W + wi) * C + c;
      if constexpr (VEC == 4) *reinterpret_cast<float4*>(dst) = *reinterpret_cast<const float4*>(src);
      else *dst = *src;
    } else {
      if constexpr (VEC == 4) *reinterpret_cast<float4*>(dst) = make_float4(0.f, 0.f, 0.f, 0.f);
      else *dst = 0.f;
    }
  }
}

// dx[n, h, w, c] = Σ_{r, s} dcols[(n, ho, wo), (r, s, c)] over the taps that read (h, w) — a gather
// (each input element summed by one thread in tap order: deterministic, no atomics)
template <int VEC>
__global__ __launch_bounds__(256) void col2im_k(const float* __restrict__ dcols, float* __restrict__ dx, int Nb, int H,
                                                int W, int C, int Ho, int Wo, int R, int S, int sh, int sw, int ph,
                                                int pw, int Kp) {
  const int cv = C / VEC;
  const int64_t total = (int64_t)Nb * H * W * cv;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int c = (int)(e % cv) * VEC;
    const int64_t pix = e / cv;
    const int w = (int)(pix % W), hh = (int)((pix / W) % H), n = (int)(pix / ((int64_t)W * H));
    float acc[VEC];
#pragma unroll
    for (int q = 0; q < VEC; ++q) acc[q] = 0.f;
    for (int r = 0; r < R; ++r) {
      const int th = hh + ph - r;
      if (th < 0 || th % sh) continue;
      const int ho = th / sh;
      if (ho >= Ho) continue;
      for (int s = 0; s < S; ++s) {
        const int tw = w + pw - s;
        if (tw < 0 || tw % sw) continue;
        const int wo = tw / sw;
        if (wo >= Wo) continue;
        const float* src = dcols + (((int64_t)n * Ho + ho) * Wo + wo) * Kp + (int64_t)(r * S + s) * C + c;
        if constexpr (VEC == 4) {
          const float4 v = *reinterpret_cast<const float4*>(src);
          acc[0] += v.x, acc[1] += v.y, acc[2] += v.z, acc[3] += v.w;
        } else {
          acc[0] += *src;
        }
      }
    }
    float* dst = dx + pix * C + c;
    if constexpr (VEC == 4) *reinterpret_cast<float4*>(dst) = make_float4(acc[0], acc[1], acc[2], acc[3]);
    else *dst = acc[0];
  }
}

int grid_for(int64_t work) { return (int)std::min<int64_t>((work + 255) / 256, 8192); }

}  // namespace

bool gemm_f32_supported(int M, int N, int K, bool a_tr, bool b_tr, int lda, int ldb, int ldc) {
  if (M <= 0 || N <= 0 || K <= 0 || lda % 4 || ldb % 4 || ldc < N) return false;
  if (!a_tr && (K % 4 || lda < K)) return false;
  if (a_tr && (M % 4 || lda < M)) return false;
  if (!b_tr && (K % 4 || ldb < K)) return false;
  if (b_tr && (N % 4 || ldb < N)) return false;
  return true;
}

namespace {
// (BM, BN, workgroups per CU): 128x128, 256x64, 64x256 (2 per CU: 64-80 KiB of LDS), 256x128,
// 128x256 (1 per CU: 96 KiB)
constexpr int kNumShapes = 5;
constexpr int kShapes[kNumShapes][3] = {{128, 128, 2}, {256, 64, 2}, {64, 256, 2}, {256, 128, 1}, {128, 256, 1}};

// Launch plan: the tile shape and split count minimising a cost model of the MFMA-bound kernel —
// 256 CUs each time-slice their resident workgroups, so the time is the number of 256-workgroup
// "waves" of the grid times the slices per workgroup (+1.5 for the prologue and epilogue), plus
// the split-K slab traffic (write + the reduce's read, ~4 TB/s) in the same units (~1.7 us per
// slice of a 4-wave 64x64-per-wave tile).
void plan(int M, int N, int K, int req, int req_shape, int* shape, int* splits, int* per_out) {
  const int nk = (K + kBK - 1) / kBK;
  double best = 1e30;
  int bs = req_shape >= 0 && req_shape < kNumShapes ? req_shape : 0, bsp = 1, bper = nk;
  for (int t = 0; t < kNumShapes; ++t) {
    if (req_shape >= 0 && t != req_shape) continue;
    const int bm = kShapes[t][0], bn = kShapes[t][1], occ = kShapes[t][2];
    const int64_t tiles = (int64_t)((M + bm - 1) / bm) * ((N + bn - 1) / bn);
    for (int s = 1; s <= std::min(nk, 128); ++s) {
      if (req > 0 && s != std::min(req, nk)) continue;
      const int per = (nk + s - 1) / s, se = (nk + per - 1) / per;
      if (se != s) continue;
      // a 1-per-CU tile does twice the MFMA work per slice of a 2-per-CU one in the same time slot
      const int64_t waves = (tiles * s + 256 * occ - 1) / (256 * occ);
      double est = (double)waves * (per + 1.5) * (occ == 1 ? 2.0 : 1.0);
      if (s > 1) est += ((double)M * N * 4.0 * (s + 1) / 4.0e6 + 3.0) / 1.7;
      if (est < best * 0.98) {
        best = est;
        bs = t;
        bsp = s;
        bper = per;
      }
    }
  }
  *shape = bs;
  *splits = bsp;
  *per_out = bper;
}

template <int WM, int WN, int FM, int FN>
void launch_shape(const F32Args& p, bool a_tr, bool b_tr, int nwg, hipStream_t st) {
  const dim3 grid(nwg), block(kThreads);
  if (!a_tr && !b_tr) hipLaunchKernelGGL((gemm_f32_k<WM, WN, FM, FN, false, false>), grid, block, 0, st, p);
  else if (!a_tr && b_tr) hipLaunchKernelGGL((gemm_f32_k<WM, WN, FM, FN, false, true>), grid, block, 0, st, p);
  else if (a_tr && !b_tr) hipLaunchKernelGGL((gemm_f32_k<WM, WN, FM, FN, true, false>), grid, block, 0, st, p);
  else hipLaunchKernelGGL((gemm_f32_k<WM, WN, FM, FN, true, true>), grid, block, 0, st, p);
}
}  // namespace

int gemm_f32_splits(int M, int N, int K, int splits, int shape) {
  int t, sp, per;
  plan(M, N, K, splits, shape, &t, &sp, &per);
  return sp;
}

hipError_t gemm_f32(const float* A, const float* B, float* C, float* part, const float* bias, const float* zero,
                    int M, int N, int K, bool a_tr, bool b_tr, int lda, int ldb, int ldc, float alpha, float beta,
                    int relu, int splits, int shape, hipStream_t st) {
  if (!gemm_f32_supported(M, N, K, a_tr, b_tr, lda, ldb, ldc) || zero == nullptr) return hipErrorInvalidValue;
  int per;
  plan(M, N, K, splits, shape, &shape, &splits, &per);
  if (splits > 1 && part == nullptr) return hipErrorInvalidValue;
  F32Args p{A, B, C, part, bias, zero, M, N, K, lda, ldb, ldc, per * kBK, splits, alpha, beta, relu};
  const int bm = kShapes[shape][0], bn = kShapes[shape][1];
  const int nwg = ((M + bm - 1) / bm) * ((N + bn - 1) / bn) * splits;
  if (shape == 0) launch_shape<2, 2, 2, 2>(p, a_tr, b_tr, nwg, st);
  else if (shape == 1) launch_shape<4, 1, 2, 2>(p, a_tr, b_tr, nwg, st);
  else if (shape == 2) launch_shape<1, 4, 2, 2>(p, a_tr, b_tr, nwg, st);
  else if (shape == 3) launch_shape<2, 2, 4, 2>(p, a_tr, b_tr, nwg, st);
  else launch_shape<2, 2, 2, 4>(p, a_tr, b_tr, nwg, st);
  if (splits == 1) return hipGetLastError();
  const bool v4 = N % 4 == 0 && ldc % 4 == 0 && reinterpret_cast<uintptr_t>(C) % 16 == 0;
  const int64_t work = (int64_t)M * N / (v4 ? 4 : 1);
  if (v4) hipLaunchKernelGGL(gemm_f32_reduce_k<4>, dim3(grid_for(work)), dim3(256), 0, st, p);
  else hipLaunchKernelGGL(gemm_f32_reduce_k<1>, dim3(grid_for(work)), dim3(256), 0, st, p);
  return hipGetLastError();
}

hipError_t im2col_f32(const float* x, float* cols, int Nb, int H, int W, int C, int Ho, int Wo, int R, int S, int sh,
                      int sw, int ph, int pw, int Kp, hipStream_t st) {
  if (Kp < R * S * C) return hipErrorInvalidValue;
  if (C % 4 == 0 && Kp % 4 == 0)
    hipLaunchKernelGGL((im2col_k<4>), dim3(grid_for((int64_t)Nb * Ho * Wo * (Kp / 4))), dim3(256), 0, st, x, cols, Nb,
                       H, W, C, Ho, Wo, R, S, sh, sw, ph, pw, Kp);
  else
    hipLaunchKernelGGL((im2col_k<1>), dim3(grid_for((int64_t)Nb * Ho * Wo * Kp)), dim3(256), 0, st, x, cols, Nb, H, W,
                       C, Ho, Wo, R, S, sh, sw, ph, pw, Kp);
  return hipGetLastError();
}

hipError_t col2im_f32(const float* dcols, float* dx, int Nb, int H, int W, int C, int Ho, int Wo, int R, int S, int sh,
                      int sw, int ph, int pw, int Kp, hipStream_t st) {
  if (Kp < R * S * C) return hipErrorInvalidValue;
  if (C % 4 == 0 && Kp % 4 == 0)
    hipLaunchKernelGGL((col2im_k<4>), dim3(grid_for((int64_t)Nb * H * W * (C / 4))), dim3(256), 0, st, dcols, dx, Nb,
                       H, W, C, Ho, Wo, R, S, sh, sw, ph, pw, Kp);
  else
    hipLaunchKernelGGL((col2im_k<1>), dim3(grid_for((int64_t)Nb * H * W * C)), dim3(256), 0, st, dcols, dx, Nb, H, W,
                       C, Ho, Wo, R, S, sh, sw, ph, pw, Kp);
  return hipGetLastError();
}

}  // namespace hyp

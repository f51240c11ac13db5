// Flash-style softmax attention, forward + backward, on gfx950 MFMA (v_mfma_f32_16x16x32_{bf16,f16}).
//
// Replaces the SDPA math path the reference fell back to ("not compiled with memory efficient
// attention", baseline_performance.ipynb:37) inside nn.MultiheadAttention / HF Llama
// (SURVEY §2.4 "Softmax attention"; shapes §2.5: S = 16/127/128, head_dim 64/128, causal for
// Llama, dropout 0.1 for nn.TransformerEncoderLayer).
//
// Layout: q/k/v/o are [B, S, H, D] tensors given by (batch, seq, head) element strides with the
// head dim contiguous — so the packed QKV projection output is consumed in place (no permute).
//
// Forward: 128 query rows per workgroup on the 32x32x16 MFMA (details at attn_fwd_k); dropout on P
// by a counter-based hash of (seed, b, h, q, key) — regenerated in backward; writes O and the
// log2-domain log-sum-exp per row.
// Backward (one workgroup = 64 keys of one (b, h); wave w owns 16 keys; loop over query tiles):
//   * S and dP recomputed with the query on rows, key on the lane; their C tiles are directly the
//     B operands of dVᵀ += dOᵀ·P and dKᵀ += Qᵀ·dS (accumulator-as-operand, §3) — no LDS trip;
//   * dQ = dS·K goes through one bf16 LDS image of dS and is accumulated across key blocks with
//     fp32 atomics into a [B,H,S,D] workspace, converted by a final pass.
#include "hyp_common.h"
#include "hyp_kernels.h"

namespace hyp {
namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));
typedef uint16_t u16x4 __attribute__((ext_vector_type(4)));

template <typename T>
struct MM;
template <>
struct MM<bf16_t> {
  static __device__ __forceinline__ f32x4 mfma(u16x8 a, u16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c,
                                                   0, 0, 0);
  }
  static __device__ __forceinline__ uint16_t cvt(float f) { return float_to_bf16(f); }
  static __device__ __forceinline__ float tof(uint16_t v) { return bf16_to_float(v); }
};
template <>
struct MM<f16_t> {
  static __device__ __forceinline__ f32x4 mfma(u16x8 a, u16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, a), __builtin_bit_cast(f16x8_t, b), c, 0,
                                                  0, 0);
  }
  static __device__ __forceinline__ uint16_t cvt(float f) { return __builtin_bit_cast(uint16_t, (f16_t)f); }
  static __device__ __forceinline__ float tof(uint16_t v) { return (float)__builtin_bit_cast(f16_t, v); }
};

constexpr int KB = 64;         // keys (fwd) / queries (bwd) per LDS tile
constexpr int TS = KB + 4;     // transposed-image row stride (elements): 136 B rows, conflict-free b64 reads

__device__ __forceinline__ uint32_t hash_keep(uint64_t seed, uint64_t idx) {
  uint64_t z = seed + 0x9E3779B97F4A7C15ull * (idx + 1);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (uint32_t)z;
}

// A [64 rows][D] tile of a [S, D] (strided) slab held in registers between its global load and its
// LDS store: every thread's loads are issued together (the old load-store loop waited one memory
// round trip per 16-byte chunk), and the NEXT tile's loads are issued before the current tile's
// MFMA work, so they are in flight while it computes.  Out-of-range rows are zero.
template <int D>
struct TileRegs {
  static constexpr int N = KB * D / 8 / 256;  // 16-byte chunks per thread
  u16x8 v[N];
};

template <int D>
__device__ __forceinline__ void load_tile(const uint16_t* __restrict__ base, int64_t sstride, int row0, int S,
                                          TileRegs<D>& t) {
  constexpr int NCH = D / 8;
#pragma unroll
  for (int i = 0; i < TileRegs<D>::N; ++i) {
    const int c = threadIdx.x + 256 * i, r = c / NCH, ch = c - r * NCH;
    u16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
    if (row0 + r < S) v = *reinterpret_cast<const u16x8*>(base + (int64_t)(row0 + r) * sstride + ch * 8);
    t.v[i] = v;
  }
}

// registers -> a swizzled row image and/or a transposed image
template <int D, bool ROWS, bool TRANS>
__device__ __forceinline__ void store_tile(const TileRegs<D>& t, uint16_t* __restrict__ rows_img,
                                           uint16_t* __restrict__ t_img) {
  constexpr int NCH = D / 8;
#pragma unroll
  for (int i = 0; i < TileRegs<D>::N; ++i) {
    const int c = threadIdx.x + 256 * i, r = c / NCH, ch = c - r * NCH;
    if (ROWS) *reinterpret_cast<u16x8*>(rows_img + r * D + ((ch ^ (r & 7)) * 8)) = t.v[i];
    if (TRANS) {
#pragma unroll
      for (int e = 0; e < 8; ++e) t_img[(ch * 8 + e) * TS + r] = t.v[i][e];
    }
  }
}

template <int D, bool ROWS, bool TRANS>
__device__ __forceinline__ void stage_tile(const uint16_t* __restrict__ base, int64_t sstride, int row0, int S,
                                           uint16_t* __restrict__ rows_img, uint16_t* __restrict__ t_img) {
  TileRegs<D> t;
  load_tile<D>(base, sstride, row0, S, t);
  store_tile<D, ROWS, TRANS>(t, rows_img, t_img);
}

__device__ __forceinline__ u16x8 read_row_chunk(const uint16_t* img, int D, int r, int ch) {
  return *reinterpret_cast<const u16x8*>(img + r * D + ((ch ^ (r & 7)) * 8));
}

// 8 elements of transposed-image row `d`: columns [c0, c0+4) and [c1, c1+4)
__device__ __forceinline__ u16x8 read_t_pair(const uint16_t* t_img, int d, int c0, int c1) {
  const u16x4 a = *reinterpret_cast<const u16x4*>(t_img + d * TS + c0);
  const u16x4 b = *reinterpret_cast<const u16x4*>(t_img + d * TS + c1);
  u16x8 o = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return o;
}

// ============================================================================ forward
// One workgroup = 4 wave64s = FQ = 128 query rows of one (b, h); wave w owns 32 rows and runs the
// 32x32x16 MFMA (v_mfma_f32_32x32x16_{bf16,f16}): per 64-key tile 16 MFMAs for Sᵀ and 16 for O.
//  * Sᵀ = K·Qᵀ: A = K rows from LDS (ds_read_b128), B = this lane's query row held in registers for
//    the whole kernel; the accumulator leaves lane l with 32 scores of ONE query (q = l & 31) —
//    the row max needs one cross-half exchange, the row sum none until the end.
//  * Oᵀ += Vᵀ·Pᵀ: the score accumulator IS the B operand (registers 8s..8s+7 → bf16, §3
//    "accumulator tile as the next MFMA's operand"); Vᵀ comes from the row-major V tile through
//    ds_read_b64_tr_b16 (T10) with the matching permuted key order.  Oᵀ keeps the query on the
//    lane, so the online-softmax rescale is lane-local.
//  * K and V share one LDS image layout, `img_off`, conflict-free for both the b128 row reads and
//    the transposed reads.
//  * K/V tiles arrive by LDS-DMA into a 2-deep ring (no staging registers: the 32 Q + 64 O + 32 S
//    accumulator registers fit two waves per SIMD); tile kt+1's DMA flies under tile kt's MFMAs,
//    one barrier per tile.
//  * XCD-aware block order: the query blocks of one (b, h) — which share K/V — run on one XCD
//    (one L2), heaviest (causal) block first.
constexpr int FQ = 128;

template <typename T>
struct MM32;
template <>
struct MM32<bf16_t> {
  static __device__ __forceinline__ f32x16 mfma(u16x8 a, u16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b),
                                                   c, 0, 0, 0);
  }
};
template <>
struct MM32<f16_t> {
  static __device__ __forceinline__ f32x16 mfma(u16x8 a, u16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8_t, a), __builtin_bit_cast(f16x8_t, b), c,
                                                  0, 0, 0);
  }
};

// [64][D] tile image (cdna_hip_programming T10 form (a)): 8-row x 32-column subtiles of 512 B,
// the 4 chunks of a subtile row XOR-ed with (row >> 2) & 3.  Conflict-free for the 32x32x16 row
// reads (ds_read_b128) and transposed reads (ds_read_b64_tr_b16), and the reads of one wave differ
// by lane-independent constants — 2 address registers for all K reads, 2 for all V reads.
// Element offset of 16-byte chunk `ch` of row `row`:
template <int D>
__device__ __forceinline__ int img_off(int row, int ch) {
  return (row >> 3) * (8 * D) + (ch >> 2) * 256 + (row & 7) * 32 + (((ch & 3) ^ ((row >> 2) & 3)) << 3);
}

__device__ __forceinline__ u16x4 read_tr(const uint16_t* lds, int off) {
  const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(reinterpret_cast<uintptr_t>(lds + off)));
  return __builtin_bit_cast(u16x4, v);
}

template <typename T, int D, bool DROP>
__global__ __launch_bounds__(256, 2) void attn_fwd_k(AttnParams p) {
  constexpr int NS = D / 16;              // k-steps of the score product
  constexpr int NDB = D / 32;             // 32-wide head-dim blocks of Oᵀ
  constexpr int NCH = D / 8;              // 16-byte chunks per row
  constexpr int NPC = KB * D * 2 / 1024;  // 1-KiB DMA pieces per tile
  __shared__ __attribute__((aligned(16))) uint16_t Ks[2][KB * D];
  __shared__ __attribute__((aligned(16))) uint16_t Vs[2][KB * D];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 31, hh = lane >> 5;
  const int nqb = (p.S + FQ - 1) / FQ;
  const int total = nqb * p.B * p.H;
  int bid = blockIdx.x;
  {
    const int q8 = total / 8, r8 = total % 8, xcd = bid % 8, idx = bid / 8;
    bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + idx;
  }
  const int bh = bid / nqb, qblk = nqb - 1 - (bid - bh * nqb);
  const int b = bh / p.H, hd = bh - b * p.H;
  const int q0 = qblk * FQ;
  const int wq0 = q0 + 32 * w;  // this wave's first query
  const int qrow = wq0 + r;     // this lane's query
  const uint16_t* qb = static_cast<const uint16_t*>(p.q) + b * p.sqb + hd * p.sqh;
  const uint16_t* kb = static_cast<const uint16_t*>(p.k) + b * p.skb + hd * p.skh;
  const uint16_t* vb = static_cast<const uint16_t*>(p.v) + b * p.svb + hd * p.svh;

  u16x8 qf[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    u16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
    qf[s] = qrow < p.S ? *reinterpret_cast<const u16x8*>(qb + (int64_t)qrow * p.sqs + 16 * s + 8 * hh) : z;
  }
  f32x16 o[NDB];
#pragma unroll
  for (int n = 0; n < NDB; ++n)
#pragma unroll
    for (int e = 0; e < 16; ++e) o[n][e] = 0.f;
  float m = -INFINITY, l = 0.f;
  const float inv_keep = DROP ? 1.f / (1.f - p.p_drop) : 1.f;
  const uint32_t thr = (uint32_t)(p.p_drop * 4294967296.0);
  const uint64_t seed = DROP ? rng_key(p.rng) : 0;  // graph-safe generator state
  const uint8_t* kpm = p.kpm ? p.kpm + (int64_t)b * p.S : nullptr;

  int nkt = (p.S + KB - 1) / KB;
  if (p.causal) nkt = min(nkt, (min(q0 + FQ, p.S) - 1) / KB + 1);
  const int wave_last_q = min(wq0 + 31, p.S - 1);

  // tile kt -> LDS buffer kt & 1 by LDS-DMA (global_load_lds, 16 B per lane, 1 KiB per wave
  // instruction = two 512-B subtiles): the image is lane-linear, so the chunk XOR goes on the per-lane
  // SOURCE; rows past S re-read row S-1 (their scores are masked, their P is 0)
  auto dma_kv = [&](int k0, int buf) {
#pragma unroll
    for (int i = 0; i < NPC / 4; ++i) {
      const int pc = 4 * i + w, t = 2 * pc + (lane >> 5);  // subtile
      const int row = 8 * (t / (NCH / 4)) + ((lane & 31) >> 2);
      const int ch = 4 * (t % (NCH / 4)) + ((lane & 3) ^ ((row >> 2) & 3));
      const int64_t gr = min(k0 + row, p.S - 1);
      __builtin_amdgcn_global_load_lds((const void*)(kb + gr * p.sks + ch * 8),
                                       (void __attribute__((address_space(3)))*)(Ks[buf] + pc * 512), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(vb + gr * p.svs + ch * 8),
                                       (void __attribute__((address_space(3)))*)(Vs[buf] + pc * 512), 16, 0, 0);
    }
  };
  dma_kv(0, 0);
  // transposed-read addressing (T10): lane i of a 16-lane group supplies row (i >> 2), columns
  // 4 (i & 3) .. +3 of its group's 4 x 16 block; the group's columns are 16 (g & 1) .. +15 of a 32-wide
  // head-dim block and its rows 4 hh .. +3 (+8 for elements 4..7) of a 16-key k-step
  const int tr_row = 4 * hh + ((lane & 15) >> 2);
  const int tr_ch = 2 * ((lane >> 4) & 1) + ((lane & 3) >> 1);
  // img_off folded into per-lane bases + lane-independent constants (immediate offsets):
  //   K row read (block j, k-step s):   kbase[s & 1] + 32 D j + 256 (s >> 1)
  //   V tr read (k-step ks, block n, rows +8 hi): vbase[hi] + 16 D ks + 256 n
  int kbase[2], vbase[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    kbase[i] = (r >> 3) * 8 * D + (r & 7) * 32 + (((2 * i + hh) ^ ((r >> 2) & 3)) << 3);
    vbase[i] = i * 8 * D + tr_row * 32 + ((tr_ch ^ (hh + 2 * i)) << 3) + 4 * (lane & 1);
  }

  for (int kt = 0; kt < nkt; ++kt) {
    const int k0 = kt * KB;
    __builtin_amdgcn_s_waitcnt(0);  // this wave's DMA of tile kt has landed ...
    __syncthreads();                // ... every wave's; and tile kt-1's buffer is free
    if (kt + 1 < nkt) dma_kv(k0 + KB, (kt + 1) & 1);
    if (p.causal && k0 > wave_last_q) continue;  // wave-uniform: every key of the tile is masked
    const uint16_t* Kc = Ks[kt & 1];
    const uint16_t* Vc = Vs[kt & 1];

    f32x16 sacc[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
#pragma unroll
      for (int e = 0; e < 16; ++e) sacc[j][e] = 0.f;
#pragma unroll
      for (int s = 0; s < NS; ++s)
        sacc[j] = MM32<T>::mfma(*reinterpret_cast<const u16x8*>(Kc + kbase[s & 1] + 32 * D * j + 256 * (s >> 1)),
                                qf[s], sacc[j]);
    }
    // mask where the tile needs it (raw scores; the scale goes into the exponent below).  Key of
    // register e of block j: k0 + 32 j + 4 hh + crow(e), crow(e) = (e & 3) + 8 (e >> 2)
    if ((k0 + KB > p.S) || (p.causal && k0 + KB - 1 > wq0) || kpm) {  // wave-uniform
      uint64_t valid = ~0ull;  // bit kl: key k0 + kl may be attended (before the causal cut)
      if (k0 + KB > p.S) valid = (1ull << (p.S - k0)) - 1;
      if (kpm) valid &= ~__ballot(k0 + lane < p.S && kpm[k0 + lane] != 0);
      const int lim = (p.causal ? qrow - k0 : KB) - 4 * hh;  // causal: 32 j + crow(e) <= lim
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const uint32_t word = (uint32_t)(valid >> (32 * j)) >> (4 * hh);  // bit crow(e)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int cr = (e & 3) + 8 * (e >> 2);
          if (!((word >> cr) & 1) || 32 * j + cr > lim) sacc[j][e] = -INFINITY;
        }
      }
    }
    float mt = -INFINITY;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) mt = fmaxf(mt, sacc[j][e]);
    mt = fmaxf(mt, __shfl_xor(mt, 32, 64)) * p.scale_log2;  // scale > 0: max commutes with it
    const float mnew = fmaxf(m, mt);
    const float base = mnew == -INFINITY ? 0.f : mnew;
    const float alpha = exp2f(m - base);
    m = mnew;
    l *= alpha;
#pragma unroll
    for (int n = 0; n < NDB; ++n)
#pragma unroll
      for (int e = 0; e < 16; ++e) o[n][e] *= alpha;
    u16x8 pb[4];  // B fragments of the 4 key k-steps: step 2j + s = registers 8s..8s+7 of block j
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const float ex = exp2f(fmaf(sacc[j][e], p.scale_log2, -base));
        l += ex;
        sacc[j][e] = ex;
      }
    if constexpr (DROP) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int key = k0 + 32 * j + (e & 3) + 8 * (e >> 2) + 4 * hh;
          const uint64_t idx = (((uint64_t)bh * p.S + qrow) * p.S) + key;
          sacc[j][e] = hash_keep(seed, idx) >= thr ? sacc[j][e] * inv_keep : 0.f;
        }
    }
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) pb[2 * j + (e >> 3)][e & 7] = MM<T>::cvt(sacc[j][e]);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
#pragma unroll
      for (int n = 0; n < NDB; ++n) {
        const u16x4 lo = read_tr(Vc, vbase[0] + 16 * D * ks + 256 * n);
        const u16x4 hi = read_tr(Vc, vbase[1] + 16 * D * ks + 256 * n);
        const u16x8 a = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        o[n] = MM32<T>::mfma(a, pb[ks], o[n]);
      }
    }
  }
  l += __shfl_xor(l, 32, 64);
  const float inv = l > 0.f ? 1.f / l : 0.f;
  if (hh == 0 && qrow < p.S && p.lse) p.lse[(int64_t)bh * p.S + qrow] = l > 0.f ? m + log2f(l) : INFINITY;
  if (qrow < p.S) {
    uint16_t* orow = static_cast<uint16_t*>(p.o) + b * p.sob + hd * p.soh + (int64_t)qrow * p.sos;
    // Oᵀ register e of block n = head dim 32 n + 8 (e >> 2) + 4 hh + (e & 3)
#pragma unroll
    for (int n = 0; n < NDB; ++n)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        u16x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = MM<T>::cvt(o[n][4 * g + e] * inv);
        *reinterpret_cast<u16x4*>(orow + 32 * n + 8 * g + 4 * hh) = v;
      }
  }
}

// ============================================================================ backward
// delta[bh, q] = Σ_d dO·O ; also zero the fp32 dQ accumulator rows
template <typename T, int D>
__global__ __launch_bounds__(256) void attn_bwd_pre_k(AttnBwdParams p) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);  // over B*H*S
  if (row >= (int64_t)p.B * p.H * p.S) return;
  const int q = (int)(row % p.S);
  const int bh = (int)(row / p.S);
  const int b = bh / p.H, hd = bh - b * p.H;
  const uint16_t* o = static_cast<const uint16_t*>(p.o) + b * p.sob + hd * p.soh + (int64_t)q * p.sos;
  const uint16_t* g = static_cast<const uint16_t*>(p.dout) + b * p.sdob + hd * p.sdoh + (int64_t)q * p.sdos;
  float acc = 0.f;
  for (int d = lane; d < D; d += 64) acc += MM<T>::tof(o[d]) * MM<T>::tof(g[d]);
  acc = wave_sum(acc);
  if (lane == 0) p.delta[row] = acc;
  float* dq = p.dq_acc + row * D;
  for (int d = lane; d < D; d += 64) dq[d] = 0.f;
}

template <typename T, int D>
__global__ __launch_bounds__(256) void attn_bwd_k(AttnBwdParams p) {
  constexpr int NKK = D / 32;
  constexpr int NN = D / 16;
  __shared__ __attribute__((aligned(16))) uint16_t Qs[KB * D];
  __shared__ __attribute__((aligned(16))) uint16_t Qt[D * TS];
  __shared__ __attribute__((aligned(16))) uint16_t dOs[KB * D];
  __shared__ __attribute__((aligned(16))) uint16_t dOt[D * TS];
  __shared__ __attribute__((aligned(16))) uint16_t Kt[D * TS];
  __shared__ __attribute__((aligned(16))) uint16_t dSs[KB * (KB + 8)];
  __shared__ float lse_s[KB];
  __shared__ float delta_s[KB];

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 4, c16 = lane & 15;
  const int bh = blockIdx.y, b = bh / p.H, hd = bh - b * p.H;
  const int k0 = blockIdx.x * KB;
  const int key = k0 + 16 * w + c16;  // this lane's key (C-tile column)
  const uint16_t* qb = static_cast<const uint16_t*>(p.q) + b * p.sqb + hd * p.sqh;
  const uint16_t* kb = static_cast<const uint16_t*>(p.k) + b * p.skb + hd * p.skh;
  const uint16_t* vb = static_cast<const uint16_t*>(p.v) + b * p.svb + hd * p.svh;
  const uint16_t* gb = static_cast<const uint16_t*>(p.dout) + b * p.sdob + hd * p.sdoh;

  u16x8 kf[NKK], vf[NKK];
#pragma unroll
  for (int kk = 0; kk < NKK; ++kk) {
    u16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
    kf[kk] = key < p.S ? *reinterpret_cast<const u16x8*>(kb + (int64_t)key * p.sks + 8 * h + 32 * kk) : z;
    vf[kk] = key < p.S ? *reinterpret_cast<const u16x8*>(vb + (int64_t)key * p.svs + 8 * h + 32 * kk) : z;
  }
  stage_tile<D, false, true>(kb, p.sks, k0, p.S, nullptr, Kt);

  f32x4 dvt[NN], dkt[NN];
#pragma unroll
  for (int n = 0; n < NN; ++n) dvt[n] = dkt[n] = f32x4{0.f, 0.f, 0.f, 0.f};
  const float inv_keep = p.p_drop > 0.f ? 1.f / (1.f - p.p_drop) : 1.f;
  const uint32_t thr = (uint32_t)(p.p_drop * 4294967296.0);
  const uint64_t seed = p.p_drop > 0.f ? rng_key(p.rng) : 0;  // graph-safe generator state
  const bool key_masked = key >= p.S || (p.kpm && p.kpm[(int64_t)b * p.S + key] != 0);

  const int nq = (p.S + KB - 1) / KB;
  const int qt0 = p.causal ? k0 / KB : 0;
  TileRegs<D> qr, gr;  // the next query tile, in flight while the current one computes
  float lse_r = INFINITY, delta_r = 0.f;
  auto load_q = [&](int q0n) {
    load_tile<D>(qb, p.sqs, q0n, p.S, qr);
    load_tile<D>(gb, p.sdos, q0n, p.S, gr);
    if (threadIdx.x < KB) {
      const int qq = q0n + threadIdx.x;
      lse_r = qq < p.S ? p.lse[(int64_t)bh * p.S + qq] : INFINITY;
      delta_r = qq < p.S ? p.delta[(int64_t)bh * p.S + qq] : 0.f;
    }
  };
  if (qt0 < nq) load_q(qt0 * KB);
  for (int qt = qt0; qt < nq; ++qt) {
    const int q0 = qt * KB;
    __syncthreads();
    store_tile<D, true, true>(qr, Qs, Qt);
    store_tile<D, true, true>(gr, dOs, dOt);
    if (threadIdx.x < KB) {
      lse_s[threadIdx.x] = lse_r;
      delta_s[threadIdx.x] = delta_r;
    }
    if (qt + 1 < nq) load_q(q0 + KB);
    __syncthreads();

    float pd[4][4], ds[4][4];
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      f32x4 s = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < NKK; ++kk) {
        s = MM<T>::mfma(read_row_chunk(Qs, D, 16 * qq + c16, h + 4 * kk), kf[kk], s);
        dp = MM<T>::mfma(read_row_chunk(dOs, D, 16 * qq + c16, h + 4 * kk), vf[kk], dp);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ql = 16 * qq + 4 * h + r;
        const int qg = q0 + ql;
        bool ok = !key_masked;
        if (p.causal) ok = ok && key <= qg;
        const float pv = ok ? exp2f(s[r] * p.scale_log2 - lse_s[ql]) : 0.f;
        float dpv = dp[r];
        float pdv = pv;
        if (p.p_drop > 0.f) {
          const uint64_t idx = (((uint64_t)bh * p.S + qg) * p.S) + key;
          const bool keep = hash_keep(seed, idx) >= thr;
          pdv = keep ? pv * inv_keep : 0.f;
          dpv = keep ? dpv * inv_keep : 0.f;
        }
        pd[qq][r] = pdv;
        ds[qq][r] = pv * (dpv - delta_s[ql]);
      }
    }
    // dVᵀ += dOᵀ·P_drop ; dKᵀ += Qᵀ·dS    (k = query, permuted order within each 32-step)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      u16x8 bp, bs;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        bp[r] = MM<T>::cvt(pd[2 * s2][r]);
        bp[4 + r] = MM<T>::cvt(pd[2 * s2 + 1][r]);
        bs[r] = MM<T>::cvt(ds[2 * s2][r]);
        bs[4 + r] = MM<T>::cvt(ds[2 * s2 + 1][r]);
      }
#pragma unroll
      for (int n = 0; n < NN; ++n) {
        const int d = 16 * n + c16;
        dvt[n] = MM<T>::mfma(read_t_pair(dOt, d, 32 * s2 + 4 * h, 32 * s2 + 16 + 4 * h), bp, dvt[n]);
        dkt[n] = MM<T>::mfma(read_t_pair(Qt, d, 32 * s2 + 4 * h, 32 * s2 + 16 + 4 * h), bs, dkt[n]);
      }
    }
    // dQ: dS image [q][key] in LDS, then wave w reduces its 16 query rows over the 64 keys
#pragma unroll
    for (int qq = 0; qq < 4; ++qq)
#pragma unroll
      for (int r = 0; r < 4; ++r) dSs[(16 * qq + 4 * h + r) * (KB + 8) + 16 * w + c16] = MM<T>::cvt(ds[qq][r]);
    __syncthreads();
#pragma unroll
    for (int n = 0; n < NN; ++n) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const u16x8 a = *reinterpret_cast<const u16x8*>(dSs + (16 * w + c16) * (KB + 8) + 32 * s2 + 8 * h);
        const u16x8 bk = *reinterpret_cast<const u16x8*>(Kt + (16 * n + c16) * TS + 32 * s2 + 8 * h);
        acc = MM<T>::mfma(a, bk, acc);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int qg = q0 + 16 * w + 4 * h + r;
        if (qg < p.S) atomicAdd(p.dq_acc + ((int64_t)bh * p.S + qg) * D + 16 * n + c16, acc[r] * p.scale);
      }
    }
  }
  // write dK, dV: lane holds [d = 16n + 4h + r][key] for r = 0..3 (4 consecutive d)
  if (key < p.S) {
    uint16_t* dk = static_cast<uint16_t*>(p.dk) + b * p.sdkb + hd * p.sdkh + (int64_t)key * p.sdks;
    uint16_t* dv = static_cast<uint16_t*>(p.dv) + b * p.sdvb + hd * p.sdvh + (int64_t)key * p.sdvs;
#pragma unroll
    for (int n = 0; n < NN; ++n) {
      u16x4 kv, vv;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        kv[r] = MM<T>::cvt(dkt[n][r] * p.scale);
        vv[r] = MM<T>::cvt(dvt[n][r]);
      }
      *reinterpret_cast<u16x4*>(dk + 16 * n + 4 * h) = kv;
      *reinterpret_cast<u16x4*>(dv + 16 * n + 4 * h) = vv;
    }
  }
}

template <typename T, int D>
__global__ __launch_bounds__(256) void attn_bwd_post_k(AttnBwdParams p) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // over B*H*S*D/4
  const int64_t total = (int64_t)p.B * p.H * p.S * (D / 4);
  if (i >= total) return;
  const int64_t row = i / (D / 4);
  const int d = (int)(i - row * (D / 4)) * 4;
  const int q = (int)(row % p.S);
  const int bh = (int)(row / p.S);
  const int b = bh / p.H, hd = bh - b * p.H;
  const float4 v = *reinterpret_cast<const float4*>(p.dq_acc + row * D + d);
  uint16_t* dq = static_cast<uint16_t*>(p.dq) + b * p.sdqb + hd * p.sdqh + (int64_t)q * p.sdqs + d;
  u16x4 o = {MM<T>::cvt(v.x), MM<T>::cvt(v.y), MM<T>::cvt(v.z), MM<T>::cvt(v.w)};
  *reinterpret_cast<u16x4*>(dq) = o;
}

template <typename T, int D>
hipError_t fwd_launch(const AttnParams& p, hipStream_t st) {
  const dim3 grid(((p.S + FQ - 1) / FQ) * p.B * p.H);
  if (p.p_drop > 0.f) hipLaunchKernelGGL((attn_fwd_k<T, D, true>), grid, dim3(256), 0, st, p);
  else hipLaunchKernelGGL((attn_fwd_k<T, D, false>), grid, dim3(256), 0, st, p);
  return hipGetLastError();
}

template <typename T, int D>
hipError_t bwd_launch(const AttnBwdParams& p, hipStream_t st) {
  const int64_t rows = (int64_t)p.B * p.H * p.S;
  hipLaunchKernelGGL((attn_bwd_pre_k<T, D>), dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, st, p);
  const dim3 grid((p.S + KB - 1) / KB, p.B * p.H);
  hipLaunchKernelGGL((attn_bwd_k<T, D>), grid, dim3(256), 0, st, p);
  const int64_t tot = rows * (D / 4);
  hipLaunchKernelGGL((attn_bwd_post_k<T, D>), dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, p);
  return hipGetLastError();
}

}  // namespace

bool attention_supported(int dtype, int D) { return (dtype == kBF16 || dtype == kF16) && (D == 64 || D == 128); }

hipError_t attention_forward(int dtype, const AttnParams& p, hipStream_t st) {
  if (!attention_supported(dtype, p.D)) return hipErrorInvalidValue;
  if (dtype == kBF16) return p.D == 64 ? fwd_launch<bf16_t, 64>(p, st) : fwd_launch<bf16_t, 128>(p, st);
  return p.D == 64 ? fwd_launch<f16_t, 64>(p, st) : fwd_launch<f16_t, 128>(p, st);
}

hipError_t attention_backward(int dtype, const AttnBwdParams& p, hipStream_t st) {
  if (!attention_supported(dtype, p.D)) return hipErrorInvalidValue;
  if (dtype == kBF16) return p.D == 64 ? bwd_launch<bf16_t, 64>(p, st) : bwd_launch<bf16_t, 128>(p, st);
  return p.D == 64 ? bwd_launch<f16_t, 64>(p, st) : bwd_launch<f16_t, 128>(p, st);
}

}  // namespace hyp

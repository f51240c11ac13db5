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
// Backward: 128 keys per workgroup on the 32x32x16 MFMA (details at attn_bwd_k); dQ stored directly
// when one key block covers the sequence, else accumulated with fp32 atomics.
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
constexpr int FQ = 128;  // query rows of the default (4-wave) forward workgroup
// attn_set_fwd_narrow (A/B, default off): one-wave forward workgroups measured no faster on the
// Llama LoRA step (14.58-14.60 vs 14.54-14.57 ms, profiles/r05/attn_fwd_narrow_ab.txt)
int g_attn_fwd_narrow = 0;

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

// NWV: waves per workgroup (FQ = 32 NWV query rows).  4 by default; 1 (opt-in) for grids that would
// leave most CUs idle (Llama-2-7B at batch 1, S = 128: 32 workgroups of 4 waves -> 128 of 1)
template <typename T, int D, bool DROP, int NWV = 4>
__global__ __launch_bounds__(64 * NWV, 2) void attn_fwd_k(AttnParams p) {
  constexpr int FQ = 32 * NWV;
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
    for (int i = 0; i < NPC / NWV; ++i) {
      const int pc = NWV * i + w, t = 2 * pc + (lane >> 5);  // subtile
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
    if (wq0 >= p.S) continue;  // wave-uniform: the padded query tail (S = 197: rows 224-255) — nothing stored
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
// delta[bh, q] = Σ_d dO·O ; also zero the fp32 dQ accumulator rows (when there is one).
// D / 8 lanes per row, one 16-byte load of O and of dO per lane, a shuffle reduction in the group.
template <typename T, int D>
__global__ __launch_bounds__(256) void attn_bwd_pre_k(AttnBwdParams p) {
  constexpr int LPR = D / 8;  // lanes per row
  const int64_t row = ((int64_t)blockIdx.x * 256 + threadIdx.x) / LPR;  // over B*H*S
  const int c = threadIdx.x % LPR;
  const bool ok = row < (int64_t)p.B * p.H * p.S;
  float acc = 0.f;
  if (ok) {
    const int q = (int)(row % p.S);
    const int bh = (int)(row / p.S);
    const int b = bh / p.H, hd = bh - b * p.H;
    const u16x8 o = *reinterpret_cast<const u16x8*>(static_cast<const uint16_t*>(p.o) + b * p.sob + hd * p.soh +
                                                    (int64_t)q * p.sos + 8 * c);
    const u16x8 g = *reinterpret_cast<const u16x8*>(static_cast<const uint16_t*>(p.dout) + b * p.sdob +
                                                    hd * p.sdoh + (int64_t)q * p.sdos + 8 * c);
#pragma unroll
    for (int e = 0; e < 8; ++e) acc += MM<T>::tof(o[e]) * MM<T>::tof(g[e]);
    if (p.dq_acc && p.dq_slabs == 0) {  // (slab mode: every slab row is stored, nothing to clear)
      float4* dq = reinterpret_cast<float4*>(p.dq_acc + row * D + 8 * c);
      dq[0] = make_float4(0.f, 0.f, 0.f, 0.f);
      dq[1] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
#pragma unroll
  for (int m = 1; m < LPR; m <<= 1) acc += __shfl_xor(acc, m, 64);
  if (ok && c == 0) p.delta[row] = acc;
}

// One workgroup = 4 wave64s = BKB = 128 keys of one (b, h); wave w owns keys kw0 = k0 + 32 w .. +31
// and keeps dKᵀ, dVᵀ of them in registers ([d][key] 32x32 blocks: key on the lane) while the
// workgroup sweeps query slices of QS rows (32 for D = 128, 64 for D = 64) — 32x32x16 MFMAs:
//  * S = Q·Kᵀ and dP = dO·Vᵀ with the KEY on the lane (A = Q / dO rows from LDS, B = this wave's
//    K rows from LDS / V rows held in registers): their accumulators are directly the B operands
//    of dVᵀ += dOᵀ·P and dKᵀ += Qᵀ·dS (§3 accumulator-as-operand; Aᵀ by ds_read_b64_tr_b16 from the
//    same Q / dO images);
//  * dS crosses LDS once, as a [key][q] image written 8 bytes per lane, and dQ = dS·K is one
//    32x32 block per wave (A = dS by transposed reads, B = K by transposed reads of the K image);
//  * S <= 128 (one key block per (b, h): Llama / LM sequence lengths): dQ is complete inside the
//    workgroup and is stored directly — no fp32 workspace, no atomics, no conversion pass;
//    longer sequences add it with fp32 atomics into dq_acc (zeroed by attn_bwd_pre_k, converted by
//    attn_bwd_post_k);
//  * Q / dO slices (and their LSE / delta rows) arrive by LDS-DMA into a 2-deep ring, one barrier
//    pair per slice; XCD-grouped blocks, heaviest (causal) key block first.
constexpr int BKB = 128;

// D = 128 keeps 128 accumulator + 32 V-operand registers per lane live across the sweep: one wave
// per SIMD with the whole register file (a 256-register cap spilled the V operand to scratch);
// D = 64 fits two workgroups per CU.
// ROPE (D = 128): dQ and dK leave through the inverse rotary embedding (the forward applied RoPE to
// q and k in the projection epilogue) — the rotate-half partner of a dK column is in the same lane,
// the partner of a dQ block is the block of wave w ^ 2 (exchanged through LDS).
template <typename T, int D, bool DROP, bool DIRECT, bool ROPE = false>
__global__ __launch_bounds__(256, D == 128 ? 1 : 2) void attn_bwd_k(AttnBwdParams p) {
  constexpr int NS = D / 16;    // k-steps over the head dim
  constexpr int NDB = D / 32;   // 32-wide head-dim blocks
  constexpr int NCH = D / 8;    // 16-byte chunks per row
  constexpr int QS = 4096 / D;  // query rows per slice
  constexpr int NQB = QS / 32;  // 32-row query blocks per slice
  constexpr int SPC = QS * D * 2 / 1024;   // 1-KiB DMA pieces per Q (or dO) slice
  constexpr int KPC = BKB * D * 2 / 1024;  // ... per K tile
  constexpr int DSU = QS / 4;              // 8-byte units per dSᵀ row
  __shared__ __attribute__((aligned(16))) uint16_t Ks[BKB * D];
  __shared__ __attribute__((aligned(16))) uint16_t Qs[2][QS * D];
  __shared__ __attribute__((aligned(16))) uint16_t dOs[2][QS * D];
  __shared__ __attribute__((aligned(16))) uint16_t dSt[BKB * QS];
  __shared__ __attribute__((aligned(16))) float lse_s[2][64];
  __shared__ __attribute__((aligned(16))) float del_s[2][64];
  __shared__ float rope_x[ROPE ? 4 * 16 * 64 : 1];  // dQ blocks of the 4 waves [wave][e][lane]
  // direct D = 128 (one key block per (b, h): each query slice is visited once): delta = rowsum(dO·O)
  // is computed here from an O slice staged beside dO — no separate pre-pass launch
  constexpr bool FDELTA = DIRECT && D == 128;
  __shared__ __attribute__((aligned(16))) uint16_t Os[FDELTA ? 2 : 1][FDELTA ? QS * D : 8];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 31, hh = lane >> 5;
  const int nkb = (p.S + BKB - 1) / BKB;
  const int qsplit = DIRECT ? p.qsplit : 1;  // query-slice split of one (b, h) (adjacent ids: one XCD)
  const int total = nkb * p.B * p.H * qsplit;
  int bid = blockIdx.x;
  {
    const int q8 = total / 8, r8 = total % 8, xcd = bid % 8, idx = bid / 8;
    bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + idx;
  }
  const int zq = bid % qsplit;
  bid /= qsplit;
  const int bh = bid / nkb, kblk = bid - bh * nkb;
  const int b = bh / p.H, hd = bh - b * p.H;
  const int k0 = kblk * BKB, kw0 = k0 + 32 * w, key = kw0 + r;
  const uint16_t* qb = static_cast<const uint16_t*>(p.q) + b * p.sqb + hd * p.sqh;
  const uint16_t* kb = static_cast<const uint16_t*>(p.k) + b * p.skb + hd * p.skh;
  const uint16_t* vb = static_cast<const uint16_t*>(p.v) + b * p.svb + hd * p.svh;
  const uint16_t* gb = static_cast<const uint16_t*>(p.dout) + b * p.sdob + hd * p.sdoh;
  const float* lse_g = p.lse + (int64_t)bh * p.S;
  const float* del_g = p.delta + (int64_t)bh * p.S;

  auto dma_rows = [&](const uint16_t* base, int64_t sstride, int row0, uint16_t* img, int npieces) {
    for (int pc = w; pc < npieces; pc += 4) {
      const int t = 2 * pc + (lane >> 5);
      const int row = 8 * (t / (NCH / 4)) + ((lane & 31) >> 2);
      const int ch = 4 * (t % (NCH / 4)) + ((lane & 3) ^ ((row >> 2) & 3));
      const int64_t gr = min(row0 + row, p.S - 1);
      __builtin_amdgcn_global_load_lds((const void*)(base + gr * sstride + ch * 8),
                                       (void __attribute__((address_space(3)))*)(img + pc * 512), 16, 0, 0);
    }
  };
  const uint16_t* ob = static_cast<const uint16_t*>(p.o) + b * p.sob + hd * p.soh;
  auto dma_slice = [&](int q0, int buf) {
    dma_rows(qb, p.sqs, q0, Qs[buf], SPC);
    dma_rows(gb, p.sdos, q0, dOs[buf], SPC);
    if constexpr (FDELTA) dma_rows(ob, p.sos, q0, Os[buf], SPC);
    if (w < (FDELTA ? 1 : 2)) {
      const float* src = (w == 0 ? lse_g : del_g) + min(q0 + lane, p.S - 1);
      __builtin_amdgcn_global_load_lds((const void*)src,
                                       (void __attribute__((address_space(3)))*)(w == 0 ? lse_s[buf] : del_s[buf]),
                                       4, 0, 0);
    }
  };

  // this wave's V rows as the B operand of dP (key on the lane)
  u16x8 vf[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    u16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
    vf[s] = key < p.S ? *reinterpret_cast<const u16x8*>(vb + (int64_t)key * p.svs + 16 * s + 8 * hh) : z;
  }
  const bool key_ok = key < p.S && !(p.kpm && p.kpm[(int64_t)b * p.S + key] != 0);
  const float inv_keep = DROP ? 1.f / (1.f - p.p_drop) : 1.f;
  const uint32_t thr = (uint32_t)(p.p_drop * 4294967296.0);
  const uint64_t seed = DROP ? rng_key(p.rng) : 0;  // graph-safe generator state

  const int qstart = p.causal ? (k0 / QS) * QS : 0;
  const int nsl = qstart < p.S ? (p.S - qstart + QS - 1) / QS : 0;
  dma_rows(kb, p.sks, k0, Ks, KPC);
  if (zq < nsl) dma_slice(qstart + zq * QS, 0);

  f32x16 dvt[NDB], dkt[NDB];
#pragma unroll
  for (int n = 0; n < NDB; ++n)
#pragma unroll
    for (int e = 0; e < 16; ++e) dvt[n][e] = dkt[n][e] = 0.f;

  // per-lane LDS bases (reads of a wave differ by lane-independent constants)
  const int tr_row = 4 * hh + ((lane & 15) >> 2);
  const int tr_ch = 2 * ((lane >> 4) & 1) + ((lane & 3) >> 1);
  int rbase[2], tbase[2];  // row reads (k-step parity) / transposed reads (+8 rows) of a Q-like image
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    rbase[i] = (r >> 3) * 8 * D + (r & 7) * 32 + (((2 * i + hh) ^ ((r >> 2) & 3)) << 3);
    tbase[i] = i * 8 * D + tr_row * 32 + ((tr_ch ^ (hh + 2 * i)) << 3) + 4 * (lane & 1);
  }
  // dQ block of this wave and the dSᵀ image swizzle (8-byte units of 4 queries)
  const int dq_qb = w / NDB, dq_db = w % NDB;
  auto dsw = [](int row) { return QS == 32 ? ((row >> 1) & 7) : ((row & 15) ^ (((row >> 1) & 1) << 3)); };
  // dQ operands by transposed reads, key k-step ks (16 keys) at + 16 QS ks / + 16 D ks:
  //   A = dS[q][key] from the dSᵀ image, B = K[key][d] from the K image; lane (group g, i = 4 qq + pp)
  //   addresses key row 16 ks + 8 hh + 4 t + qq, query / head-dim columns 16 (g & 1) + 4 pp .. +3
  int dqa[2], dqb[2];
  {
    const int gq = 16 * ((lane >> 4) & 1), qq = (lane & 15) >> 2, pp = lane & 3;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int row = 8 * hh + 4 * t + qq;
      const int u = (32 * dq_qb + gq) / 4 + pp;
      dqa[t] = row * QS + 4 * (u ^ dsw(row));
      dqb[t] = img_off<D>(row, 4 * dq_db + (gq >> 3) + (pp >> 1)) + 4 * (pp & 1);
    }
  }
  // dSᵀ write of register group g (block qbk): row 32 w + r, unit 8 qbk + 2 g + hh
  const int ds_row = 32 * w + r;

  for (int sl = zq, it = 0; sl < nsl; sl += qsplit, ++it) {  // this workgroup's slices zq, zq + qsplit, ...
    const int q0 = qstart + sl * QS, cur = it & 1;
    __builtin_amdgcn_s_waitcnt(0);  // this wave's DMA of slice sl (and the K tile) has landed ...
    __syncthreads();                // ... every wave's; the previous slice's buffers and dSt are free
    if (sl + qsplit < nsl) dma_slice(q0 + qsplit * QS, cur ^ 1);
    const uint16_t* Qc = Qs[cur];
    const uint16_t* Gc = dOs[cur];
    if constexpr (FDELTA) {  // delta[q] = Σ_d dO·O: 8 threads per query row, 16 columns each
      const int row = tid >> 3, part = tid & 7;
      float acc = 0.f;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int off = img_off<D>(row, 2 * part + c);
        const u16x8 g8 = *reinterpret_cast<const u16x8*>(Gc + off);
        const u16x8 o8 = *reinterpret_cast<const u16x8*>(Os[cur] + off);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc += MM<T>::tof(g8[e]) * MM<T>::tof(o8[e]);
      }
      acc += __shfl_xor(acc, 1, 64);
      acc += __shfl_xor(acc, 2, 64);
      acc += __shfl_xor(acc, 4, 64);
      if (part == 0) del_s[cur][row] = acc;
      __syncthreads();
    }
#pragma unroll
    for (int qbk = 0; qbk < NQB; ++qbk) {
      const int qbase = q0 + 32 * qbk;
      // wave-uniform: the whole block is masked (causal), past the sequence end (the padded query
      // tail of S = 197: ViT), or this wave's 32 keys are all past it — P = dS = 0 there, so only
      // the zero dSᵀ entries are needed (dV / dK / dQ terms of the block are exactly zero)
      if ((p.causal && kw0 > qbase + 31) || qbase >= p.S || kw0 >= p.S) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int u = 8 * qbk + 2 * g + hh;
          *reinterpret_cast<uint2*>(dSt + ds_row * QS + 4 * (u ^ dsw(ds_row))) = make_uint2(0u, 0u);
        }
        continue;
      }
      f32x16 sacc, dpacc;
#pragma unroll
      for (int e = 0; e < 16; ++e) sacc[e] = dpacc[e] = 0.f;
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const int qo = rbase[s & 1] + 32 * D * qbk + 256 * (s >> 1);
        const u16x8 kf = *reinterpret_cast<const u16x8*>(Ks + rbase[s & 1] + 32 * D * w + 256 * (s >> 1));
        sacc = MM32<T>::mfma(*reinterpret_cast<const u16x8*>(Qc + qo), kf, sacc);
        dpacc = MM32<T>::mfma(*reinterpret_cast<const u16x8*>(Gc + qo), vf[s], dpacc);
      }
      // P, dS; register e holds query qbase + crow(e), crow(e) = (e & 3) + 8 (e >> 2) + 4 hh
      const bool edge = !key_ok || (p.causal && kw0 + 31 > qbase) || qbase + 32 > p.S;
      u16x8 pb[2], sb[2];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int ql = 32 * qbk + 8 * g + 4 * hh;  // slice-local query of register 4g
        const float4 ls = *reinterpret_cast<const float4*>(&lse_s[cur][ql]);
        const float4 dl = *reinterpret_cast<const float4*>(&del_s[cur][ql]);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int e = 4 * g + i;
          float pv = exp2f(fmaf(sacc[e], p.scale_log2, -(&ls.x)[i]));
          if (edge) {
            const int qg = q0 + ql + i;
            if (!key_ok || qg >= p.S || (p.causal && key > qg)) pv = 0.f;
          }
          float dpv = dpacc[e], pdv = pv;
          if constexpr (DROP) {
            const int qg = q0 + ql + i;
            const uint64_t idx = (((uint64_t)bh * p.S + qg) * p.S) + key;
            const bool keep = hash_keep(seed, idx) >= thr;
            pdv = keep ? pv * inv_keep : 0.f;
            dpv = keep ? dpv * inv_keep : 0.f;
          }
          pb[e >> 3][e & 7] = MM<T>::cvt(pdv);
          sb[e >> 3][e & 7] = MM<T>::cvt(pv * (dpv - (&dl.x)[i]));
        }
      }
      // dVᵀ += dOᵀ·P, dKᵀ += Qᵀ·dS  (k = query, the accumulator's permuted order)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int n = 0; n < NDB; ++n) {
          const int off = 32 * D * qbk + 16 * D * s2 + 256 * n;
          const u16x4 glo = read_tr(Gc, tbase[0] + off), ghi = read_tr(Gc, tbase[1] + off);
          const u16x4 qlo = read_tr(Qc, tbase[0] + off), qhi = read_tr(Qc, tbase[1] + off);
          const u16x8 ga = {glo[0], glo[1], glo[2], glo[3], ghi[0], ghi[1], ghi[2], ghi[3]};
          const u16x8 qa = {qlo[0], qlo[1], qlo[2], qlo[3], qhi[0], qhi[1], qhi[2], qhi[3]};
          dvt[n] = MM32<T>::mfma(ga, pb[s2], dvt[n]);
          dkt[n] = MM32<T>::mfma(qa, sb[s2], dkt[n]);
        }
      // dSᵀ image: registers 4g..4g+3 = queries 32 qbk + 8 g + 4 hh + 0..3 of key row 32 w + r
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int u = 8 * qbk + 2 * g + hh;
        const u16x8& src = sb[g >> 1];
        const int o4 = 4 * (g & 1);
        const uint2 v = make_uint2((uint32_t)src[o4] | ((uint32_t)src[o4 + 1] << 16),
                                   (uint32_t)src[o4 + 2] | ((uint32_t)src[o4 + 3] << 16));
        *reinterpret_cast<uint2*>(dSt + ds_row * QS + 4 * (u ^ dsw(ds_row))) = v;
      }
    }
    __syncthreads();  // dSᵀ complete
    // dQ[32 dq_qb + .., 32 dq_db + ..] = Σ_key dS·K over the workgroup's 128 keys
    {
      f32x16 acc;
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[e] = 0.f;
      float2 rcs[ROPE ? 16 : 1];  // (cos, sin) of this lane's 16 dQ entries, in flight under the MFMAs
      if constexpr (ROPE) {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int qg = min(q0 + 32 * dq_qb + (e & 3) + 8 * (e >> 2) + 4 * hh, p.S - 1);
          rcs[e] = p.rope_cs[(int64_t)qg * 64 + ((32 * dq_db + r) & 63)];
        }
      }
#pragma unroll
      for (int ks = 0; ks < BKB / 16; ++ks) {
        const u16x4 a0 = read_tr(dSt, dqa[0] + 16 * QS * ks), a1 = read_tr(dSt, dqa[1] + 16 * QS * ks);
        const u16x4 b0 = read_tr(Ks, dqb[0] + 16 * D * ks), b1 = read_tr(Ks, dqb[1] + 16 * D * ks);
        const u16x8 a = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
        const u16x8 bk = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
        acc = MM32<T>::mfma(a, bk, acc);
      }
      // acc[e] = dQ[query q0 + 32 dq_qb + crow(e)][head dim 32 dq_db + r]
      const int d = 32 * dq_db + r;
      if constexpr (ROPE) {  // inverse rotation: partner head-dim block dq_db ^ 2 lives in wave w ^ 2
        static_assert(D == 128, "fused RoPE backward: head_dim 128");
#pragma unroll
        for (int e = 0; e < 16; ++e) rope_x[(w * 16 + e) * 64 + lane] = acc[e];
        __syncthreads();
        const bool lo = dq_db < 2;  // this block holds x0 (first half of the head)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const float other = rope_x[(((w ^ 2) * 16) + e) * 64 + lane];
          acc[e] = lo ? acc[e] * rcs[e].x + other * rcs[e].y : acc[e] * rcs[e].x - other * rcs[e].y;
        }
      }
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int qg = q0 + 32 * dq_qb + (e & 3) + 8 * (e >> 2) + 4 * hh;
        if (qg < p.S) {
          if constexpr (DIRECT) {
            uint16_t* dq = static_cast<uint16_t*>(p.dq) + b * p.sdqb + hd * p.sdqh + (int64_t)qg * p.sdqs;
            dq[d] = MM<T>::cvt(acc[e] * p.scale);
          } else {
            if (p.dq_slabs)  // one fp32 slab per key block, summed in order by attn_bwd_post_k
              p.dq_acc[(((int64_t)kblk * p.B * p.H + bh) * p.S + qg) * D + d] = acc[e] * p.scale;
            else
              atomicAdd(p.dq_acc + ((int64_t)bh * p.S + qg) * D + d, acc[e] * p.scale);
          }
        }
      }
    }
  }
  // dK, dV: lane holds [d = 32 n + 8 g + 4 hh + 0..3][key]
  if (key < p.S) {
    uint16_t* dk = static_cast<uint16_t*>(p.dk) + b * p.sdkb + hd * p.sdkh + (int64_t)key * p.sdks;
    uint16_t* dv = static_cast<uint16_t*>(p.dv) + b * p.sdvb + hd * p.sdvh + (int64_t)key * p.sdvs;
    if constexpr (ROPE) {  // inverse rotation of dK: columns d and d + 64 are blocks n and n + 2 of this lane
      float2 kcs[2][16];
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int e = 0; e < 16; ++e) kcs[n][e] = p.rope_cs[(int64_t)key * 64 + 32 * n + 8 * (e >> 2) + 4 * hh + (e & 3)];
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const float x0 = dkt[n][e], x1 = dkt[n + 2][e];
          dkt[n][e] = x0 * kcs[n][e].x + x1 * kcs[n][e].y;
          dkt[n + 2][e] = x1 * kcs[n][e].x - x0 * kcs[n][e].y;
        }
    }
    if (qsplit > 1) {  // partial sums over this workgroup's query slices: fp32, summed by attn_bwd_kv_sum_k
      const int64_t plane = (int64_t)p.B * p.H * p.S * D;
      float* pk = p.dkv_part + (int64_t)zq * 2 * plane + ((int64_t)bh * p.S + key) * D;
      float* pv = pk + plane;
#pragma unroll
      for (int n = 0; n < NDB; ++n)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          *reinterpret_cast<float4*>(pk + 32 * n + 8 * g + 4 * hh) =
              make_float4(dkt[n][4 * g] * p.scale, dkt[n][4 * g + 1] * p.scale, dkt[n][4 * g + 2] * p.scale,
                          dkt[n][4 * g + 3] * p.scale);
          *reinterpret_cast<float4*>(pv + 32 * n + 8 * g + 4 * hh) =
              make_float4(dvt[n][4 * g], dvt[n][4 * g + 1], dvt[n][4 * g + 2], dvt[n][4 * g + 3]);
        }
      return;
    }
#pragma unroll
    for (int n = 0; n < NDB; ++n)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        u16x4 kv, vv;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          kv[i] = MM<T>::cvt(dkt[n][4 * g + i] * p.scale);
          vv[i] = MM<T>::cvt(dvt[n][4 * g + i]);
        }
        *reinterpret_cast<u16x4*>(dk + 32 * n + 8 * g + 4 * hh) = kv;
        *reinterpret_cast<u16x4*>(dv + 32 * n + 8 * g + 4 * hh) = vv;
      }
  }
}

// dK, dV = Σ_z partial[z] (fixed order: deterministic) of the query-split direct backward
template <typename T, int D>
__global__ __launch_bounds__(256) void attn_bwd_kv_sum_k(AttnBwdParams p) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // over 2 * B*H*S*D/4 quads
  const int64_t plane = (int64_t)p.B * p.H * p.S * D;
  const int64_t half = plane / 4;
  if (i >= 2 * half) return;
  const int which = i >= half ? 1 : 0;
  const int64_t e = (i - which * half) * 4;
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int z = 0; z < p.qsplit; ++z) {
    const float4 u = *reinterpret_cast<const float4*>(p.dkv_part + ((int64_t)z * 2 + which) * plane + e);
    v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
  }
  const int64_t row = e / D;
  const int d = (int)(e - row * D);
  const int key = (int)(row % p.S);
  const int bh = (int)(row / p.S);
  const int b = bh / p.H, hd = bh - b * p.H;
  uint16_t* dst = which == 0 ? static_cast<uint16_t*>(p.dk) + b * p.sdkb + hd * p.sdkh + (int64_t)key * p.sdks + d
                             : static_cast<uint16_t*>(p.dv) + b * p.sdvb + hd * p.sdvh + (int64_t)key * p.sdvs + d;
  u16x4 o = {MM<T>::cvt(v.x), MM<T>::cvt(v.y), MM<T>::cvt(v.z), MM<T>::cvt(v.w)};
  *reinterpret_cast<u16x4*>(dst) = o;
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
  float4 v;
  if (p.dq_slabs) {  // key blocks whose slice range covers q (causal: key block j starts at query 128 j)
    v = make_float4(0.f, 0.f, 0.f, 0.f);
    const int64_t slab = (int64_t)p.B * p.H * p.S * D;
    const int nk = p.causal ? min(p.dq_slabs, q / BKB + 1) : p.dq_slabs;
    for (int j = 0; j < nk; ++j) {
      const float4 u = *reinterpret_cast<const float4*>(p.dq_acc + j * slab + row * D + d);
      v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
    }
  } else {
    v = *reinterpret_cast<const float4*>(p.dq_acc + row * D + d);
  }
  uint16_t* dq = static_cast<uint16_t*>(p.dq) + b * p.sdqb + hd * p.sdqh + (int64_t)q * p.sdqs + d;
  u16x4 o = {MM<T>::cvt(v.x), MM<T>::cvt(v.y), MM<T>::cvt(v.z), MM<T>::cvt(v.w)};
  *reinterpret_cast<u16x4*>(dq) = o;
}

template <typename T, int D>
hipError_t fwd_launch(const AttnParams& p, hipStream_t st) {
  const int64_t bh = (int64_t)p.B * p.H;
  if (g_attn_fwd_narrow && bh * ((p.S + FQ - 1) / FQ) < 128) {  // one wave per workgroup
    const dim3 grid(((p.S + 31) / 32) * bh);
    if (p.p_drop > 0.f) hipLaunchKernelGGL((attn_fwd_k<T, D, true, 1>), grid, dim3(64), 0, st, p);
    else hipLaunchKernelGGL((attn_fwd_k<T, D, false, 1>), grid, dim3(64), 0, st, p);
    return hipGetLastError();
  }
  const dim3 grid(((p.S + FQ - 1) / FQ) * p.B * p.H);
  if (p.p_drop > 0.f) hipLaunchKernelGGL((attn_fwd_k<T, D, true>), grid, dim3(256), 0, st, p);
  else hipLaunchKernelGGL((attn_fwd_k<T, D, false>), grid, dim3(256), 0, st, p);
  return hipGetLastError();
}

template <typename T, int D>
hipError_t bwd_launch(const AttnBwdParams& p, hipStream_t st) {
  const int64_t rows = (int64_t)p.B * p.H * p.S;
  const bool direct = p.S <= BKB;
  if (!direct && !p.dq_acc) return hipErrorInvalidValue;
  if (!(direct && D == 128))  // (direct D = 128 computes delta in the main kernel)
    hipLaunchKernelGGL((attn_bwd_pre_k<T, D>), dim3((unsigned)((rows * (D / 8) + 255) / 256)), dim3(256), 0, st, p);
  const dim3 grid(((p.S + BKB - 1) / BKB) * p.B * p.H);
  const bool drop = p.p_drop > 0.f;
  const bool rope = p.rope != 0;
  if (rope && (D != 128 || drop)) return hipErrorInvalidValue;
  if (direct) {
    AttnBwdParams q = p;
    q.dq_acc = nullptr;
    constexpr int QS = 4096 / D;
    const int nsl = (p.S + QS - 1) / QS;
    if (q.qsplit < 1 || q.dkv_part == nullptr) q.qsplit = 1;
    if (q.qsplit > nsl) return hipErrorInvalidValue;  // every split must own a slice (its partial is summed)
    const dim3 g2(grid.x * q.qsplit);
    if (rope) hipLaunchKernelGGL((attn_bwd_k<T, D, false, true, D == 128>), g2, dim3(256), 0, st, q);
    else if (drop) hipLaunchKernelGGL((attn_bwd_k<T, D, true, true>), g2, dim3(256), 0, st, q);
    else hipLaunchKernelGGL((attn_bwd_k<T, D, false, true>), g2, dim3(256), 0, st, q);
    if (q.qsplit > 1) {
      const int64_t quads = 2 * (int64_t)p.B * p.H * p.S * D / 4;
      hipLaunchKernelGGL((attn_bwd_kv_sum_k<T, D>), dim3((unsigned)((quads + 255) / 256)), dim3(256), 0, st, q);
    }
    return hipGetLastError();
  }
  if (rope) hipLaunchKernelGGL((attn_bwd_k<T, D, false, false, D == 128>), grid, dim3(256), 0, st, p);
  else if (drop) hipLaunchKernelGGL((attn_bwd_k<T, D, true, false>), grid, dim3(256), 0, st, p);
  else hipLaunchKernelGGL((attn_bwd_k<T, D, false, false>), grid, dim3(256), 0, st, p);
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

void attn_set_fwd_narrow(int on) { g_attn_fwd_narrow = on; }

hipError_t attention_backward(int dtype, const AttnBwdParams& p, hipStream_t st) {
  if (!attention_supported(dtype, p.D)) return hipErrorInvalidValue;
  if (dtype == kBF16) return p.D == 64 ? bwd_launch<bf16_t, 64>(p, st) : bwd_launch<bf16_t, 128>(p, st);
  return p.D == 64 ? bwd_launch<f16_t, 64>(p, st) : bwd_launch<f16_t, 128>(p, st);
}

}  // namespace hyp

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
// Forward (one workgroup = 4 wave64s = 64 query rows of one (b, h); wave w owns 16 rows):
//   * K tile [64 keys][D] staged in LDS with a 16-B-chunk XOR swizzle (conflict-free
//     ds_read_b128 row reads, cdna_hip_programming §5.5 T2); V staged transposed [D][64+4].
//   * Sᵀ = K·Qᵀ ("swapped" product, T12): each lane ends up holding 16 scores of ONE query row,
//     so the online-softmax row max / sum needs only two __shfl_xor steps.
//   * P·V consumes P straight from registers: the 8 scores a lane holds for a 32-key step form
//     its A fragment under a permuted k order; the V fragment is read with the same permutation
//     (two ds_read_b64 from the transposed image, padded rows => conflict-free).
//   * dropout on P by a counter-based hash of (seed, b, h, q, key) — regenerated in backward.
//   * writes O and the log2-domain log-sum-exp per row.
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

// stage rows [row0, row0+64) of a [S, D] (strided) slab into a swizzled row image and/or a
// transposed image; out-of-range rows are zero.
template <int D, bool ROWS, bool TRANS>
__device__ __forceinline__ void stage_tile(const uint16_t* __restrict__ base, int64_t sstride, int row0, int S,
                                           uint16_t* __restrict__ rows_img, uint16_t* __restrict__ t_img) {
  constexpr int NCH = D / 8;
  for (int c = threadIdx.x; c < KB * NCH; c += 256) {
    const int r = c / NCH, ch = c - r * NCH;
    u16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
    if (row0 + r < S) v = *reinterpret_cast<const u16x8*>(base + (int64_t)(row0 + r) * sstride + ch * 8);
    if (ROWS) *reinterpret_cast<u16x8*>(rows_img + r * D + ((ch ^ (r & 7)) * 8)) = v;
    if (TRANS) {
#pragma unroll
      for (int i = 0; i < 8; ++i) t_img[(ch * 8 + i) * TS + r] = v[i];
    }
  }
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
template <typename T, int D>
__global__ __launch_bounds__(256) void attn_fwd_k(AttnParams p) {
  constexpr int NKK = D / 32;  // 32-deep k-steps over the head dim
  constexpr int NN = D / 16;   // 16-wide output column tiles
  __shared__ __attribute__((aligned(16))) uint16_t Ks[KB * D];
  __shared__ __attribute__((aligned(16))) uint16_t Vt[D * TS];

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 4, c16 = lane & 15;
  const int bh = blockIdx.y, b = bh / p.H, hd = bh - b * p.H;
  const int q0 = blockIdx.x * KB;
  const int qrow = q0 + 16 * w + c16;  // this lane's query (Sᵀ column)
  const uint16_t* qb = static_cast<const uint16_t*>(p.q) + b * p.sqb + hd * p.sqh;
  const uint16_t* kb = static_cast<const uint16_t*>(p.k) + b * p.skb + hd * p.skh;
  const uint16_t* vb = static_cast<const uint16_t*>(p.v) + b * p.svb + hd * p.svh;

  u16x8 qf[NKK];
#pragma unroll
  for (int kk = 0; kk < NKK; ++kk) {
    u16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
    qf[kk] = qrow < p.S ? *reinterpret_cast<const u16x8*>(qb + (int64_t)qrow * p.sqs + 8 * h + 32 * kk) : z;
  }
  f32x4 o[NN];
#pragma unroll
  for (int n = 0; n < NN; ++n) o[n] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;
  const float inv_keep = p.p_drop > 0.f ? 1.f / (1.f - p.p_drop) : 1.f;
  const uint32_t thr = (uint32_t)(p.p_drop * 4294967296.0);
  const uint64_t seed = p.p_drop > 0.f ? rng_key(p.rng) : 0;  // graph-safe generator state
  const uint8_t* kpm = p.kpm ? p.kpm + (int64_t)b * p.S : nullptr;

  int kt_end = (p.S + KB - 1) / KB;
  if (p.causal) {
    const int last_q = min(q0 + KB, p.S) - 1;
    kt_end = min(kt_end, last_q / KB + 1);
  }
  for (int kt = 0; kt < kt_end; ++kt) {
    const int k0 = kt * KB;
    __syncthreads();
    stage_tile<D, true, false>(kb, p.sks, k0, p.S, Ks, nullptr);
    stage_tile<D, false, true>(vb, p.svs, k0, p.S, nullptr, Vt);
    __syncthreads();

    float x[4][4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < NKK; ++kk) acc = MM<T>::mfma(read_row_chunk(Ks, D, 16 * t + c16, h + 4 * kk), qf[kk], acc);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = k0 + 16 * t + 4 * h + r;
        bool ok = key < p.S;
        if (p.causal) ok = ok && key <= qrow;
        if (kpm) ok = ok && (key >= p.S || kpm[key] == 0);
        x[t][r] = ok ? acc[r] * p.scale_log2 : -INFINITY;
      }
    }
    float mt = -INFINITY;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) mt = fmaxf(mt, x[t][r]);
    mt = fmaxf(mt, __shfl_xor(mt, 16, 64));
    mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
    const float mnew = fmaxf(m, mt);
    const float base = mnew == -INFINITY ? 0.f : mnew;
    const float alpha = exp2f(m - base);
    float pr[4][4];
    float ls = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float e = exp2f(x[t][r] - base);
        ls += e;
        float pd = e;
        if (p.p_drop > 0.f) {
          const int key = k0 + 16 * t + 4 * h + r;
          const uint64_t idx = (((uint64_t)bh * p.S + qrow) * p.S) + key;
          pd = hash_keep(seed, idx) >= thr ? e * inv_keep : 0.f;
        }
        pr[t][r] = pd;
      }
    l = l * alpha + ls;
    m = mnew;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float ar = __shfl(alpha, 4 * h + r, 64);
#pragma unroll
      for (int n = 0; n < NN; ++n) o[n][r] *= ar;
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      u16x8 a;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        a[r] = MM<T>::cvt(pr[2 * s][r]);
        a[4 + r] = MM<T>::cvt(pr[2 * s + 1][r]);
      }
#pragma unroll
      for (int n = 0; n < NN; ++n) {
        const u16x8 bv = read_t_pair(Vt, 16 * n + c16, 32 * s + 4 * h, 32 * s + 16 + 4 * h);
        o[n] = MM<T>::mfma(a, bv, o[n]);
      }
    }
  }
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);
  const float inv = l > 0.f ? 1.f / l : 0.f;
  if (h == 0 && qrow < p.S && p.lse) p.lse[(int64_t)bh * p.S + qrow] = l > 0.f ? m + log2f(l) : INFINITY;
  uint16_t* ob = static_cast<uint16_t*>(p.o) + b * p.sob + hd * p.soh;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float ir = __shfl(inv, 4 * h + r, 64);
    const int qr = q0 + 16 * w + 4 * h + r;
    if (qr < p.S) {
#pragma unroll
      for (int n = 0; n < NN; ++n) ob[(int64_t)qr * p.sos + 16 * n + c16] = MM<T>::cvt(o[n][r] * ir);
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
  for (int qt = qt0; qt < nq; ++qt) {
    const int q0 = qt * KB;
    __syncthreads();
    stage_tile<D, true, true>(qb, p.sqs, q0, p.S, Qs, Qt);
    stage_tile<D, true, true>(gb, p.sdos, q0, p.S, dOs, dOt);
    if (threadIdx.x < KB) {
      const int qq = q0 + threadIdx.x;
      lse_s[threadIdx.x] = qq < p.S ? p.lse[(int64_t)bh * p.S + qq] : INFINITY;
      delta_s[threadIdx.x] = qq < p.S ? p.delta[(int64_t)bh * p.S + qq] : 0.f;
    }
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
  const dim3 grid((p.S + KB - 1) / KB, p.B * p.H);
  hipLaunchKernelGGL((attn_fwd_k<T, D>), grid, dim3(256), 0, st, p);
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

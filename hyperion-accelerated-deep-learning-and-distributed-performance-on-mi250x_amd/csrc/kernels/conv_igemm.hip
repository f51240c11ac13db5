// NHWC implicit-GEMM convolution on gfx950 MFMA, with an optional fused BatchNorm-statistics
// epilogue.  Also serves as the stride-1 data-gradient (a forward conv of dY with the flipped,
// transposed filter).
//
// Reference: ResNet-18/50 convolutions ran through MIOpen (cuDNN API) with BatchNorm statistics in
// a separate pass (SURVEY §2.4 "Convolution + BatchNorm + ReLU", §2.5 ResNet rows).  Here
//
//   out[m = (n,p,q), k] = Σ_{r,s,c} in[n, p*sh + r - ph, q*sw + s - pw, c] · W[k, r, s, c]
//
// is a GEMM with M = N·P·Q rows (output pixels), N = K columns (output channels) and a reduction
// over (r, s, c) in exactly the channels-last filter's memory order (W is [K, R·S·C], reduction
// contiguous), so B tiles are plain row slices of W and A tiles are 64-channel runs of one input
// pixel (128 contiguous bytes) — one 16-byte global_load_lds per lane, straight into LDS.
// Padding / out-of-range rows are served from a zero page: the LDS-DMA cannot write zeros, so
// the lane's SOURCE address is redirected instead (no branches around the load).
//
// Tiles BM x BN x 64 (BM, BN ∈ {64, 128}), 4 waves as 2 x 2, v_mfma_f32_16x16x32_{bf16,f16},
// double-buffered LDS with the (row >> 1) & 7 chunk swizzle of gemm_mfma.hip, XCD-aware tile
// order.  Epilogue: bf16/f16 store + (optional) per-channel Σy, Σy² over the tile's rows of the
// ROUNDED outputs, written as one partial row per M-tile — exactly the partial layout the BN
// finalize kernel (bn_act.hip) consumes, so BN's separate statistics pass over y disappears.
// Requirements: C % 64 == 0 (every ResNet conv but the 3-channel stem), 16-byte aligned tensors.
#include "hyp_common.h"
#include "hyp_kernels.h"

namespace hyp {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));

constexpr int kBK = 64, kThreads = 256;

template <typename T>
__device__ __forceinline__ f32x4 mma(u16x8 a, u16x8 b, f32x4 c);
template <>
__device__ __forceinline__ f32x4 mma<bf16_t>(u16x8 a, u16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                 0, 0);
}
template <>
__device__ __forceinline__ f32x4 mma<f16_t>(u16x8 a, u16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0,
                                                0);
}

__device__ __forceinline__ int swz(int row) { return (row >> 1) & 7; }

__device__ __forceinline__ void glds16(const uint16_t* src, uint16_t* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const void*)src, (void __attribute__((address_space(3)))*)lds_wave_base, 16, 0,
                                   0);
}

__device__ __forceinline__ u16x8 frag(const uint16_t* lds, int row, int chunk) {
  return *reinterpret_cast<const u16x8*>(lds + row * kBK + ((chunk ^ swz(row)) * 8));
}

struct ConvArgs {
  const uint16_t* in;    // [N, H, W, C]
  const uint16_t* w;     // [K, R, S, C]
  uint16_t* out;         // [N, P, Q, K]
  const uint16_t* zero;  // >= 1 KiB of zeros
  float* psum;           // [Mtiles, K] or null
  float* psq;
  int N, H, W, C, K, P, Q, R, S, sh, sw, ph, pw;
  int M;                 // N*P*Q
};

template <typename T, int BM, int BN, bool STATS>
__global__ __launch_bounds__(kThreads) void conv_fwd_k(const ConvArgs a) {
  constexpr int FM = BM / 32, FN = BN / 32;  // 16x16 fragments per wave (wave tile BM/2 x BN/2)
  constexpr int IA = BM / 32, IB = BN / 32;  // glds instructions per wave per slice
  constexpr int kBuf = (BM + BN) * kBK;
  __shared__ __attribute__((aligned(16))) uint16_t smem[2 * kBuf];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  const int tiles_m = (a.M + BM - 1) / BM, tiles_n = (a.K + BN - 1) / BN, nwg = tiles_m * tiles_n;
  int bid = blockIdx.x;
  {  // XCD-aware remap (bijective for any nwg)
    const int q = nwg / 8, r = nwg % 8, xcd = bid % 8, idx = bid / 8;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
  }
  constexpr int kGroup = 8;
  const int group = kGroup * tiles_n;
  const int first_m = (bid / group) * kGroup;
  const int gsize = min(tiles_m - first_m, kGroup);
  const int tm = first_m + (bid % group) % gsize;
  const int tn = (bid % group) / gsize;
  const int m0 = tm * BM, n0 = tn * BN;

  // ---- per-lane A-row bookkeeping (rows fixed for the whole K loop)
  const int slot = lane & 7;
  int64_t a_off[IA];
  int a_h0[IA], a_w0[IA];
  bool a_ok[IA];
  const int PQ = a.P * a.Q;
#pragma unroll
  for (int i = 0; i < IA; ++i) {
    const int row = (i * 4 + wave) * 8 + (lane >> 3);
    const int m = m0 + row;
    const int chunk = slot ^ swz(row);
    a_ok[i] = m < a.M;
    const int mm = a_ok[i] ? m : 0;
    const int n = mm / PQ, pq = mm - n * PQ, p = pq / a.Q, q = pq - p * a.Q;
    a_h0[i] = p * a.sh - a.ph;
    a_w0[i] = q * a.sw - a.pw;
    a_off[i] = (((int64_t)n * a.H + a_h0[i]) * a.W + a_w0[i]) * a.C + chunk * 8;
  }
  const int64_t ldw = (int64_t)a.R * a.S * a.C;
  const uint16_t* b_src[IB];
#pragma unroll
  for (int i = 0; i < IB; ++i) {
    const int row = (i * 4 + wave) * 8 + (lane >> 3);
    const int k = n0 + row;
    const int chunk = slot ^ swz(row);
    b_src[i] = k < a.K ? a.w + (int64_t)k * ldw + chunk * 8 : nullptr;
  }
  const uint16_t* zero = a.zero + slot * 8;

  const int cpb = a.C / kBK;  // 64-channel slices per filter tap
  const int nk = a.R * a.S * cpb;

  auto stage = [&](int t, uint16_t* buf) {
    const int rs = t / cpb, c0 = (t - rs * cpb) * kBK;
    const int r = rs / a.S, s = rs - r * a.S;
    const int64_t tap = ((int64_t)r * a.W + s) * a.C + c0;
#pragma unroll
    for (int i = 0; i < IA; ++i) {
      const int h = a_h0[i] + r, w = a_w0[i] + s;
      const bool ok = a_ok[i] && (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W;
      glds16(ok ? a.in + a_off[i] + tap : zero, buf + (i * 4 + wave) * 8 * kBK);
    }
    const int64_t kofs = (int64_t)t * kBK;
#pragma unroll
    for (int i = 0; i < IB; ++i)
      glds16(b_src[i] ? b_src[i] + kofs : zero, buf + BM * kBK + (i * 4 + wave) * 8 * kBK);
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  stage(0, smem);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  const int r16 = lane & 15, c4 = lane >> 4;
  for (int t = 0; t < nk; ++t) {
    const int cur = t & 1;
    if (t + 1 < nk) stage(t + 1, smem + (cur ^ 1) * kBuf);
    const uint16_t* as = smem + cur * kBuf;
    const uint16_t* bs = as + BM * kBK;
#pragma unroll
    for (int ks = 0; ks < kBK / 32; ++ks) {
      u16x8 fa[FM], fb[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) fa[i] = frag(as, wm * (BM / 2) + i * 16 + r16, ks * 4 + c4);
#pragma unroll
      for (int j = 0; j < FN; ++j) fb[j] = frag(bs, wn * (BN / 2) + j * 16 + r16, ks * 4 + c4);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mma<T>(fa[i], fb[j], acc[i][j]);
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
  }

  // ---- epilogue.  acc[i][j][e] is out[m0 + wm*BM/2 + i*16 + c4*4 + e][n0 + wn*BN/2 + j*16 + r16].
  // Values are rounded to T once; the BN statistics use the rounded values (what BN will read),
  // and the tile is transposed through LDS so the global stores are whole 16-byte row chunks
  // (a raw accumulator store would be 2-byte scattered writes).
  constexpr int kLd = BN + 8;  // padded LDS row (elements)
  uint16_t* tile = smem;       // [BM][kLd] of T (the K loop ended with a barrier: smem is free)
  float* red = reinterpret_cast<float*>(smem + BM * kLd);  // [2 (wm)][2 (sum, sq)][BN]
  float csum[FN], csq[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) csum[j] = csq[j] = 0.f;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int lr = wm * (BM / 2) + i * 16 + c4 * 4 + e;
      const bool row_ok = m0 + lr < a.M;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int lc = wn * (BN / 2) + j * 16 + r16;
        const float v = rnd<T>(acc[i][j][e]);
        st1<T>(reinterpret_cast<T*>(tile) + lr * kLd + lc, v);
        if (STATS && row_ok) {
          csum[j] += v;
          csq[j] += v * v;
        }
      }
    }
  }
  if (STATS) {
    // reduce over the 4 row groups of the wave (lanes l, l^16, l^32, l^48 share a column)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      csum[j] += __shfl_xor(csum[j], 16, 64);
      csum[j] += __shfl_xor(csum[j], 32, 64);
      csq[j] += __shfl_xor(csq[j], 16, 64);
      csq[j] += __shfl_xor(csq[j], 32, 64);
    }
    if (c4 == 0) {
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int col = wn * (BN / 2) + j * 16 + r16;
        red[(wm * 2 + 0) * BN + col] = csum[j];
        red[(wm * 2 + 1) * BN + col] = csq[j];
      }
    }
  }
  __syncthreads();
  constexpr int kChunksPerRow = BN / 8;
#pragma unroll
  for (int it = 0; it < BM * kChunksPerRow / kThreads; ++it) {
    const int idx = it * kThreads + tid;
    const int lr = idx / kChunksPerRow, ch = idx - lr * kChunksPerRow;
    const int m = m0 + lr, k = n0 + ch * 8;
    if (m < a.M && k < a.K) {
      const uint4 v = *reinterpret_cast<const uint4*>(tile + lr * kLd + ch * 8);
      *reinterpret_cast<uint4*>(a.out + (int64_t)m * a.K + k) = v;
    }
  }
  if (STATS && tid < BN) {
    const int k = n0 + tid;
    if (k < a.K) {
      a.psum[(int64_t)tm * a.K + k] = red[0 * BN + tid] + red[2 * BN + tid];
      a.psq[(int64_t)tm * a.K + k] = red[1 * BN + tid] + red[3 * BN + tid];
    }
  }
}

template <typename T, int BM, int BN>
hipError_t launch(const ConvArgs& a, bool stats, hipStream_t st) {
  const int tiles = ((a.M + BM - 1) / BM) * ((a.K + BN - 1) / BN);
  if (stats)
    hipLaunchKernelGGL((conv_fwd_k<T, BM, BN, true>), dim3(tiles), dim3(kThreads), 0, st, a);
  else
    hipLaunchKernelGGL((conv_fwd_k<T, BM, BN, false>), dim3(tiles), dim3(kThreads), 0, st, a);
  return hipGetLastError();
}

}  // namespace

// Tile choice: the largest tile that still gives >= 2 workgroups per CU (256 CUs), else 64 x 64.
void conv_fwd_tile(int M, int K, int* bm, int* bn) {
  auto tiles = [&](int m, int n) { return (int64_t)((M + m - 1) / m) * ((K + n - 1) / n); };
  if (K <= 64) {  // a 128-wide tile would compute half zeros
    *bm = tiles(128, 64) >= 256 ? 128 : 64, *bn = 64;
  } else if (tiles(128, 128) >= 512) {
    *bm = 128, *bn = 128;
  } else if (K <= 64 || tiles(128, 64) >= 512) {
    *bm = 128, *bn = 64;
  } else {
    *bm = 64, *bn = 64;
  }
}

bool conv_fwd_supported(int C, int K) { return C % 64 == 0 && K % 8 == 0; }

hipError_t conv_fwd(int dtype, const void* in, const void* w, void* out, const void* zero, float* psum, float* psq,
                    int N, int H, int W, int C, int K, int P, int Q, int R, int S, int sh, int sw, int ph, int pw,
                    int bm, int bn, hipStream_t st) {
  if (!conv_fwd_supported(C, K) || dtype == kF32) return hipErrorInvalidValue;
  const int64_t M64 = (int64_t)N * P * Q;
  if (M64 <= 0 || M64 > INT32_MAX) return hipErrorInvalidValue;
  ConvArgs a{static_cast<const uint16_t*>(in), static_cast<const uint16_t*>(w), static_cast<uint16_t*>(out),
             static_cast<const uint16_t*>(zero), psum, psq, N, H, W, C, K, P, Q, R, S, sh, sw, ph, pw, (int)M64};
  const bool stats = psum != nullptr && psq != nullptr;
  if (dtype == kBF16) {
    if (bm == 128 && bn == 128) return launch<bf16_t, 128, 128>(a, stats, st);
    if (bm == 128 && bn == 64) return launch<bf16_t, 128, 64>(a, stats, st);
    return launch<bf16_t, 64, 64>(a, stats, st);
  }
  if (bm == 128 && bn == 128) return launch<f16_t, 128, 128>(a, stats, st);
  if (bm == 128 && bn == 64) return launch<f16_t, 128, 64>(a, stats, st);
  return launch<f16_t, 64, 64>(a, stats, st);
}

}  // namespace hyp

// The weight-gradient kernels' device code (the design is described in conv_wgrad.hip): shared by
// conv_wgrad.hip (the plain launches) and conv_dual.hip (a data gradient and a weight gradient
// horizontally fused into one launch).  Anonymous namespace: each including TU instantiates what
// it launches.
#pragma once
#include "hyp_common.h"
#include "hyp_kernels.h"
#include "mfma_lds.h"

namespace hyp {

// (namespace hyp, not the anonymous one: conv_wgrad.hip and conv_dual.hip pass it between TUs)
struct WgradArgs {
  const uint16_t* dy;    // [M, K]   (M = N*P*Q output pixels, channels-last)
  const uint16_t* x;     // [N, H, W, C]
  void* out;             // splits == 1: dW [K, R, S, C] in T; else fp32 partials [splits, K, R*S*C]
  const uint16_t* zero;  // >= 1 KiB of zeros
  int N, H, W, C, K, P, Q, R, S, sh, sw, ph, pw;
  int M, splits, steps_per_split;
  uint64_t mq, mpq;  // magic multipliers: floor(m / Q) = (m * mq) >> 36 (same for P*Q)
  float alpha;       // output scale (splits == 1: applied in the store; else in the reduce)
  int dn, dpq;       // one 64-pixel stage = dn images + dpq pixels (kBP = dn * P*Q + dpq)
  int pix;           // x's pixel stride in elements (C, or the stem's 16: see hyp_kernels.h)
  WgradPendingReduce pr;  // an EARLIER weight gradient's split-K reduce, run by extra workgroups
  int nwg_main;           // workgroups of this gradient (blockIdx.x >= nwg_main: the pending reduce)
};

namespace {

using namespace mfl;


constexpr int kBP = 64;  // pixels (reduction) per LDS stage
#ifndef HYP_CONV_KTHREADS
#define HYP_CONV_KTHREADS
constexpr int kThreads = 256;
#endif


// The deferred split-K reduce of a previous weight gradient (WgradPendingReduce): workgroup b of
// the extra range sums quads [64 b, 64 b + 64) (stride: every extra workgroup) — 4 split lanes per
// quad combined in lane order through LDS, the fixed order of splitk_reduce4_k (deterministic).
__device__ __forceinline__ void pending_reduce_block(const WgradPendingReduce& pr, int b, int nb, f32x4* red) {
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int64_t nq = pr.n / 4, sn = nq;
  for (int64_t q0 = (int64_t)b * 64; q0 < nq; q0 += (int64_t)nb * 64) {
    const int64_t iq = q0 + tx;
    const bool ok = iq < nq;
    f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0;
    if (ok) {
      const f32x4* src = reinterpret_cast<const f32x4*>(pr.part) + iq;
      int s = ty;
      for (; s + 4 < pr.splits; s += 8) {
        a0 += __builtin_nontemporal_load(src + (int64_t)s * sn);
        a1 += __builtin_nontemporal_load(src + (int64_t)(s + 4) * sn);
      }
      if (s < pr.splits) a0 += __builtin_nontemporal_load(src + (int64_t)s * sn);
    }
    f32x4 acc = a0 + a1;
    __syncthreads();
    if (ty > 0) red[(ty - 1) * 64 + tx] = acc;
    __syncthreads();
    if (ty == 0 && ok) {
      acc = ((acc + red[tx]) + red[64 + tx]) + red[128 + tx];
      acc *= pr.alpha;
      if (pr.dtype == kBF16) {
#pragma unroll
        for (int e = 0; e < 4; ++e) st1<bf16_t>(static_cast<bf16_t*>(pr.out) + iq * 4 + e, acc[e]);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) st1<f16_t>(static_cast<f16_t*>(pr.out) + iq * 4 + e, acc[e]);
      }
    }
  }
}

// floor(x / d) with magic = ceil(2^36 / d): exact while x * d < 2^36 (host: M < 2^22, P*Q < 2^14)
__device__ __forceinline__ int fdiv(int x, uint64_t magic) { return (int)(((uint64_t)(uint32_t)x * magic) >> 36); }

// Epilogue of both weight-gradient kernels, staged through LDS so the global stores are whole
// rows (16 B per lane): acc[i][j][e] = dW[k0 + wm*BM/2 + i*16 + (lane>>4)*4 + e]
//                                        [col0 + wn*BN/2 + j*16 + (lane&15)]
// splits == 1: alpha * acc in T into dW; else the fp32 partial slab of this split.
template <typename T, int BM, int BN>
__device__ __forceinline__ void wgrad_store_tile(const f32x4 (&acc)[BM / 32][BN / 32], uint16_t* smem,
                                                 const WgradArgs& a, int k0, int col0, int split, int RSC) {
  constexpr int FM = BM / 32, FN = BN / 32;
  constexpr int kLdo = BN + 4;  // staging row (floats): the 4 row groups of a store land on distinct banks
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  __syncthreads();  // every wave's last LDS reads are done before the ring is overwritten
  float* st = reinterpret_cast<float*>(smem);
  const int r16 = lane & 15, c4 = lane >> 4;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        st[(wm * (BM / 2) + i * 16 + c4 * 4 + e) * kLdo + wn * (BN / 2) + j * 16 + r16] = acc[i][j][e];
  __syncthreads();
  constexpr int Q4 = BN / 4;  // float4 quads per tile row
  const bool direct = a.splits == 1;
  float* part = reinterpret_cast<float*>(a.out) + (int64_t)split * a.K * RSC;
  T* outT = reinterpret_cast<T*>(a.out);
#pragma unroll
  for (int it = 0; it < BM * Q4 / kThreads; ++it) {
    const int idx = it * kThreads + tid, row = idx / Q4, q4 = idx - row * Q4;
    const int k = k0 + row;
    if (k >= a.K) continue;
    const f32x4 v = *reinterpret_cast<const f32x4*>(st + row * kLdo + q4 * 4);
    const int64_t off = (int64_t)k * RSC + col0 + q4 * 4;
    if (direct) {
      T o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) st1<T>(o + e, a.alpha * v[e]);
      *reinterpret_cast<uint2*>(outT + off) = *reinterpret_cast<const uint2*>(o);
    } else {
      st16_wt(part + off, __builtin_bit_cast(uint4, v));
    }
  }
}

template <int BM, int BN, int NB>
constexpr int wgrad_smem_bytes() {
  return NB * (BM + BN) * kBP * 2 > BM * (BN + 4) * 4 ? NB * (BM + BN) * kBP * 2 : BM * (BN + 4) * 4;
}

// DENSE: 1x1, stride 1, no padding — X is the plain [M, C] matrix, so both operands are row-major
// over the pixels and each lane's source is a pointer advanced by one stage per issue.  Otherwise
// each lane tracks its row's (image, pixel) pair incrementally (no per-stage division by P*Q) and
// gathers the shifted / strided input pixel with a 32-bit element offset (host: |X| < 2^31).
// The main workgroups' body (blk < a.nwg_main; conv_dual.hip runs it inside a fused launch)
template <typename T, int BM, int BN, int NB, bool DENSE>
__device__ __forceinline__ void conv_wgrad_body(const WgradArgs& a, const int blk, uint16_t* smem) {
  constexpr int FM = BM / 32, FN = BN / 32;          // 16x16 fragments per wave (wave tile BM/2 x BN/2)
  constexpr int IA = BM / 32, IB = BN / 32;          // glds per wave per stage (8-row blocks)
  constexpr int CA = BM / 8, CB = BN / 8;            // 16-byte chunks per image row
  constexpr int kBuf = (BM + BN) * kBP;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  const int RSC = a.R * a.S * a.C;
  const int tiles_k = (a.K + BM - 1) / BM, tiles_c = RSC / BN, ntiles = tiles_k * tiles_c;
  const int nwg = ntiles * a.splits;
  int bid = blk;
  bid = xcd_remap(bid, nwg);  // consecutive logical tiles (same pixel split) share an XCD's L2
  const int split = bid / ntiles, tile = bid - split * ntiles;
  const int tk = tile % tiles_k, tc = tile / tiles_k;
  const int k0 = tk * BM;
  const int col0 = tc * BN;               // column in (r, s, c) order; BN | C so one tap per tile
  const int rs = col0 / a.C, c0 = col0 - rs * a.C;
  const int r = rs / a.S, s = rs - r * a.S;
  const int mbeg = split * a.steps_per_split * kBP;
  const int nsteps = min(a.steps_per_split, (a.M - mbeg + kBP - 1) / kBP);

  // ---- per-lane staging state: lane covers image row (i*4 + wave)*R? + lane/C? of each operand (a
  // wave instruction writes 1024 B = 1024 / (2*BM) rows of the A image)
  constexpr int RA = 1024 / (2 * BM), RB = 1024 / (2 * BN);  // rows per wave instruction
  const uint16_t* pa[IA];
  int ma[IA];
  const uint16_t* pb[IB];
  int mb[IB], nb_[IB], pqb[IB], cb[IB];
  const int PQ = a.P * a.Q;
#pragma unroll
  for (int i = 0; i < IB; ++i) {
    const int row = (i * 4 + wave) * RB + lane / CB;
    cb[i] = c0 + (((lane % CB) ^ swz_tr<BN>(row)) << 3);
  }
  // lane state at stage tp of this split
  auto init = [&](int tp) {
    const int m0 = mbeg + tp * kBP;
#pragma unroll
    for (int i = 0; i < IA; ++i) {
      const int row = (i * 4 + wave) * RA + lane / CA;
      const int col = k0 + (((lane % CA) ^ swz_tr<BM>(row)) << 3);
      // a column past K (K % BM != 0) reads as pixel >= M: zeros
      ma[i] = col < a.K ? m0 + row : a.M;
      pa[i] = a.dy + (int64_t)(m0 + row) * a.K + col;
    }
#pragma unroll
    for (int i = 0; i < IB; ++i) {
      const int row = (i * 4 + wave) * RB + lane / CB;
      mb[i] = m0 + row;
      if (DENSE) {
        pb[i] = a.x + (int64_t)mb[i] * a.C + cb[i];
      } else {
        nb_[i] = fdiv(mb[i], a.mpq);
        pqb[i] = mb[i] - nb_[i] * PQ;
      }
    }
  };
  init(0);
  const uint16_t* zero = a.zero;
  const int64_t da = (int64_t)kBP * a.K, db = (int64_t)kBP * a.C;

  // stages are issued in order t = 0, 1, 2, ...: each call advances the lane state by one stage
  auto stage = [&](uint16_t* buf) {
#pragma unroll
    for (int i = 0; i < IA; ++i) {
      glds16(ma[i] < a.M ? pa[i] : zero, buf + (i * 4 + wave) * 512);
      ma[i] += kBP;
      pa[i] += da;
    }
#pragma unroll
    for (int i = 0; i < IB; ++i) {
      const uint16_t* src;
      if (DENSE) {
        src = mb[i] < a.M ? pb[i] : zero;
        pb[i] += db;
      } else {
        const int p = fdiv(pqb[i], a.mq), q = pqb[i] - p * a.Q;
        const int h = p * a.sh + r - a.ph, w = q * a.sw + s - a.pw;
        const bool ok = mb[i] < a.M && (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W;
        src = ok ? a.x + (((nb_[i] * a.H + h) * a.W + w) * a.pix + cb[i]) : zero;
        pqb[i] += a.dpq;
        nb_[i] += a.dn;
        if (pqb[i] >= PQ) {
          pqb[i] -= PQ;
          nb_[i] += 1;
        }
      }
      mb[i] += kBP;
      glds16(src, buf + BM * kBP + (i * 4 + wave) * 512);
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // NB-deep ring (see mfma_lds.h wait_stage): stage t+NB-1 is issued after the barrier that
  // retires stage t-1's buffer
#pragma unroll
  for (int i = 0; i < NB - 1; ++i)
    if (i < nsteps) stage(smem + i * kBuf);
  for (int t = 0; t < nsteps; ++t) {
    wait_stage<IA + IB, NB>(min(NB - 2, nsteps - 1 - t));
    barrier_keep_vm();
    if (t + NB - 1 < nsteps) stage(smem + ((t + NB - 1) % NB) * kBuf);
    const uint16_t* as = smem + (t % NB) * kBuf;
    const uint16_t* bs = as + BM * kBP;
#pragma unroll
    for (int ks = 0; ks < kBP / 32; ++ks) {
      u16x8 fa[FM], fb[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) fa[i] = frag_tr<BM>(as, ks * 32, wm * (BM / 2) + i * 16, lane);
#pragma unroll
      for (int j = 0; j < FN; ++j) fb[j] = frag_tr<BN>(bs, ks * 32, wn * (BN / 2) + j * 16, lane);
      lds_reads_done();  // the asm transposed reads (see mfma_lds.h) have returned
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mma16<T>(fa[i], fb[j], acc[i][j]);
    }
  }

  wgrad_store_tile<T, BM, BN>(acc, smem, a, k0, col0, split, RSC);
}

// Lean main loop for DENSE operands (1x1 stride-1 weight gradients, linear-layer weight
// gradients): dY and X are plain [M, ld] matrices, so a lane's source is a FIXED 32-bit byte
// offset from a wave-uniform base that advances one stage per issue (scalar arithmetic), the
// LDS destination is wave-uniform (M0 from scalars), and the transposed fragment reads take their
// row offsets as immediates.  Measured on conv_wgrad_k (scripts/wgrad_probe.py ablations): with
// loads and MFMAs both removed its loop still cost 450-970 cycles per stage — the per-lane
// address VALU (8-11 vector instructions per 16x16x32 MFMA, whose shadow holds ~2) bounded it,
// not HBM/L2 or the matrix cores.  Here the vector work per stage is FM+FN adds.  Stages whose
// 64 pixels are all < M in a tile whose BM rows are all < K take the lean path; the partial last
// stage and a K tail select the zero page per lane.
// One 32-deep k-step of a wave's (FM x FN) 16x16 fragments out of a transposed stage image.
template <typename T, int BM, int BN, int R0>
__device__ __forceinline__ void wgrad_kstep(const unsigned (&pa)[BM / 32], const unsigned (&pb)[BN / 32],
                                            f32x4 (&acc)[BM / 32][BN / 32]) {
  constexpr int FM = BM / 32, FN = BN / 32;
  u16x8 fa[FM], fb[FN];
#pragma unroll
  for (int i = 0; i < FM; ++i) fa[i] = frag_tr_at<BM, R0>(pa[i]);
#pragma unroll
  for (int j = 0; j < FN; ++j) fb[j] = frag_tr_at<BN, R0>(pb[j]);
  lds_reads_done();
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = mma16<T>(fa[i], fb[j], acc[i][j]);
}

// LDS bytes of a conv_wgrad_dense_k workgroup
template <int BM, int BN, int NB, int KP>
constexpr int wgrad_dense_smem_bytes() {
  return NB * (BM + BN) * KP * 2 > BM * (BN + 4) * 4 ? NB * (BM + BN) * KP * 2 : BM * (BN + 4) * 4;
}

template <typename T, int BM, int BN, int NB, int KP>
__device__ __forceinline__ void conv_wgrad_dense_body(const WgradArgs& a, const int blk,
                                                      uint16_t* smem) {
  static_assert(KP == 64 || KP == 128, "pixels per stage");
  static_assert(NB * (BM + BN) * KP * 2 <= 160 * 1024, "LDS ring exceeds 160 KiB");
  constexpr int FM = BM / 32, FN = BN / 32;
  constexpr int IA = KP * BM / 2048, IB = KP * BN / 2048;  // 1 KiB wave pieces per stage (4 waves)
  constexpr int CA = BM / 8, CB = BN / 8;
  constexpr int kBuf = (BM + BN) * KP;
  constexpr int RA = 1024 / (2 * BM), RB = 1024 / (2 * BN);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;

  const int K = a.K, C = a.C, M = a.M;
  const int tiles_k = (K + BM - 1) / BM, tiles_c = C / BN, ntiles = tiles_k * tiles_c;
  const int bid = xcd_remap(blk, ntiles * a.splits);
  const int split = bid / ntiles, tile = bid - split * ntiles;
  const int tk = tile % tiles_k, tc = tile / tiles_k;
  const int k0 = tk * BM, c0 = tc * BN;
  const int mbeg = split * a.steps_per_split * kBP;
  const int mend = min(M, mbeg + a.steps_per_split * kBP);  // this split's pixels: [mbeg, mend)
  const int nsteps = (mend - mbeg + KP - 1) / KP;
  const bool ktail = k0 + BM > K;

  unsigned va[IA], vb[IB];  // lane byte offsets from the stage's first pixel row
#pragma unroll
  for (int i = 0; i < IA; ++i) {
    const int row = (i * 4 + wave) * RA + lane / CA;
    va[i] = (unsigned)(row * K + k0 + (((lane % CA) ^ swz_tr<BM>(row)) << 3)) * 2u;
  }
#pragma unroll
  for (int i = 0; i < IB; ++i) {
    const int row = (i * 4 + wave) * RB + lane / CB;
    vb[i] = (unsigned)(row * C + c0 + (((lane % CB) ^ swz_tr<BN>(row)) << 3)) * 2u;
  }
  const char* ga = reinterpret_cast<const char*>(a.dy + (int64_t)mbeg * K);
  const char* gb = reinterpret_cast<const char*>(a.x + (int64_t)mbeg * C);
  const int64_t sa = (int64_t)KP * K * 2, sb = (int64_t)KP * C * 2;
  int mcur = mbeg;

  auto stage = [&](uint16_t* buf) {
    if (!ktail && mcur + KP <= mend) {
#pragma unroll
      for (int i = 0; i < IA; ++i)
        glds16(reinterpret_cast<const uint16_t*>(ga + va[i]), buf + (i * 4 + wave) * 512);
#pragma unroll
      for (int i = 0; i < IB; ++i)
        glds16(reinterpret_cast<const uint16_t*>(gb + vb[i]), buf + BM * KP + (i * 4 + wave) * 512);
    } else {
#pragma unroll
      for (int i = 0; i < IA; ++i) {
        const int row = (i * 4 + wave) * RA + lane / CA;
        const int col = k0 + (((lane % CA) ^ swz_tr<BM>(row)) << 3);
        const bool ok = mcur + row < mend && col < K;
        glds16(ok ? reinterpret_cast<const uint16_t*>(ga + va[i]) : a.zero, buf + (i * 4 + wave) * 512);
      }
#pragma unroll
      for (int i = 0; i < IB; ++i) {
        const int row = (i * 4 + wave) * RB + lane / CB;
        glds16(mcur + row < mend ? reinterpret_cast<const uint16_t*>(gb + vb[i]) : a.zero,
               buf + BM * KP + (i * 4 + wave) * 512);
      }
    }
    ga += sa;
    gb += sb;
    mcur += KP;
  };

  unsigned fo_a[FM], fo_b[FN];  // lane byte offsets of the fragments inside a stage buffer
#pragma unroll
  for (int i = 0; i < FM; ++i) fo_a[i] = frag_tr_lane<BM>(wm * (BM / 2) + i * 16, lane);
#pragma unroll
  for (int j = 0; j < FN; ++j) fo_b[j] = frag_tr_lane<BN>(wn * (BN / 2) + j * 16, lane) + BM * KP * 2;
  const unsigned sbase = lds_addr(smem);

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int i = 0; i < NB - 1; ++i)
    if (i < nsteps) stage(smem + i * kBuf);
  for (int t = 0; t < nsteps; ++t) {
    wait_stage<IA + IB, NB>(min(NB - 2, nsteps - 1 - t));
    barrier_keep_vm();
    if (t + NB - 1 < nsteps) stage(smem + ((t + NB - 1) % NB) * kBuf);
    const unsigned buf = sbase + (unsigned)((t % NB) * kBuf * 2);
    unsigned pa_[FM], pb_[FN];
#pragma unroll
    for (int i = 0; i < FM; ++i) pa_[i] = buf + fo_a[i];
#pragma unroll
    for (int j = 0; j < FN; ++j) pb_[j] = buf + fo_b[j];
    wgrad_kstep<T, BM, BN, 0>(pa_, pb_, acc);
    wgrad_kstep<T, BM, BN, 32>(pa_, pb_, acc);
    if constexpr (KP == 128) {
      wgrad_kstep<T, BM, BN, 64>(pa_, pb_, acc);
      wgrad_kstep<T, BM, BN, 96>(pa_, pb_, acc);
    }
  }
  wgrad_store_tile<T, BM, BN>(acc, smem, a, k0, c0, split, C);
}

template <typename T, int BM, int BN, int NB, bool DENSE>
__global__ __launch_bounds__(kThreads) void conv_wgrad_k(const WgradArgs a) {
  __shared__ __attribute__((aligned(16))) uint16_t smem[wgrad_smem_bytes<BM, BN, NB>() / 2];
  if ((int)blockIdx.x >= a.nwg_main) {
    pending_reduce_block(a.pr, blockIdx.x - a.nwg_main, gridDim.x - a.nwg_main, reinterpret_cast<f32x4*>(smem));
    return;
  }
  conv_wgrad_body<T, BM, BN, NB, DENSE>(a, blockIdx.x, smem);
}

template <typename T, int BM, int BN, int NB, int KP>
__global__ __launch_bounds__(kThreads) void conv_wgrad_dense_k(const WgradArgs a) {
  __shared__ __attribute__((aligned(16))) uint16_t smem[wgrad_dense_smem_bytes<BM, BN, NB, KP>() / 2];
  if ((int)blockIdx.x >= a.nwg_main) {
    pending_reduce_block(a.pr, blockIdx.x - a.nwg_main, gridDim.x - a.nwg_main, reinterpret_cast<f32x4*>(smem));
    return;
  }
  conv_wgrad_dense_body<T, BM, BN, NB, KP>(a, blockIdx.x, smem);
}

}  // namespace
}  // namespace hyp

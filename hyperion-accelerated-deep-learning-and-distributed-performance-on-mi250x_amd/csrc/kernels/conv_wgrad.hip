// NHWC convolution WEIGHT gradient on gfx950 MFMA (split-K implicit GEMM).
//
// Reference: ResNet-50/18 weight gradients ran through MIOpen's `igemm_wrw` / CK batched-GEMM
// solvers plus their zero-fill and cast kernels (3-4 launches per conv; SURVEY §2.4
// "Convolution + BatchNorm + ReLU" backward, §2.5 ResNet rows).  Here
//
//   dW[k, r, s, c] = Σ_{m = (n,p,q)} dY[m, k] · X[n, p*sh + r - ph, q*sw + s - pw, c]
//
// is a GEMM with rows = output channels k, columns = (r, s, c) in the channels-last filter's own
// order, and a reduction over the N·P·Q output pixels.  BOTH operands have the reduction (pixel)
// dimension strided in memory — dY rows and input pixels are channel-contiguous — so tiles are
// staged pixel-major straight from HBM with 16-byte global_load_lds (a pixel's BM/BN-channel run
// is one contiguous row), and the MFMA operands are read back TRANSPOSED with gfx950's
// ds_read_b64_tr_b16 (guide T10): no register transpose, no ds_permute.
//
// LDS image per operand: [64 pixels][W channels] with W*2-byte rows and an XOR swizzle of the
// 16-byte chunks chosen so every 32-lane half of a transposed read touches 64 distinct banks
// (rows 0..7 of a read half land on disjoint chunk pairs).  The pixel <-> MFMA k-slot mapping is
// free (both operands sum over the same pixels), so each 16-lane group reads 4 consecutive rows.
//
// Work split: tiles BM x BN (k x c) of one filter tap, 4 waves as 2 x 2, 16x16x32 bf16/f16 MFMA;
// the pixel reduction is split over `splits` workgroups (the outputs of a ResNet wgrad are small —
// 64 x 576 for a layer1 3x3 — while the reduction is up to 10^5 pixels long).  splits == 1 stores
// the result in the parameter dtype; otherwise fp32 partials [splits][K][R·S·C] are summed (in a
// fixed order: deterministic) and cast by conv_wgrad_reduce_k.
#include "hyp_common.h"
#include "hyp_kernels.h"
#include "mfma_lds.h"

namespace hyp {
namespace {

using namespace mfl;

constexpr int kBP = 64;  // pixels (reduction) per LDS stage
constexpr int kThreads = 256;

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
      *reinterpret_cast<f32x4*>(part + off) = v;
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
template <typename T, int BM, int BN, int NB, bool DENSE>
__global__ __launch_bounds__(kThreads) void conv_wgrad_k(const WgradArgs a) {
  constexpr int FM = BM / 32, FN = BN / 32;          // 16x16 fragments per wave (wave tile BM/2 x BN/2)
  constexpr int IA = BM / 32, IB = BN / 32;          // glds per wave per stage (8-row blocks)
  constexpr int CA = BM / 8, CB = BN / 8;            // 16-byte chunks per image row
  constexpr int kBuf = (BM + BN) * kBP;
  __shared__ __attribute__((aligned(16))) uint16_t smem[wgrad_smem_bytes<BM, BN, NB>() / 2];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  if ((int)blockIdx.x >= a.nwg_main) {
    pending_reduce_block(a.pr, blockIdx.x - a.nwg_main, gridDim.x - a.nwg_main, reinterpret_cast<f32x4*>(smem));
    return;
  }
  const int RSC = a.R * a.S * a.C;
  const int tiles_k = (a.K + BM - 1) / BM, tiles_c = RSC / BN, ntiles = tiles_k * tiles_c;
  const int nwg = ntiles * a.splits;
  int bid = blockIdx.x;
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

template <typename T, int BM, int BN, int NB, int KP>
__global__ __launch_bounds__(kThreads) void conv_wgrad_dense_k(const WgradArgs a) {
  static_assert(KP == 64 || KP == 128, "pixels per stage");
  static_assert(NB * (BM + BN) * KP * 2 <= 160 * 1024, "LDS ring exceeds 160 KiB");
  constexpr int FM = BM / 32, FN = BN / 32;
  constexpr int IA = KP * BM / 2048, IB = KP * BN / 2048;  // 1 KiB wave pieces per stage (4 waves)
  constexpr int CA = BM / 8, CB = BN / 8;
  constexpr int kBuf = (BM + BN) * KP;
  constexpr int RA = 1024 / (2 * BM), RB = 1024 / (2 * BN);
  constexpr int kSm = NB * kBuf * 2 > BM * (BN + 4) * 4 ? NB * kBuf * 2 : BM * (BN + 4) * 4;
  __shared__ __attribute__((aligned(16))) uint16_t smem[kSm / 2];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;

  if ((int)blockIdx.x >= a.nwg_main) {
    pending_reduce_block(a.pr, blockIdx.x - a.nwg_main, gridDim.x - a.nwg_main, reinterpret_cast<f32x4*>(smem));
    return;
  }
  const int K = a.K, C = a.C, M = a.M;
  const int tiles_k = (K + BM - 1) / BM, tiles_c = C / BN, ntiles = tiles_k * tiles_c;
  const int bid = xcd_remap(blockIdx.x, ntiles * a.splits);
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

// out = alpha * Σ_s part[s] (fixed order: deterministic), cast to T; 4 elements per thread
// (16-byte loads).  Optional rank-r epilogue (the LoRA update fused into the base GEMM's reduce):
//   out[m, n] += beta * (mask ? mask[m, n] : 1) * Σ_j U[m, j] · V[j * sv_j + n * sv_n]
// with U [M, r] and V any 2D view (B of y += t·Bᵀ is V = Bᵀ: sv_j = 1, sv_n = r).
// 64-thread blocks (a wgrad output can be only 37K floats: 256-thread blocks left ~36 workgroups
// on 256 CUs) and 4 independent accumulators, so 4 slab loads are in flight per thread.
constexpr int kRedThreads = 64;

template <typename T, bool LOWRANK, bool AFF>
__global__ __launch_bounds__(kRedThreads) void splitk_reduce_k(const float* __restrict__ part, T* __restrict__ out,
                                                               int64_t n, int splits, float alpha, SplitkEpilogue ep) {
  const int64_t i4 = ((int64_t)blockIdx.x * kRedThreads + threadIdx.x) * 4;
  if (i4 >= n) return;
  const f32x4* src = reinterpret_cast<const f32x4*>(part + i4);
  const int64_t sn = n / 4;  // slab stride in f32x4
  f32x4 a0 = __builtin_nontemporal_load(src), a1 = {0.f, 0.f, 0.f, 0.f}, a2 = a1, a3 = a1;
  int s = 1;
  for (; s + 3 < splits; s += 4) {
    a0 += __builtin_nontemporal_load(src + (int64_t)s * sn);
    a1 += __builtin_nontemporal_load(src + (int64_t)(s + 1) * sn);
    a2 += __builtin_nontemporal_load(src + (int64_t)(s + 2) * sn);
    a3 += __builtin_nontemporal_load(src + (int64_t)(s + 3) * sn);
  }
  for (; s < splits; ++s) a0 += __builtin_nontemporal_load(src + (int64_t)s * sn);
  f32x4 acc = (a0 + a1) + (a2 + a3);
  acc *= alpha;
  if (LOWRANK) {
    // r % 8 == 0, r <= 64: U's row and V's rows / columns are read as 16- / 8-byte vectors
    const int64_t m = i4 / ep.N, n0 = i4 - m * ep.N;  // N % 4 == 0: the 4 elements share a row
    const T* u = reinterpret_cast<const T*>(ep.U) + m * ep.r;
    const T* v = reinterpret_cast<const T*>(ep.V);
    f32x4 lr = {0.f, 0.f, 0.f, 0.f};
    for (int j0 = 0; j0 < ep.r; j0 += 8) {
      float uj[8];
      Vec8<T>::load(u + j0, uj);
      if (ep.sv_n != 1) {  // V = [N, r] (row n holds the r coefficients of output column n)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float vv[8];
          Vec8<T>::load(v + (n0 + e) * ep.sv_n + j0, vv);
#pragma unroll
          for (int q = 0; q < 8; ++q) lr[e] += uj[q] * vv[q];
        }
      } else {  // V = [r, N]: 4 consecutive outputs = one 8-byte run per coefficient row
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const uint2 raw = *reinterpret_cast<const uint2*>(v + (int64_t)(j0 + q) * ep.sv_j + n0);
          const T* h = reinterpret_cast<const T*>(&raw);
#pragma unroll
          for (int e = 0; e < 4; ++e) lr[e] += uj[q] * ld1<T>(h + e);
        }
      }
    }
    if (ep.mask != nullptr) {
      const uint2 raw = *reinterpret_cast<const uint2*>(reinterpret_cast<const T*>(ep.mask) + i4);
      const T* mk = reinterpret_cast<const T*>(&raw);
#pragma unroll
      for (int e = 0; e < 4; ++e) lr[e] *= ld1<T>(mk + e);
    }
    acc += ep.beta * lr;
  }
  if (AFF) {  // eval BN folded in: act(round(acc) * scale + shift (+ residual)), N % 4 == 0
    const int64_t n0 = i4 % ep.N;
    const T* res = static_cast<const T*>(ep.residual);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float v = fmaf(rnd<T>(acc[e]), ep.scale[n0 + e], ep.shift[n0 + e]);
      if (res != nullptr) v += ld1<T>(res + i4 + e);
      acc[e] = ep.act ? fmaxf(v, 0.f) : v;
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) st1<T>(out + i4 + e, acc[e]);
}

// Small outputs with many splits (weight gradients: 37K-262K elements, 8-256 splits): 4 split
// lanes per output quad (split s goes to lane s % 4, summed in increasing s), combined in lane
// order through LDS — still a fixed order, 4x the loads in flight of splitk_reduce_k.
template <typename T>
__global__ __launch_bounds__(256) void splitk_reduce4_k(const float* __restrict__ part, T* __restrict__ out,
                                                        int64_t n, int splits, float alpha) {
  __shared__ f32x4 red[3][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int64_t i4 = ((int64_t)blockIdx.x * 64 + tx) * 4;
  const bool ok = i4 < n;
  f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0;
  if (ok) {
    const f32x4* src = reinterpret_cast<const f32x4*>(part + i4);
    const int64_t sn = n / 4;
    int s = ty;
    for (; s + 4 < splits; s += 8) {
      a0 += __builtin_nontemporal_load(src + (int64_t)s * sn);
      a1 += __builtin_nontemporal_load(src + (int64_t)(s + 4) * sn);
    }
    if (s < splits) a0 += __builtin_nontemporal_load(src + (int64_t)s * sn);
  }
  f32x4 acc = a0 + a1;
  if (ty > 0) red[ty - 1][tx] = acc;
  __syncthreads();
  if (ty == 0 && ok) {
    acc = ((acc + red[0][tx]) + red[1][tx]) + red[2][tx];
    acc *= alpha;
#pragma unroll
    for (int e = 0; e < 4; ++e) st1<T>(out + i4 + e, acc[e]);
  }
}

template <typename T>
hipError_t reduce_launch(const float* part, T* out, int64_t n, int splits, float alpha, const SplitkEpilogue* ep,
                         hipStream_t st) {
  const int blocks = (int)((n / 4 + kRedThreads - 1) / kRedThreads);
  if (ep != nullptr && ep->U != nullptr)
    hipLaunchKernelGGL((splitk_reduce_k<T, true, false>), dim3(blocks), dim3(kRedThreads), 0, st, part, out, n, splits,
                       alpha, *ep);
  else if (ep != nullptr && ep->scale != nullptr)
    hipLaunchKernelGGL((splitk_reduce_k<T, false, true>), dim3(blocks), dim3(kRedThreads), 0, st, part, out, n, splits,
                       alpha, *ep);
  else if (splits >= 8 && n / 4 <= (1 << 16))
    hipLaunchKernelGGL((splitk_reduce4_k<T>), dim3((int)((n / 4 + 63) / 64)), dim3(256), 0, st, part, out, n, splits,
                       alpha);
  else
    hipLaunchKernelGGL((splitk_reduce_k<T, false, false>), dim3(blocks), dim3(kRedThreads), 0, st, part, out, n,
                       splits, alpha, SplitkEpilogue{});
  return hipGetLastError();
}

}  // namespace

namespace {
// Split-K reduce of a convolution's [splits, M, K] fp32 partials with the BN-statistics epilogue
// of conv_fwd_k: out = Σ_s part[s] rounded to T, and per-channel Σy, Σy² of the ROUNDED outputs
// over kStatRows-row blocks, added atomically into psum[K] / psq[K] (the sums the BN apply
// finalizes inline).  Used when a forward conv has too few output tiles to fill 256 CUs
// (ResNet-50 layer3/4: 200-392 tiles, 55 us at 0.8 workgroups per CU).  Block = 64 column quads
// (256 channels, 16-byte loads) x 4 row lanes.
template <typename T>
__global__ __launch_bounds__(256) void splitk_reduce_stats_k(const float* __restrict__ part, T* __restrict__ out,
                                                             int M, int K, int splits, int rows,
                                                             double* __restrict__ psum, double* __restrict__ psq) {
  __shared__ float red[2][4][256];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = blockIdx.y * 256 + tx * 4;
  const int r0 = blockIdx.x * rows;
  const int r1 = min(M, r0 + rows);
  const int64_t slab = (int64_t)M * K;
  f32x4 cs = {0.f, 0.f, 0.f, 0.f}, cq = cs;
  if (c < K) {
    for (int r = r0 + ty; r < r1; r += 4) {
      const float* src = part + (int64_t)r * K + c;
      f32x4 a0 = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(src)), a1 = {0.f, 0.f, 0.f, 0.f};
      int s = 1;
      for (; s + 1 < splits; s += 2) {
        a0 += __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(src + (int64_t)s * slab));
        a1 += __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(src + (int64_t)(s + 1) * slab));
      }
      if (s < splits) a0 += __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(src + (int64_t)s * slab));
      const f32x4 acc = a0 + a1;
      T* o = out + (int64_t)r * K + c;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float v = rnd<T>(acc[e]);
        st1<T>(o + e, v);
        cs[e] += v;
        cq[e] += v * v;
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    red[0][ty][tx * 4 + e] = cs[e];
    red[1][ty][tx * 4 + e] = cq[e];
  }
  __syncthreads();
  // one atomic per channel per block: 64 consecutive channels per wave instruction (256-byte runs)
  if (threadIdx.x < 256) {
    const int j = threadIdx.x, ch = blockIdx.y * 256 + j;
    if (ch < K) {
      const int64_t slot = (int64_t)(blockIdx.x % kStatSlots) * 2 * K;
      unsafeAtomicAdd(psum + slot + ch, (double)((red[0][0][j] + red[0][1][j]) + (red[0][2][j] + red[0][3][j])));
      unsafeAtomicAdd(psq + slot + ch, (double)((red[1][0][j] + red[1][1][j]) + (red[1][2][j] + red[1][3][j])));
    }
  }
}
}  // namespace

hipError_t splitk_reduce_stats(int dtype, const float* part, void* out, int M, int K, int splits, double* psum,
                               double* psq, hipStream_t st) {
  if (K % 4 != 0 || splits < 1 || M < 1) return hipErrorInvalidValue;
  // kStatRows-row blocks (fewer atomic adders per channel) unless that leaves < 512 blocks
  const int cb = (K + 255) / 256;
  const int rows = (int64_t)((M + kStatRows - 1) / kStatRows) * cb >= 512 ? kStatRows : 16;
  const dim3 grid((M + rows - 1) / rows, cb);
  if (dtype == kBF16)
    hipLaunchKernelGGL(splitk_reduce_stats_k<bf16_t>, grid, dim3(256), 0, st, part, static_cast<bf16_t*>(out), M, K,
                       splits, rows, psum, psq);
  else if (dtype == kF16)
    hipLaunchKernelGGL(splitk_reduce_stats_k<f16_t>, grid, dim3(256), 0, st, part, static_cast<f16_t*>(out), M, K,
                       splits, rows, psum, psq);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

namespace {
// Split-K reduce of a stride-1 data gradient with the BN-backward epilogue (conv_igemm.hip's BNB
// epilogue for the split case): out = dz = round(round(Σ_s part[s]) + addend) · mask and Σdz,
// Σdz·x per channel into slot blockIdx.x % kStatSlots of bnb.sums.  Same block shape as
// splitk_reduce_stats_k (64 column quads x 4 row lanes, `rows` rows per block).
template <typename T>
__global__ __launch_bounds__(256) void splitk_reduce_bnb_k(const float* __restrict__ part, T* __restrict__ out,
                                                           const T* __restrict__ addend, int M, int K, int splits,
                                                           int rows, BnBwdEpilogue bnb) {
  __shared__ float red[2][4][256];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = blockIdx.y * 256 + tx * 4;
  const int r0 = blockIdx.x * rows;
  const int r1 = min(M, r0 + rows);
  const int64_t slab = (int64_t)M * K;
  const T* xb = static_cast<const T*>(bnb.x);
  const T* yb = static_cast<const T*>(bnb.y);
  float msc[4] = {0.f, 0.f, 0.f, 0.f}, msh[4] = {0.f, 0.f, 0.f, 0.f};
  if (bnb.mode == 1 && c < K) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float sc = (bnb.w ? bnb.w[c + e] : 1.f) * bnb.invstd[c + e];
      msc[e] = sc;
      msh[e] = (bnb.b ? bnb.b[c + e] : 0.f) - bnb.mean[c + e] * sc;
    }
  }
  f32x4 cs = {0.f, 0.f, 0.f, 0.f}, cq = cs;
  if (c < K) {
    for (int r = r0 + ty; r < r1; r += 4) {
      const int64_t off = (int64_t)r * K + c;
      const float* src = part + off;
      f32x4 a0 = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(src)), a1 = {0.f, 0.f, 0.f, 0.f};
      int s = 1;
      for (; s + 1 < splits; s += 2) {
        a0 += __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(src + (int64_t)s * slab));
        a1 += __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(src + (int64_t)(s + 1) * slab));
      }
      if (s < splits) a0 += __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(src + (int64_t)s * slab));
      const f32x4 acc = a0 + a1;
      // 4 channels = one 8-byte run of each 2-byte operand
      const uint2 rx = *reinterpret_cast<const uint2*>(xb + off);
      const uint2 ry = bnb.mode == 2 ? *reinterpret_cast<const uint2*>(yb + off) : uint2{0u, 0u};
      const uint2 rd = addend != nullptr ? *reinterpret_cast<const uint2*>(addend + off) : uint2{0u, 0u};
      const T* hx = reinterpret_cast<const T*>(&rx);
      const T* hy = reinterpret_cast<const T*>(&ry);
      const T* hd = reinterpret_cast<const T*>(&rd);
      T ov[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v = rnd<T>(acc[e]);
        if (addend != nullptr) v = rnd<T>(v + ld1<T>(hd + e));
        const float xv = ld1<T>(hx + e);
        const bool keep = bnb.mode == 0 || (bnb.mode == 1 ? fmaf(xv, msc[e], msh[e]) > 0.f : ld1<T>(hy + e) > 0.f);
        v = keep ? v : 0.f;
        st1<T>(ov + e, v);
        cs[e] += v;
        cq[e] += v * xv;
      }
      *reinterpret_cast<uint2*>(out + off) = *reinterpret_cast<const uint2*>(ov);
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    red[0][ty][tx * 4 + e] = cs[e];
    red[1][ty][tx * 4 + e] = cq[e];
  }
  __syncthreads();
  const int j = threadIdx.x, ch = blockIdx.y * 256 + j;
  if (ch < K) {
    double* slot = bnb.sums + (int64_t)(blockIdx.x % kStatSlots) * 2 * K;
    unsafeAtomicAdd(slot + ch, (double)((red[0][0][j] + red[0][1][j]) + (red[0][2][j] + red[0][3][j])));
    unsafeAtomicAdd(slot + K + ch, (double)((red[1][0][j] + red[1][1][j]) + (red[1][2][j] + red[1][3][j])));
  }
}
}  // namespace

hipError_t splitk_reduce_bnb(int dtype, const float* part, void* out, const void* addend, int M, int K, int splits,
                             const BnBwdEpilogue& bnb, hipStream_t st) {
  if (K % 4 != 0 || splits < 1 || M < 1) return hipErrorInvalidValue;
  const int cb = (K + 255) / 256;
  const int rows = (int64_t)((M + kStatRows - 1) / kStatRows) * cb >= 512 ? kStatRows : 16;
  const dim3 grid((M + rows - 1) / rows, cb);
  if (dtype == kBF16)
    hipLaunchKernelGGL(splitk_reduce_bnb_k<bf16_t>, grid, dim3(256), 0, st, part, static_cast<bf16_t*>(out),
                       static_cast<const bf16_t*>(addend), M, K, splits, rows, bnb);
  else if (dtype == kF16)
    hipLaunchKernelGGL(splitk_reduce_bnb_k<f16_t>, grid, dim3(256), 0, st, part, static_cast<f16_t*>(out),
                       static_cast<const f16_t*>(addend), M, K, splits, rows, bnb);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t splitk_reduce(int dtype, const float* part, void* out, int64_t n, int splits, hipStream_t st, float alpha,
                         const SplitkEpilogue* ep) {
  if (n % 4 != 0 || splits < 1) return hipErrorInvalidValue;
  if (ep != nullptr && ep->U != nullptr && (ep->N % 4 != 0 || ep->r < 8 || ep->r % 8 != 0 || n % ep->N != 0))
    return hipErrorInvalidValue;
  if (ep != nullptr && ep->scale != nullptr && (ep->N % 4 != 0 || n % ep->N != 0 || ep->shift == nullptr))
    return hipErrorInvalidValue;
  if (dtype == kBF16) return reduce_launch<bf16_t>(part, static_cast<bf16_t*>(out), n, splits, alpha, ep, st);
  if (dtype == kF16) return reduce_launch<f16_t>(part, static_cast<f16_t*>(out), n, splits, alpha, ep, st);
  return hipErrorInvalidValue;
}

namespace {

uint64_t magic36(int d) { return ((1ull << 36) + (uint64_t)d - 1) / (uint64_t)d; }

// tuning overrides (conv_wgrad_set_stages, for sweeps); 0 = the plan's choice
int g_wgrad_stages = 0;  // LDS ring depth
int g_wgrad_lean = 1;    // dense shapes on conv_wgrad_dense_k (0: the general kernel)
int g_wgrad_kp = 0;      // pixels per LDS stage of the dense kernel

template <typename T, int BM, int BN, bool DENSE>
hipError_t launch_d(const WgradArgs& a, hipStream_t st, int nb, int kp) {
  const int tiles = ((a.K + BM - 1) / BM) * (a.R * a.S * a.C / BN);
  const dim3 grid(tiles * a.splits + a.pr.blocks);
  if (DENSE && g_wgrad_lean) {
    if (kp == 128) {  // 3 stages of 128 pixels fit 160 KiB of LDS up to 128 x 64 tiles
      if constexpr (BM + BN <= 192) {
        if (nb >= 3) {
          hipLaunchKernelGGL((conv_wgrad_dense_k<T, BM, BN, 3, 128>), grid, dim3(kThreads), 0, st, a);
          return hipGetLastError();
        }
      }
      hipLaunchKernelGGL((conv_wgrad_dense_k<T, BM, BN, 2, 128>), grid, dim3(kThreads), 0, st, a);
    } else {
      if (nb == 2) hipLaunchKernelGGL((conv_wgrad_dense_k<T, BM, BN, 2, 64>), grid, dim3(kThreads), 0, st, a);
      else if (nb == 3) hipLaunchKernelGGL((conv_wgrad_dense_k<T, BM, BN, 3, 64>), grid, dim3(kThreads), 0, st, a);
      else hipLaunchKernelGGL((conv_wgrad_dense_k<T, BM, BN, 4, 64>), grid, dim3(kThreads), 0, st, a);
    }
  } else {
    if (nb == 2) hipLaunchKernelGGL((conv_wgrad_k<T, BM, BN, 2, DENSE>), grid, dim3(kThreads), 0, st, a);
    else if (nb == 3) hipLaunchKernelGGL((conv_wgrad_k<T, BM, BN, 3, DENSE>), grid, dim3(kThreads), 0, st, a);
    else hipLaunchKernelGGL((conv_wgrad_k<T, BM, BN, 4, DENSE>), grid, dim3(kThreads), 0, st, a);
  }
  return hipGetLastError();
}

// Ring depth / stage size: dense shapes with long reductions (ResNet layer1 1x1, M ~ 10^5) run
// 3 stages of 128 pixels (conv_wgrad_dense_k: 15.0 -> 12.2 us on MI355X, scripts/wgrad_probe.py);
// everything else 2 stages of 64 (deeper rings measured slower on the 3x3 shapes).
template <typename T, int BM, int BN>
hipError_t launch(const WgradArgs& a, hipStream_t st) {
  const bool dense = a.R == 1 && a.S == 1 && a.sh == 1 && a.sw == 1 && a.ph == 0 && a.pw == 0;
  const bool longk = dense && a.M >= 65536;
  const int nb = g_wgrad_stages > 0 ? g_wgrad_stages : (longk ? 3 : 2);
  const int kp = g_wgrad_kp > 0 ? g_wgrad_kp : (longk && g_wgrad_stages == 0 ? 128 : 64);
  return dense ? launch_d<T, BM, BN, true>(a, st, nb, kp) : launch_d<T, BM, BN, false>(a, st, nb, kp);
}

}  // namespace

bool conv_wgrad_supported(int C, int K) { return C % 64 == 0 && K % 8 == 0; }

void conv_wgrad_set_stages(int nb) {
  g_wgrad_stages = (nb & 7) >= 2 && (nb & 7) <= 4 ? (nb & 7) : 0;
  g_wgrad_lean = ((nb >> 4) & 1) ^ 1;  // tuning: bit 4 sends dense shapes to the general kernel
  g_wgrad_kp = (nb >> 5) & 1 ? 128 : 0;  // tuning: bit 5 stages 128 pixels (dense kernel)
}

// Plan (from the per-layer sweep of bench/conv_shapes.py over ResNet-50 at batch 32 on MI355X,
// profiles/conv_r01/conv_shapes_wgrad_sweep.json): 64 x 64 tiles win at every layer (more workgroups in flight;
// the kernel is latency- not MFMA-bound at these sizes), and the best pixel split keeps each
// workgroup at ~16-25 stages of 64 pixels — enough to amortize the prologue/epilogue, short enough
// that the grid fills the chip.  Fewer splits also bound the fp32 partial traffic (splits*K*RSC*8 B).
void conv_wgrad_plan(int M, int K, int C, int R, int S, int* bm, int* bn, int* splits, int* steps_per_split) {
  (void)K, (void)C, (void)R, (void)S;
  *bm = 64;
  *bn = 64;
  const int total_steps = (M + kBP - 1) / kBP;
  const int per = max(16, (total_steps + 63) / 64);
  *steps_per_split = per;
  *splits = (total_steps + per - 1) / per;
}

hipError_t conv_wgrad(int dtype, const void* dy, const void* x, void* dw, float* partials, const void* zero, int N,
                      int H, int W, int C, int K, int P, int Q, int R, int S, int sh, int sw, int ph, int pw, int bm,
                      int bn, int splits, int steps_per_split, hipStream_t st, float alpha,
                      const WgradPendingReduce* pending, bool defer_reduce, int pix) {
  if (!conv_wgrad_supported(C, K) || dtype == kF32) return hipErrorInvalidValue;
  if (C % bn != 0 || (bm != 64 && bm != 128) || (bn != 64 && bn != 128) || splits < 1) return hipErrorInvalidValue;
  const int64_t M64 = (int64_t)N * P * Q;
  // fdiv's 36-bit magic is exact for numerators < 2^22 and divisors < 2^14
  if (M64 <= 0 || M64 >= (1ll << 22) || (int64_t)P * Q >= (1 << 14)) return hipErrorInvalidValue;
  if ((int64_t)splits * steps_per_split * kBP < M64) return hipErrorInvalidValue;
  if (splits > 1 && partials == nullptr) return hipErrorInvalidValue;
  if ((int64_t)N * H * W * C >= (1ll << 31)) return hipErrorInvalidValue;  // 32-bit gather offsets
  WgradArgs a{static_cast<const uint16_t*>(dy), static_cast<const uint16_t*>(x),
              splits > 1 ? static_cast<void*>(partials) : dw, static_cast<const uint16_t*>(zero), N, H, W, C, K, P, Q,
              R, S, sh, sw, ph, pw, (int)M64, splits, steps_per_split, magic36(Q), magic36(P * Q), alpha,
              kBP / (P * Q), kBP % (P * Q)};
  a.pix = pix > 0 ? pix : C;
  if (pix > 0 && (pix % 8 != 0 || (R == 1 && S == 1 && sh == 1 && sw == 1 && ph == 0 && pw == 0)))
    return hipErrorInvalidValue;  // (the DENSE 1x1 path reads x as a plain [M, C] matrix)
  a.pr = WgradPendingReduce{};
  if (pending != nullptr && pending->part != nullptr) {
    if (pending->n % 4 != 0 || pending->splits < 1 || (pending->dtype != kBF16 && pending->dtype != kF16))
      return hipErrorInvalidValue;
    a.pr = *pending;
    // one extra workgroup per 64 output quads, at most 256 (they loop)
    const int64_t want = (pending->n / 4 + 63) / 64;
    a.pr.blocks = (int)(want < 256 ? want : 256);
  }
  a.nwg_main = ((K + bm - 1) / bm) * (R * S * C / bn) * splits;
  hipError_t e;
  if (dtype == kBF16) {
    if (bm == 128 && bn == 128) e = launch<bf16_t, 128, 128>(a, st);
    else if (bm == 128) e = launch<bf16_t, 128, 64>(a, st);
    else if (bn == 128) e = launch<bf16_t, 64, 128>(a, st);
    else e = launch<bf16_t, 64, 64>(a, st);
  } else {
    if (bm == 128 && bn == 128) e = launch<f16_t, 128, 128>(a, st);
    else if (bm == 128) e = launch<f16_t, 128, 64>(a, st);
    else if (bn == 128) e = launch<f16_t, 64, 128>(a, st);
    else e = launch<f16_t, 64, 64>(a, st);
  }
  if (e != hipSuccess || splits == 1 || defer_reduce) return e;
  return splitk_reduce(dtype, partials, dw, (int64_t)K * R * S * C, splits, st, alpha);  // C % 64 == 0: n % 4 == 0
}

}  // namespace hyp

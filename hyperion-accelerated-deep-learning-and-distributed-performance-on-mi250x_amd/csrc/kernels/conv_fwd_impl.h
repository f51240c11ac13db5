// conv_fwd_k's device code (the design is described in conv_igemm.hip): shared by conv_igemm.hip
// (the plain launches) and conv_dual.hip (a data gradient and a weight gradient horizontally fused
// into one launch).  Everything lives in an anonymous namespace: each including TU instantiates
// what it launches.
#pragma once
#include "hyp_common.h"
#include "hyp_kernels.h"
#include "mfma_lds.h"
#include "bn_fin.h"

namespace hyp {

// (namespace hyp, not the anonymous one: conv_igemm.hip and conv_dual.hip pass it between TUs)
struct ConvArgs {
  const uint16_t* in;    // [N, H, W, C]
  const uint16_t* w;     // [K, R, S, C]
  uint16_t* out;         // [N, P, Q, K]
  const uint16_t* zero;  // >= 1 KiB of zeros
  double* psum;          // Σy accumulator [kStatSlots][2][K] (fp64, zeroed by the caller) or null
  double* psq;           // psum + K: Σy²
  int N, H, W, C, K, P, Q, R, S, sh, sw, ph, pw;
  int M;                 // N*P*Q
  int pix;               // input pixel stride in elements (C, or the stem's 16: see hyp_kernels.h)
  int sd;                // DGRAD only: 2 = stride-2 data gradient by output phase (below), else 1
  int Hx, Wx;            // sd == 2: dX's spatial size (2P x 2Q); the tile grid is one phase's [N, P, Q]
  int nb;                // host only: LDS ring depth of this launch (0 = conv_set_stages / default 2)
  int direct;            // host only: forward + statistics with the DIRECT store epilogue (see conv_fwd_k)
  uint64_t mq, mpq;      // 36-bit magic multipliers of Q and P*Q (0: plain division; see fdiv36)
  int group;             // M-tiles per tile-order group (see conv_fwd_group)
  int splits, steps_per_split;  // split-K over the reduction (splits > 1: fp32 partials, no STATS)
  float* part;                  // [splits, M, K] fp32 when splits > 1
  const uint16_t* addend;       // optional [M, K] tensor added to the rounded output (no split)
  BnBwdEpilogue bnb;            // STATS && DGRAD: the BatchNorm-backward epilogue
  const float* aff_scale;       // !STATS: out = act(round(acc) * scale[k] + shift[k] (+ addend)) (eval BN)
  const float* aff_shift;
  int aff_act;
  int kvalid;                   // B rows that exist (< K only for a padded linear-CE vocabulary chunk)
  CeEpilogue ce;                // EPI 1 / 2: fused linear + cross-entropy (see linear_ce)
  unsigned long long* stamps;   // diagnostic timeline (conv_set_stamps), null in normal runs
  // XF: the input BatchNorm + ReLU applied to the A operand (hyp_kernels.h ConvInXform)
  FwdFin xfin;                  // the producer's statistics -> scale / shift (bn_fin.h)
  uint16_t* xf_out;             // side output relu(x * scale + shift) [N, H, W, C], or null
  int xf_on;
  int xf_dbg;                   // diagnostic (conv_set_xf_debug): 1 no transform, 2 no finalize, 4 no side store
};

// conv_dual.hip: the data-gradient launch of `a` (variant 0 plain, 1 BN-backward LEAN, 2 BN-backward
// full; tiles bm x bn, LDS ring nb) with the weight gradient `d` in the same grid.  Returns
// hipErrorNotSupported for a combination conv_dual.hip does not instantiate (nothing launched).
hipError_t conv_dual_launch(const ConvArgs& a, int dtype, int bm, int bn, int nb, int variant, const DualWgrad& d,
                            hipStream_t st);

namespace {

using mfl::bf16x8;
using mfl::f16x8;
using mfl::f32x4;
using mfl::u16x8;
using mfl::glds16;

constexpr int kBK = 64;
#ifndef HYP_CONV_KTHREADS
#define HYP_CONV_KTHREADS
constexpr int kThreads = 256;  // every conv kernel (and conv_dual.hip's fused launch) runs 4 waves
#endif

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

template <typename T>
__device__ __forceinline__ uint32_t pack2(float lo, float hi);
template <>
__device__ __forceinline__ uint32_t pack2<bf16_t>(float lo, float hi) { return pack_bf16x2(lo, hi); }
template <>
__device__ __forceinline__ uint32_t pack2<f16_t>(float lo, float hi) { return pack_f16x2(lo, hi); }

// floor(x / d) by a host-precomputed 36-bit magic (exact for x < 2^22, d < 2^14): the prologue's
// per-row (n, p, q) decomposition without integer-division sequences; magic 0 = plain division
__device__ __forceinline__ int fdiv36(int x, uint64_t magic, int d) {
  return magic ? (int)(((uint64_t)(uint32_t)x * magic) >> 36) : x / d;
}

__device__ __forceinline__ u16x8 frag(const uint16_t* lds, int row, int chunk) {
  return *reinterpret_cast<const u16x8*>(lds + row * kBK + ((chunk ^ swz(row)) * 8));
}


// relu(v * scale + shift) of 8 consecutive channels, rounded to T: the fp32 FMAs as packed pairs
// (v_pk_fma_f32), then the ReLU on the rounded 16-bit pairs as a signed-integer max with 0
// (v_pk_max_i16: a negative bf16 / f16 is a negative int16, -0 included) — the same values as the
// standalone apply's round(max(fma, 0)) for every finite input (a NaN stays NaN here)
typedef float xf_f2 __attribute__((ext_vector_type(2)));
typedef short xf_s2 __attribute__((ext_vector_type(2)));
template <typename T>
__device__ __forceinline__ u16x8 xf_apply(u16x8 v, const xf_f2 (&sc)[4], const xf_f2 (&sh)[4]) {
  const uint4 w = __builtin_bit_cast(uint4, v);
  const uint32_t wi[4] = {w.x, w.y, w.z, w.w};
  uint32_t o[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    xf_f2 f;
    if constexpr (sizeof(T) == 2 && __is_same(T, bf16_t)) {
      f = xf_f2{__uint_as_float(wi[q] << 16), __uint_as_float(wi[q] & 0xffff0000u)};
    } else {
      f = xf_f2{f16_lo(wi[q]), f16_hi(wi[q])};
    }
    f = __builtin_elementwise_fma(f, sc[q], sh[q]);
    const uint32_t pk = __is_same(T, bf16_t) ? pack_bf16x2(f.x, f.y) : pack_f16x2(f.x, f.y);
    const xf_s2 r = __builtin_elementwise_max(__builtin_bit_cast(xf_s2, pk), xf_s2{0, 0});
    o[q] = __builtin_bit_cast(uint32_t, r);
  }
  return __builtin_bit_cast(u16x8, (uint4){o[0], o[1], o[2], o[3]});
}

// Diagnostic per-workgroup timeline: s_memrealtime (100 MHz, chip-wide) at entry, before and
// after the K loop and at the end, plus HW_ID / XCC_ID, then (EPI 0 stores) after the epilogue's
// LDS transpose and after its store loop — 8 words per workgroup.  Never on in
// timed runs (the stamp's lgkmcnt(0) forbids overlaps); read its SHARES, not its length.
__device__ __forceinline__ unsigned long long realtime_stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

// DGRAD = false: W is [K, R, S, C] (reduction contiguous; B tiles are row slices, read row-wise).
// DGRAD = true:  the stride-1 data gradient dX = conv(dY, flip(W) with C <-> K, pad R-1-p), run on
//   the ORIGINAL filter [C_dgrad_in = a.C][R][S][K_dgrad_out = a.K]: a B tile is 64 reduction rows
//   of W[c, R-1-r, S-1-s, n0 : n0+BN] (output channels contiguous), staged row-permuted
//   (tr_row_to_k) and read transposed with ds_read_b64_tr_b16 — no flipped/transposed filter copy.
// EPI 0: the stores above; 1: linear-CE log-sum-exp partials (no output tensor); 2: linear-CE
// softmax gradient written in place of the logits (see linear_ce)
// LEAN (BN-backward epilogue only): mode 0/1 without an addend — no y / addend prefetch registers
// (64x64: 119 -> 104 VGPR+AGPR, 128x64: 191 -> 158, one more resident wave per SIMD there)
// XF (forward only): the A operand is the producer's raw conv output, transformed at fragment-read
// time into relu(x * scale + shift) — the training BatchNorm apply + ReLU of the previous layer
// fused into this conv (no standalone apply pass: one launch and one read + write of the
// activation fewer).  scale / shift are finalized per workgroup from the producer's statistics
// sums into an LDS table; the first output-channel tile's workgroups also store the transformed
// activation (the backward's saved input) at the centre tap.
// DIRECT (forward + BN statistics only, no addend / affine): the epilogue stores the lane-pair
// packed accumulators straight to global memory (32-byte row segments per 8 lanes) instead of
// transposing the tile through LDS into 16-byte row chunks — no LDS round trip or barrier before
// the stores (the transpose was ~2 us of a 1x1 forward tile's ~6 us)
// LDS (uint16 elements) of one conv_fwd_k workgroup: the ring, or (NB == 1: one stage) at least the
// epilogue's transpose tile + its reduction scratch
template <int BM, int BN, int NB>
constexpr int conv_fwd_smem() {
  constexpr int kBuf = (BM + BN) * kBK;
  constexpr int kEpi = BM * (BN + 8) + 16 * BN, kCe = 8 * BM;
  return NB * kBuf > kEpi ? (NB * kBuf > kCe ? NB * kBuf : kCe) : (kEpi > kCe ? kEpi : kCe);
}

// The workgroup body: `blk` is the workgroup's linear id within this conv's grid (the hardware id
// for a plain launch, a remapped id inside conv_dual.hip's horizontally fused dgrad + wgrad
// launch), `smem` its conv_fwd_smem<BM, BN, NB>() LDS elements.
template <typename T, int BM, int BN, bool STATS, bool DGRAD, int NB, int EPI = 0, bool LEAN = false,
          bool DIRECT = false, bool XF = false>
__device__ __forceinline__ void conv_fwd_body(const ConvArgs& a, const int blk, uint16_t* smem) {
  constexpr int FM = BM / 32, FN = BN / 32;  // 16x16 fragments per wave (wave tile BM/2 x BN/2)
  constexpr int IA = BM / 32, IB = BN / 32;  // glds instructions per wave per slice
  constexpr int kBuf = (BM + BN) * kBK;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  unsigned long long tsa = 0, tsb = 0, tsc = 0;
  if (a.stamps != nullptr) tsa = realtime_stamp();

  const int tiles_m = (a.M + BM - 1) / BM, tiles_n = (a.K + BN - 1) / BN, nwg = tiles_m * tiles_n;
  // Stride-2 data gradient (sd2): dX pixel (2i + pa, 2j + pb) only receives taps r ≡ pa + ph,
  // s ≡ pb + pw (mod 2), from dY pixel (i + (pa + ph - r) / 2, j + (pb + pw - s) / 2) — so each of
  // the 4 output phases is a small stride-1 conv over dY (1x1, 1x2, 2x1, 2x2 taps for a 3x3
  // filter, padding 1) and one launch runs all four: the tile grid is one phase's [N, P, Q] x C,
  // the phase index runs fastest (every XCD gets the same mix of light and heavy phases), and the
  // epilogue stores each row at its interleaved dX pixel.
  const bool sd2 = DGRAD && a.sd == 2;
  int bid, split, phase = 0;
  if (sd2) {
    const int lb = mfl::xcd_remap(blk, nwg * 4);
    phase = lb & 3;
    bid = lb >> 2;
    split = 0;
  } else {
    // split-major logical order: an XCD's contiguous range is tiles of ONE reduction split
    bid = mfl::xcd_remap(blk, nwg * a.splits);
    split = bid / nwg;
    bid -= split * nwg;
  }
  const int ph_a = phase >> 1, ph_b = phase & 1;
  const int r0 = sd2 ? ((ph_a + a.ph) & 1) : 0, s0 = sd2 ? ((ph_b + a.pw) & 1) : 0;
  const int nr = sd2 ? (a.R - r0 + 1) / 2 : a.R, ns = sd2 ? (a.S - s0 + 1) / 2 : a.S;
  const int kGroup = a.group;
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
    const int n = fdiv36(mm, a.mpq, PQ), pq = mm - n * PQ, p = fdiv36(pq, a.mq, a.Q), q = pq - p * a.Q;
    a_h0[i] = sd2 ? p + (ph_a + a.ph - r0) / 2 : p * a.sh - a.ph;
    a_w0[i] = sd2 ? q + (ph_b + a.pw - s0) / 2 : q * a.sw - a.pw;
    a_off[i] = (((int64_t)n * a.H + a_h0[i]) * a.W + a_w0[i]) * a.pix + chunk * 8;
  }
  const int64_t ldw = (int64_t)a.R * a.S * a.C;
  const uint16_t* b_src[IB];
#pragma unroll
  for (int i = 0; i < IB; ++i) {
    if (!DGRAD) {
      const int row = (i * 4 + wave) * 8 + (lane >> 3);
      const int k = n0 + row;
      const int chunk = slot ^ swz(row);
      b_src[i] = k < a.kvalid ? a.w + (int64_t)k * ldw + chunk * 8 : nullptr;
    } else {  // image [64 reduction rows][BN]: a wave instruction fills 1024 / (2 BN) rows
      constexpr int RB = 1024 / (2 * BN), CB = BN / 8;
      const int row = (i * 4 + wave) * RB + lane / CB;
      const int col = n0 + (((lane % CB) ^ mfl::swz_tr<BN>(row)) << 3);
      b_src[i] = col < a.K ? a.w + (int64_t)mfl::tr_row_to_k(row) * a.R * a.S * a.K + col : nullptr;
    }
  }
  const uint16_t* zero = a.zero + slot * 8;

  const int cpb = a.C / kBK;  // 64-channel slices per filter tap
  const int kt0 = split * a.steps_per_split;  // this split's reduction steps [kt0, kt0 + nk)
  const int nk = sd2 ? nr * ns * cpb : max(0, min(a.R * a.S * cpb - kt0, a.steps_per_split));

  // reduction position of the NEXT stage to issue, advanced incrementally (stages are issued in
  // order): filter tap (r, s) and channel slice c0 — no per-stage integer divisions
  int st_r, st_s, st_c0;
  {
    const int rs = kt0 / cpb;
    st_c0 = (kt0 - rs * cpb) * kBK;
    st_r = rs / a.S;
    st_s = rs - st_r * a.S;
  }
  int64_t st_t = kt0;
  auto stage = [&](uint16_t* buf) {
    const int r = st_r, s = st_s, c0 = st_c0;
    const int dh = sd2 ? -r : r, dw = sd2 ? -s : s;  // sd2: (r, s) count the phase's taps
    const int64_t tap = ((int64_t)dh * a.W + dw) * a.pix + c0;
#pragma unroll
    for (int i = 0; i < IA; ++i) {
      const int h = a_h0[i] + dh, w = a_w0[i] + dw;
      const bool ok = a_ok[i] & ((unsigned)h < (unsigned)a.H) & ((unsigned)w < (unsigned)a.W);
      glds16(ok ? a.in + a_off[i] + tap : zero, buf + (i * 4 + wave) * 8 * kBK);
    }
    // DGRAD: filter tap (R-1-r, S-1-s) of reduction channels c0 .. c0+63 (sd2: tap (r0 + 2r, s0 + 2s))
    const int64_t kofs =
        DGRAD ? ((int64_t)c0 * a.R * a.S + (sd2 ? (r0 + 2 * r) * a.S + s0 + 2 * s : (a.R - 1 - r) * a.S + (a.S - 1 - s))) * a.K
              : st_t * kBK;
#pragma unroll
    for (int i = 0; i < IB; ++i)
      glds16(b_src[i] ? b_src[i] + kofs : zero, buf + BM * kBK + (i * 4 + wave) * 512);
    ++st_t;
    st_c0 += kBK;
    if (st_c0 == a.C) {
      st_c0 = 0;
      if (++st_s == ns) {
        st_s = 0;
        ++st_r;
      }
    }
  };
  // dX row (in units of K elements) of tile row m: m itself, or (sd2) its interleaved phase pixel
  auto orow = [&](int m) -> int64_t {
    if (!sd2) return m;
    const int n = fdiv36(m, a.mpq, PQ), pq = m - n * PQ, p = fdiv36(pq, a.mq, a.Q), q = pq - p * a.Q;
    return ((int64_t)n * a.Hx + 2 * p + ph_a) * a.Wx + 2 * q + ph_b;
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // XF: channel tid's statistics loads go out ahead of the first stages (their arithmetic runs
  // after the stage issue, so the two round trips overlap); channels >= 256 (C = 512) after
  __shared__ float xtab[XF ? 2 * kXfMaxC : 1];  // [scale | shift] of the input channels
  double xsa[kStatSlots], xsq[kStatSlots];
  float xw = 0.f, xb = 0.f;
  if constexpr (XF) {
    if (tid < a.C && !(a.xf_dbg & 2)) fwd_const_load(a.xfin, a.C, tid, xsa, xsq, xw, xb);
  }
  __builtin_amdgcn_sched_barrier(0);
  // NB-deep ring: stage t+NB-1 is issued right after the barrier that retires stage t-1's buffer
  // (NB == 1: stage 0 is issued here too, ahead of the epilogue loads below)
#pragma unroll
  for (int i = 0; i < (NB > 1 ? NB - 1 : 1); ++i)
    if (i < nk) stage(smem + i * kBuf);
  __builtin_amdgcn_sched_barrier(0);
  // XF: the consumed stage's filter tap / channel slice, advanced per K step
  int cs_r = 0, cs_s = 0, cs_c0 = 0;
  bool xside = false;
  if constexpr (XF) {
    const bool writer = blk == 0;
    if (a.xf_dbg & 2) {
      for (int c = tid; c < a.C; c += kThreads) xtab[c] = 1.f, xtab[kXfMaxC + c] = 0.f;
    } else {
      if (tid < a.C) fwd_const_from(a.xfin, tid, xsa, xsq, xw, xb, writer, xtab[tid], xtab[kXfMaxC + tid]);
      for (int c = tid + kThreads; c < a.C; c += kThreads) fwd_const1(a.xfin, a.C, c, writer, xtab[c], xtab[kXfMaxC + c]);
    }
    mfl::barrier_keep_vm();  // the table is read before the K loop's first barrier (xf_pass)
    const int rs = kt0 / cpb;
    cs_c0 = (kt0 - rs * cpb) * kBK;
    cs_r = rs / a.S;
    cs_s = rs - cs_r * a.S;
    xside = a.xf_out != nullptr && tn == 0 && !(a.xf_dbg & 4);
  }
  // Epilogue operand prefetch: the addend / BN-backward x, y chunks this thread will store, issued
  // BEFORE the K loop so their HBM round trip overlaps the loads and MFMAs of the whole tile
  // (issued after the loop, the BN-backward epilogue waited ~2 us for x on every workgroup; inside
  // the store loop, a round trip per iteration: +18 us on a layer1 dgrad).  Issued right after the
  // first stages (which the K loop needs first) and ahead of the epilogue constants; a counted
  // stage wait that sees them behind stage 0 only over-waits.  (Split-K tiles store fp32 partials
  // instead: no prefetch.)
  constexpr bool FSTATS = STATS && !DGRAD, BNB = STATS && DGRAD;
  constexpr int kChunksPerRow = BN / 8;
  constexpr int kIt = BM * kChunksPerRow / kThreads;
  uint4 pd[kIt], px[kIt], py[kIt];
  const bool has_add = !FSTATS && !LEAN && a.addend != nullptr;
  const bool stores_here = a.splits == 1 || sd2;
#pragma unroll
  for (int it = 0; it < kIt; ++it) {
    const int idx = it * kThreads + tid;
    const int lr = idx / kChunksPerRow, ch = idx - lr * kChunksPerRow;
    const int m = m0 + lr, k = n0 + ch * 8;
    const bool ok = stores_here && m < a.M && k < a.K;
    const int64_t off = (ok ? orow(m) : 0) * a.K + k;
    pd[it] = px[it] = py[it] = uint4{0u, 0u, 0u, 0u};
    if (has_add && ok) pd[it] = *reinterpret_cast<const uint4*>(a.addend + off);
    if (BNB && ok) {
      px[it] = *reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(a.bnb.x) + off);
      if (!LEAN && a.bnb.mode == 2)
        py[it] = *reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(a.bnb.y) + off);
    }
  }

  // per-channel epilogue constants of this thread's store column (the eval-BN affine or the
  // BN-backward ReLU-mask scale/shift), loaded before the main loop so the epilogue never waits
  // on them (loaded there, they cost a full memory round trip per tile) — but AFTER the first
  // stages are issued: the BN-backward scale/shift arithmetic consumes its loads at once, and
  // ahead of the stage issue that vmcnt(0) serialised a whole HBM round trip (~2 us per
  // workgroup) in front of the K loop; here it overlaps the stages' own latency
  float asc[8], ash[8];
  {
    constexpr int kCpr = BN / 8;
    const int my_k = n0 + (tid % kCpr) * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) asc[e] = ash[e] = 0.f;
    // (8 channels = two 16-byte loads per array: my_k % 8 == 0 and the [K] fp32 arrays are aligned)
    auto ld8 = [](const float* p, float (&v)[8]) {
      const float4 x0 = reinterpret_cast<const float4*>(p)[0], x1 = reinterpret_cast<const float4*>(p)[1];
      v[0] = x0.x; v[1] = x0.y; v[2] = x0.z; v[3] = x0.w; v[4] = x1.x; v[5] = x1.y; v[6] = x1.z; v[7] = x1.w;
    };
    if (!STATS && a.aff_scale != nullptr && my_k < a.K) {
      ld8(a.aff_scale + my_k, asc);
      ld8(a.aff_shift + my_k, ash);
    }
    if (STATS && DGRAD && a.bnb.mode == 1 && my_k < a.K) {  // ReluMask<MASKX> arithmetic of bn_act.hip
      float wv[8], iv[8], bv[8], mv[8];
      ld8(a.bnb.invstd + my_k, iv);
      ld8(a.bnb.mean + my_k, mv);
#pragma unroll
      for (int e = 0; e < 8; ++e) wv[e] = 1.f, bv[e] = 0.f;
      if (a.bnb.w) ld8(a.bnb.w + my_k, wv);
      if (a.bnb.b) ld8(a.bnb.b + my_k, bv);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float sc = wv[e] * iv[e];
        asc[e] = sc;
        ash[e] = bv[e] - mv[e] * sc;
      }
    }
  }

  // XF: every thread transforms, in place, the A chunks its own LDS-DMA wrote (row
  // (i*4 + wave)*8 + lane/8, physical 16-byte slot lane%8 = logical chunk slot ^ swz(row)) once its
  // own loads have landed and BEFORE the barrier that publishes the stage: each element is
  // transformed once, the K loop's fragment reads and MFMAs stay as they are.  Padding taps and
  // rows past M read the zero page and stay zero.
  auto xf_pass = [&](uint16_t* buf) {
    if (a.xf_dbg & 1) return;
    const bool center = xside && cs_r == a.ph && cs_s == a.pw;
    // the thread's logical chunk is the same in all IA rows (swz = (row >> 1) & 7, rows 32 apart)
    const int cb = cs_c0 + ((slot ^ swz(wave * 8 + (lane >> 3))) << 3);
    xf_f2 sc[4], sh[4];
    {
      const float4* ps = reinterpret_cast<const float4*>(xtab + cb);
      const float4* pt = reinterpret_cast<const float4*>(xtab + kXfMaxC + cb);
      const float4 s0 = ps[0], s1 = ps[1], t0 = pt[0], t1 = pt[1];
      sc[0] = xf_f2{s0.x, s0.y}; sc[1] = xf_f2{s0.z, s0.w}; sc[2] = xf_f2{s1.x, s1.y}; sc[3] = xf_f2{s1.z, s1.w};
      sh[0] = xf_f2{t0.x, t0.y}; sh[1] = xf_f2{t0.z, t0.w}; sh[2] = xf_f2{t1.x, t1.y}; sh[3] = xf_f2{t1.z, t1.w};
    }
    u16x8 v[IA];
    bool ok[IA];
#pragma unroll
    for (int i = 0; i < IA; ++i) {  // every read first (no write can alias a later read)
      const int h = a_h0[i] + cs_r, w = a_w0[i] + cs_s;
      ok[i] = a_ok[i] & ((unsigned)h < (unsigned)a.H) & ((unsigned)w < (unsigned)a.W);
      v[i] = *reinterpret_cast<const u16x8*>(buf + (i * 4 + wave) * 8 * kBK + lane * 8);
    }
#pragma unroll
    for (int i = 0; i < IA; ++i) {
      if (ok[i]) {  // padding taps / rows past M read the zero page and stay zero
        v[i] = xf_apply<T>(v[i], sc, sh);
        *reinterpret_cast<u16x8*>(buf + (i * 4 + wave) * 8 * kBK + lane * 8) = v[i];
      }
    }
    if (center) {  // centre tap: this row's input pixel is its output pixel (stride 1, "same" padding)
#pragma unroll
      for (int i = 0; i < IA; ++i)
        if (ok[i])
          *reinterpret_cast<u16x8*>(a.xf_out + (int64_t)(m0 + (i * 4 + wave) * 8 + (lane >> 3)) * a.C + cb) = v[i];
    }
  };

  const int r16 = lane & 15, c4 = lane >> 4;
  if (a.stamps != nullptr) tsb = realtime_stamp();
  for (int t = 0; t < nk; ++t) {
    if (NB == 1) {
      // single buffer (short reductions: LDS for more resident workgroups instead of a ring):
      // wait until every wave has read stage t-1, refill, wait for the DMA, publish
      if (t > 0) {
        mfl::barrier_keep_vm();
        stage(smem);
      }
      mfl::wait_vmcnt<0>();
      if constexpr (XF) xf_pass(smem);
      mfl::barrier_keep_vm();
    } else {
      mfl::wait_stage<IA + IB, NB>(min(NB - 2, nk - 1 - t));
      if constexpr (XF) xf_pass(smem + (t % NB) * kBuf);
      mfl::barrier_keep_vm();  // stage t visible to all waves; every wave is done with buffer (t-1) % NB
      if (t + NB - 1 < nk) stage(smem + ((t + NB - 1) % NB) * kBuf);
    }
    const uint16_t* as = smem + (t % NB) * kBuf;
    const uint16_t* bs = as + BM * kBK;
#pragma unroll
    for (int ks = 0; ks < kBK / 32; ++ks) {
      u16x8 fa[FM], fb[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) fa[i] = frag(as, wm * (BM / 2) + i * 16 + r16, ks * 4 + c4);
#pragma unroll
      for (int j = 0; j < FN; ++j)
        fb[j] = DGRAD ? mfl::frag_tr<BN>(bs, ks * 32, wn * (BN / 2) + j * 16, lane)
                      : frag(bs, wn * (BN / 2) + j * 16 + r16, ks * 4 + c4);
      if (DGRAD) mfl::lds_reads_done();  // the asm transposed reads (see mfma_lds.h) have returned
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mma<T>(fa[i], fb[j], acc[i][j]);
    }
    if constexpr (XF) {  // the next consumed stage's tap / channel slice
      cs_c0 += kBK;
      if (cs_c0 == a.C) {
        cs_c0 = 0;
        if (++cs_s == a.S) {
          cs_s = 0;
          ++cs_r;
        }
      }
    }
  }
  __syncthreads();  // the epilogue reuses the ring
  if (a.stamps != nullptr) tsc = realtime_stamp();
  // (the end stamp is written when the kernel returns, on every epilogue path)
  unsigned long long tsd = 0, tse = 0;
  struct StampEnd {
    const ConvArgs& a;
    const int blk;
    unsigned long long s0, s1, s2;
    const unsigned long long& s4;
    const unsigned long long& s5;
    __device__ ~StampEnd() {
      if (a.stamps != nullptr && threadIdx.x == 0) {
        const unsigned long long s3 = realtime_stamp();
        unsigned long long* o = a.stamps + (size_t)blk * 8;
        o[0] = s0;
        o[1] = s1;
        o[2] = s2;
        o[3] = s3;
        o[4] = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_REG_HW_ID
        o[5] = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
        o[6] = s4;
        o[7] = s5;
      }
    }
  } stamp_end{a, blk, tsa, tsb, tsc, tsd, tse};

  if (EPI != 0) {
    // ---- fused linear + cross-entropy.  Class n0 + n of this tile is vocabulary index
    // col_off + n; z = round(acc + bias) (the bf16 logit the unfused path would store).
    // EPI 1: per-row (max, Σexp) over the tile's classes -> ce.part[tile_n][m], the target
    //        logit -> ce.zt[m]; the logits are never written.
    // EPI 2: acc <- (exp(z - lse[m]) - [class == target]) * scale (0 for ignored rows and padded
    //        classes), then the regular store epilogue writes dz.
    const CeEpilogue& ce = a.ce;
    float bcol[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = n0 + wn * (BN / 2) + j * 16 + r16;
      bcol[j] = (ce.bias != nullptr && n < a.kvalid) ? ce.bias[a.ce.col_off + n] : 0.f;
    }
    const float gscale = EPI == 2 ? *ce.scale : 0.f;
    float* ls = reinterpret_cast<float*>(smem);  // EPI 1: [2 (wn)][BM][2] (row max, row Σexp)
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int lr = wm * (BM / 2) + i * 16 + c4 * 4 + e;
        const int m = m0 + lr;
        const int64_t tg = m < a.M ? ce.target[m] : ce.ignore;
        if (EPI == 1) {
          float v[FN], mx = -INFINITY;
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            const int n = n0 + wn * (BN / 2) + j * 16 + r16;
            v[j] = -INFINITY;
            if (n < a.kvalid) {
              v[j] = rnd<T>(acc[i][j][e] + bcol[j]);
              if (m < a.M && (int64_t)(ce.col_off + n) == tg) ce.zt[m] = v[j];
            }
            mx = fmaxf(mx, v[j]);
          }
#pragma unroll
          for (int o = 1; o < 16; o <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));  // the row's 16 lanes
          float sm = 0.f;
          if (mx != -INFINITY) {
#pragma unroll
            for (int j = 0; j < FN; ++j) sm += __expf(v[j] - mx);  // exp(-inf) = 0 for padding
          }
#pragma unroll
          for (int o = 1; o < 16; o <<= 1) sm += __shfl_xor(sm, o, 64);
          if (r16 == 0) {
            ls[(wn * BM + lr) * 2 + 0] = mx;
            ls[(wn * BM + lr) * 2 + 1] = sm;
          }
        } else {
          const float lse = m < a.M ? ce.lse[m] : 0.f;
          const float sc = (m < a.M && tg != ce.ignore) ? gscale : 0.f;
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            const int n = n0 + wn * (BN / 2) + j * 16 + r16;
            float g = 0.f;
            if (n < a.kvalid) {
              const float z = rnd<T>(acc[i][j][e] + bcol[j]);
              g = (__expf(z - lse) - ((int64_t)(ce.col_off + n) == tg ? 1.f : 0.f)) * sc;
            }
            acc[i][j][e] = g;
          }
        }
      }
    }
    if (EPI == 1) {
      __syncthreads();
      for (int lr = tid; lr < BM; lr += kThreads) {
        const int m = m0 + lr;
        if (m < a.M) {
          const float m0v = ls[lr * 2], s0 = ls[lr * 2 + 1];
          const float m1v = ls[(BM + lr) * 2], s1 = ls[(BM + lr) * 2 + 1];
          const float mx = fmaxf(m0v, m1v);
          float sm = 0.f;
          if (mx != -INFINITY) sm = s0 * __expf(m0v - mx) + s1 * __expf(m1v - mx);
          ce.part[(int64_t)tn * a.M + m] = make_float2(mx, sm);
        }
      }
      return;
    }
  }

  if (a.splits > 1 && !sd2) {  // split-K: raw fp32 partials (16 lanes = one 64-byte row segment per store)
    float* part = a.part + (int64_t)split * a.M * a.K;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + wm * (BM / 2) + i * 16 + c4 * 4 + e;
        if (m < a.M) {
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            const int n = n0 + wn * (BN / 2) + j * 16 + r16;
            if (n < a.K) part[(int64_t)m * a.K + n] = acc[i][j][e];
          }
        }
      }
    return;
  }

  // ---- epilogue.  acc[i][j][e] is out[m0 + wm*BM/2 + i*16 + c4*4 + e][n0 + wn*BN/2 + j*16 + r16].
  // STATS && !DGRAD: forward BN statistics; STATS && DGRAD: the BN-backward epilogue (a.bnb).
  // Values are rounded to T once; the BN statistics use the rounded values (what BN will read),
  // and the tile is transposed through LDS so the global stores are whole 16-byte row chunks
  // (a raw accumulator store would be 2-byte scattered writes).
  constexpr int kLd = BN + 8;  // padded LDS row (elements)
  uint16_t* tile = smem;       // [BM][kLd] of T (the K loop ended with a barrier: smem is free)
  float* red = reinterpret_cast<float*>(smem + BM * kLd);  // [2 (wm)][2 (sum, sq)][BN]
  float csum[FN], csq[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) csum[j] = csq[j] = 0.f;
  // acc -> LDS as 32-bit column pairs: neighbour lanes (r16, r16 ^ 1) hold adjacent columns of the
  // same 4 rows, so one lane^1 exchange per row pair lets the even lane store rows e, the odd lane
  // rows e + 1, each as (column 2c, 2c + 1) — half the LDS write instructions of 2-byte stores
  const bool odd = r16 & 1;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int lc = wn * (BN / 2) + j * 16 + (r16 & ~1);
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = rnd<T>(acc[i][j][e]);
        if (FSTATS && m0 + wm * (BM / 2) + i * 16 + c4 * 4 + e < a.M) {
          csum[j] += v[e];
          csq[j] += v[e] * v[e];
        }
      }
#pragma unroll
      for (int ep = 0; ep < 4; ep += 2) {
        // lane ^ 1 exchange on the DPP path (quad_perm [1,0,3,2]): no LDS traffic, unlike __shfl_xor
        const float got = __builtin_bit_cast(
            float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, odd ? v[ep] : v[ep + 1]), 0xB1, 0xF, 0xF, false));
        const int lr = wm * (BM / 2) + i * 16 + c4 * 4 + ep + (odd ? 1 : 0);
        const uint32_t pk = pack2<T>(odd ? got : v[ep], odd ? v[ep + 1] : got);
        if (DIRECT) {
          if (m0 + lr < a.M && n0 + lc < a.K)
            *reinterpret_cast<uint32_t*>(a.out + (int64_t)(m0 + lr) * a.K + n0 + lc) = pk;
        } else {
          *reinterpret_cast<uint32_t*>(reinterpret_cast<T*>(tile) + lr * kLd + lc) = pk;
        }
      }
    }
  }
  if (FSTATS) {
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
  if (a.stamps != nullptr) tsd = realtime_stamp();
  // one no-return f64 atomic per channel per tile, issued BEFORE the tile's stores so their
  // ~1 us memory-side latency overlaps the store phase instead of extending the workgroup's drain
  if (FSTATS && tid < BN) {
    const int k = n0 + tid;
    if (k < a.K) {
      const int64_t slot = (int64_t)(tm % kStatSlots) * 2 * a.K;
      unsafeAtomicAdd(a.psum + slot + k, (double)(red[0 * BN + tid] + red[2 * BN + tid]));
      unsafeAtomicAdd(a.psq + slot + k, (double)(red[1 * BN + tid] + red[3 * BN + tid]));
    }
  }
  if (DIRECT) return;  // (stored above; the statistics atomics are issued)
  // BNB: every thread keeps ONE 8-channel chunk column (kThreads % kChunksPerRow == 0) across its rows
  float bs[8], bq[8];
  if (BNB) {
#pragma unroll
    for (int e = 0; e < 8; ++e) bs[e] = bq[e] = 0.f;
  }
#pragma unroll
  for (int it = 0; it < BM * kChunksPerRow / kThreads; ++it) {
    const int idx = it * kThreads + tid;
    const int lr = idx / kChunksPerRow, ch = idx - lr * kChunksPerRow;
    const int m = m0 + lr, k = n0 + ch * 8;
    if (m < a.M && k < a.K) {
      uint4 v = *reinterpret_cast<const uint4*>(tile + lr * kLd + ch * 8);
      if (BNB) {
        // dz = round(round(acc) + addend) * mask; Σdz, Σdz·x over the stored (rounded) values
        float o[8], xv[8], yv[8] = {};
        Vec8<T>::load(reinterpret_cast<const T*>(&v), o);
        if (has_add) {
          float d[8];
          Vec8<T>::load(reinterpret_cast<const T*>(&pd[it]), d);
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = rnd<T>(o[e] + d[e]);
        }
        Vec8<T>::load(reinterpret_cast<const T*>(&px[it]), xv);
        if (!LEAN) Vec8<T>::load(reinterpret_cast<const T*>(&py[it]), yv);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const bool keep =
              a.bnb.mode == 0 || ((LEAN || a.bnb.mode == 1) ? fmaf(xv[e], asc[e], ash[e]) > 0.f : yv[e] > 0.f);
          o[e] = keep ? o[e] : 0.f;
          bs[e] += o[e];
          bq[e] += o[e] * xv[e];
        }
        Vec8<T>::store(reinterpret_cast<T*>(&v), o);
      } else if (!STATS && (has_add || a.aff_scale != nullptr)) {
        // out = round(round(acc) + addend): the same two roundings as a separate T add kernel;
        // eval BN: out = round(act(round(acc) * scale + shift (+ addend))), the conv -> BN(eval)
        // (-> + residual) (-> ReLU) composition in one store
        float o[8];
        Vec8<T>::load(reinterpret_cast<const T*>(&v), o);
        if (a.aff_scale != nullptr) {
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = fmaf(o[e], asc[e], ash[e]);
        }
        if (has_add) {
          float d[8];
          Vec8<T>::load(reinterpret_cast<const T*>(&pd[it]), d);
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] += d[e];
        }
        if (a.aff_act) {
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = fmaxf(o[e], 0.f);
        }
        Vec8<T>::store(reinterpret_cast<T*>(&v), o);
      }
      st16_wt(a.out + orow(m) * a.K + k, v);
    }
  }
  if (a.stamps != nullptr) tse = realtime_stamp();
  if (BNB) {
    // column sums: the lanes of a wave that share a chunk column (lane % kChunksPerRow) by xor
    // shuffles, then the 4 waves through LDS in fixed order
    static_assert(64 % kChunksPerRow == 0, "chunk columns repeat within a wave");
#pragma unroll
    for (int o = kChunksPerRow; o < 64; o <<= 1) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        bs[e] += __shfl_xor(bs[e], o, 64);
        bq[e] += __shfl_xor(bq[e], o, 64);
      }
    }
    float* wred = reinterpret_cast<float*>(smem + BM * kLd);  // [4 waves][kChunksPerRow][16]
    if (lane < kChunksPerRow) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        wred[(wave * kChunksPerRow + lane) * 16 + e] = bs[e];
        wred[(wave * kChunksPerRow + lane) * 16 + 8 + e] = bq[e];
      }
    }
    __syncthreads();
    if (tid < BN && n0 + tid < a.K) {
      const int chn = tid >> 3, e = tid & 7;
      float sa = 0.f, sb = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        sa += wred[(w * kChunksPerRow + chn) * 16 + e];
        sb += wred[(w * kChunksPerRow + chn) * 16 + 8 + e];
      }
      double* slot = a.bnb.sums + (int64_t)(tm % kStatSlots) * 2 * a.K;
      unsafeAtomicAdd(slot + n0 + tid, (double)sa);
      unsafeAtomicAdd(slot + a.K + n0 + tid, (double)sb);
    }
  }
}

template <typename T, int BM, int BN, bool STATS, bool DGRAD, int NB, int EPI = 0, bool LEAN = false,
          bool DIRECT = false, bool XF = false>
__global__ __launch_bounds__(kThreads) void conv_fwd_k(const ConvArgs a) {
  __shared__ __attribute__((aligned(16))) uint16_t smem[conv_fwd_smem<BM, BN, NB>()];
  conv_fwd_body<T, BM, BN, STATS, DGRAD, NB, EPI, LEAN, DIRECT, XF>(a, blockIdx.x, smem);
}

}  // namespace
}  // namespace hyp

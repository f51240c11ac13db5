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
// ROUNDED outputs, added atomically into the [2][K] sums the BN apply finalizes inline
// (bn_act.hip), so BN's separate statistics pass over y and its finalize launch disappear.
// Requirements: C % 64 == 0 (every ResNet conv but the 3-channel stem), 16-byte aligned tensors.
#include <type_traits>

#include "conv_fwd_impl.h"
#include "conv_persist.h"

namespace hyp {
namespace {

template <typename T, int BM, int BN, int NB>
hipError_t launch_nb(const ConvArgs& a, bool stats, bool dgrad, hipStream_t st) {
  const int tiles = ((a.M + BM - 1) / BM) * ((a.K + BN - 1) / BN) * a.splits;
  if (a.xf_on && stats)
    hipLaunchKernelGGL((conv_fwd_k<T, BM, BN, true, false, NB, 0, false, false, true>), dim3(tiles), dim3(kThreads), 0,
                       st, a);
  else if (a.xf_on)
    hipLaunchKernelGGL((conv_fwd_k<T, BM, BN, false, false, NB, 0, false, false, true>), dim3(tiles), dim3(kThreads), 0,
                       st, a);
  else if (dgrad && stats && a.bnb.mode <= 1 && a.addend == nullptr)
    hipLaunchKernelGGL((conv_fwd_k<T, BM, BN, true, true, NB, 0, true>), dim3(tiles), dim3(kThreads), 0, st, a);
  else if (dgrad && stats)
    hipLaunchKernelGGL((conv_fwd_k<T, BM, BN, true, true, NB>), dim3(tiles), dim3(kThreads), 0, st, a);
  else if (dgrad)
    hipLaunchKernelGGL((conv_fwd_k<T, BM, BN, false, true, NB>), dim3(tiles), dim3(kThreads), 0, st, a);
  else if (stats && a.direct)
    hipLaunchKernelGGL((conv_fwd_k<T, BM, BN, true, false, NB, 0, false, true>), dim3(tiles), dim3(kThreads), 0, st,
                       a);
  else if (stats)
    hipLaunchKernelGGL((conv_fwd_k<T, BM, BN, true, false, NB>), dim3(tiles), dim3(kThreads), 0, st, a);
  else
    hipLaunchKernelGGL((conv_fwd_k<T, BM, BN, false, false, NB>), dim3(tiles), dim3(kThreads), 0, st, a);
  return hipGetLastError();
}

// Persistent launch (conv_persist.h) of the supported variants: grid = the resident capacity
// (occupancy query x CUs), tiles spread evenly, a multiple of 8 workgroups
int g_persist = 0;  // conv_set_persist

template <typename T, int BM, int BN, bool STATS, bool DGRAD, int NB, bool LEAN>
hipError_t launch_persist_k(const ConvArgs& a, int ntiles, hipStream_t st) {
  auto kern = conv_persist_k<T, BM, BN, STATS, DGRAD, NB, LEAN>;
  static int cap = 0;  // per instantiation: resident workgroups on the whole device
  if (cap == 0) {
    int occ = 0, dev = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, kThreads, 0) != hipSuccess || occ < 1) occ = 1;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 256;
    cap = occ * cus;
  }
  const int per = (ntiles + cap - 1) / cap;
  int nblk = (ntiles + per - 1) / per;
  nblk = (nblk + 7) / 8 * 8;  // tile blk + i * nblk stays on its plain-launch XCD
  hipLaunchKernelGGL(kern, dim3(nblk), dim3(kThreads), 0, st, a, nblk);
  return hipGetLastError();
}

template <typename T, int BM, int BN, int NB>
hipError_t launch_persist_nb(const ConvArgs& a, bool stats, bool dgrad, hipStream_t st) {
  const int ntiles = ((a.M + BM - 1) / BM) * ((a.K + BN - 1) / BN) * (a.sd == 2 ? 4 : 1);
  if (dgrad && stats && a.bnb.mode <= 1 && a.addend == nullptr)
    return launch_persist_k<T, BM, BN, true, true, NB, true>(a, ntiles, st);
  if (dgrad && stats) return launch_persist_k<T, BM, BN, true, true, NB, false>(a, ntiles, st);
  if (dgrad) return launch_persist_k<T, BM, BN, false, true, NB, false>(a, ntiles, st);
  if (stats) return launch_persist_k<T, BM, BN, true, false, NB, false>(a, ntiles, st);
  return hipErrorNotSupported;
}

int g_stages = 0;  // 0 = automatic (conv_set_stages, for tuning sweeps)
int g_xf_dbg = 0;  // conv_set_xf_debug (diagnostics only)
unsigned long long* g_stamps = nullptr;  // diagnostic timeline buffer (conv_set_stamps)

template <typename T, int BM, int BN>
hipError_t launch(const ConvArgs& a, bool stats, bool dgrad, hipStream_t st) {
  // 2 stages: the deeper rings (3/4, counted vmcnt across raw barriers) measured no better on any
  // ResNet-50 layer or Llama projection (profiles/conv_r01, profiles/llama_r01) — at 2-5
  // workgroups per CU the other workgroups already hide the glds latency (guide: "regime-gated")
  const int nb = a.nb > 0 ? a.nb : (g_stages > 0 ? g_stages : 2);
  if (nb == 1) return launch_nb<T, BM, BN, 1>(a, stats, dgrad, st);
  if (nb == 2) return launch_nb<T, BM, BN, 2>(a, stats, dgrad, st);
  if (nb == 3) return launch_nb<T, BM, BN, 3>(a, stats, dgrad, st);
  return launch_nb<T, BM, BN, 4>(a, stats, dgrad, st);
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

// Tile order: ids run M-fastest inside groups of `group` M-tiles, and each XCD takes a contiguous
// 1/8 of the ids, so an XCD's L2 holds ~group A-slices and ~(tiles/8)/group filter slices.  A
// filter slice is R*S*BN/BM times an activation slice; the footprint group*a + (T/8/group)*b is
// smallest at group = sqrt(T*b / (8a)).  (ResNet layer4 3x3: 200 tiles -> group 15; the old fixed
// 8 made every XCD stream all 4.7 MB of filter through a 4 MB L2.)
int g_group_mode = 0;  // conv_set_group (A/B sweeps): 0 the model below, > 0 fixed, -1 x2, -2 x0.5

int conv_fwd_group(int M, int K, int RS, int bm, int bn) {
  const int tm = (M + bm - 1) / bm, tn = (K + bn - 1) / bn;
  double g = sqrt((double)tm * tn * RS * bn / (8.0 * bm));
  if (g_group_mode > 0) g = g_group_mode;
  else if (g_group_mode == -1) g *= 2.0;
  else if (g_group_mode == -2) g *= 0.5;
  return max(1, min(tm, (int)(g + 0.5)));
}

void conv_set_group(int mode) { g_group_mode = mode; }

void conv_set_stamps(void* buf) { g_stamps = static_cast<unsigned long long*>(buf); }

void conv_set_stages(int nb) { g_stages = (nb >= 1 && nb <= 4) ? nb : 0; }

void conv_set_persist(int on) { g_persist = on; }

void conv_set_xf_debug(int bits) { g_xf_dbg = bits & 7; }

// Below ~2 workgroups per CU a conv runs latency-bound on its long reduction (ResNet-50 layer4
// 3x3: 200 tiles x 72 K-steps, 55 us).  Split the reduction until ~768 workgroups run, keeping
// >= 6 K-steps per split.  The reduce launch costs ~5 us, so at 300-480 tiles only long
// reductions split (MI355X, bench profile: layer3 3x3 (392 tiles, 36 steps) 31 -> 23 + 5 us;
// layer3 1x1 (392 tiles, 16 steps) 18 -> 16 + 5 us, a loss).
int conv_fwd_splits(int M, int K, int nk, int bm, int bn) {
  const int tiles = ((M + bm - 1) / bm) * ((K + bn - 1) / bn);
  if (tiles >= 480 || (tiles >= 300 && nk < 32)) return 1;
  int sp = (768 + tiles - 1) / tiles;
  sp = min(sp, nk / 6);
  return max(1, sp);
}

hipError_t conv_fwd(int dtype, const void* in, const void* w, void* out, const void* zero, double* psum, double* psq,
                    int N, int H, int W, int C, int K, int P, int Q, int R, int S, int sh, int sw, int ph, int pw,
                    int bm, int bn, int dgrad, int splits, float* part, hipStream_t st, float alpha,
                    const SplitkEpilogue* ep, const void* addend, const BnBwdEpilogue* bnb, int pix, int dgrad_stride,
                    int Hx, int Wx, int nb, const ConvInXform* xf, const DualWgrad* dual) {
  if (!conv_fwd_supported(C, K) || dtype == kF32) return hipErrorInvalidValue;
  if (dual != nullptr && !dgrad) return hipErrorInvalidValue;
  if (dgrad && (psum != nullptr || sh != 1 || sw != 1)) return hipErrorInvalidValue;
  const bool sd2 = dgrad_stride == 2;
  if (sd2 && (!dgrad || Hx != 2 * P || Wx != 2 * Q || alpha != 1.f || ep != nullptr)) return hipErrorInvalidValue;
  if (dgrad_stride != 1 && !sd2) return hipErrorInvalidValue;
  if (splits > 1 && part == nullptr) return hipErrorInvalidValue;
  if (addend != nullptr && ((splits > 1 && bnb == nullptr) || psum != nullptr)) return hipErrorInvalidValue;
  if (bnb != nullptr && (!dgrad || bnb->sums == nullptr || bnb->x == nullptr || (bnb->mode == 2 && bnb->y == nullptr) ||
                         (bnb->mode == 1 && (bnb->mean == nullptr || bnb->invstd == nullptr)) || alpha != 1.f ||
                         (ep != nullptr && ep->U != nullptr)))
    return hipErrorInvalidValue;
  // alpha / the rank-r epilogue live in the split-K reduce
  if ((alpha != 1.f || (ep != nullptr && ep->U != nullptr)) && splits < 2) return hipErrorInvalidValue;
  const bool aff = ep != nullptr && ep->scale != nullptr;
  if (aff && (ep->shift == nullptr || ep->U != nullptr || dgrad || psum != nullptr || addend != nullptr || alpha != 1.f))
    return hipErrorInvalidValue;
  const int64_t M64 = (int64_t)N * P * Q;
  if (M64 <= 0 || M64 > INT32_MAX) return hipErrorInvalidValue;
  if (xf != nullptr &&
      (dgrad || C > kXfMaxC || pix > 0 || xf->sums == nullptr || xf->save_mean == nullptr || xf->save_invstd == nullptr ||
       addend != nullptr || aff || alpha != 1.f || ep != nullptr || (int64_t)N * H * W < 2 ||
       (xf->out != nullptr && (sh != 1 || sw != 1 || P != H || Q != W || 2 * ph != R - 1 || 2 * pw != S - 1))))
    return hipErrorInvalidValue;
  ConvArgs a{static_cast<const uint16_t*>(in), static_cast<const uint16_t*>(w), static_cast<uint16_t*>(out),
             static_cast<const uint16_t*>(zero), psum, psq, N, H, W, C, K, P, Q, R, S, sh, sw, ph, pw, (int)M64};
  a.group = conv_fwd_group(a.M, K, R * S, bm, bn);
  a.kvalid = K;
  a.stamps = g_stamps;
  a.pix = pix > 0 ? pix : C;
  a.sd = sd2 ? 2 : 1;
  {
    auto magic36 = [](int d) -> uint64_t { return ((1ull << 36) + (uint64_t)d - 1) / (uint64_t)d; };
    const bool exact = M64 < (1 << 22) && (int64_t)P * Q < (1 << 14);
    a.mq = exact ? magic36(Q) : 0;
    a.mpq = exact ? magic36(P * Q) : 0;
  }
  // nb: LDS ring depth 1..4 (0 = automatic); + 16: the DIRECT store epilogue (forward + statistics)
  a.direct = (nb & 16) && psum != nullptr && !dgrad && addend == nullptr && !aff && xf == nullptr ? 1 : 0;
  a.xf_on = xf != nullptr ? 1 : 0;
  a.xf_dbg = g_xf_dbg;
  a.xf_out = nullptr;
  if (xf != nullptr) {
    const double Mi = (double)N * H * W;  // the producer's rows (this conv's input pixels)
    a.xfin = FwdFin{xf->sums, xf->weight, xf->bias, xf->running_mean, xf->running_var, xf->momentum, xf->eps,
                    xf->save_mean, xf->save_invstd, 1.0 / Mi, Mi / (Mi - 1.0)};
    a.xf_out = static_cast<uint16_t*>(xf->out);
  }
  nb &= 15;
  a.nb = (nb >= 1 && nb <= 4) ? nb : 0;
  a.Hx = Hx;
  a.Wx = Wx;
  if (pix > 0 && (dgrad || pix % 8 != 0)) return hipErrorInvalidValue;
  const int nk = R * S * (C / kBK);
  splits = max(1, min(splits, nk));
  a.steps_per_split = (nk + splits - 1) / splits;
  a.splits = (nk + a.steps_per_split - 1) / a.steps_per_split;  // no empty splits
  if (sd2) {  // one launch over the 4 output phases (the grid's "splits" are the phases), no split-K
    a.steps_per_split = nk;
    a.splits = 4;
  }
  a.part = part;
  a.addend = static_cast<const uint16_t*>(addend);
  if (bnb != nullptr) a.bnb = *bnb;
  a.aff_scale = aff ? ep->scale : nullptr;
  a.aff_shift = aff ? ep->shift : nullptr;
  a.aff_act = aff ? ep->act : 0;
  if (aff && a.splits == 1) a.addend = static_cast<const uint16_t*>(ep->residual);
  // the weight gradient riding on this data gradient: in the same launch when conv_dual.hip has the
  // combination, else launched right after (the split-K data gradient, f16, other tiles)
  auto wgrad_after = [&]() -> hipError_t {
    if (dual == nullptr) return hipSuccess;
    return conv_wgrad(dtype, dual->dy, dual->x, dual->dw, dual->partials, zero, dual->N, dual->H, dual->W, dual->C,
                      dual->K, dual->P, dual->Q, dual->R, dual->S, dual->sh, dual->sw, dual->ph, dual->pw, dual->bm,
                      dual->bn,
                      dual->splits, dual->steps_per_split, st, 1.f, dual->pending, dual->defer_reduce);
  };
  if (a.splits > 1 && !sd2) {
    hipError_t e;
    if (dtype == kBF16) {
      if (bm == 128 && bn == 128) e = launch<bf16_t, 128, 128>(a, false, dgrad, st);
      else if (bm == 128 && bn == 64) e = launch<bf16_t, 128, 64>(a, false, dgrad, st);
      else e = launch<bf16_t, 64, 64>(a, false, dgrad, st);
    } else {
      if (bm == 128 && bn == 128) e = launch<f16_t, 128, 128>(a, false, dgrad, st);
      else if (bm == 128 && bn == 64) e = launch<f16_t, 128, 64>(a, false, dgrad, st);
      else e = launch<f16_t, 64, 64>(a, false, dgrad, st);
    }
    if (e != hipSuccess) return e;
    if (bnb != nullptr) {
      e = splitk_reduce_bnb(dtype, part, out, addend, a.M, K, a.splits, *bnb, st);
      return e != hipSuccess ? e : wgrad_after();
    }
    if (psum != nullptr) {  // BN statistics from the reduce (atomics per kStatRows-row block)
      if (alpha != 1.f || (ep != nullptr && ep->U != nullptr)) return hipErrorInvalidValue;
      return splitk_reduce_stats(dtype, part, out, a.M, K, a.splits, psum, psq, st);
    }
    e = splitk_reduce(dtype, part, out, (int64_t)a.M * K, a.splits, st, alpha, ep);
    return e != hipSuccess ? e : wgrad_after();
  }
  const bool stats = (psum != nullptr && psq != nullptr) || bnb != nullptr;
  // persistent launch: bf16, no split-K / XF / DIRECT / affine epilogue; forward only with BN
  // statistics (no addend); every data-gradient variant (also the stride-2 phase split)
  const bool persist_ok = g_persist && dual == nullptr && dtype == kBF16 && xf == nullptr && !a.direct && !aff &&
                          ep == nullptr && (dgrad || (stats && addend == nullptr)) && a.splits == (a.sd == 2 ? 4 : 1);
  if (persist_ok) {
    const int nbv = a.nb > 0 ? a.nb : (g_stages > 0 ? g_stages : 2);
    hipError_t e = hipErrorNotSupported;
    if (nbv >= 1 && nbv <= 3) {
      auto go = [&](auto nbc) -> hipError_t {
        constexpr int NBv = decltype(nbc)::value;
        if (bm == 128 && bn == 128) return launch_persist_nb<bf16_t, 128, 128, NBv>(a, stats, dgrad, st);
        if (bm == 128 && bn == 64) return launch_persist_nb<bf16_t, 128, 64, NBv>(a, stats, dgrad, st);
        if (bm == 64 && bn == 64) return launch_persist_nb<bf16_t, 64, 64, NBv>(a, stats, dgrad, st);
        return hipErrorNotSupported;  // other tiles: the plain launch
      };
      e = nbv == 1 ? go(std::integral_constant<int, 1>{})
                   : (nbv == 2 ? go(std::integral_constant<int, 2>{}) : go(std::integral_constant<int, 3>{}));
    }
    if (e != hipErrorNotSupported) return e;
  }
  if (dual != nullptr) {
    // launch_nb's variant choice for a data gradient: LEAN BN-backward (mode 0/1, no addend), full
    // BN-backward, plain
    const int variant = !stats ? 0 : (a.bnb.mode <= 1 && a.addend == nullptr ? 1 : 2);
    const int nbv = a.nb > 0 ? a.nb : (g_stages > 0 ? g_stages : 2);
    const hipError_t e = conv_dual_launch(a, dtype, bm, bn, nbv, variant, *dual, st);
    if (e != hipErrorNotSupported) return e;
    hipError_t e1;
    if (dtype == kBF16) {
      if (bm == 128 && bn == 128) e1 = launch<bf16_t, 128, 128>(a, stats, dgrad, st);
      else if (bm == 128 && bn == 64) e1 = launch<bf16_t, 128, 64>(a, stats, dgrad, st);
      else e1 = launch<bf16_t, 64, 64>(a, stats, dgrad, st);
    } else {
      if (bm == 128 && bn == 128) e1 = launch<f16_t, 128, 128>(a, stats, dgrad, st);
      else if (bm == 128 && bn == 64) e1 = launch<f16_t, 128, 64>(a, stats, dgrad, st);
      else e1 = launch<f16_t, 64, 64>(a, stats, dgrad, st);
    }
    return e1 != hipSuccess ? e1 : wgrad_after();
  }
  if (dtype == kBF16) {
    if (bm == 128 && bn == 128) return launch<bf16_t, 128, 128>(a, stats, dgrad, st);
    if (bm == 128 && bn == 64) return launch<bf16_t, 128, 64>(a, stats, dgrad, st);
    return launch<bf16_t, 64, 64>(a, stats, dgrad, st);
  }
  if (bm == 128 && bn == 128) return launch<f16_t, 128, 128>(a, stats, dgrad, st);
  if (bm == 128 && bn == 64) return launch<f16_t, 128, 64>(a, stats, dgrad, st);
  return launch<f16_t, 64, 64>(a, stats, dgrad, st);
}

// Fused linear + cross-entropy GEMM passes (ops/cross_entropy.py): z = x[M, E] · w[classes]ᵀ (+ b)
// on the MFMA implicit-GEMM kernel (R = S = 1), 128 x bn tiles, classes [col_off, col_off + kvalid)
// of the vocabulary (w points at row col_off; kcols = kvalid rounded up to 8 for mode 2's store).
//   mode 1: ce.part [ceil(kcols / bn), M] (row max, row Σexp) + ce.zt — the logits never stored;
//   mode 2: out [M, kcols] = dz of those classes (the softmax gradient, ready for the dX / dW GEMMs).
hipError_t linear_ce(int dtype, int mode, const void* x, const void* w, void* out, const void* zero, int M, int E,
                     int kcols, int kvalid, const CeEpilogue& ce, hipStream_t st, int bn) {
  if (E % kBK != 0 || kcols % 8 != 0 || kvalid > kcols || kvalid < 1 || M < 1 || (mode != 1 && mode != 2) ||
      (dtype != kBF16 && dtype != kF16) || (bn != 64 && bn != 128))
    return hipErrorInvalidValue;
  if (mode == 1 && (ce.part == nullptr || ce.zt == nullptr)) return hipErrorInvalidValue;
  if (mode == 2 && (out == nullptr || ce.lse == nullptr || ce.scale == nullptr)) return hipErrorInvalidValue;
  ConvArgs a{static_cast<const uint16_t*>(x), static_cast<const uint16_t*>(w), static_cast<uint16_t*>(out),
             static_cast<const uint16_t*>(zero), nullptr, nullptr, M, 1, 1, E, kcols, 1, 1, 1, 1, 1, 1, 0, 0, M};
  constexpr int BM = 128;
  a.group = conv_fwd_group(M, kcols, 1, BM, bn);
  a.kvalid = kvalid;
  a.pix = E;
  a.splits = 1;
  a.steps_per_split = E / kBK;
  a.ce = ce;
  const int tiles = ((M + BM - 1) / BM) * ((kcols + bn - 1) / bn);
#define HYP_CE_LAUNCH(TT, BNV, MODE) \
  hipLaunchKernelGGL((conv_fwd_k<TT, BM, BNV, false, false, 2, MODE>), dim3(tiles), dim3(kThreads), 0, st, a)
  if (dtype == kBF16) {
    if (bn == 128) {
      if (mode == 1) HYP_CE_LAUNCH(bf16_t, 128, 1);
      else HYP_CE_LAUNCH(bf16_t, 128, 2);
    } else {
      if (mode == 1) HYP_CE_LAUNCH(bf16_t, 64, 1);
      else HYP_CE_LAUNCH(bf16_t, 64, 2);
    }
  } else {
    if (bn == 128) {
      if (mode == 1) HYP_CE_LAUNCH(f16_t, 128, 1);
      else HYP_CE_LAUNCH(f16_t, 128, 2);
    } else {
      if (mode == 1) HYP_CE_LAUNCH(f16_t, 64, 1);
      else HYP_CE_LAUNCH(f16_t, 64, 2);
    }
  }
#undef HYP_CE_LAUNCH
  return hipGetLastError();
}

}  // namespace hyp

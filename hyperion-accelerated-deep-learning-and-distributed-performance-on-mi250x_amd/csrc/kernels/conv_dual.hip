// A convolution's data gradient and weight gradient in ONE launch (horizontal fusion).
//
// Reference: the ResNet backward ran MIOpen's bwd-data and bwd-weights solvers as separate kernels
// on one stream (SURVEY §2.4 "Convolution + BatchNorm + ReLU", §2.5 ResNet rows).  In the Hyperion
// ResNet-50 step both are latency-bound launches of 10-35 us at 1-4 workgroups per CU (per
// workgroup ~2-3 us of first loads, ~1-3 us of epilogue around a short K loop), and the ~50 weight
// gradients sit on the critical path: skipping them takes the step from 4.79 to 3.81 ms
// (profiles/r05/dual_ab.txt).  Nothing in the backward reads a weight gradient, so
// dW = Xᵀ·dY of a layer can run in the SAME grid as dX = dY ⊛ Wᵀ of that layer — one launch fewer
// per layer, no ramp / tail of a second kernel, and the two gradients' workgroups fill each
// other's latency (a data-gradient tile waiting on its epilogue loads beside a weight-gradient
// tile streaming its K loop).  A side stream was measured instead and lost (5.25 ms: the graph's
// cross-queue dependencies, profiles/r05/dual_ab.txt).
//
// Grid layout: workgroups are taken in 8-wide groups (the hardware deals workgroup ids round-robin
// over the 8 XCDs, so a group is one workgroup per XCD); a group belongs to the data gradient or to
// the weight gradient in Bresenham proportion (order 0) or data-gradient groups first (order 1),
// and a kind's local id keeps local % 8 == hardware id % 8 — each gradient's own XCD-aware tile
// order (mfl::xcd_remap) sees exactly the id sequence of its plain launch.  Past the groups run the
// pending split-K reduce workgroups of an EARLIER weight gradient (conv_wgrad.hip), as in a plain
// weight-gradient launch.
//
// Instantiated for bf16 with every data-gradient tile / LDS depth / epilogue variant the conv plans
// use and a 64 x 64 weight-gradient tile (dense 1x1: the lean kernel, 2 x 64-pixel stages; strided /
// 3x3: the general kernel, 2 stages); the fused kernel's registers and LDS are the larger of the
// two bodies'.  (The plain launch's 3 x 128-pixel ring for long dense reductions takes 96 KiB of
// LDS: one workgroup per CU for BOTH kinds here, so the fused launch keeps 2 x 64.)
#include "conv_fwd_impl.h"
#include "conv_wgrad_impl.h"

namespace hyp {
namespace {

struct DualMap {
  int nd, nw;  // data- / weight-gradient workgroups
  int gd, gw;  // 8-wide groups of each (the last one of a kind may be partial: its extra ids exit)
  int np;      // pending-reduce workgroups after the 8 * (gd + gw) group ids
  int order;   // 0 interleaved, 1 data gradient first
};

// kind 0 data gradient, 1 weight gradient, 2 pending reduce; local id within the kind
__device__ __forceinline__ void dual_decode(const DualMap& m, int b, int& kind, int& local) {
  const int G = m.gd + m.gw, g = b >> 3, l8 = b & 7;
  if (g >= G) {
    kind = 2;
    local = b - 8 * G;
    return;
  }
  if (m.order == 1) {
    kind = g < m.gd ? 0 : 1;
    local = 8 * (g < m.gd ? g : g - m.gd) + l8;
    return;
  }
  // data-gradient groups among groups [0, g) and [0, g]: floor(g * gd / G), floor((g + 1) * gd / G)
  const int d0 = (int)(((int64_t)g * m.gd) / G), d1 = (int)(((int64_t)(g + 1) * m.gd) / G);
  kind = d1 > d0 ? 0 : 1;
  local = 8 * (d1 > d0 ? d0 : g - d0) + l8;
}

constexpr int cmax(int a, int b) { return a > b ? a : b; }

// VARIANT 0: plain data gradient; 1: BN-backward epilogue LEAN; 2: BN-backward epilogue full.
// WK 0: dense 1x1 weight gradient (64-pixel stages, NB 2); 1: general weight gradient (strided /
// RxS, NB 2).
template <int BM, int BN, int NB, int VARIANT, int WK>
__global__ __launch_bounds__(kThreads) void conv_dual_k(const ConvArgs da, const WgradArgs wa, const DualMap mp) {
  using T = bf16_t;
  constexpr int kDg = conv_fwd_smem<BM, BN, NB>() * 2;
  constexpr int kWg = WK == 0 ? wgrad_dense_smem_bytes<64, 64, 2, 64>() : wgrad_smem_bytes<64, 64, 2>();
  constexpr int kPr = 3 * 64 * 16;  // pending_reduce_block's f32x4 [3][64]
  __shared__ __attribute__((aligned(16))) uint16_t smem[cmax(cmax(kDg, kWg), kPr) / 2];
  int kind, local;
  dual_decode(mp, blockIdx.x, kind, local);
  if (kind == 0) {
    if (local < mp.nd) conv_fwd_body<T, BM, BN, VARIANT != 0, true, NB, 0, VARIANT == 1>(da, local, smem);
  } else if (kind == 1) {
    if (local < mp.nw) {
      if constexpr (WK == 0) conv_wgrad_dense_body<T, 64, 64, 2, 64>(wa, local, smem);
      else conv_wgrad_body<T, 64, 64, 2, false>(wa, local, smem);
    }
  } else {
    pending_reduce_block(wa.pr, local, mp.np, reinterpret_cast<f32x4*>(smem));
  }
}

template <int BM, int BN, int NB, int VARIANT>
hipError_t launch_wk(const ConvArgs& a, const WgradArgs& w, const DualMap& mp, int wk, hipStream_t st) {
  const dim3 grid(8 * (mp.gd + mp.gw) + mp.np);
  if (wk == 0) hipLaunchKernelGGL((conv_dual_k<BM, BN, NB, VARIANT, 0>), grid, dim3(kThreads), 0, st, a, w, mp);
  else hipLaunchKernelGGL((conv_dual_k<BM, BN, NB, VARIANT, 1>), grid, dim3(kThreads), 0, st, a, w, mp);
  return hipGetLastError();
}

template <int BM, int BN, int NB>
hipError_t launch_var(const ConvArgs& a, const WgradArgs& w, const DualMap& mp, int variant, int wk, hipStream_t st) {
  if (variant == 0) return launch_wk<BM, BN, NB, 0>(a, w, mp, wk, st);
  if (variant == 1) return launch_wk<BM, BN, NB, 1>(a, w, mp, wk, st);
  return launch_wk<BM, BN, NB, 2>(a, w, mp, wk, st);
}

template <int BM, int BN>
hipError_t launch_nb(const ConvArgs& a, const WgradArgs& w, const DualMap& mp, int nb, int variant, int wk,
                     hipStream_t st) {
  if (nb == 1) return launch_var<BM, BN, 1>(a, w, mp, variant, wk, st);
  if (nb == 2) return launch_var<BM, BN, 2>(a, w, mp, variant, wk, st);
  if (nb == 3) return launch_var<BM, BN, 3>(a, w, mp, variant, wk, st);
  return hipErrorNotSupported;
}

int g_dual_order = -1;  // conv_dual_set_order (A/B): -1 = the DualWgrad's own

}  // namespace

void conv_dual_set_order(int order) { g_dual_order = order; }

hipError_t conv_dual_launch(const ConvArgs& a, int dtype, int bm, int bn, int nb, int variant, const DualWgrad& d,
                            hipStream_t st) {
  if (dtype != kBF16 || nb < 1 || nb > 3 || variant < 0 || variant > 2) return hipErrorNotSupported;
  if (!((bm == 64 && bn == 64) || (bm == 128 && bn == 64) || (bm == 128 && bn == 128))) return hipErrorNotSupported;
  if (a.splits != 1 && a.sd != 2) return hipErrorNotSupported;  // split-K data gradients need their reduce first
  if (d.bm != 64 || d.bn != 64) return hipErrorNotSupported;
  WgradArgs w;
  hipError_t e = conv_wgrad_prepare(&w, dtype, d, a.zero);
  if (e != hipSuccess) return e;
  const bool dense = d.R == 1 && d.S == 1 && d.sh == 1 && d.sw == 1 && d.ph == 0 && d.pw == 0;
  const int wk = dense ? 0 : 1;
  DualMap mp;
  mp.nd = ((a.M + bm - 1) / bm) * ((a.K + bn - 1) / bn) * a.splits;  // (sd2: the 4 phases)
  mp.nw = w.nwg_main;
  mp.gd = (mp.nd + 7) / 8;
  mp.gw = (mp.nw + 7) / 8;
  mp.np = w.pr.part != nullptr ? w.pr.blocks : 0;
  mp.order = g_dual_order >= 0 ? g_dual_order : d.order;
  if (bm == 64) e = launch_nb<64, 64>(a, w, mp, nb, variant, wk, st);
  else if (bn == 64) e = launch_nb<128, 64>(a, w, mp, nb, variant, wk, st);
  else e = launch_nb<128, 128>(a, w, mp, nb, variant, wk, st);
  if (e != hipSuccess || d.splits == 1 || d.defer_reduce) return e;
  return splitk_reduce(dtype, d.partials, d.dw, (int64_t)d.K * d.R * d.S * d.C, d.splits, st, 1.f);
}

}  // namespace hyp

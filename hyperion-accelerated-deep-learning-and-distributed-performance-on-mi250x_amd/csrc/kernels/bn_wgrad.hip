// A layer's BatchNorm-backward dx pass and the weight gradient of the conv above it in ONE launch.
//
// Reference: MIOpen's batch-norm backward and bwd-weights solvers ran as separate kernels on one
// stream (SURVEY §2.4 "Convolution + BatchNorm + ReLU", §2.5 ResNet rows).  In the Hyperion
// ResNet-50 backward each layer is  data gradient (dz + the BN reduce in its epilogue) ->
// BN dx pass (dC = A·dz + B·x + C) -> the next data gradient, a chain of latency-bound launches,
// and the weight gradients (~1 ms of a 4.8 ms step, profiles/r05/dual_ab.txt) do not feed it.
// The weight gradient of conv j reads dC_j and x_j, both ready once the BN dx pass of layer j has
// run — so it can share the launch of the NEXT BN dx pass (layer j-1's), whose memory-bound
// workgroups (a few us of streaming) then run beside the weight gradient's long K loops instead of
// as a separate latency-bound launch between two data gradients; the data gradients themselves
// keep their own tuned kernels and occupancy (conv_dual.hip fused them with the weight gradient
// instead: both are slot-bound, so that pairing hid ~0.1 ms; this one hides the dx passes).
//
// Grid: [BN dx blocks (row block x channel chunk, flattened), padded to a multiple of 8]
//       [weight-gradient tiles: ids keep hardware % 8 == local % 8, so its XCD-aware tile order
//        is that of a plain launch] [pending split-K reduce of an earlier weight gradient].
// Every workgroup of a launch takes the kernel's LDS and registers, BN dx blocks included, so the
// weight gradient runs lean rings only: 2 x 64-pixel stages (dense 1x1) or the general kernel's 2
// stages, tiles 64 x 64 / 128 x 64 / 64 x 128 (35-52 KiB of LDS: 3-4 workgroups per CU; the plain
// launch's 3 x 128-pixel ring or a 128 x 128 tile would leave the BN blocks 1-2 per CU).
#include "bn_bwd_impl.h"
#include "conv_wgrad_impl.h"

namespace hyp {
namespace {

struct BnDxArgs {
  const uint16_t* dz;
  const uint16_t* x;
  uint16_t* dx;
  BwdFin fin;
  int64_t M;
  int C, tpr, rpi;
  int64_t rpb;
  int P, nb, nbp;  // BN row blocks (grid.x of a plain launch), BN blocks (P * gy), padded to 8
  int np;          // pending-reduce workgroups
};

constexpr int cmax(int a, int b) { return a > b ? a : b; }

// WK 0: dense, NB x 64-pixel stages; 1: general (NB stages)
template <int BM, int BN, int NB, int WK>
constexpr int wk_smem() {
  return WK == 0 ? wgrad_dense_smem_bytes<BM, BN, NB, 64>() : wgrad_smem_bytes<BM, BN, NB>();
}

template <int BM, int BN, int NB, int WK>
__global__ __launch_bounds__(kThreads) void bn_dx_wgrad_k(const BnDxArgs b, const WgradArgs w) {
  using T = bf16_t;
  __shared__ __attribute__((aligned(16))) uint16_t smem[cmax(wk_smem<BM, BN, NB, WK>(), 3 * 64 * 16) / 2];
  const int blk = blockIdx.x;
  if (blk < b.nbp) {
    if (blk < b.nb) {
      const int by = blk / b.P, bx = blk - by * b.P;
      bn_bwd_dx_body<T, false, false, false>(reinterpret_cast<const T*>(b.dz), reinterpret_cast<const T*>(b.x),
                                             nullptr, reinterpret_cast<T*>(b.dx), nullptr, b.fin, b.M, b.C, b.tpr,
                                             b.rpi, b.rpb, nullptr, bx, by);
    }
    return;
  }
  const int local = blk - b.nbp;
  if (local < w.nwg_main) {
    if constexpr (WK == 0) conv_wgrad_dense_body<T, BM, BN, NB, 64>(w, local, smem);
    else conv_wgrad_body<T, BM, BN, NB, false>(w, local, smem);
  } else {
    pending_reduce_block(w.pr, local - w.nwg_main, b.np, reinterpret_cast<f32x4*>(smem));
  }
}

template <int BM, int BN>
hipError_t launch_tile(const BnDxArgs& b, const WgradArgs& w, bool dense, hipStream_t st) {
  const dim3 grid(b.nbp + w.nwg_main + b.np);
  if (dense) hipLaunchKernelGGL((bn_dx_wgrad_k<BM, BN, 2, 0>), grid, dim3(kThreads), 0, st, b, w);
  else hipLaunchKernelGGL((bn_dx_wgrad_k<BM, BN, 2, 1>), grid, dim3(kThreads), 0, st, b, w);
  return hipGetLastError();
}

}  // namespace

hipError_t bn_backward_dx_wgrad(int dtype, const void* dz, const void* x, void* dx, int64_t M, int C,
                                const float* weight, const float* save_mean, const float* save_invstd, int training,
                                const double* sums, float* dweight, float* dbias, const DualWgrad& d,
                                const void* zero, hipStream_t stream) {
  if (dtype != kBF16) return hipErrorNotSupported;
  BnGeom ga;
  if (!apply_geom(M, C, ga)) return hipErrorInvalidValue;
  WgradArgs w;
  hipError_t e = conv_wgrad_prepare(&w, dtype, d, zero);
  if (e != hipSuccess) return e;
  BnDxArgs b;
  b.dz = static_cast<const uint16_t*>(dz);
  b.x = static_cast<const uint16_t*>(x);
  b.dx = static_cast<uint16_t*>(dx);
  b.fin = BwdFin{weight, save_mean, save_invstd, training, dweight, dbias, sums, 1.0 / (double)M};
  b.M = M, b.C = C, b.tpr = ga.tpr, b.rpi = ga.rpi, b.rpb = ga.rows_per_block;
  b.P = ga.P;
  b.nb = ga.P * ga.gy;
  b.nbp = (b.nb + 7) / 8 * 8;
  b.np = w.pr.part != nullptr ? w.pr.blocks : 0;
  const bool dense = d.R == 1 && d.S == 1 && d.sh == 1 && d.sw == 1 && d.ph == 0 && d.pw == 0;
  if (d.bm == 64 && d.bn == 64) e = launch_tile<64, 64>(b, w, dense, stream);
  else if (d.bm == 128 && d.bn == 64) e = launch_tile<128, 64>(b, w, dense, stream);
  else if (d.bm == 64 && d.bn == 128) e = launch_tile<64, 128>(b, w, dense, stream);
  else return hipErrorNotSupported;  // (128 x 128: the caller picks a narrower tile)
  if (e != hipSuccess || d.splits == 1 || d.defer_reduce) return e;
  return splitk_reduce(dtype, d.partials, d.dw, (int64_t)d.K * d.R * d.S * d.C, d.splits, stream, 1.f);
}

}  // namespace hyp

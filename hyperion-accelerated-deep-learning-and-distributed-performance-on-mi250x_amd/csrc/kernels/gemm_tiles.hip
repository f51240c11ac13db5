// Classic deep-pipelined tiles (gemm_tile_k) and the host side of the tiled GEMM: planner,
// split-K, dispatch.  Kernels and their documentation: gemm_tiles_impl.h.
#include <mutex>

#include "kernels/gemm_tiles_impl.h"

namespace hyp {
namespace gt {

template <typename T, typename OutT>
hipError_t launch_tile(const GemmP& p, bool atr, bool btr, int tile, int nwg, hipStream_t st) {
  switch (tile) {
    case 0: return launch_layout<T, OutT, 256, 256, 2, 4, false, 4>(p, atr, btr, nwg, st);
    case 1: return launch_layout<T, OutT, 256, 128, 4, 2, false, 4>(p, atr, btr, nwg, st);
    case 2: return launch_layout<T, OutT, 128, 128, 2, 2, false, 4>(p, atr, btr, nwg, st);
    case 4: return launch_layout<T, OutT, 64, 64, 2, 1, false, 4>(p, atr, btr, nwg, st);
    case 5: return launch_layout<T, OutT, 128, 64, 2, 1, false, 4>(p, atr, btr, nwg, st);
    case 6: return launch_layout<T, OutT, 64, 128, 2, 2, false, 4>(p, atr, btr, nwg, st);
    case 7: return launch_layout<T, OutT, 192, 128, 2, 2, false, 4>(p, atr, btr, nwg, st);
    default: return launch_layout<T, OutT, 128, 128, 2, 2, true, 4>(p, atr, btr, nwg, st);
  }
}

// Split-K arrival counters: one hipMalloc'd, zeroed pool per device (the last arriver of a tile
// resets its counter, so a range is reusable by the next launch in stream order).  Eager launches
// cycle through the first kEagerRing counters (a range is reused only ~kEagerRing / tiles
// launches later); launches under hipGraph capture take never-reused ranges after it (the graph
// replays them), and fall back to the separate reduce kernel when that region is exhausted or
// the pool does not exist yet (no hipMalloc inside a capture).
constexpr int64_t kEagerRing = 1 << 20, kCntTotal = 1 << 22;
struct CntPool {
  unsigned* base = nullptr;
  int64_t eager_next = 0, cap_next = kEagerRing;
};
std::mutex g_cnt_mu;
CntPool g_cnt[64];

unsigned* splitk_counters(int ntiles, hipStream_t st) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64 || ntiles <= 0 || ntiles > kEagerRing / 8) return nullptr;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(g_cnt_mu);
  CntPool& c = g_cnt[dev];
  if (c.base == nullptr) {
    if (cs != hipStreamCaptureStatusNone) return nullptr;
    void* b = nullptr;
    if (hipMalloc(&b, kCntTotal * sizeof(unsigned)) != hipSuccess) return nullptr;
    if (hipMemset(b, 0, kCntTotal * sizeof(unsigned)) != hipSuccess) return nullptr;
    c.base = static_cast<unsigned*>(b);
  }
  if (cs == hipStreamCaptureStatusNone) {
    if (c.eager_next + ntiles > kEagerRing) c.eager_next = 0;
    unsigned* r = c.base + c.eager_next;
    c.eager_next += ntiles;
    return r;
  }
  if (c.cap_next + ntiles > kCntTotal) return nullptr;
  unsigned* r = c.base + c.cap_next;
  c.cap_next += ntiles;
  return r;
}

int g_splitk_inkernel = 0;  // gemm_set_splitk_inkernel (A/B; off: measured slower, profiles/r05/splitk_last_arriver_ab.txt)

}  // namespace gt

using namespace gt;

void gemm_set_splitk_inkernel(int on) { g_splitk_inkernel = on; }

void gemm_tiled_plan(int M, int N, int K, int* tile, int* splits) { gemm_tiled_plan_layout(M, N, K, false, false, tile, splits); }

// the fast kernels stage a ragged last slice per lane (zero page past K; gemm_tiled has already
// checked the K % 8 != 0 rule); the ping-pong kernel also needs a whole number of KS-slice steps
bool fast_k(int tile, int K) {
  const int ks = kTiles[tile].ks > 0 ? kTiles[tile].ks : 1;
  return ((K + kBK - 1) / kBK) % ks == 0;
}

// slices per split-K slice for `tile` (a multiple of the ping-pong step) and the resulting split count
void split_plan(int tile, int K, int splits_req, int* per_out, int* splits_out) {
  const int nk = (K + kBK - 1) / kBK;
  const int ks = tile >= 0 && tile < kNumTiles && kTiles[tile].ks > 0 ? kTiles[tile].ks : 1;
  int per = (nk + splits_req - 1) / splits_req;
  per = (per + ks - 1) / ks * ks;
  *per_out = per;
  *splits_out = (nk + per - 1) / per;  // no empty slices
}

void gemm_tiled_plan_layout(int M, int N, int K, bool a_tr, bool b_tr, int* tile, int* splits) {
  const int cus = 256;
  double best = 1e30;
  int bt = 2, bs = 1;
  for (int t = 0; t < kNumTiles; ++t) {
    if (t == 3 || !tile_layout_ok(t, a_tr, b_tr) || M < kTiles[t].bm || N < kTiles[t].bn) continue;
    const TileCfg& c = kTiles[t];
    if (!fast_k(t, K)) continue;
    const int64_t tiles = (int64_t)((M + c.bm - 1) / c.bm) * ((N + c.bn - 1) / c.bn);
    for (int s = 1; s <= 16; ++s) {
      int per, sp;
      split_plan(t, K, s, &per, &sp);
      if (sp != s) continue;
      if (s > 1 && per < 8) break;  // >= 256-deep slices
      const int64_t wgs = tiles * s;
      const int64_t rounds = (wgs + (int64_t)cus * c.occ - 1) / ((int64_t)cus * c.occ);
      // time ~ rounds x one tile-slice (per-CU MFMA work / efficiency), in 256x256x32-step units
      double est = (double)rounds * ((double)c.bm * c.bn / (256.0 * 256.0)) * (per + 6) / (c.eff * c.occ);
      if (s > 1) est += 4.0 + (double)M * N * 4.0 * (s + 1) / (cus * 64.0 * 1024.0);  // slab traffic + launch
      if (est < best * 0.97) {
        best = est;
        bt = t;
        bs = s;
      }
    }
  }
  *tile = bt;
  *splits = bs;
}

hipError_t gemm_tiled(const GemmTiledArgs& a, hipStream_t st) {
  if (a.in_dtype == kF32 || a.K <= 0 || a.M <= 0 || a.N <= 0) return hipErrorInvalidValue;
  if (a.N % 4 != 0 || a.lda % 8 != 0 || a.ldb % 8 != 0) return hipErrorInvalidValue;
  // K % 8 != 0: the SAFE kernel reads a row-form operand in 8-element chunks past K (its row
  // stride must cover them and the caller keeps those pad elements finite) and a transposed
  // operand's rows past K as zeros — so at most one operand may be row-form
  const int k8 = (a.K + 7) / 8 * 8;
  if (a.K % 8 != 0 && ((!a.a_tr && !a.b_tr) || (!a.a_tr && a.lda < k8) || (!a.b_tr && a.ldb < k8)))
    return hipErrorInvalidValue;
  const int nb = a.b_rows > 0 ? a.b_rows : a.N;
  if (nb > a.N || (nb < a.N && a.b_tr)) return hipErrorInvalidValue;
  if ((a.a_tr && a.M % 8 != 0) || (a.b_tr && a.N % 8 != 0)) return hipErrorInvalidValue;
  // per-lane staging offsets are 32-bit byte offsets from the per-piece base (< 16 rows apart)
  if ((int64_t)a.lda * 64 >= ((int64_t)1 << 31) || (int64_t)a.ldb * 64 >= ((int64_t)1 << 31)) return hipErrorInvalidValue;
  int tile = a.tile, splits = a.splits;
  if (tile < 0 || splits < 1) {
    int t, s;
    gemm_tiled_plan_layout(a.M, a.N, a.K, a.a_tr, a.b_tr, &t, &s);
    if (tile < 0) tile = t;
    if (splits < 1) splits = s;
  }
  if (tile >= kNumTiles) return hipErrorInvalidValue;
  if (!tile_layout_ok(tile, a.a_tr, a.b_tr)) return hipErrorInvalidValue;
  if (tile != 3) {  // the fast (unclamped) kernels: see gemm_tile_k's SAFE
    const TileCfg& f = kTiles[tile];
    const bool ragged = a.M % f.bm != 0 || a.N % f.bn != 0;
    const bool fast = a.M >= f.bm && a.N >= f.bn && fast_k(tile, a.K) && nb == a.N &&
                      !(ragged && (a.beta != 0.f || (a.R != nullptr && a.R == a.C)));
    if (!fast) tile = 3;
  }
  int per;
  split_plan(tile, a.K, splits, &per, &splits);
  if (splits > 1 && a.part == nullptr) return hipErrorInvalidValue;
  GemmP p;
  p.A = static_cast<const uint16_t*>(a.A);
  p.B = static_cast<const uint16_t*>(a.B);
  p.zero = static_cast<const uint16_t*>(a.zero);
  p.part = splits > 1 ? a.part : nullptr;
  p.cnt = nullptr;
  p.e = Epi{a.C, a.aux, a.bias, a.R, a.alpha, a.beta, a.ldc, a.ldr, a.act, a.bias_dtype, 0u, 0.f, a.drng};
  if (a.drop_p > 0.f) {
    if (a.act == 0 || a.R != nullptr || a.drop_p >= 1.f) return hipErrorInvalidValue;
    p.e.dthr = (uint32_t)fminf(a.drop_p * 4294967296.f, 4294967295.f);  // dropout.hip's threshold
    p.e.dscale = 1.f / (1.f - a.drop_p);
  }
  p.M = a.M;
  p.N = a.N;
  p.K = a.K;
  p.lda = a.lda;
  p.ldb = a.ldb;
  p.nb = nb;
  p.kper = per * kBK;
  p.splits = splits;
  p.a_ext = a.a_tr ? (int64_t)(a.K - 1) * a.lda + a.M : (int64_t)(a.M - 1) * a.lda + k8;
  p.b_ext = a.b_tr ? (int64_t)(a.K - 1) * a.ldb + a.N : (int64_t)(nb - 1) * a.ldb + k8;
  const TileCfg& c = kTiles[tile];
  const int ntiles = ((a.M + c.bm - 1) / c.bm) * ((a.N + c.bn - 1) / c.bn);
  const int nwg = ntiles * splits;
  if (splits > 1 && g_splitk_inkernel && c.ks == 0) p.cnt = splitk_counters(ntiles, st);
  hipError_t err;
  if (c.ks > 0) {
    err = launch_pp_tile(a.in_dtype, a.out_dtype, p, a.a_tr, a.b_tr, tile, nwg, st);
  } else if (a.in_dtype == kBF16) {
    HYP_DISPATCH_FLOAT(a.out_dtype, TO, { err = launch_tile<bf16_t, TO>(p, a.a_tr, a.b_tr, tile, nwg, st); });
  } else {
    HYP_DISPATCH_FLOAT(a.out_dtype, TO, { err = launch_tile<f16_t, TO>(p, a.a_tr, a.b_tr, tile, nwg, st); });
  }
  if (err != hipSuccess || splits == 1 || p.cnt != nullptr) return err;
  const int64_t n4 = (int64_t)a.M * a.N / 4;
  const int blocks = (int)std::min<int64_t>((n4 + 255) / 256, 2048);
  HYP_DISPATCH_FLOAT(a.out_dtype, TO, {
    hipLaunchKernelGGL((gemm_splitk_epi_k<TO>), dim3(blocks), dim3(256), 0, st, a.part, p.e, a.M, a.N, splits);
  });
  return hipGetLastError();
}

int gemm_tiled_splits(const GemmTiledArgs& a) {
  int tile = a.tile, splits = a.splits;
  if (tile < 0 || splits < 1) {
    int t, s;
    gemm_tiled_plan_layout(a.M, a.N, a.K, a.a_tr, a.b_tr, &t, &s);
    if (tile < 0) tile = t;
    if (splits < 1) splits = s;
  }
  if (tile >= 0 && tile < kNumTiles && tile != 3) {  // mirror gemm_tiled's fast-path fallback
    const TileCfg& f = kTiles[tile];
    const int nb = a.b_rows > 0 ? a.b_rows : a.N;
    if (!(a.M >= f.bm && a.N >= f.bn && fast_k(tile, a.K) && nb == a.N)) tile = 3;
  }
  int per, sp;
  split_plan(tile, a.K, splits, &per, &sp);
  return sp;
}

}  // namespace hyp

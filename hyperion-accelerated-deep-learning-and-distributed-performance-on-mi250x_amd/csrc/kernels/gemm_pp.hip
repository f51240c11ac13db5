// Ping-pong MFMA GEMM tiles (gemm_pp_k, documented in gemm_tiles_impl.h): their own translation
// unit so the classic tiles and these compile in parallel.
#include "kernels/gemm_tiles_impl.h"

namespace hyp {
namespace gt {

template <typename T, typename OutT>
hipError_t launch_pp_typed(const GemmP& p, bool atr, bool btr, int tile, int nwg, hipStream_t st) {
  switch (tile) {
    // R (last template argument): LDS-DMA pieces per slice issued from the MFMA interval (measured:
    // profiles/r06/gemm_pp_refill_split*.jsonl — 256²: R 3 of 4; 256x128 / 128x256: R 2 of 3)
    case 8: return launch_pp<T, OutT, 256, 256, 1, 4, 1, 4, 3>(p, atr, btr, nwg, st);
    case 9: return launch_pp<T, OutT, 256, 128, 2, 2, 2, 6, 2>(p, atr, btr, nwg, st);
    case 10: return launch_pp<T, OutT, 128, 256, 1, 4, 2, 6, 2>(p, atr, btr, nwg, st);
    case 11: return launch_pp<T, OutT, 128, 128, 2, 2, 2, 6, 1>(p, atr, btr, nwg, st);
    case 12: return launch_pp<T, OutT, 256, 256, 1, 4, 1, 5, 3>(p, atr, btr, nwg, st);  // all 160 KiB: 5-deep ring
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_pp_tile(int in_dtype, int out_dtype, const GemmP& p, bool atr, bool btr, int tile, int nwg,
                          hipStream_t st) {
  hipError_t err = hipErrorInvalidValue;
  if (in_dtype == kBF16) {
    HYP_DISPATCH_FLOAT(out_dtype, TO, { err = launch_pp_typed<bf16_t, TO>(p, atr, btr, tile, nwg, st); });
  } else {
    HYP_DISPATCH_FLOAT(out_dtype, TO, { err = launch_pp_typed<f16_t, TO>(p, atr, btr, tile, nwg, st); });
  }
  return err;
}

}  // namespace gt
}  // namespace hyp

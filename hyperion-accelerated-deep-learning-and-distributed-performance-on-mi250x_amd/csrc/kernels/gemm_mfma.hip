// LDS-tiled MFMA GEMM for gfx950:  C[M, N] = A[M, K] · B[N, K]ᵀ  (bf16 / f16 in, f32 accumulate).
//
// Replaces the reference's `torch.matmul` microbenchmark path (hipBLASLt/rocBLAS behind
// `01_hardware_exploration.ipynb:208-242`, SURVEY C3 / §2.4 "GEMM") with a hand-written CDNA4
// kernel, and is the GEMM building block for the fused ops.
//
// Structure (cdna_hip_programming.md §5 "canonical CDNA GEMM", the 128²-tile 2-barrier form):
//  * 128 x 128 output tile per 256-thread workgroup (4 waves as 2 x 2, 64 x 64 per wave =
//    4 x 4 accumulators of v_mfma_f32_16x16x32_{bf16,f16});
//  * K staged through LDS in BK-deep slices, double-buffered, with global_load_lds_dwordx4
//    (16 B per lane straight into LDS, no VGPR round trip): the load of slice t+1 is issued
//    before the MFMAs of slice t;
//  * LDS rows are 128 B (64 elements); the 16-byte chunk index is XOR-swizzled with
//    (row >> 1) & 7 so the 16 lanes of a ds_read_b128 fragment read (16 consecutive rows, one
//    logical chunk) hit 16 distinct bank groups.  global_load_lds writes LDS lane-linearly, so the
//    swizzle is applied to the per-lane GLOBAL source address and undone on the read (rule 21);
//  * XCD-aware workgroup remap (T1): consecutive tile ids land on the same XCD (own L2), and tiles
//    are walked in GROUP_M-row super-rows so neighbouring workgroups share A and B panels.
// Requirements (checked on the host): M % 128 == 0, N % 128 == 0, K % BK == 0, 16-byte aligned
// rows (lda, ldb multiples of 8).
#include "hyp_common.h"
#include "hyp_kernels.h"

namespace hyp {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));

constexpr int kBM = 128, kBN = 128, kThreads = 256, kGroupM = 8;

template <typename T>
__device__ __forceinline__ f32x4 mfma16(u16x8 a, u16x8 b, f32x4 c);
template <>
__device__ __forceinline__ f32x4 mfma16<bf16_t>(u16x8 a, u16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                 0, 0);
}
template <>
__device__ __forceinline__ f32x4 mfma16<f16_t>(u16x8 a, u16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0,
                                                0);
}

__device__ __forceinline__ int swz(int row) { return (row >> 1) & 7; }

// Stage a [128 rows x BK] slice of a K-contiguous matrix into LDS (rows of BK elements; BK = 64
// -> 128 B rows, 8 chunks).  Every wave instruction covers 8 rows (64 lanes x 16 B).
template <int BK>
__device__ __forceinline__ void stage(const uint16_t* __restrict__ g, int ld, int row0, int k0, uint16_t* lds,
                                      int wave, int lane) {
  constexpr int kChunks = BK / 8;          // 16-byte chunks per row
  constexpr int kRowsPerInstr = 64 / kChunks;
  constexpr int kInstr = kBM / kRowsPerInstr / 4;  // per wave (4 waves)
#pragma unroll
  for (int i = 0; i < kInstr; ++i) {
    const int r0 = (i * 4 + wave) * kRowsPerInstr;
    const int row = r0 + lane / kChunks;
    const int slot = lane % kChunks;
    const int chunk = slot ^ (swz(row) & (kChunks - 1));
    const uint16_t* src = g + (int64_t)(row0 + row) * ld + k0 + chunk * 8;
    __builtin_amdgcn_global_load_lds((const void*)src,
                                     (void __attribute__((address_space(3)))*)(lds + r0 * BK), 16, 0, 0);
  }
}

template <int BK>
__device__ __forceinline__ u16x8 frag(const uint16_t* lds, int row, int chunk) {
  constexpr int kChunks = BK / 8;
  const int slot = chunk ^ (swz(row) & (kChunks - 1));
  return *reinterpret_cast<const u16x8*>(lds + row * BK + slot * 8);
}

template <typename T, typename OutT, int BK>
__global__ __launch_bounds__(kThreads) void gemm_nt_k(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B,
                                                      OutT* __restrict__ C, int M, int N, int K, int lda, int ldb,
                                                      int ldc, float alpha) {
  __shared__ __attribute__((aligned(16))) uint16_t smem[2 * 2 * kBM * BK];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  // ---- XCD-aware remap + grouped tile order
  const int tiles_m = M / kBM, tiles_n = N / kBN, nwg = tiles_m * tiles_n;
  int bid = blockIdx.x;
  {
    const int q = nwg / 8, r = nwg % 8, xcd = bid % 8, idx = bid / 8;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
  }
  const int group = kGroupM * tiles_n;
  const int gid = bid / group, first_m = gid * kGroupM;
  const int gsize = min(tiles_m - first_m, kGroupM);
  const int tm = first_m + (bid % group) % gsize;
  const int tn = (bid % group) / gsize;
  const int m0 = tm * kBM, n0 = tn * kBN;

  // buffer b: A slice at smem + b * 2*kBM*BK, B slice right after it
  constexpr int kBuf = 2 * kBM * BK;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / BK;
  stage<BK>(A, lda, m0, 0, smem, wave, lane);
  stage<BK>(B, ldb, n0, 0, smem + kBM * BK, wave, lane);
  __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0) lgkmcnt(0): slice 0 landed
  __syncthreads();

  const int r16 = lane & 15, c4 = lane >> 4;
  for (int t = 0; t < nk; ++t) {
    const int cur = t & 1;
    if (t + 1 < nk) {
      uint16_t* nb = smem + (cur ^ 1) * kBuf;
      stage<BK>(A, lda, m0, (t + 1) * BK, nb, wave, lane);
      stage<BK>(B, ldb, n0, (t + 1) * BK, nb + kBM * BK, wave, lane);
    }
    const uint16_t* as = smem + cur * kBuf;
    const uint16_t* bs = as + kBM * BK;
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      u16x8 a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = frag<BK>(as, wm * 64 + i * 16 + r16, ks * 4 + c4);
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = frag<BK>(bs, wn * 64 + j * 16 + r16, ks * 4 + c4);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16<T>(a[i], b[j], acc[i][j]);
    }
    __builtin_amdgcn_s_waitcnt(0);  // next slice's LDS-DMA complete (this wave)
    __syncthreads();                // ... for every wave; also: everyone done reading `cur`
  }

  // ---- epilogue: acc[i][j][e] = C[m0 + wm*64 + i*16 + (lane>>4)*4 + e][n0 + wn*64 + j*16 + (lane&15)]
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = m0 + wm * 64 + i * 16 + c4 * 4 + e;
        const int col = n0 + wn * 64 + j * 16 + r16;
        st1<OutT>(C + (int64_t)row * ldc + col, acc[i][j][e] * alpha);
      }
}

}  // namespace

bool gemm_nt_supported(int M, int N, int K, int lda, int ldb, int bk) {
  return M % kBM == 0 && N % kBN == 0 && (bk == 32 || bk == 64) && K % bk == 0 && lda % 8 == 0 && ldb % 8 == 0 &&
         M > 0 && N > 0 && K > 0;
}

hipError_t gemm_nt(int in_dtype, int out_dtype, const void* A, const void* B, void* C, int M, int N, int K, int lda,
                   int ldb, int ldc, float alpha, int bk, hipStream_t st) {
  if (!gemm_nt_supported(M, N, K, lda, ldb, bk) || in_dtype == kF32) return hipErrorInvalidValue;
  const dim3 grid((M / kBM) * (N / kBN)), block(kThreads);
  const uint16_t* a = static_cast<const uint16_t*>(A);
  const uint16_t* b = static_cast<const uint16_t*>(B);
#define HYP_GEMM_LAUNCH(TI, BKV)                                                                                 \
  HYP_DISPATCH_FLOAT(out_dtype, TO, {                                                                            \
    hipLaunchKernelGGL((gemm_nt_k<TI, TO, BKV>), grid, block, 0, st, a, b, static_cast<TO*>(C), M, N, K, lda, ldb, \
                       ldc, alpha);                                                                              \
  })
  if (in_dtype == kBF16) {
    if (bk == 64) HYP_GEMM_LAUNCH(bf16_t, 64) else HYP_GEMM_LAUNCH(bf16_t, 32)
  } else {
    if (bk == 64) HYP_GEMM_LAUNCH(f16_t, 64) else HYP_GEMM_LAUNCH(f16_t, 32)
  }
#undef HYP_GEMM_LAUNCH
  return hipGetLastError();
}

}  // namespace hyp

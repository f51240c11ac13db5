// FP32 GEMM on the gfx950 fp32-input matrix cores:  C[M, N] = alpha · A[M, K] · B[N, K]ᵀ.
//
// Reference: the fp32 rows of the matmul precision sweep (`torch.matmul` of fp32 N x N operands,
// `Phase 1/01_hardware_exploration.ipynb:208-242`, SURVEY C3 / §2.4 "GEMM": "fp32 via fp32 MFMA").
// gfx950 has no xf32 (TF32-like) MFMA, but it does have exact fp32-in / fp32-accumulate MFMA at the
// fp32 VALU peak (cdna_hip_programming.md §3 "FP32-input MFMA"): v_mfma_f32_32x32x2_f32, 64 cycles
// per instruction, one float of A and of B per lane.  The result is a k-ordered fma chain — the
// same numerics as a scalar fp32 GEMM.
//
// Structure: the 128²-tile, 2-barrier form of gemm_mfma.hip with fp32 operands —
//  * 256-thread workgroup = 4 waves as 2 x 2, each wave 64 x 64 = 2 x 2 blocks of 32 x 32
//    (16 accumulator registers per block);
//  * K staged through LDS in 32-deep slices (128-byte rows: 8 chunks of 4 floats), double-buffered,
//    with global_load_lds_dwordx4 straight into LDS; the chunk index is XOR-swizzled with
//    (row >> 1) & 7 (applied to the per-lane global source, undone on the read);
//  * per 4-wide k chunk a lane reads ONE ds_read_b64 per operand block: lane (row, half h) gets
//    k = 4c + 2h, 4c + 2h + 1 and feeds the two MFMA k-steps with .x and .y — the same k
//    permutation on A and B, so the products pair up (reduction order is free), with a 2-way
//    bank conflict at most (64 lanes over all 64 banks);
//  * XCD-aware remap + grouped tile order (T1).
// Requirements (host-checked): M % 128 == 0, N % 128 == 0, K % 32 == 0, 16-byte aligned rows.
#include "hyp_common.h"
#include "hyp_kernels.h"

namespace hyp {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int kBM = 128, kBN = 128, kBK = 32, kThreads = 256, kGroupM = 8;

__device__ __forceinline__ int swz(int row) { return (row >> 1) & 7; }

// [128 rows][32 floats] slice of a K-contiguous fp32 matrix -> LDS (8 chunks of 16 B per row;
// one wave instruction = 8 rows)
__device__ __forceinline__ void stage(const float* __restrict__ g, int ld, int row0, int k0, float* lds, int wave,
                                      int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r0 = (i * 4 + wave) * 8;
    const int row = r0 + (lane >> 3);
    const int chunk = (lane & 7) ^ swz(row);
    const float* src = g + (int64_t)(row0 + row) * ld + k0 + chunk * 4;
    __builtin_amdgcn_global_load_lds((const void*)src, (void __attribute__((address_space(3)))*)(lds + r0 * kBK), 16,
                                     0, 0);
  }
}

// lane (row, h): floats k = 4c + 2h, 4c + 2h + 1 of `row`
__device__ __forceinline__ f32x2 frag(const float* lds, int row, int c, int h) {
  return *reinterpret_cast<const f32x2*>(lds + row * kBK + ((c ^ swz(row)) << 2) + 2 * h);
}

template <typename OutT>
__global__ __launch_bounds__(kThreads) void gemm_f32_nt_k(const float* __restrict__ A, const float* __restrict__ B,
                                                          OutT* __restrict__ C, int M, int N, int K, int lda, int ldb,
                                                          int ldc, float alpha) {
  __shared__ __attribute__((aligned(16))) float smem[2 * 2 * kBM * kBK];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  const int tiles_m = M / kBM, tiles_n = N / kBN, nwg = tiles_m * tiles_n;
  int bid = blockIdx.x;
  {
    const int q = nwg / 8, r = nwg % 8, xcd = bid % 8, idx = bid / 8;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
  }
  const int group = kGroupM * tiles_n;
  const int first_m = (bid / group) * kGroupM;
  const int gsize = min(tiles_m - first_m, kGroupM);
  const int tm = first_m + (bid % group) % gsize;
  const int tn = (bid % group) / gsize;
  const int m0 = tm * kBM, n0 = tn * kBN;
  constexpr int kBuf = 2 * kBM * kBK;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[i][j][v] = 0.f;

  const int nk = K / kBK;
  stage(A, lda, m0, 0, smem, wave, lane);
  stage(B, ldb, n0, 0, smem + kBM * kBK, wave, lane);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();

  const int r32 = lane & 31, h = lane >> 5;
  for (int t = 0; t < nk; ++t) {
    const int cur = t & 1;
    if (t + 1 < nk) {
      float* nb = smem + (cur ^ 1) * kBuf;
      stage(A, lda, m0, (t + 1) * kBK, nb, wave, lane);
      stage(B, ldb, n0, (t + 1) * kBK, nb + kBM * kBK, wave, lane);
    }
    const float* as = smem + cur * kBuf;
    const float* bs = as + kBM * kBK;
#pragma unroll
    for (int c = 0; c < kBK / 4; ++c) {
      f32x2 a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = frag(as, wm * 64 + i * 32 + r32, c, h);
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = frag(bs, wn * 64 + j * 32 + r32, c, h);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].x, b[j].x, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].y, b[j].y, acc[i][j], 0, 0, 0);
        }
    }
    __builtin_amdgcn_s_waitcnt(0);  // next slice's LDS-DMA (this wave)
    __syncthreads();                // ... every wave's; everyone done with `cur`
  }

  // acc[i][j][v] = C[m0 + wm*64 + i*32 + 8 (v / 4) + 4 h + (v % 4)][n0 + wn*64 + j*32 + r32]
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int row = m0 + wm * 64 + i * 32 + 8 * (v >> 2) + 4 * h + (v & 3);
        const int col = n0 + wn * 64 + j * 32 + r32;
        st1<OutT>(C + (int64_t)row * ldc + col, acc[i][j][v] * alpha);
      }
}

}  // namespace

bool gemm_f32_nt_supported(int M, int N, int K, int lda, int ldb) {
  return M > 0 && N > 0 && K > 0 && M % kBM == 0 && N % kBN == 0 && K % kBK == 0 && lda % 4 == 0 && ldb % 4 == 0;
}

hipError_t gemm_f32_nt(int out_dtype, const float* A, const float* B, void* C, int M, int N, int K, int lda, int ldb,
                       int ldc, float alpha, hipStream_t st) {
  if (!gemm_f32_nt_supported(M, N, K, lda, ldb)) return hipErrorInvalidValue;
  const dim3 grid((M / kBM) * (N / kBN)), block(kThreads);
  HYP_DISPATCH_FLOAT(out_dtype, TO, {
    hipLaunchKernelGGL((gemm_f32_nt_k<TO>), grid, block, 0, st, A, B, static_cast<TO*>(C), M, N, K, lda, ldb, ldc,
                       alpha);
  })
  return hipGetLastError();
}

}  // namespace hyp

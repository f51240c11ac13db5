#pragma once
// Deep-pipelined MFMA GEMM for gfx950 with fused epilogues — the transformer training GEMM.
//
//   C[M, N] = epi( alpha · Σ_k A(m, k) · B(n, k) )
//
// Each operand is either K-contiguous ("row" form: X(i, k) at X + i·ld + k — nn.Linear weights,
// activations in the forward) or MN-contiguous ("tr" form: X(i, k) at X + k·ld + i — the weight in
// a data gradient, both operands of a weight gradient).  One kernel covers forward (NT), data
// gradient (NN) and weight gradient (TN) of every linear layer without transposed copies.
//
// Replaces the reference's hipBLASLt/rocBLAS GEMMs behind nn.Linear / TransformerEncoderLayer /
// ViT MLP (SURVEY §2.4 "GEMM", C3/C5/C14/C15; reference `distributed_utils.py:75-88`), with the
// bias / GELU / ReLU / residual / accumulate epilogues fused into the store.
//
// Structure (cdna_hip_programming.md §5):
//  * 256x256 (8 waves as 2x4, 128x64 per wave), 256x128 (8 waves as 4x2) or 128x128 (4 waves as
//    2x2) output tiles; 16x16x32 bf16/f16 MFMA; per wave FM x FN accumulators;
//  * K staged in 32-deep slices through an NB = 4 LDS ring filled by global_load_lds_dwordx4
//    (LDS-DMA, no VGPR round trip): stages t+1, t+2 stay in flight across the barrier that
//    publishes stage t (counted vmcnt, raw s_barrier — never vmcnt(0) in the loop);
//  * row-form images [rows][32] (64-byte rows) with the 16-byte chunk XOR-swizzled by
//    ((row>>2)&1)<<1: conflict-free for ds_read_b128's lane groups; tr-form images
//    [32 k-rows][128 cols] read with ds_read_b64_tr_b16 (guide T10), their rows permuted by
//    tr_row_to_k so both forms deliver reduction index 8g+e in element e of lane group g;
//    the swizzles are applied to the per-lane GLOBAL source address (glds writes lane-linearly);
//  * XCD-aware workgroup order (T1) with GROUP_M super-rows; split-K slices of a tile are
//    adjacent ids (same XCD) and write fp32 slabs reduced by gemm_splitk_epi_k;
//  * epilogue through a per-wave fp32 LDS patch (conflict-free padded rows) so every lane stores
//    4 consecutive outputs: alpha, beta·C_old, +bias[n], aux = pre-activation, ReLU/GELU,
//    +residual, rounding to the output dtype.
// Out-of-range rows/columns read clamped (discarded) or the zero page; the reduction tail reads
// the zero page, so any K % 8 == 0 works.
#include "hyp_common.h"
#include "hyp_kernels.h"
#include "mfma_lds.h"

namespace hyp {
namespace gt {  // shared by gemm_tiles.hip (classic tiles, host code) and gemm_pp.hip
using namespace mfl;

constexpr int kBK = 32;
// LDS ring depth: a template parameter (NBR) — 4 for the 2-workgroups-per-CU tiles, 6-8 for the
// deep-ring tiles that run one workgroup per CU and keep 5-7 stages in flight (the k-loop of the
// small transformer GEMMs is latency-bound: a 32-deep stage per ~latency / (NBR - 1))
constexpr int kGroupM = 8;

typedef int i32x4 __attribute__((ext_vector_type(4)));

// lgkmcnt(0) pinned between two scheduling fences: hipcc moves register-only MFMAs across an asm
// waitcnt (guide §5.4 rule 18) — without the leading fence it hoisted the wait above 15 of the 16
// MFMAs it was meant to overlap with the in-flight fragment reads.
__device__ __forceinline__ void lds_wait_fenced() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ u16x8 ds_read_b128_asm(unsigned addr) {
  i32x4 v;
  asm volatile("ds_read_b128 %0, %1" HYP_LDS_SYNC : "=v"(v) : "v"(addr) : "memory");
  return __builtin_bit_cast(u16x8, v);
}

// ---- staging ------------------------------------------------------------------------------------
// Each stage is kL LDS-DMA pieces per lane (one 1 KiB wave-instruction each), issued one at a time
// between MFMA groups.  Fast path: source = wave-uniform byte base (SGPRs) + ONE loop-invariant
// 32-bit lane offset per operand (the saddr form of global_load_lds; per-piece 64-bit lane
// pointers spilled the 256x256 kernel past its 256 VGPRs).  The stage holding the ragged end of the
// reduction and ragged tiles take the per-lane path (SAFE kernels: zero page past K, clamped rows /
// columns past M / N — discarded outputs).
//
// Row form: image [R rows][32]; piece i fills rows r0 .. r0+15 (4 lanes x 16 B per row).  The
// 16-byte chunk is XOR-swizzled by ((row >> 2) & 1) << 1: with ds_read_b128's lane groups
// ({0-3,12-15,20-27}, {4-11,16-19,28-31}, +32; MI355X_MICROARCH §LDS) every group of a fragment
// read then covers 16 distinct 16-byte bank slots (the (row >> 2) & 3 swizzle, designed for
// 16-consecutive-lane groups, was 2-way: 3.8 conflict cycles per LDS instruction in the PMC pass).
// For 16-aligned r0 it reduces to ((lane >> 4) & 1) << 1, so the lane offset
// (lane >> 2)·ld + chunk·8 is the same for every piece.
__device__ __forceinline__ unsigned row_lane(int ld, int lane) {
  return (unsigned)(((lane >> 2) * ld + ((lane & 3) ^ (((lane >> 4) & 1) << 1)) * 8) * 2);
}

template <int R, int NW, bool SAFE>
__device__ __forceinline__ void row_issue(const uint16_t* g, int ld, int row0, int nrows, unsigned lp, int i, int k0,
                                          int K, uint16_t* img, int wave, int lane, const uint16_t* zero, int64_t ext) {
  static_assert(R / (16 * NW) >= 1 && R % (16 * NW) == 0, "row image rows per wave instruction");
  const int r0 = (i * NW + wave) * 16;
  uint16_t* dst = img + r0 * kBK;
  if constexpr (!SAFE) {
    asm volatile("" : "+v"(lp));  // keep the add per stage (no hoisted per-piece lane pointers)
    const char* base = reinterpret_cast<const char*>(g + (int64_t)(row0 + r0) * ld + k0);
    HYP_DASSERT(reinterpret_cast<const uint16_t*>(base + lp) >= g && reinterpret_cast<const uint16_t*>(base + lp) + 8 <= g + ext);
    glds16(reinterpret_cast<const uint16_t*>(base + lp), dst);
  } else {
    // rows past the operand's end read the zero page: their outputs are either discarded (past
    // M / N) or, for a B operand with fewer rows than output columns (b_rows < N: the LM head's
    // padded class columns), exactly zero
    const int chunk = (lane & 3) ^ (((lane >> 4) & 1) << 1);
    const int gr = row0 + r0 + (lane >> 2);
    const int kk = k0 + chunk * 8;
    HYP_DASSERT(kk >= K || gr >= nrows || (g + (int64_t)gr * ld + kk + 8 <= g + ext));
    glds16(kk < K && gr < nrows ? g + (int64_t)gr * ld + kk : zero, dst);
  }
}

// Tr form: image = C/128 blocks of [32 k-rows][128 cols]; piece i fills image rows rr .. rr+3 of
// block blk (rr = 4·(ins & 7)); image row rho holds reduction index tr_row_to_k(rho), which is
// tr_row_to_k(rr) + (rho & 3) for these rows, and the chunk swizzle (rho & 7) << 1 depends on the
// lane and on rr & 4 = 4·(wave & 1) only: one lane offset per wave.
template <int NW>
__device__ __forceinline__ unsigned tr_lane_off(int ld, int wave, int lane) {
  const int x = lane >> 4, rho = ((wave & 1) << 2) + x;  // rr & 4 == (ins & 1) * 4 == (wave & 1) * 4 (NW even)
  static_assert(NW % 2 == 0, "tr staging assumes an even wave count");
  const int chunk = (lane & 15) ^ swz_tr<128>(rho);
  return (unsigned)((x * ld + chunk * 8) * 2);
}

template <int C, int NW, bool SAFE>
__device__ __forceinline__ void tr_issue(const uint16_t* g, int ld, int col0, int ncols, unsigned lp, int i, int k0,
                                         int K, uint16_t* img, int wave, int lane, const uint16_t* zero, int64_t ext) {
  static_assert((C / 128) * 8 / NW >= 1 && ((C / 128) * 8) % NW == 0, "tr image instructions per wave");
  const int ins = i * NW + wave, blk = ins >> 3, rr = (ins & 7) * 4;
  uint16_t* dst = img + blk * (kBK * 128) + rr * 128;
  if constexpr (!SAFE) {
    asm volatile("" : "+v"(lp));
    const char* base = reinterpret_cast<const char*>(g + (int64_t)(k0 + tr_row_to_k(rr)) * ld + col0 + blk * 128);
    HYP_DASSERT(reinterpret_cast<const uint16_t*>(base + lp) >= g && reinterpret_cast<const uint16_t*>(base + lp) + 8 <= g + ext);
    glds16(reinterpret_cast<const uint16_t*>(base + lp), dst);
  } else {
    const int rho = rr + (lane >> 4);
    const int chunk = (lane & 15) ^ swz_tr<128>(rho);
    const int k = k0 + tr_row_to_k(rho);
    const int c = min(col0 + blk * 128 + chunk * 8, ncols - 8);
    HYP_DASSERT(k >= K || (g + (int64_t)k * ld + c + 8 <= g + ext));
    glds16(k < K ? g + (int64_t)k * ld + c : zero, dst);
  }
}

// ---- fragment reads -----------------------------------------------------------------------------
// row form: rows ro + (lane & 15), chunk lane >> 4 (reduction 8g .. 8g+7)
__device__ __forceinline__ u16x8 frag_row(unsigned img_addr, int ro, int lane) {
  const int r16 = lane & 15, g = lane >> 4;
  const int row = ro + r16;
  const int slot = g ^ (((row >> 2) & 1) << 1);
  return ds_read_b128_asm(img_addr + (unsigned)((row * kBK + slot * 8) * 2));
}

// tr form: columns co + (lane & 15) of the [32][128]-block image — frag_tr<128> with the lane terms
// factored: row 4g+q and the half-row select give a fixed byte offset L, and for the even chunk
// index c = cb/8 of a 16-aligned column base, (c + (p>>1)) ^ swz(row) == c ^ Y with
// Y = swz(row) | (p>>1).  The second 16-row half is the +4 KiB immediate.  Y is made opaque per
// batch of reads so hipcc recomputes c ^ Y (2 VALU) instead of hoisting one VGPR per fragment.
struct TrLane {
  unsigned L, Y;
};
__device__ __forceinline__ TrLane tr_lane(int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int row = 4 * g + q;
  return TrLane{(unsigned)((row * 128 + ((p & 1) << 2)) * 2), (unsigned)(swz_tr<128>(row) | (p >> 1))};
}

__device__ __forceinline__ u16x8 frag_col(const uint16_t* img, int co, TrLane tl) {
  const unsigned base = lds_addr(img + (co >> 7) * (kBK * 128));
  const unsigned addr = base + tl.L + (((unsigned)((co & 127) >> 3) ^ tl.Y) << 4);
  const s16x4 v0 = ds_read_tr16_imm<0>(addr);
  const s16x4 v1 = ds_read_tr16_imm<16 * 128 * 2>(addr);
  u16x8 out;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    out[e] = (uint16_t)v0[e];
    out[4 + e] = (uint16_t)v1[e];
  }
  return out;
}

// ---- epilogue -----------------------------------------------------------------------------------
struct Epi {
  void* C;
  void* aux;         // pre-activation output (act != 0), output dtype
  const void* bias;  // [N], bias_dt
  const void* R;     // residual [M, N] (ldr), output dtype
  float alpha, beta;
  int ldc, ldr, act, bias_dt;
  uint32_t dthr;     // dropout on the activation output: keep iff rng_u32(key, row * ldc + col) >= dthr
  float dscale;      // 1 / (1 - p); 0 = no dropout
  RngState drs;
};

template <typename OutT>
__device__ __forceinline__ void ld4(const OutT* p, float (&v)[4]);
template <>
__device__ __forceinline__ void ld4<float>(const float* p, float (&v)[4]) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
}
template <>
__device__ __forceinline__ void ld4<bf16_t>(const bf16_t* p, float (&v)[4]) {
  const uint2 a = *reinterpret_cast<const uint2*>(p);
  v[0] = __uint_as_float(a.x << 16); v[1] = __uint_as_float(a.x & 0xffff0000u);
  v[2] = __uint_as_float(a.y << 16); v[3] = __uint_as_float(a.y & 0xffff0000u);
}
template <>
__device__ __forceinline__ void ld4<f16_t>(const f16_t* p, float (&v)[4]) {
  const uint2 a = *reinterpret_cast<const uint2*>(p);
  v[0] = f16_lo(a.x); v[1] = f16_hi(a.x); v[2] = f16_lo(a.y); v[3] = f16_hi(a.y);
}

template <typename OutT>
__device__ __forceinline__ void st4(OutT* p, const float (&v)[4]);
template <>
__device__ __forceinline__ void st4<float>(float* p, const float (&v)[4]) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
}
template <>
__device__ __forceinline__ void st4<bf16_t>(bf16_t* p, const float (&v)[4]) {
  *reinterpret_cast<uint2*>(p) = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
}
template <>
__device__ __forceinline__ void st4<f16_t>(f16_t* p, const float (&v)[4]) {
  *reinterpret_cast<uint2*>(p) = make_uint2(pack_f16x2(v[0], v[1]), pack_f16x2(v[2], v[3]));
}

__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_tanh(float x) {
  const float u = 0.7978845608028654f * (x + 0.044715f * x * x * x);
  return 0.5f * x * (1.f + tanhf(u));
}

// v: alpha-free accumulators of C[row, col .. col+3] (col % 4 == 0, row < M, col < N)
template <typename OutT>
__device__ __forceinline__ void epi4(const Epi& e, int row, int col, float (&v)[4]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) v[q] *= e.alpha;
  OutT* c = static_cast<OutT*>(e.C) + (int64_t)row * e.ldc + col;
  if (e.beta != 0.f) {
    float o[4];
    ld4<OutT>(c, o);
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] += e.beta * o[q];
  }
  if (e.bias != nullptr) {
    float b[4];
    if (e.bias_dt == kF32) ld4<float>(static_cast<const float*>(e.bias) + col, b);
    else if (e.bias_dt == kBF16) ld4<bf16_t>(static_cast<const bf16_t*>(e.bias) + col, b);
    else ld4<f16_t>(static_cast<const f16_t*>(e.bias) + col, b);
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] += b[q];
  }
  if (e.act != 0) {
    if (e.aux != nullptr) st4<OutT>(static_cast<OutT*>(e.aux) + (int64_t)row * e.ldc + col, v);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float x = rnd<OutT>(v[q]);  // the activation of the STORED pre-activation (aux)
      v[q] = e.act == 1 ? fmaxf(x, 0.f) : (e.act == 2 ? gelu_erf(x) : gelu_tanh(x));
    }
    if (e.dscale != 0.f) {  // dropout(act) as a separate dropout kernel over the stored act would compute it
      const uint64_t key = rng_key(e.drs);
#pragma unroll
      for (int q = 0; q < 4; ++q)
        v[q] = rng_u32(key, (uint64_t)((int64_t)row * e.ldc + col + q)) >= e.dthr ? rnd<OutT>(v[q]) * e.dscale : 0.f;
    }
  }
  if (e.R != nullptr) {
    float r[4];
    ld4<OutT>(static_cast<const OutT*>(e.R) + (int64_t)row * e.ldr + col, r);
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = rnd<OutT>(v[q]) + r[q];  // act(...) rounded, then + residual
  }
  st4<OutT>(c, v);
}

struct GemmP {
  const uint16_t* A;
  const uint16_t* B;
  const uint16_t* zero;
  float* part;  // split-K slabs [splits][M][N] fp32 (null: epilogue in-kernel)
  unsigned* cnt;  // split-K arrival counters, one per tile (null: gemm_splitk_epi_k reduces)
  Epi e;
  int M, N, K, lda, ldb, kper, splits;
  int nb;  // rows of a row-form B operand (N, or fewer: the SAFE kernel reads zeros past them)
  int64_t a_ext, b_ext;  // operand extents in elements from their bases (debug-build bounds checks)
};

// SAFE = false: every piece on the fast path — needs M >= BM, N >= BN, K % 32 == 0 (the last tile
// row / column is shifted back to end at M / N: overlapping tiles write identical values, so the
// host sends beta != 0 with ragged M / N to SAFE); SAFE = true: the per-lane path (ragged K, M < BM).
// vmcnt wait for "stage t landed" with `ahead` (<= A) later stages of L pieces each in flight
template <int L, int A>
__device__ __forceinline__ void wait_ahead_n(int ahead) {
  if constexpr (A == 0) {
    wait_vmcnt<0>();
  } else {
    if (ahead >= A) wait_vmcnt<A * L>();
    else wait_ahead_n<L, A - 1>(ahead);
  }
}

template <typename T, typename OutT, int BM, int BN, int WM, int WN, bool ATR, bool BTR, bool SAFE, int NBR>
__global__ __launch_bounds__(WM* WN * 64) void gemm_tile_k(const GemmP p) {
  constexpr int kNB = NBR;
  constexpr int NW = WM * WN;
  constexpr int FM = BM / WM / 16, FN = BN / WN / 16;
  static_assert(FN % 4 == 0, "wave tiles are 64-column multiples (epilogue patch)");
  constexpr int kA = BM * kBK, kB = BN * kBK, kStage = kA + kB;
  __shared__ __attribute__((aligned(16))) uint16_t smem[kNB * kStage];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: wave-derived bases stay in SGPRs
  const int wm = wave / WN, wn = wave % WN;

  // ---- tile / split decode: XCD remap, split slices adjacent, GROUP_M super-rows
  const int tiles_m = (p.M + BM - 1) / BM, tiles_n = (p.N + BN - 1) / BN;
  const int nwg = tiles_m * tiles_n * p.splits;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int tile = bid / p.splits, z = bid % p.splits;
  const int group = kGroupM * tiles_n;
  const int gid = tile / group, first_m = gid * kGroupM;
  const int gsize = min(tiles_m - first_m, kGroupM);
  const int tm = first_m + (tile % group) % gsize, tn = (tile % group) / gsize;
  const int m0 = SAFE ? tm * BM : min(tm * BM, p.M - BM), n0 = SAFE ? tn * BN : min(tn * BN, p.N - BN);
  const int kb = z * p.kper, ke = min(p.K, kb + p.kper);
  const int nk = (ke - kb + kBK - 1) / kBK;

  // glds per stage per lane (the counted-vmcnt unit): A pieces first, then B
  constexpr int kLA = ATR ? (BM / 128) * 8 / NW : BM / (16 * NW);
  constexpr int kLB = BTR ? (BN / 128) * 8 / NW : BN / (16 * NW);
  constexpr int kL = kLA + kLB;
  const unsigned lpA = ATR ? tr_lane_off<NW>(p.lda, wave, lane) : row_lane(p.lda, lane);
  const unsigned lpB = BTR ? tr_lane_off<NW>(p.ldb, wave, lane) : row_lane(p.ldb, lane);
  // a reduction that ends mid-slice (K % 32 != 0) stages its last slice on the per-lane path
  // (zero page past K) even in the fast kernel; every other slice takes the fast path
  const bool ragged_k = !SAFE && (ke - kb) % kBK != 0;
  auto stage_piece = [&](int t, int q) {
    uint16_t* sa = smem + (t % kNB) * kStage;
    uint16_t* sb = sa + kA;
    const int k0 = kb + t * kBK;
    if (ragged_k && t == nk - 1) {
      if (q < kLA) {
        if constexpr (ATR) tr_issue<BM, NW, true>(p.A, p.lda, m0, p.M, lpA, q, k0, ke, sa, wave, lane, p.zero, p.a_ext);
        else row_issue<BM, NW, true>(p.A, p.lda, m0, p.M, lpA, q, k0, ke, sa, wave, lane, p.zero, p.a_ext);
      } else {
        if constexpr (BTR) tr_issue<BN, NW, true>(p.B, p.ldb, n0, p.N, lpB, q - kLA, k0, ke, sb, wave, lane, p.zero, p.b_ext);
        else row_issue<BN, NW, true>(p.B, p.ldb, n0, p.nb, lpB, q - kLA, k0, ke, sb, wave, lane, p.zero, p.b_ext);
      }
      return;
    }
    if (q < kLA) {
      if constexpr (ATR) tr_issue<BM, NW, SAFE>(p.A, p.lda, m0, p.M, lpA, q, k0, ke, sa, wave, lane, p.zero, p.a_ext);
      else row_issue<BM, NW, SAFE>(p.A, p.lda, m0, p.M, lpA, q, k0, ke, sa, wave, lane, p.zero, p.a_ext);
    } else {
      if constexpr (BTR) tr_issue<BN, NW, SAFE>(p.B, p.ldb, n0, p.N, lpB, q - kLA, k0, ke, sb, wave, lane, p.zero, p.b_ext);
      else row_issue<BN, NW, SAFE>(p.B, p.ldb, n0, p.nb, lpB, q - kLA, k0, ke, sb, wave, lane, p.zero, p.b_ext);
    }
  };
  auto stage = [&](int t) {
#pragma unroll
    for (int q = 0; q < kL; ++q) stage_piece(t, q);
  };
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Software pipeline (two sub-phases per 32-deep stage; LDS fragment reads overlap the MFMAs):
  //   sub-phase 0: read A rows [FM/2, FM) of stage t   | MFMA A[0, FM/2) x B of stage t
  //   wait stage t+1 (counted vmcnt) + barrier; refill the buffer of stage t with stage t+NB
  //   sub-phase 1: read B and A rows [0, FM/2) of t+1  | MFMA A[FM/2, FM) x B of stage t
  // Every buffer's last read (sub-phase 0 of its own iteration) precedes the barrier after which
  // it is refilled; every read of stage t+1 follows the barrier that publishes it.
  constexpr int FH = FM / 2;
  const int am = wm * FM * 16, bn = wn * FN * 16;
  const TrLane trl = tr_lane(lane);
  auto opaque = [&]() {
    TrLane t2 = trl;
    asm volatile("" : "+v"(t2.Y));
    return t2;
  };
  auto read_b = [&](int t, u16x8 (&b)[FN]) {
    const uint16_t* sb = smem + (t % kNB) * kStage + kA;
    const TrLane tl = opaque();
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      if constexpr (BTR) b[j] = frag_col(sb, bn + j * 16, tl);
      else b[j] = frag_row(lds_addr(sb), bn + j * 16, lane);
    }
  };
  auto read_a = [&](int t, int half, u16x8 (&a)[FH]) {
    const uint16_t* sa = smem + (t % kNB) * kStage;
    const TrLane tl = opaque();
#pragma unroll
    for (int i = 0; i < FH; ++i) {
      if constexpr (ATR) a[i] = frag_col(sa, am + (half * FH + i) * 16, tl);
      else a[i] = frag_row(lds_addr(sa), am + (half * FH + i) * 16, lane);
    }
  };
  static_assert((kNB - 1) * kL < 64, "vmcnt is 6 bits");
  auto wait_ahead = [&](int ahead) { wait_ahead_n<kL, kNB - 1>(ahead); };  // this wave's glds of a stage landed

#pragma unroll
  for (int s = 0; s < kNB; ++s)
    if (s < nk) stage(s);
  u16x8 a0[FH], a1[FH], bc[FN];
  wait_ahead(min(kNB - 1, nk - 1));
  barrier_keep_vm();
  read_b(0, bc);
  read_a(0, 0, a0);
  lds_reads_done();

  auto mfma_half = [&](int half, const u16x8 (&a)[FH]) {
    __builtin_amdgcn_s_setprio(1);  // T5: the MFMA cluster wins issue arbitration over the partner wave's loads
#pragma unroll
    for (int i = 0; i < FH; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[half * FH + i][j] = mma16<T>(a[i], bc[j], acc[half * FH + i][j]);
    __builtin_amdgcn_s_setprio(0);
  };
  // steady state: stages 0 .. nk-2 (no MFMA under a branch: accumulators stay in place, no phi copies)
  for (int t = 0; t < nk - 1; ++t) {
    read_a(t, 1, a1);
    __builtin_amdgcn_sched_barrier(0);
    mfma_half(0, a0);
    lds_wait_fenced();
    wait_ahead(min(kNB - 2, nk - 2 - t));  // stage t+1 landed (this wave)
    barrier_keep_vm();                     // ... every wave; stage t fully read
    // sub-phase 1, interleaved in FH groups: refill stage t's buffer with stage t+NB (one LDS-DMA
    // piece at a time) between MFMA row groups — the MFMA pipe never waits on a burst of glds issue
    const bool refill = t + kNB < nk;
    constexpr int G = FH, PPG = (kL + G - 1) / G;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if (refill) {
#pragma unroll
        for (int q = g * PPG; q < kL && q < (g + 1) * PPG; ++q) stage_piece(t + kNB, q);
      }
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[FH + g][j] = mma16<T>(a1[g], bc[j], acc[FH + g][j]);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
    }
    // stage t+1's fragments after the last group, into the registers a1 / bc free (a second
    // fragment set beside the 128 accumulators spills past the 256-VGPR budget of 2 waves/SIMD)
    read_b(t + 1, bc);
    read_a(t + 1, 0, a0);
    lds_wait_fenced();
  }
  // last stage
  read_a(nk - 1, 1, a1);
  __builtin_amdgcn_sched_barrier(0);
  mfma_half(0, a0);
  lds_wait_fenced();
  mfma_half(1, a1);

  // ---- epilogue: per-wave fp32 patch of 32 rows x 64 cols (row stride 68 floats: conflict-free)
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();  // every wave done with the ring
  constexpr int kRS = 68;
  float* patch = reinterpret_cast<float*>(smem) + wave * (32 * kRS);
  const int r16 = lane & 15, g4 = lane >> 4;
  const int wrow0 = m0 + am;
#pragma unroll
  for (int hc = 0; hc < FM / 2 * (FN / 4); ++hc) {  // 32-row x 64-column pieces of the wave tile
    const int h = hc / (FN / 4), c4 = hc % (FN / 4);
    const int wcol0 = n0 + bn + c4 * 64;
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) patch[(ii * 16 + g4 * 4 + e) * kRS + j * 16 + r16] = acc[2 * h + ii][c4 * 4 + j][e];
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's patch written (wave-private region)
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int rr = it * 4 + (lane >> 4), cc = (lane & 15) * 4;
      const int row = wrow0 + h * 32 + rr, col = wcol0 + cc;
      float v[4];
      const float4 q = *reinterpret_cast<const float4*>(patch + rr * kRS + cc);
      v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
      if (row < p.M && col < p.N) {
        if (p.part == nullptr) epi4<OutT>(p.e, row, col, v);
        else if (p.cnt != nullptr) st16_wt(p.part + ((int64_t)z * p.M + row) * p.N + col, __builtin_bit_cast(uint4, q));
        else st4<float>(p.part + ((int64_t)z * p.M + row) * p.N + col, v);
      }
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // patch reads retired before the next half overwrites it
  }
  if (p.part == nullptr || p.cnt == nullptr) return;

  // ---- split-K, last arriver reduces (no gemm_splitk_epi_k launch): every slice stored its slab
  // write-through (sc1) and drained it; one lane per workgroup counts the tile's arrivals with an
  // agent-scope atomic; the workgroup whose add returns splits - 1 takes an agent-scope acquire,
  // resets the counter for the next launch, and sums the slabs in slice order z = 0 .. splits-1
  // (the same order as the separate reduce: bitwise-identical results) into the fused epilogue.
  // (MI355X_MICROARCH § visibility, Valid forms, producer row 1 with the acquire kept.)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int* flag = reinterpret_cast<int*>(smem);
  if (tid == 0) {
    const unsigned prev = __hip_atomic_fetch_add(p.cnt + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = prev == (unsigned)(p.splits - 1);
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(p.cnt + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    *flag = last;
  }
  __syncthreads();
  if (*flag == 0) return;
  constexpr int kQ = BN / 4;  // column quads per tile row
  const int64_t slab = (int64_t)p.M * p.N;
  for (int idx = tid; idx < BM * kQ; idx += NW * 64) {
    const int row = m0 + idx / kQ, col = n0 + (idx % kQ) * 4;
    if (row >= p.M || col >= p.N) continue;
    const float* src = p.part + (int64_t)row * p.N + col;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    for (int zz = 0; zz < p.splits; ++zz) {
      const float4 q = *reinterpret_cast<const float4*>(src + zz * slab);
      v[0] += q.x; v[1] += q.y; v[2] += q.z; v[3] += q.w;
    }
    epi4<OutT>(p.e, row, col, v);
  }
}

// split-K: C = epi(Σ_z part[z]) over [M, N] in groups of 4 columns
template <typename OutT>
__global__ __launch_bounds__(256) void gemm_splitk_epi_k(const float* __restrict__ part, Epi e, int M, int N,
                                                         int splits) {
  const int64_t n4 = (int64_t)M * N / 4;
  const int64_t slab = (int64_t)M * N;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const int64_t off = i * 4;
    const int row = (int)(off / N), col = (int)(off % N);
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    int z = 0;
    for (; z + 4 <= splits; z += 4) {  // four slab loads in flight, summed in slice order (as before)
      float4 q[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) q[i] = *reinterpret_cast<const float4*>(part + (z + i) * slab + off);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v[0] += q[i].x; v[1] += q[i].y; v[2] += q[i].z; v[3] += q[i].w;
      }
    }
    if (splits - z >= 2) {
      const float4 q0 = *reinterpret_cast<const float4*>(part + z * slab + off);
      const float4 q1 = *reinterpret_cast<const float4*>(part + (z + 1) * slab + off);
      v[0] += q0.x; v[1] += q0.y; v[2] += q0.z; v[3] += q0.w;
      v[0] += q1.x; v[1] += q1.y; v[2] += q1.z; v[3] += q1.w;
      z += 2;
    }
    if (z < splits) {
      const float4 q = *reinterpret_cast<const float4*>(part + z * slab + off);
      v[0] += q.x; v[1] += q.y; v[2] += q.z; v[3] += q.w;
    }
    epi4<OutT>(e, row, col, v);
  }
}

// ---- ping-pong schedule: 8 waves as two groups of 4 that alternate MFMA and load intervals ------
//
// gemm_tile_k runs every wave through the same read -> MFMA sequence between one barrier per
// 32-deep stage, so the two waves of a SIMD want the matrix pipe (and then the LDS) at the same
// time.  Here group 0 (waves 0-3, one per SIMD) and group 1 (waves 4-7, the SIMDs' second waves)
// run staggered by one barrier interval: while one group's wave issues its MFMA cluster, the
// other group's wave on the same SIMD reads its next fragments from LDS and issues the LDS-DMA
// refill of the ring (cdna_hip_programming.md §5 "256² 8-phase template": the per-phase
// ds_read || global_load_lds || MFMA interleave with counted vmcnt, raw barriers, setprio).
//
//   interval:   0          1           2           3          ...  2n-1         2n
//   group 0:    LOAD(0) |  MFMA(0)  |  LOAD(1)  |  MFMA(1)  | ... MFMA(n-1) | (idle)
//   group 1:    (idle)  |  LOAD(0)  |  MFMA(0)  |  LOAD(1)  | ... LOAD(n-1) | MFMA(n-1)
//
// A step is KS 32-deep slices.  LOAD(j) reads step j's fragments into registers (the whole wave
// tile's A and B operands) and issues the LDS-DMA of slices jKS+PD .. jKS+PD+KS-1 (PD = NB - KS
// slices ahead) into the buffers of step j-1, which group 1 finished reading in the interval
// before (retired by its lgkmcnt(0) ahead of that barrier).  Step j+1 must have landed before the
// barrier ending interval 2j+1: group 1 waits for its own pieces at the end of LOAD(j), group 0 at
// the end of MFMA(j), each with a counted vmcnt (PD - KS slices stay in flight), so every wave's
// pieces of a slice land before the barrier that precedes the slice's first read.
// Each group's wave tile: (BM/2)/WGM rows x BN/WGN (= 64) columns, so the epilogue is
// gemm_tile_k's (per-wave fp32 patches of 32 x 64).
// R (0 .. pieces per slice): the last R LDS-DMA pieces of each refilled slice are issued from the
// MFMA interval instead, between MFMA rows — it balances the two intervals: an LDS-DMA issue costs
// ~100-185 cycles in an interval of ds_reads, ~60 among bare MFMAs (MI355X_MICROARCH constants).
// Moving ALL of them measured slower (8192^3 1226 vs 1002 us on one box); of the 256² tile's 4, 2
// measured 985 vs 1180 us (R = 0) and 1037 (R = 1) on another, 3 measured 966 vs 1108 (R = 2) on a
// third (profiles/r06/gemm_pp_refill_split*.jsonl).
// With R > 0, group 1's MFMA-interval pieces of step j+1 are issued two steps ahead (PD >= 2 KS).
template <int N>
__device__ __forceinline__ void wait_vm_at_most(int n) {  // s_waitcnt vmcnt(min(n, N)), n >= 0
  if constexpr (N == 0) {
    wait_vmcnt<0>();
  } else {
    if (n >= N) wait_vmcnt<N>();
    else wait_vm_at_most<N - 1>(n);
  }
}

template <typename T, typename OutT, int BM, int BN, int WGM, int WGN, int KS, bool ATR, bool BTR, int NBR, int R>
__global__ __launch_bounds__(512) void gemm_pp_k(const GemmP p) {
  constexpr int NW = 8, kNB = NBR, PD = kNB - KS;
  static_assert(WGM * WGN == 4, "four waves per group");
  constexpr int FM = BM / 2 / WGM / 16, FN = BN / WGN / 16;
  static_assert(FN == 4 && FM % 2 == 0 && FM >= 2, "wave tiles are FM*16 x 64");
  static_assert(PD >= (R > 0 ? 2 * KS : KS), "a step's slices are issued ahead of the wait for them");
  constexpr int kA = BM * kBK, kB = BN * kBK, kStage = kA + kB;
  __shared__ __attribute__((aligned(16))) uint16_t smem[kNB * kStage];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2, wq = wave & 3, wm = wq / WGN, wn = wq % WGN;

  const int tiles_m = (p.M + BM - 1) / BM, tiles_n = (p.N + BN - 1) / BN;
  const int nwg = tiles_m * tiles_n * p.splits;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int tile = bid / p.splits, z = bid % p.splits;
  const int group = kGroupM * tiles_n;
  const int gid = tile / group, first_m = gid * kGroupM;
  const int gsize = min(tiles_m - first_m, kGroupM);
  const int tm = first_m + (tile % group) % gsize, tn = (tile % group) / gsize;
  const int m0 = min(tm * BM, p.M - BM), n0 = min(tn * BN, p.N - BN);
  const int kb = z * p.kper, ke = min(p.K, kb + p.kper);
  const int nk = (ke - kb + kBK - 1) / kBK;  // a multiple of KS (host: ceil(K / 32) % KS == 0, kper too)

  constexpr int kLA = ATR ? (BM / 128) * 8 / NW : BM / (16 * NW);
  constexpr int kLB = BTR ? (BN / 128) * 8 / NW : BN / (16 * NW);
  constexpr int kL = kLA + kLB;
  static_assert(PD * kL < 64, "vmcnt is 6 bits");
  const unsigned lpA = ATR ? tr_lane_off<NW>(p.lda, wave, lane) : row_lane(p.lda, lane);
  const unsigned lpB = BTR ? tr_lane_off<NW>(p.ldb, wave, lane) : row_lane(p.ldb, lane);
  const bool ragged_k = (ke - kb) % kBK != 0;  // the last slice ends mid-way: per-lane staging (zero page past K)
  auto stage_piece = [&](int t, int q) {
    uint16_t* sa = smem + (t % kNB) * kStage;
    uint16_t* sb = sa + kA;
    const int k0 = kb + t * kBK;
    if (ragged_k && t == nk - 1) {
      if (q < kLA) {
        if constexpr (ATR) tr_issue<BM, NW, true>(p.A, p.lda, m0, p.M, lpA, q, k0, ke, sa, wave, lane, p.zero, p.a_ext);
        else row_issue<BM, NW, true>(p.A, p.lda, m0, p.M, lpA, q, k0, ke, sa, wave, lane, p.zero, p.a_ext);
      } else {
        if constexpr (BTR) tr_issue<BN, NW, true>(p.B, p.ldb, n0, p.N, lpB, q - kLA, k0, ke, sb, wave, lane, p.zero, p.b_ext);
        else row_issue<BN, NW, true>(p.B, p.ldb, n0, p.N, lpB, q - kLA, k0, ke, sb, wave, lane, p.zero, p.b_ext);
      }
      return;
    }
    if (q < kLA) {
      if constexpr (ATR) tr_issue<BM, NW, false>(p.A, p.lda, m0, p.M, lpA, q, k0, ke, sa, wave, lane, p.zero, p.a_ext);
      else row_issue<BM, NW, false>(p.A, p.lda, m0, p.M, lpA, q, k0, ke, sa, wave, lane, p.zero, p.a_ext);
    } else {
      if constexpr (BTR) tr_issue<BN, NW, false>(p.B, p.ldb, n0, p.N, lpB, q - kLA, k0, ke, sb, wave, lane, p.zero, p.b_ext);
      else row_issue<BN, NW, false>(p.B, p.ldb, n0, p.N, lpB, q - kLA, k0, ke, sb, wave, lane, p.zero, p.b_ext);
    }
  };
  auto stage = [&](int t) {
#pragma unroll
    for (int q = 0; q < kLA + kLB; ++q) stage_piece(t, q);
  };
  auto wait_ahead = [&](int ahead) { wait_ahead_n<kL, PD - KS>(ahead); };
  static_assert(R >= 0 && R <= kL, "pieces moved into the MFMA interval");
  // pieces this wave issued after step j+1's last slice, at the end of group 1's LOAD(j): slices up to
  // jKS+PD-1 complete, the KS slices refilled by LOAD(j) with kL - R pieces each (clamped to nk)
  auto g1_outstanding = [&](int j) {
    const int last = j * KS + 2 * KS - 1;
    const int full = max(0, min(nk - 1, j * KS + PD - 1) - last);
    const int part = max(0, min(nk, j * KS + PD + KS) - max(j * KS + PD, last + 1));
    return full * kL + part * (kL - R);
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int am = grp * (BM / 2) + wm * FM * 16, bn = wn * FN * 16;
  const TrLane trl = tr_lane(lane);
  u16x8 af[KS][FM], bfr[KS][FN];
  auto read_slice = [&](int t, int ks) {
    const uint16_t* sa = smem + (t % kNB) * kStage;
    const uint16_t* sb = sa + kA;
    TrLane tl = trl;
    asm volatile("" : "+v"(tl.Y));
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      if constexpr (BTR) bfr[ks][j] = frag_col(sb, bn + j * 16, tl);
      else bfr[ks][j] = frag_row(lds_addr(sb), bn + j * 16, lane);
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      if constexpr (ATR) af[ks][i] = frag_col(sa, am + i * 16, tl);
      else af[ks][i] = frag_row(lds_addr(sa), am + i * 16, lane);
    }
  };
  auto pp_barrier = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    barrier_keep_vm();
    __builtin_amdgcn_sched_barrier(0);
  };

  // prologue: slices 0 .. PD-1 in flight; step 0 landed everywhere before the first barrier
#pragma unroll
  for (int s = 0; s < PD; ++s)
    if (s < nk) stage(s);
  wait_ahead(min(PD, nk) - KS);
  pp_barrier();
  if (grp == 1) pp_barrier();  // group 1 runs one interval behind
  const int nsteps = nk / KS;
  for (int j = 0; j < nsteps; ++j) {
    // ---- LOAD interval: step j's fragments, refill PD slices ahead (all but R pieces per slice)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) read_slice(j * KS + ks, ks);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int t = j * KS + PD + ks;
      if (t < nk) {
#pragma unroll
        for (int q = 0; q < kL - R; ++q) stage_piece(t, q);
      }
    }
    lds_wait_fenced();
    const int ahead = min(nk - 1, j * KS + PD + KS - 1) - (j * KS + 2 * KS - 1);
    if (grp == 1 && j + 1 < nsteps) {
      if constexpr (R == 0) wait_ahead(ahead);
      else wait_vm_at_most<(PD - 1) * kL>(g1_outstanding(j));
    }
    pp_barrier();
    // ---- MFMA interval (R > 0: the refill's remaining pieces between MFMA rows)
    __builtin_amdgcn_s_setprio(1);
    constexpr int RP = KS * R, RG = (KS * FM + RP) / (RP + 1);  // MFMA rows before each piece
    constexpr int RIN = RP < (KS * FM - 1) / RG ? RP : (KS * FM - 1) / RG;  // pieces issued inside the row loop
#pragma unroll
    for (int r = 0; r < KS * FM; ++r) {
      if constexpr (R > 0) {
        if (r > 0 && r % RG == 0 && r / RG <= RP) {
          const int q = r / RG - 1, t = j * KS + PD + q / R;
          if (t < nk) stage_piece(t, kL - R + q % R);
        }
      }
      const int ks = r / FM, i = r % FM;
#pragma unroll
      for (int jj = 0; jj < FN; ++jj) acc[i][jj] = mma16<T>(af[ks][i], bfr[ks][jj], acc[i][jj]);
    }
    if constexpr (R > 0) {
#pragma unroll
      for (int q = RIN; q < RP; ++q) {  // pieces the row loop did not reach
        const int t = j * KS + PD + q / R;
        if (t < nk) stage_piece(t, kL - R + q % R);
      }
    }
    __builtin_amdgcn_s_setprio(0);
    if (grp == 0 && j + 1 < nsteps) wait_ahead(ahead);
    pp_barrier();
  }
  if (grp == 0) pp_barrier();  // the interval in which group 1 runs its last MFMA cluster

  // ---- epilogue (gemm_tile_k's): per-wave fp32 patch of 32 rows x 64 cols
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  constexpr int kRS = 68;
  float* patch = reinterpret_cast<float*>(smem) + wave * (32 * kRS);
  const int r16 = lane & 15, g4 = lane >> 4;
  const int wrow0 = m0 + am, wcol0 = n0 + bn;
#pragma unroll
  for (int h = 0; h < FM / 2; ++h) {
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) patch[(ii * 16 + g4 * 4 + e) * kRS + j * 16 + r16] = acc[2 * h + ii][j][e];
    __builtin_amdgcn_s_waitcnt(0xC07F);
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int rr = it * 4 + (lane >> 4), cc = (lane & 15) * 4;
      const int row = wrow0 + h * 32 + rr, col = wcol0 + cc;
      float v[4];
      const float4 q = *reinterpret_cast<const float4*>(patch + rr * kRS + cc);
      v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
      if (row < p.M && col < p.N) {
        if (p.part == nullptr) epi4<OutT>(p.e, row, col, v);
        else st4<float>(p.part + ((int64_t)z * p.M + row) * p.N + col, v);
      }
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
  }
}

struct TileCfg {
  int bm, bn, waves, occ;
  double eff;  // relative per-CU throughput of a full tile (calibrated on MI355X)
  int ks = 0;  // > 0: the ping-pong kernel (gemm_pp_k) with KS 32-deep slices per step
};
constexpr int kNumTiles = 13;
constexpr TileCfg kTiles[kNumTiles] = {{256, 256, 8, 1, 1.0},       {256, 128, 8, 1, 0.80},     {128, 128, 4, 2, 0.62},
                                       {128, 128, 4, 2, 0.55},      {64, 64, 2, 4, 0.30},       {128, 64, 2, 3, 0.42},
                                       {64, 128, 4, 3, 0.42},       {192, 128, 4, 2, 0.70},
                                       // ping-pong tiles (gemm_pp_k): 256² KS 1 / NB 4; the others KS 2 / NB 6
                                       {256, 256, 8, 1, 1.25, 1},   {256, 128, 8, 1, 1.0, 2},
                                       {128, 256, 8, 1, 1.0, 2},    {128, 128, 8, 1, 0.70, 2},
                                       {256, 256, 8, 1, 1.25, 1}};  // 256² with a 5-deep ring

inline bool tile_layout_ok(int t, bool atr, bool btr) {
  const TileCfg& c = kTiles[t];
  return (!atr || c.bm % 128 == 0) && (!btr || c.bn % 128 == 0);
}

template <typename T, typename OutT, int BM, int BN, int WGM, int WGN, int KS, int NBR, int R = 0>
hipError_t launch_pp(const GemmP& p, bool atr, bool btr, int nwg, hipStream_t st) {
  const dim3 grid(nwg), block(512);
  if (!atr && !btr) hipLaunchKernelGGL((gemm_pp_k<T, OutT, BM, BN, WGM, WGN, KS, false, false, NBR, R>), grid, block, 0, st, p);
  else if (!atr && btr) hipLaunchKernelGGL((gemm_pp_k<T, OutT, BM, BN, WGM, WGN, KS, false, true, NBR, R>), grid, block, 0, st, p);
  else if (atr && btr) hipLaunchKernelGGL((gemm_pp_k<T, OutT, BM, BN, WGM, WGN, KS, true, true, NBR, R>), grid, block, 0, st, p);
  else hipLaunchKernelGGL((gemm_pp_k<T, OutT, BM, BN, WGM, WGN, KS, true, false, NBR, R>), grid, block, 0, st, p);
  return hipGetLastError();
}

template <typename T, typename OutT, int BM, int BN, int WM, int WN, bool SAFE, int NBR>
hipError_t launch_layout(const GemmP& p, bool atr, bool btr, int nwg, hipStream_t st) {
  // layouts a tile can stage: the row form needs BM (BN) % (16 x waves) == 0 (every tile here),
  // the transposed form 128-column image blocks (BM / BN % 128 == 0)
  const dim3 grid(nwg), block(WM * WN * 64);
  if ((atr && BM % 128 != 0) || (btr && BN % 128 != 0)) return hipErrorInvalidValue;
  if (!atr && !btr) {
    hipLaunchKernelGGL((gemm_tile_k<T, OutT, BM, BN, WM, WN, false, false, SAFE, NBR>), grid, block, 0, st, p);
  } else if (!atr && btr) {
    if constexpr (BN % 128 == 0)
      hipLaunchKernelGGL((gemm_tile_k<T, OutT, BM, BN, WM, WN, false, true, SAFE, NBR>), grid, block, 0, st, p);
  } else if (atr && btr) {
    if constexpr (BM % 128 == 0 && BN % 128 == 0)
      hipLaunchKernelGGL((gemm_tile_k<T, OutT, BM, BN, WM, WN, true, true, SAFE, NBR>), grid, block, 0, st, p);
  } else {
    if constexpr (BM % 128 == 0)
      hipLaunchKernelGGL((gemm_tile_k<T, OutT, BM, BN, WM, WN, true, false, SAFE, NBR>), grid, block, 0, st, p);
  }
  return hipGetLastError();
}

// tile 3 = the 128x128 SAFE kernel (ragged K, M or N below the tile, accumulate over ragged tiles).
// Tiles 4-7 size the grid for the small transformer GEMMs (M ~ 2k tokens): a 2032 x 768 output is
// 96 workgroups at 128x128 (37 % of the 256 CUs) but 192-384 at 64x64 / 128x64 / 64x128, and
// 2032 x 3072 is 264 at 192x128 — the vendor library's choice of one full wave of workgroups.
// Deep rings at one workgroup per CU (128x128 with 8 stages, 256x128 with 6) were measured SLOWER
// on every transformer shape (1.1-2x, profiles/r05/gemm_probe_deep_ring.json): with one wave per
// SIMD nothing hides the fragment reads behind the MFMAs.  NBR stays a template parameter.  So was
// 256x128 on 4 waves of 128x64 with a 3-deep ring (25 % fewer LDS fragment bytes per MFMA, two
// workgroups per CU): 1.5-2x slower than tile 1 on every shape, 8192^3 1186 vs 1091 us
// (profiles/r05/gemm_tile8_4wave_sweep.jsonl) — fewer waves per SIMD costs more than the LDS saves.
// the ping-pong tiles (kTiles[t].ks > 0) are instantiated in gemm_pp.hip
hipError_t launch_pp_tile(int in_dtype, int out_dtype, const GemmP& p, bool atr, bool btr, int tile, int nwg,
                          hipStream_t st);

}  // namespace gt
}  // namespace hyp

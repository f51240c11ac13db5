// Shared gfx950 MFMA / LDS building blocks for the implicit-GEMM convolution kernels.
//
// * mma16<T>      — v_mfma_f32_16x16x32_{bf16,f16}: A lane l holds row (l & 15), reduction
//                   elements 8*(l >> 4) .. +7; C lane l holds column (l & 15), rows 4*(l >> 4) + e.
// * glds16        — 16-byte global_load_lds (LDS-DMA, lane-linear destination).
// * frag_tr<W>    — a 16 x 32 MFMA operand read TRANSPOSED out of a [rows][W] bf16/f16 LDS image
//                   with ds_read_b64_tr_b16 (guide T10), for operands whose reduction dimension
//                   is the image's ROW index (pixel-major activations, k-major filters).
//                   Lane l (group g = l >> 4, q = (l >> 2) & 3, p = l & 3) addresses row
//                   r0 + 16t + 4g + q, columns cb + 4p .. +3 and receives column cb + (l & 15) of
//                   rows r0 + 16t + 4g + 0..3 as elements 4t .. 4t+3 (t = 0, 1).
// * swz_tr<W>     — 16-byte-chunk XOR swizzle of that image: every 32-lane half of a transposed
//                   read covers 8 consecutive rows x 2 chunks, which this maps onto 64 distinct
//                   banks (128-byte rows alternate bank halves by row parity -> 4 even masks;
//                   256-byte rows -> 8 even masks).
// * tr_row_to_k   — when the OTHER operand is read row-wise (element e of group g = reduction
//                   index 8g + e), a transposed image must hold reduction index
//                   8g + 4t + q in row 16t + 4g + q: this is that row -> index permutation.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hyp_common.h"

namespace hyp {
namespace mfl {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));

template <typename T>
__device__ __forceinline__ f32x4 mma16(u16x8 a, u16x8 b, f32x4 c);
template <>
__device__ __forceinline__ f32x4 mma16<bf16_t>(u16x8 a, u16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                 0, 0);
}
template <>
__device__ __forceinline__ f32x4 mma16<f16_t>(u16x8 a, u16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0,
                                                0);
}

__device__ __forceinline__ void glds16(const uint16_t* src, uint16_t* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const void*)src, (void __attribute__((address_space(3)))*)lds_wave_base, 16, 0,
                                   0);
}

template <int W>
__device__ __forceinline__ int swz_tr(int row) {
  static_assert(W == 64 || W == 128, "image rows of 64 or 128 elements");
  return W == 64 ? ((row >> 1) & 3) << 1 : (row & 7) << 1;
}

__device__ __forceinline__ int tr_row_to_k(int row) {
  return (row & ~31) | (((row >> 2) & 3) << 3) | (((row >> 4) & 1) << 2) | (row & 3);
}

// Debug builds (HYP_DEBUG: device printf checks) spill: hipcc may store an asm-read result to
// scratch right after the asm statement, before the asynchronous LDS read has returned — so there
// every asm LDS read waits for itself (HYP_LDS_SYNC).  Release kernels are verified spill-free.
#ifdef HYP_DEBUG
#define HYP_LDS_SYNC "\n\ts_waitcnt lgkmcnt(0)"
#else
#define HYP_LDS_SYNC ""
#endif

// ds_read_b64_tr_b16 as inline asm.  The builtin form makes hipcc (ROCm 7.2) wait vmcnt(0) before
// the read whenever a global_load_lds is in flight — it cannot prove the DMA's LDS destination does
// not alias — which drained the NEXT stage's prefetch before every k-step of the weight-gradient
// and data-gradient kernels (load and compute fully serialized).  The asm read is invisible to that
// pass; the caller orders it: the stage it reads was retired by wait_stage + barrier, and
// lds_reads_done() (lgkmcnt(0) + sched_barrier) precedes the MFMAs that consume the fragments.
__device__ __forceinline__ s16x4 ds_read_tr16_asm(const uint16_t* addr) {
  typedef short s16x4_t __attribute__((ext_vector_type(4)));
  s16x4_t v;
  const unsigned a = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)addr;
  asm volatile("ds_read_b64_tr_b16 %0, %1" HYP_LDS_SYNC : "=v"(v) : "v"(a) : "memory");
  return v;
}

// every LDS read issued so far (asm ones included) has returned; no instruction moves across
__device__ __forceinline__ void lds_reads_done() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

template <int W>
__device__ __forceinline__ u16x8 frag_tr(const uint16_t* img, int r0, int cb, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int chunk = (cb >> 3) + (p >> 1);
  u16x8 out;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int row = r0 + 16 * t + 4 * g + q;
    const uint16_t* addr = img + row * W + ((chunk ^ swz_tr<W>(row)) << 3) + ((p & 1) << 2);
    const s16x4 v = ds_read_tr16_asm(addr);
#pragma unroll
    for (int e = 0; e < 4; ++e) out[4 * t + e] = (uint16_t)v[e];
  }
  return out;
}

// The same transposed fragment read with the image base in one VGPR and the row offset as the
// instruction's immediate: the swizzle term of frag_tr depends only on (4g + q) for row offsets
// that are multiples of 16, so a lane's byte offset (frag_tr_lane<W>) is fixed per column block
// and every (k-step, half) variant is `base + imm` — no address VALU in the MFMA loop.
template <int OFF>
__device__ __forceinline__ s16x4 ds_read_tr16_imm(unsigned addr) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset is 16 bits");
  typedef short s16x4_t __attribute__((ext_vector_type(4)));
  s16x4_t v;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" HYP_LDS_SYNC : "=v"(v) : "v"(addr), "i"(OFF) : "memory");
  return v;
}

template <int W>
__device__ __forceinline__ unsigned frag_tr_lane(int cb, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int row = 4 * g + q;
  const int chunk = (cb >> 3) + (p >> 1);
  return (unsigned)((row * W + ((chunk ^ swz_tr<W>(row)) << 3) + ((p & 1) << 2)) * 2);
}

// frag_tr<W>(img, R0, cb, lane) == frag_tr_at<W, R0>(lds_addr(img) + frag_tr_lane<W>(cb, lane))
template <int W, int R0>
__device__ __forceinline__ u16x8 frag_tr_at(unsigned base) {
  static_assert(R0 % 16 == 0, "row offsets keep the swizzle phase");
  const s16x4 v0 = ds_read_tr16_imm<R0 * W * 2>(base);
  const s16x4 v1 = ds_read_tr16_imm<(R0 + 16) * W * 2>(base);
  u16x8 out;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    out[e] = (uint16_t)v0[e];
    out[4 + e] = (uint16_t)v1[e];
  }
  return out;
}

__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// s_waitcnt vmcnt(N) only (expcnt / lgkmcnt left at their "don't wait" maxima).  gfx9 encoding:
// vmcnt[3:0] in bits 3:0, vmcnt[5:4] in bits 15:14, expcnt in 6:4, lgkmcnt in 11:8.
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// Multi-stage LDS ring fed by global_load_lds: with NB buffers, stages t+1 .. t+NB-2 may still be
// in flight while stage t is consumed.  Every stage issues exactly L vector-memory instructions
// per lane, so "stage t has landed" is vmcnt <= L * (stages issued after t) — a compile-time
// count per tail case (the tail has fewer stages behind t).
template <int L, int NB>
__device__ __forceinline__ void wait_stage(int ahead) {
  if (NB >= 4 && ahead >= 2) wait_vmcnt<(NB >= 4 ? 2 * L : 0)>();
  else if (NB >= 3 && ahead >= 1) wait_vmcnt<(NB >= 3 ? L : 0)>();
  else wait_vmcnt<0>();
}

// Barrier that lets global_load_lds stay in flight across it: __syncthreads() fences LDS, and a
// pending LDS-DMA counts as an LDS write on the VM counter, so hipcc emits vmcnt(0) there and
// drains the whole prefetch ring (guide §5 "Pipelining across barriers").  Callers wait for the
// stage they need with wait_stage() first; this only retires the wave's own LDS reads.
__device__ __forceinline__ void barrier_keep_vm() {
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0) alone
  __builtin_amdgcn_s_barrier();
}

// XCD-aware remap of a linear workgroup id (bijective for any count): hardware dispatches
// blockIdx round-robin over the 8 XCDs; this gives each XCD a contiguous range of logical tiles
// so neighbouring tiles share that XCD's L2.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = bid % 8, idx = bid / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

}  // namespace mfl
}  // namespace hyp

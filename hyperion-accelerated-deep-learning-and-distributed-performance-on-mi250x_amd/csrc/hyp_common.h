// Shared device helpers for the Hyperion gfx950 kernels.
//
// * dtype codes shared with the Python side (hyperion/ops/_native.py): 0=f32, 1=bf16, 2=f16
// * 16-byte vector IO for 8 elements of a 2-byte type (Guideline 13: never scalar bf16 loads)
// * wave64 reductions (wavefront = 64 lanes on CDNA; __shfl_xor spans all 64)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Device-side checks of the debug build (python -m hyperion.csrc.build --debug -> _C_debug.so,
// selected by HYPERION_DEBUG_BUILD=1): a failed check prints the kernel, block, lane and the
// condition and the kernel carries on (no trap: a GPU trap can take the whole node down).  The
// release build compiles them out.
#ifdef HYP_DEBUG
#define HYP_DASSERT(cond)                                                                                   \
  do {                                                                                                     \
    if (!(cond))                                                                                           \
      printf("hyperion device check failed: %s:%d block %d thread %d: %s\n", __FILE__, __LINE__,           \
             (int)blockIdx.x, (int)threadIdx.x, #cond);                                                    \
  } while (0)
#else
#define HYP_DASSERT(cond) \
  do {                    \
  } while (0)
#endif

namespace hyp {

enum DType : int { kF32 = 0, kBF16 = 1, kF16 = 2 };

constexpr int kWave = 64;

typedef uint16_t bf16_t;  // storage type for bf16
typedef _Float16 f16_t;

__device__ __forceinline__ float bf16_to_float(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

// Plain cast: hipcc emits v_cvt_pk_bf16_f32 on gfx950 (RNE, NaN-preserving; MI355X_MICROARCH
// "Correctness boundaries").
__device__ __forceinline__ bf16_t float_to_bf16(float f) {
  __bf16 h = (__bf16)f;
  return __builtin_bit_cast(bf16_t, h);
}

__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  return (uint32_t)float_to_bf16(lo) | ((uint32_t)float_to_bf16(hi) << 16);
}

__device__ __forceinline__ uint32_t pack_f16x2(float lo, float hi) {
  f16_t a = (f16_t)lo, b = (f16_t)hi;
  return (uint32_t)__builtin_bit_cast(uint16_t, a) | ((uint32_t)__builtin_bit_cast(uint16_t, b) << 16);
}

__device__ __forceinline__ float f16_lo(uint32_t w) { return (float)__builtin_bit_cast(f16_t, (uint16_t)(w & 0xffff)); }
__device__ __forceinline__ float f16_hi(uint32_t w) { return (float)__builtin_bit_cast(f16_t, (uint16_t)(w >> 16)); }

// ---- 8-wide vector IO -------------------------------------------------------------------
// 16-byte GLOBAL store written through to memory (sc1): the line leaves the XCD's L2 at once, so a
// large output leaves no dirty lines for the kernel-end write-back (a dependent kernel boundary
// costs ~1.5 us + the dirty bytes / ~6 TB/s; writer + trivial successor in a hipGraph, MI355X:
// 16 MB 6.21 -> 5.03 us, 32 MB 8.67 -> 7.07 us, profiles/r05/boundary_wt.jsonl).  Global
// addresses only.  HYP_WT_STORES=0 compiles plain stores (A/B).  The store is inline asm, which the
// compiler's hazard recognizer does not see: a VALU writing the store's data VGPRs in the next
// cycles would race the store's read of them (gfx9 "VMEM store data > 8 bytes" hazard: observed as
// dx = dres in the small-M BN backward, whose next pack reuses the registers at once), so the asm
// carries its own wait states (s_nop 1).  Its vmcnt bookkeeping does not see the store either,
// which only ever makes its waits stricter.
#ifndef HYP_WT_STORES
#define HYP_WT_STORES 1
#endif
__device__ __forceinline__ void st16_wt(void* p, uint4 v) {
#if HYP_WT_STORES
  typedef unsigned hyp_u32x4 __attribute__((ext_vector_type(4)));
  const hyp_u32x4 w = {v.x, v.y, v.z, v.w};
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(w) : "memory");
#else
  *reinterpret_cast<uint4*>(p) = v;
#endif
}

template <typename T>
struct Vec8;

template <>
struct Vec8<float> {
  static __device__ __forceinline__ void load(const float* __restrict__ p, float (&v)[8]) {
    const float4 a = reinterpret_cast<const float4*>(p)[0];
    const float4 b = reinterpret_cast<const float4*>(p)[1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  static __device__ __forceinline__ void store(float* __restrict__ p, const float (&v)[8]) {
    reinterpret_cast<float4*>(p)[0] = make_float4(v[0], v[1], v[2], v[3]);
    reinterpret_cast<float4*>(p)[1] = make_float4(v[4], v[5], v[6], v[7]);
  }
  static __device__ __forceinline__ void store_wt(float* __restrict__ p, const float (&v)[8]) {
    st16_wt(p, uint4{__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])});
    st16_wt(p + 4, uint4{__float_as_uint(v[4]), __float_as_uint(v[5]), __float_as_uint(v[6]), __float_as_uint(v[7])});
  }
};

template <>
struct Vec8<bf16_t> {
  static __device__ __forceinline__ void load(const bf16_t* __restrict__ p, float (&v)[8]) {
    const uint4 r = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(w[i] << 16);
      v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
  static __device__ __forceinline__ void store(bf16_t* __restrict__ p, const float (&v)[8]) {
    uint4 r;
    r.x = pack_bf16x2(v[0], v[1]);
    r.y = pack_bf16x2(v[2], v[3]);
    r.z = pack_bf16x2(v[4], v[5]);
    r.w = pack_bf16x2(v[6], v[7]);
    *reinterpret_cast<uint4*>(p) = r;
  }
  static __device__ __forceinline__ void store_wt(bf16_t* __restrict__ p, const float (&v)[8]) {
    st16_wt(p, uint4{pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]),
                     pack_bf16x2(v[6], v[7])});
  }
};

template <>
struct Vec8<f16_t> {
  static __device__ __forceinline__ void load(const f16_t* __restrict__ p, float (&v)[8]) {
    const uint4 r = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = f16_lo(w[i]);
      v[2 * i + 1] = f16_hi(w[i]);
    }
  }
  static __device__ __forceinline__ void store(f16_t* __restrict__ p, const float (&v)[8]) {
    uint4 r;
    r.x = pack_f16x2(v[0], v[1]);
    r.y = pack_f16x2(v[2], v[3]);
    r.z = pack_f16x2(v[4], v[5]);
    r.w = pack_f16x2(v[6], v[7]);
    *reinterpret_cast<uint4*>(p) = r;
  }
  static __device__ __forceinline__ void store_wt(f16_t* __restrict__ p, const float (&v)[8]) {
    st16_wt(p, uint4{pack_f16x2(v[0], v[1]), pack_f16x2(v[2], v[3]), pack_f16x2(v[4], v[5]),
                     pack_f16x2(v[6], v[7])});
  }
};

// scalar load/store in float
template <typename T>
__device__ __forceinline__ float ld1(const T* p);
template <>
__device__ __forceinline__ float ld1<float>(const float* p) { return *p; }
template <>
__device__ __forceinline__ float ld1<bf16_t>(const bf16_t* p) { return bf16_to_float(*p); }
template <>
__device__ __forceinline__ float ld1<f16_t>(const f16_t* p) { return (float)*p; }

template <typename T>
__device__ __forceinline__ void st1(T* p, float v);
template <>
__device__ __forceinline__ void st1<float>(float* p, float v) { *p = v; }
template <>
__device__ __forceinline__ void st1<bf16_t>(bf16_t* p, float v) { *p = float_to_bf16(v); }
template <>
__device__ __forceinline__ void st1<f16_t>(f16_t* p, float v) { *p = (f16_t)v; }

// round a float to T's precision and back (keeps fused outputs bit-consistent with stored ones)
template <typename T>
__device__ __forceinline__ float rnd(float v);
template <>
__device__ __forceinline__ float rnd<float>(float v) { return v; }
template <>
__device__ __forceinline__ float rnd<bf16_t>(float v) { return bf16_to_float(float_to_bf16(v)); }
template <>
__device__ __forceinline__ float rnd<f16_t>(float v) { return (float)(f16_t)v; }

// ---- counter-based RNG (dropout) ----------------------------------------------------------
// The (seed, offset) pair comes from torch's default generator (PhiloxCudaState) so streams
// advance like torch's own dropout AND stay hipGraph-safe: under capture the kernel reads the
// seed and the graph's extragraph offset from device memory at replay time (the bindings pass
// whichever form the generator handed out).
struct RngState {
  uint64_t seed, offset;       // not captured
  const int64_t* seed_ptr;     // captured: *seed_ptr, *offset_ptr + intra
  const int64_t* offset_ptr;
  uint64_t intra;
  int captured;
};

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// one 64-bit key per (seed, offset): element streams are rng_u32(key, element index)
__device__ __forceinline__ uint64_t rng_key(const RngState& s) {
  const uint64_t seed = s.captured ? (uint64_t)*s.seed_ptr : s.seed;
  const uint64_t off = s.captured ? (uint64_t)*s.offset_ptr + s.intra : s.offset;
  return splitmix64(seed ^ splitmix64(off));
}

__device__ __forceinline__ uint32_t rng_u32(uint64_t key, uint64_t ctr) {
  return (uint32_t)(splitmix64(key + 0xD1B54A32D192ED03ull * (ctr + 1)) >> 32);
}

// LoRA-dropout keep mask (ops/llama_fused.py): one cheap 32-bit hash per element index, keyed by the
// call's rng_key — regenerated identically by every forward and backward kernel that needs it.
__device__ __forceinline__ uint32_t lowbias32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

// keep (probability 1 - thr / 2^32) for element `idx` = (proj * M + m) * K + k
__device__ __forceinline__ bool lora_keep(uint64_t key, uint32_t idx, uint32_t thr) {
  return lowbias32(lowbias32(idx ^ (uint32_t)key) ^ (uint32_t)(key >> 32)) >= thr;
}

// ---- wave / block reductions ------------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x <= 1024; `scratch` needs blockDim.x/64 floats.
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += scratch[i];
  return t;
}

__device__ __forceinline__ float block_max(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float t = -INFINITY;
  for (int i = 0; i < nw; ++i) t = fmaxf(t, scratch[i]);
  return t;
}

// Dispatch a templated launcher over the three floating dtypes.
#define HYP_DISPATCH_FLOAT(DT, T, ...)                 \
  switch (DT) {                                        \
    case ::hyp::kF32: { typedef float T; __VA_ARGS__; break; }   \
    case ::hyp::kBF16: { typedef ::hyp::bf16_t T; __VA_ARGS__; break; } \
    case ::hyp::kF16: { typedef ::hyp::f16_t T; __VA_ARGS__; break; }   \
    default: return hipErrorInvalidValue;             \
  }

}  // namespace hyp

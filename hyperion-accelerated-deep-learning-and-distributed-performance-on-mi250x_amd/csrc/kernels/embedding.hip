// Token embedding forward (row gather) and backward (fp32 atomic row accumulation).
//
// Reference: ``nn.Embedding`` in SimpleTransformerLM (V = 50257, E = 256 / 768; C14/C15) and HF
// Llama's ``embed_tokens`` (V = 32000, E = 4096; C26) — PyTorch's index_select forward and
// ``embedding_dense_backward`` (SURVEY §2.4 "Embedding fwd/bwd").
//
// Forward: one wave per token, 16-byte vectors along the row.
// Backward: fp32 atomic accumulation into a zeroed [V, E] buffer, one wave per token (full-rate
// 256-byte atomic runs), then one cast pass for bf16/f16 weights.  (A first, deterministic
// sorted-run version serialized each id's run in one wave: the LM's pad token is ~1/3 of all
// tokens, so one wave summed ~1300 rows — 1.35 ms per step; profiles/lm_r01.)
#include <algorithm>

#include "hyp_common.h"
#include "hyp_kernels.h"

namespace hyp {
namespace {

template <typename T>
__global__ __launch_bounds__(256) void embed_fwd_k(const int64_t* __restrict__ ids, const T* __restrict__ w,
                                                   T* __restrict__ out, int64_t n, int E, int64_t V) {
  const int64_t tok = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (tok >= n) return;
  const int lane = threadIdx.x & 63;
  int64_t id = ids[tok];
  id = id < 0 ? 0 : (id >= V ? V - 1 : id);  // clamp: an out-of-range id must not fault the GPU
  const T* src = w + id * E;
  T* dst = out + tok * E;
  for (int c = lane * 8; c < E; c += 64 * 8) {
    float v[8];
    Vec8<T>::load(src + c, v);
    Vec8<T>::store(dst + c, v);
  }
}

// One wave per token: dW[id, :] += dY[token, :] with no-return fp32 atomics, one dword per lane so
// each wave instruction adds a contiguous 256-byte run (the full-rate shape: MI355X_MICROARCH
// "Global float atomics").  The pad id gets no gradient.
template <typename T>
__global__ __launch_bounds__(256) void embed_bwd_atomic_k(const int64_t* __restrict__ ids, const T* __restrict__ dy,
                                                          float* __restrict__ dw, int64_t n, int E, int64_t V,
                                                          int64_t pad_idx) {
  const int64_t tok = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (tok >= n) return;
  const int64_t id = ids[tok];
  if (id < 0 || id >= V || id == pad_idx) return;
  const int lane = threadIdx.x & 63;
  const T* src = dy + tok * E;
  float* dst = dw + id * E;
  for (int c = lane; c < E; c += 64) atomicAdd(dst + c, ld1<T>(src + c));
}

// Touched rows only (one wave per token; a repeated id rewrites the same row with the same values):
// ZERO = true clears the fp32 accumulator row before the atomics, ZERO = false rounds the finished
// row into the weight-dtype gradient.  The accumulator's untouched rows are never initialized or
// read, and the low-precision gradient is zero-filled by one memset — the two full [V, E] passes
// of a dense fp32 buffer (zero fill + cast: ~55 us for GPT-2's 50257 x 768) become ~2 x 6 MB.
template <typename T, bool ZERO>
__global__ __launch_bounds__(256) void embed_rows_k(const int64_t* __restrict__ ids, float* __restrict__ dw32,
                                                    T* __restrict__ dw, int64_t n, int E, int64_t V, int64_t pad_idx) {
  const int64_t tok = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (tok >= n) return;
  const int64_t id = ids[tok];
  if (id < 0 || id >= V || id == pad_idx) return;
  const int lane = threadIdx.x & 63;
  float* row = dw32 + id * E;
  for (int c = lane * 8; c < E; c += 64 * 8) {
    float v[8];
    if (ZERO) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = 0.f;
      Vec8<float>::store(row + c, v);
    } else {
      Vec8<float>::load(row + c, v);
      Vec8<T>::store(dw + id * E + c, v);
    }
  }
}

// zero fill in 16-byte stores (a kernel rather than hipMemsetAsync: a memset issued while a stream
// captures a segmented hipGraph was not replayed — the FSDP segmented step read stale gradient rows)
__global__ __launch_bounds__(256) void zero16_k(uint4* __restrict__ p, int64_t n16) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256)
    p[i] = make_uint4(0u, 0u, 0u, 0u);
}

}  // namespace

hipError_t embedding_forward(int dtype, const int64_t* ids, const void* w, void* out, int64_t n, int E, int64_t V,
                             hipStream_t st) {
  if (E % 8 != 0) return hipErrorInvalidValue;
  if (n == 0) return hipSuccess;
  HYP_DISPATCH_FLOAT(dtype, T, {
    hipLaunchKernelGGL(embed_fwd_k<T>, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st, ids, (const T*)w, (T*)out, n,
                       E, V);
  });
  return hipGetLastError();
}

// dw32: [V, E] fp32 accumulator — for f32 it is the result itself and must be ZEROED by the caller;
// for bf16 / f16 it may be uninitialized (only the rows of the ids are cleared, accumulated and
// rounded into dw, which is zero-filled here)
hipError_t embedding_backward(int dtype, const int64_t* ids, const void* dy, float* dw32, void* dw, int64_t n, int E,
                              int64_t V, int64_t pad_idx, hipStream_t st) {
  if (E % 8 != 0) return hipErrorInvalidValue;
  const dim3 grid((unsigned)((n + 3) / 4)), block(256);
  HYP_DISPATCH_FLOAT(dtype, T, {
    if (dtype != kF32) {
      const int64_t n16 = V * E * (int64_t)sizeof(T) / 16;  // E % 8 == 0: whole 16-byte chunks
      hipLaunchKernelGGL(zero16_k, dim3((unsigned)std::min<int64_t>((n16 + 255) / 256, 8192)), block, 0, st,
                         static_cast<uint4*>(dw), n16);
      if (n > 0) hipLaunchKernelGGL((embed_rows_k<T, true>), grid, block, 0, st, ids, dw32, (T*)dw, n, E, V, pad_idx);
    }
    if (n > 0)
      hipLaunchKernelGGL(embed_bwd_atomic_k<T>, grid, block, 0, st, ids, (const T*)dy, dw32, n, E, V, pad_idx);
    if (dtype != kF32 && n > 0)
      hipLaunchKernelGGL((embed_rows_k<T, false>), grid, block, 0, st, ids, dw32, (T*)dw, n, E, V, pad_idx);
  });
  return hipGetLastError();
}

}  // namespace hyp

// Token embedding forward (row gather) and a deterministic backward (sorted-segment row sums).
//
// Reference: ``nn.Embedding`` in SimpleTransformerLM (V = 50257, E = 256 / 768; C14/C15) and HF
// Llama's ``embed_tokens`` (V = 32000, E = 4096; C26) — PyTorch's index_select forward and
// ``embedding_dense_backward`` (SURVEY §2.4 "Embedding fwd/bwd").
//
// Forward: one wave per token, 16-byte vectors along the row.
// Backward: the token ids are sorted once (with their positions); one wave per sorted position,
// and only the wave that starts a run of equal ids sums the run's gradient rows (fp32, in sorted
// order: deterministic) and writes that id's row.  Rows of ids that never occur are zeroed by the
// same launch (a second grid stripe walks the "absent" rows), so the dense [V, E] gradient is
// written exactly once, with no atomics and no separate memset.
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

// blocks [0, nrun_blocks): one wave per sorted position (run heads write their row);
// blocks [nrun_blocks, ...): one wave per row id, zeroing rows whose id is absent (present[id] == 0).
template <typename T>
__global__ __launch_bounds__(256) void embed_bwd_k(const int64_t* __restrict__ sorted_ids,
                                                   const int64_t* __restrict__ order, const T* __restrict__ dy,
                                                   T* __restrict__ dw, const uint8_t* __restrict__ present, int64_t n,
                                                   int E, int64_t V, int nrun_blocks, int64_t pad_idx) {
  const int lane = threadIdx.x & 63;
  if ((int)blockIdx.x < nrun_blocks) {
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= n) return;
    const int64_t id = sorted_ids[i];
    if (i > 0 && sorted_ids[i - 1] == id) return;  // not a run head
    if (id < 0 || id >= V) return;
    int64_t j1 = i + 1;
    while (j1 < n && sorted_ids[j1] == id) ++j1;
    for (int c = lane * 8; c < E; c += 64 * 8) {
      float acc[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] = 0.f;
      if (id != pad_idx) {
        for (int64_t j = i; j < j1; ++j) {
          float v[8];
          Vec8<T>::load(dy + order[j] * E + c, v);
#pragma unroll
          for (int q = 0; q < 8; ++q) acc[q] += v[q];
        }
      }
      Vec8<T>::store(dw + id * E + c, acc);
    }
    return;
  }
  const int64_t row = (int64_t)(blockIdx.x - nrun_blocks) * 4 + (threadIdx.x >> 6);
  if (row >= V || present[row]) return;
  float z[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) z[q] = 0.f;
  for (int c = lane * 8; c < E; c += 64 * 8) Vec8<T>::store(dw + row * E + c, z);
}

__global__ __launch_bounds__(256) void mark_present_k(const int64_t* __restrict__ ids, uint8_t* __restrict__ present,
                                                      int64_t n, int64_t V) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) {
    const int64_t id = ids[i];
    if (id >= 0 && id < V) present[id] = 1;
  }
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

// present: [V] uint8 scratch, ZEROED by the caller
hipError_t embedding_backward(int dtype, const int64_t* sorted_ids, const int64_t* order, const void* dy, void* dw,
                              uint8_t* present, int64_t n, int E, int64_t V, int64_t pad_idx, hipStream_t st) {
  if (E % 8 != 0) return hipErrorInvalidValue;
  if (n > 0)
    hipLaunchKernelGGL(mark_present_k, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, sorted_ids, present, n, V);
  const int nrun = (int)((n + 3) / 4);
  const int nrow = (int)((V + 3) / 4);
  HYP_DISPATCH_FLOAT(dtype, T, {
    hipLaunchKernelGGL(embed_bwd_k<T>, dim3(nrun + nrow), dim3(256), 0, st, sorted_ids, order, (const T*)dy, (T*)dw,
                       present, n, E, V, nrun, pad_idx);
  });
  return hipGetLastError();
}

}  // namespace hyp

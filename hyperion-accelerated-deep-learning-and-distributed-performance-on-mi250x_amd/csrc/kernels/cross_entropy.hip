// Softmax cross-entropy forward + backward in ONE pass pair over the logits, in place.
//
// Reference: every LM trainer computes `CrossEntropyLoss(ignore_index=pad)(fc(x), y)` over
// V = 50257 (distributed_utils.py:161,177; core_framework.ipynb:243-262) — PyTorch runs
// log_softmax, nll_loss, nll_loss_backward and log_softmax_backward as four kernels with an
// fp32 [N, V] intermediate each (SURVEY §2.4 "Cross-entropy", §2.5 LM-256: 4064 x 50257).
//
// Here (the CE half of hyperion.ops.cross_entropy.fused_linear_cross_entropy):
//   pass 1  online max / sum-exp over the row            -> lse, loss = lse - z[target]
//   pass 2  z <- (softmax(z) - onehot(target)) * scale  (written over the logits, same dtype)
// so the logits buffer becomes dlogits and the caller runs the two backward GEMMs on it
// directly.  `scale` is read from device memory (1 / #non-ignored tokens, computed on device), so
// no host sync and the whole loss is hipGraph-capturable.  Rows are processed by one 512-thread
// workgroup each (8 waves); V need not be a multiple of 8 (50257): each row is split into an
// unaligned scalar head, a 16-byte-vector body and a scalar tail.  The second pass re-reads the
// row (≤ 100 KB bf16) from L2, not HBM.
#include "hyp_common.h"
#include "hyp_kernels.h"

namespace hyp {
namespace {

constexpr int kCeThreads = 512;

struct MaxSum {
  float m, s;
};

__device__ __forceinline__ MaxSum ms_combine(MaxSum a, MaxSum b) {
  const float m = fmaxf(a.m, b.m);
  if (m == -INFINITY) return {m, 0.f};
  return {m, a.s * __expf(a.m - m) + b.s * __expf(b.m - m)};
}

__device__ __forceinline__ void ms_add(MaxSum& a, float x) {
  if (x > a.m) {
    a.s = a.s * __expf(a.m - x) + 1.f;
    a.m = x;
  } else {
    a.s += __expf(x - a.m);
  }
}

template <typename T>
__global__ __launch_bounds__(kCeThreads) void ce_fwd_bwd_k(T* __restrict__ logits, int64_t ld,
                                                            const int64_t* __restrict__ target,
                                                            float* __restrict__ loss_rows, float* __restrict__ lse_out,
                                                            const float* __restrict__ scale_ptr, float scale_mul,
                                                            int V, int64_t ignore_index, int write_grad) {
  __shared__ float red_m[kCeThreads / 64], red_s[kCeThreads / 64];
  const int64_t row = blockIdx.x;
  T* z = logits + row * ld;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;

  // split into scalar head | vector body | scalar tail by the row's 16-byte alignment
  const int64_t eoff = (int64_t)(reinterpret_cast<uintptr_t>(z) % 16) / sizeof(T);
  const int vecw = 16 / sizeof(T) == 4 ? 4 : 8;  // elements per 16 B (fp32: 4, 2-byte: 8)
  int head = (int)((vecw - eoff) % vecw);
  if (head > V) head = V;
  const int nvec = (V - head) / vecw;
  const int body_end = head + nvec * vecw;

  MaxSum acc{-INFINITY, 0.f};
  if (tid < head) ms_add(acc, ld1<T>(z + tid));
  if (tid < V - body_end) ms_add(acc, ld1<T>(z + body_end + tid));
  if constexpr (sizeof(T) == 4) {
    const float4* zv = reinterpret_cast<const float4*>(z + head);
    for (int i = tid; i < nvec; i += kCeThreads) {
      const float4 q = zv[i];
      ms_add(acc, q.x); ms_add(acc, q.y); ms_add(acc, q.z); ms_add(acc, q.w);
    }
  } else {
    for (int i = tid; i < nvec; i += kCeThreads) {
      float v[8];
      Vec8<T>::load(z + head + (int64_t)i * 8, v);
      float mx = v[0];
#pragma unroll
      for (int j = 1; j < 8; ++j) mx = fmaxf(mx, v[j]);
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) s += __expf(v[j] - mx);
      acc = ms_combine(acc, MaxSum{mx, s});
    }
  }
  // wave then block combine
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    MaxSum other{__shfl_xor(acc.m, o, 64), __shfl_xor(acc.s, o, 64)};
    acc = ms_combine(acc, other);
  }
  if (lane == 0) {
    red_m[wid] = acc.m;
    red_s[wid] = acc.s;
  }
  __syncthreads();
  MaxSum tot{red_m[0], red_s[0]};
#pragma unroll
  for (int w = 1; w < kCeThreads / 64; ++w) tot = ms_combine(tot, MaxSum{red_m[w], red_s[w]});
  const float lse = tot.m + __logf(tot.s);

  const int64_t t = target[row];
  const bool valid = t != ignore_index && t >= 0 && t < V;
  if (tid == 0) {
    loss_rows[row] = valid ? (lse - ld1<T>(z + t)) : 0.f;
    if (lse_out) lse_out[row] = lse;
  }
  if (!write_grad) return;
  __syncthreads();  // z[t] was read above before any thread overwrites it
  const float sc = (scale_ptr ? *scale_ptr : 1.f) * scale_mul;
  const float g = valid ? sc : 0.f;         // ignored rows get zero gradient
  const int64_t tt = valid ? t : -1;        // one-hot column (folded into the element that owns it)
  if (tid < head) st1<T>(z + tid, __expf(ld1<T>(z + tid) - lse) * g - (tid == tt ? g : 0.f));
  if (tid < V - body_end) {
    const int c = body_end + tid;
    st1<T>(z + c, __expf(ld1<T>(z + c) - lse) * g - (c == tt ? g : 0.f));
  }
  if constexpr (sizeof(T) == 4) {
    float4* zv = reinterpret_cast<float4*>(z + head);
    for (int i = tid; i < nvec; i += kCeThreads) {
      float4 q = zv[i];
      const int64_t c0 = head + (int64_t)i * 4;
      q.x = __expf(q.x - lse) * g - (c0 == tt ? g : 0.f);
      q.y = __expf(q.y - lse) * g - (c0 + 1 == tt ? g : 0.f);
      q.z = __expf(q.z - lse) * g - (c0 + 2 == tt ? g : 0.f);
      q.w = __expf(q.w - lse) * g - (c0 + 3 == tt ? g : 0.f);
      zv[i] = q;
    }
  } else {
    for (int i = tid; i < nvec; i += kCeThreads) {
      float v[8];
      const int64_t c0 = head + (int64_t)i * 8;
      T* p = z + c0;
      Vec8<T>::load(p, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = __expf(v[j] - lse) * g - (c0 + j == tt ? g : 0.f);
      Vec8<T>::store(p, v);
    }
  }
}

}  // namespace

hipError_t cross_entropy_fwd_bwd(int dtype, void* logits, int64_t rows, int V, int64_t ld, const int64_t* target,
                                 float* loss_rows, float* lse, const float* scale_ptr, float scale_mul,
                                 int64_t ignore_index, int write_grad, hipStream_t st) {
  if (rows == 0) return hipSuccess;
  if (V <= 0 || ld < V) return hipErrorInvalidValue;
  HYP_DISPATCH_FLOAT(dtype, T, {
    hipLaunchKernelGGL(ce_fwd_bwd_k<T>, dim3((unsigned)rows), dim3(kCeThreads), 0, st, reinterpret_cast<T*>(logits),
                       ld, target, loss_rows, lse, scale_ptr, scale_mul, V, ignore_index, write_grad);
  });
  return hipGetLastError();
}

namespace {
// One wave per row: merge the GEMM tiles' (max, Σexp) partials of the row (fixed order within a
// lane, then a wave tree: deterministic) into lse and the per-row loss.
__global__ __launch_bounds__(256) void ce_lse_combine_k(const float2* __restrict__ part, int tiles, int M,
                                                        const float* __restrict__ zt,
                                                        const int64_t* __restrict__ target, int64_t ignore,
                                                        float* __restrict__ lse, float* __restrict__ loss_rows) {
  const int lane = threadIdx.x & 63;
  const int m = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= M) return;
  float mx = -INFINITY, sm = 0.f;
  for (int t = lane; t < tiles; t += 64) {
    const float2 p = part[(int64_t)t * M + m];
    if (p.x == -INFINITY) continue;
    if (p.x > mx) {
      sm = sm * __expf(mx - p.x) + p.y;
      mx = p.x;
    } else {
      sm += p.y * __expf(p.x - mx);
    }
  }
  const float gmx = wave_max(mx);
  float s = mx == -INFINITY ? 0.f : sm * __expf(mx - gmx);
  s = wave_sum(s);
  if (lane == 0) {
    const float l = gmx + __logf(s);
    lse[m] = l;
    loss_rows[m] = target[m] == ignore ? 0.f : l - zt[m];
  }
}
}  // namespace

hipError_t ce_lse_combine(const float2* part, int tiles, int M, const float* zt, const int64_t* target,
                          int64_t ignore, float* lse, float* loss_rows, hipStream_t st) {
  if (tiles < 1 || M < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(ce_lse_combine_k, dim3((M + 3) / 4), dim3(256), 0, st, part, tiles, M, zt, target, ignore, lse,
                     loss_rows);
  return hipGetLastError();
}

}  // namespace hyp

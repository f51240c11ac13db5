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
                                                            const float* __restrict__ bias,
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

  auto bz = [&](int64_t c) { return bias ? bias[c] : 0.f; };
  MaxSum acc{-INFINITY, 0.f};
  if (tid < head) ms_add(acc, ld1<T>(z + tid) + bz(tid));
  if (tid < V - body_end) ms_add(acc, ld1<T>(z + body_end + tid) + bz(body_end + tid));
  if constexpr (sizeof(T) == 4) {
    const float4* zv = reinterpret_cast<const float4*>(z + head);
    for (int i = tid; i < nvec; i += kCeThreads) {
      const float4 q = zv[i];
      const int64_t c0 = head + (int64_t)i * 4;
      ms_add(acc, q.x + bz(c0)); ms_add(acc, q.y + bz(c0 + 1)); ms_add(acc, q.z + bz(c0 + 2));
      ms_add(acc, q.w + bz(c0 + 3));
    }
  } else {
    for (int i = tid; i < nvec; i += kCeThreads) {
      float v[8];
      Vec8<T>::load(z + head + (int64_t)i * 8, v);
      if (bias) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] += bias[head + (int64_t)i * 8 + j];
      }
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
    loss_rows[row] = valid ? (lse - ld1<T>(z + t) - bz(t)) : 0.f;
    if (lse_out) lse_out[row] = lse;
  }
  if (!write_grad) return;
  __syncthreads();  // z[t] was read above before any thread overwrites it
  const float sc = (scale_ptr ? *scale_ptr : 1.f) * scale_mul;
  const float g = valid ? sc : 0.f;         // ignored rows get zero gradient
  const int64_t tt = valid ? t : -1;        // one-hot column (folded into the element that owns it)
  if (tid < head) st1<T>(z + tid, __expf(ld1<T>(z + tid) + bz(tid) - lse) * g - (tid == tt ? g : 0.f));
  if (tid < V - body_end) {
    const int c = body_end + tid;
    st1<T>(z + c, __expf(ld1<T>(z + c) + bz(c) - lse) * g - (c == tt ? g : 0.f));
  }
  if constexpr (sizeof(T) == 4) {
    float4* zv = reinterpret_cast<float4*>(z + head);
    for (int i = tid; i < nvec; i += kCeThreads) {
      float4 q = zv[i];
      const int64_t c0 = head + (int64_t)i * 4;
      q.x = __expf(q.x + bz(c0) - lse) * g - (c0 == tt ? g : 0.f);
      q.y = __expf(q.y + bz(c0 + 1) - lse) * g - (c0 + 1 == tt ? g : 0.f);
      q.z = __expf(q.z + bz(c0 + 2) - lse) * g - (c0 + 2 == tt ? g : 0.f);
      q.w = __expf(q.w + bz(c0 + 3) - lse) * g - (c0 + 3 == tt ? g : 0.f);
      zv[i] = q;
    }
  } else {
    for (int i = tid; i < nvec; i += kCeThreads) {
      float v[8];
      const int64_t c0 = head + (int64_t)i * 8;
      T* p = z + c0;
      Vec8<T>::load(p, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = __expf(v[j] + bz(c0 + j) - lse) * g - (c0 + j == tt ? g : 0.f);
      Vec8<T>::store(p, v);
    }
  }
}

// Register-resident variant (16-byte aligned rows, V <= 8 * 1024 * NCH): each of 1024 threads
// keeps NCH 8-element chunks of the row in registers, so the row is read from HBM once and the
// gradient written from registers — one read + one write per logit instead of the two-pass
// kernel's two reads + one write (its second pass misses L2 once ~2 rows per CU are in flight:
// 4064 x 50257 bf16 rows are 100 KB each).  Chunk i of thread t covers columns 8 (t + 1024 i).
constexpr int kCeRegThreads = 1024;

template <typename T, int NCH>
__global__ __launch_bounds__(kCeRegThreads) void ce_fwd_bwd_reg_k(T* __restrict__ logits, int64_t ld,
                                                                   const float* __restrict__ bias,
                                                                   const int64_t* __restrict__ target,
                                                                   float* __restrict__ loss_rows,
                                                                   float* __restrict__ lse_out,
                                                                   const float* __restrict__ scale_ptr,
                                                                   float scale_mul, int V, int64_t ignore_index,
                                                                   int write_grad) {
  __shared__ float red_m[kCeRegThreads / 64], red_s[kCeRegThreads / 64];
  __shared__ float zt_s;
  const int64_t row = blockIdx.x;
  T* z = logits + row * ld;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const int64_t t = target[row];
  const bool valid = t != ignore_index && t >= 0 && t < V;
  float v[NCH][8];
  MaxSum acc{-INFINITY, 0.f};
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int c0 = (tid + i * kCeRegThreads) * 8;
    if (c0 + 8 <= V) {
      Vec8<T>::load(z + c0, v[i]);
      if (bias) {
        const float4 b0 = *reinterpret_cast<const float4*>(bias + c0);
        const float4 b1 = *reinterpret_cast<const float4*>(bias + c0 + 4);
        v[i][0] += b0.x; v[i][1] += b0.y; v[i][2] += b0.z; v[i][3] += b0.w;
        v[i][4] += b1.x; v[i][5] += b1.y; v[i][6] += b1.z; v[i][7] += b1.w;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        v[i][j] = c0 + j < V ? ld1<T>(z + c0 + j) + (bias ? bias[c0 + j] : 0.f) : -INFINITY;
    }
    float mx = v[i][0];
#pragma unroll
    for (int j = 1; j < 8; ++j) mx = fmaxf(mx, v[i][j]);
    if (mx != -INFINITY) {
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) s += __expf(v[i][j] - mx);
      acc = ms_combine(acc, MaxSum{mx, s});
    }
  }
  // the target logit, from the thread that holds it
  if (valid && tid == (int)((t >> 3) % kCeRegThreads)) {
    const int ti = (int)((t >> 3) / kCeRegThreads), tj = (int)(t & 7);
    float zt = 0.f;
#pragma unroll
    for (int i = 0; i < NCH; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (i == ti && j == tj) zt = v[i][j];
    zt_s = zt;
  }
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
  for (int w = 1; w < kCeRegThreads / 64; ++w) tot = ms_combine(tot, MaxSum{red_m[w], red_s[w]});
  const float lse = tot.m + __logf(tot.s);
  if (tid == 0) {
    loss_rows[row] = valid ? lse - zt_s : 0.f;
    if (lse_out) lse_out[row] = lse;
  }
  if (!write_grad) return;
  const float g = valid ? (scale_ptr ? *scale_ptr : 1.f) * scale_mul : 0.f;
  const int64_t tt = valid ? t : -1;
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int c0 = (tid + i * kCeRegThreads) * 8;
    if (c0 >= V) continue;
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = __expf(v[i][j] - lse) * g - (c0 + j == tt ? g : 0.f);
    if (c0 + 8 <= V) {
      Vec8<T>::store(z + c0, o);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (c0 + j < V) st1<T>(z + c0 + j, o[j]);
    }
  }
}

}  // namespace

hipError_t cross_entropy_fwd_bwd(int dtype, void* logits, int64_t rows, int V, int64_t ld, const int64_t* target,
                                 float* loss_rows, float* lse, const float* scale_ptr, float scale_mul,
                                 int64_t ignore_index, int write_grad, hipStream_t st, const float* bias) {
  if (rows == 0) return hipSuccess;
  if (V <= 0 || ld < V) return hipErrorInvalidValue;
  if (bias && reinterpret_cast<uintptr_t>(bias) % 16) return hipErrorInvalidValue;
  const int chunks = (V + 7) / 8;
  const bool aligned = ld % 8 == 0 && reinterpret_cast<uintptr_t>(logits) % 16 == 0;
  if (aligned && chunks <= 8 * kCeRegThreads) {
    const int nch = chunks <= kCeRegThreads ? 1 : chunks <= 2 * kCeRegThreads ? 2 : chunks <= 4 * kCeRegThreads ? 4 : 8;
    HYP_DISPATCH_FLOAT(dtype, T, {
      auto* k = nch == 1 ? ce_fwd_bwd_reg_k<T, 1> : nch == 2 ? ce_fwd_bwd_reg_k<T, 2>
                : nch == 4 ? ce_fwd_bwd_reg_k<T, 4> : ce_fwd_bwd_reg_k<T, 8>;
      hipLaunchKernelGGL(k, dim3((unsigned)rows), dim3(kCeRegThreads), 0, st, reinterpret_cast<T*>(logits), ld, bias,
                         target, loss_rows, lse, scale_ptr, scale_mul, V, ignore_index, write_grad);
    });
    return hipGetLastError();
  }
  HYP_DISPATCH_FLOAT(dtype, T, {
    hipLaunchKernelGGL(ce_fwd_bwd_k<T>, dim3((unsigned)rows), dim3(kCeThreads), 0, st, reinterpret_cast<T*>(logits),
                       ld, bias, target, loss_rows, lse, scale_ptr, scale_mul, V, ignore_index, write_grad);
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

// Host-side launcher declarations for every Hyperion gfx950 kernel.  Implementations live in
// csrc/kernels/*.hip (pure HIP, no torch headers); csrc/bindings/*.cpp wraps them for Python.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hyp_common.h"

namespace hyp {

// ---- bn_act.hip ----------------------------------------------------------------------------
// Statistics sums are [kStatSlots][2][C] fp64: producer block / tile b adds into slot b % kStatSlots,
// so a burst of tiles finishing together queues <= 1/kStatSlots of its atomics on any one 64-byte
// line (the memory-side atomic unit serializes per line: 784 layer1 tiles on one slot cost ~13 us);
// consumers sum the slots in fixed order.
constexpr int kStatSlots = 8;
// Training statistics are per-channel fp64 sums [kStatSlots][2][C] (Σx, Σx²) accumulated with atomics: every
// `sums` argument must point at ZEROED memory before its producer runs.  Consumers finalize inline.
hipError_t bn_stats(int dtype, const void* x, int64_t M, int C, double* sums, hipStream_t stream);
hipError_t bn_forward(int dtype, const void* x, const void* res, void* y, int64_t M, int C, const float* weight,
                      const float* bias, float* running_mean, float* running_var, float momentum, float eps,
                      int training, int act, double* sums, float* save_mean, float* save_invstd, float* scale,
                      float* shift, hipStream_t stream);
hipError_t bn_forward_from_sums(int dtype, const void* x, const void* res, void* y, int64_t M, int C,
                                const float* weight, const float* bias, float* running_mean, float* running_var,
                                float momentum, float eps, int act, const double* sums, float* save_mean,
                                float* save_invstd, hipStream_t stream);
// small-M one-launch backward (M <= 2048); 0 disables (A/B, tests)
void bn_set_small_paths(int on);
// y == nullptr with act: the ReLU mask is recomputed from x (training, no residual gradient only).
// sums: zeroed [kStatSlots][2][C] workspace for Σdz, Σdz·x.
hipError_t bn_backward(int dtype, const void* dy, const void* x, const void* y, void* dx, void* dres, int64_t M, int C,
                       const float* weight, const float* bias, const float* save_mean, const float* save_invstd,
                       int training, int act, double* sums, float* dweight, float* dbias, hipStream_t stream);
// dz already masked and its sums [kStatSlots][2][C] (Σdz, Σdz·x) complete: the dx pass only.
hipError_t bn_backward_dx(int dtype, const void* dz, const void* x, void* dx, int64_t M, int C, const float* weight,
                          const float* save_mean, const float* save_invstd, int training, const double* sums,
                          float* dweight, float* dbias, hipStream_t stream);

// ---- adam.hip ------------------------------------------------------------------------------
// param_dtype kF32: ptrs = [param, grad, m, v]; kBF16/kF16: ptrs = [lowp param, grad, m, v, fp32 master]
hipError_t adam_multi_tensor(int grad_dtype, int param_dtype, const int64_t* ptrs, const int64_t* sizes,
                             const int* blocks, int nblocks, int T, int chunk, float lr, float b1, float b2, float eps,
                             float wd, int adamw, const float* lr_t, const float* step_t, const float* inv_scale,
                             const float* found_inf, hipStream_t stream, int zero_grad = 0);
hipError_t unscale_multi_tensor(int grad_dtype, const int64_t* ptrs, const int64_t* sizes, const int* blocks,
                                int nblocks, int chunk, const float* inv_scale, float* found_inf, hipStream_t stream);
hipError_t sumsq_multi_tensor(int grad_dtype, const int64_t* ptrs, const int64_t* sizes, const int* blocks, int nblocks,
                              int chunk, float* partials, float* out, hipStream_t stream);
hipError_t copy_multi_tensor(int src_dtype, int dst_dtype, const int64_t* ptrs, const int64_t* sizes, const int* blocks,
                             int nblocks, int T, int chunk, hipStream_t stream);
hipError_t clip_multi_tensor(int grad_dtype, const int64_t* ptrs, const int64_t* sizes, const int* blocks, int nblocks,
                             int chunk, const float* total_sq, float max_norm, hipStream_t stream);

// ---- stream_bw.hip -------------------------------------------------------------------------
hipError_t stream_op(int op, const float* a, const float* b, float* c, float s, int64_t n, int nontemporal,
                     int blocks, hipStream_t stream);

}  // namespace hyp

namespace hyp {
// ---- layernorm.hip ---------------------------------------------------------------------------
bool layernorm_supported(int d);
void layernorm_bwd_geom(int64_t rows, int d, int* P, int* rows_per_wave);
// wt = 1: w / b (and dw / db) are in the activation dtype instead of fp32 (pointers reinterpreted)
// drop_p > 0 (d <= 2048; forward needs r): s = r + dropout(x) with the dropout.hip mask of *rs; the
// backward then also writes dxa = dropout(dx), the gradient of the dropped input.
void ln_set_waves(int waves);  // LayerNorm narrow-row grids: target wave count (0 = defaults)
hipError_t layernorm_forward(int dtype, int rms, const void* x, const void* r, void* s, void* y, const float* w,
                             const float* b, float* mean, float* rstd, int64_t rows, int d, float eps,
                             hipStream_t st, int wt = 0, float drop_p = 0.f, const struct RngState* rs = nullptr);
hipError_t layernorm_backward(int dtype, int rms, const void* dy, const void* xin, const float* w, const float* mean,
                              const float* rstd, const void* dres, void* dx, float* pdw, float* pdb, void* dw,
                              void* db, int64_t rows, int d, int P, int rows_per_wave, hipStream_t st, int wt = 0,
                              void* dxa = nullptr, float drop_p = 0.f, const struct RngState* rs = nullptr,
                              void* dbs = nullptr, int dbs_dtype = -1);
// dbs (d <= 2048): also Σ_rows of the branch gradient as stored (dxa when dropping, else dx) — the
// bias gradient of the linear layer that produced the norm's input, combined in the same launch as
// dγ / dβ.  dbs_dtype < 0: the weight dtype, at dw + d (no bias) or dw + 2d (with db); else any
// buffer of that dtype (the linear's bias dtype: no cast kernel when the norm keeps fp32 weights)
}  // namespace hyp

namespace hyp {
// ---- attention.hip ---------------------------------------------------------------------------
struct AttnParams {
  const void* q; const void* k; const void* v; void* o;
  int64_t sqb, sqs, sqh, skb, sks, skh, svb, svs, svh, sob, sos, soh;  // element strides (batch, seq, head)
  float* lse;            // [B*H, S] log2-domain log-sum-exp (may be null in inference)
  const uint8_t* kpm;    // [B, S] key padding mask, nonzero = ignore (may be null)
  int B, H, S, D;
  float scale_log2;      // softmax scale * log2(e)
  int causal;
  float p_drop;
  RngState rng;  // dropout stream (torch generator seed / offset; graph-safe)
};
struct AttnBwdParams {
  const void* q; const void* k; const void* v; const void* o; const void* dout;
  void* dq; void* dk; void* dv;
  int64_t sqb, sqs, sqh, skb, sks, skh, svb, svs, svh, sob, sos, soh;
  int64_t sdob, sdos, sdoh, sdqb, sdqs, sdqh, sdkb, sdks, sdkh, sdvb, sdvs, sdvh;
  const float* lse; float* delta; float* dq_acc;  // delta [B*H*S], dq_acc [B*H*S*D] fp32 workspaces
  int dq_slabs;  // > 0: dq_acc holds one fp32 dQ slab per key block (plain stores, no zeroing / atomics)
  int qsplit;         // S <= 128: query slices split over qsplit workgroups per (b, h) (few heads: fill the CUs)
  float* dkv_part;    // qsplit > 1: [qsplit][2 (dK, dV)][B*H][S][D] fp32 partials, summed by attn_bwd_kv_sum_k
  int rope; const float2* rope_cs;  // rope: dQ / dK through the inverse rotary embedding (D = 128, no
                                    // dropout); rope_cs [S][64] (cos, sin) of position x inv_freq(i)
  const uint8_t* kpm;
  int B, H, S, D;
  float scale, scale_log2;
  int causal;
  float p_drop;
  RngState rng;  // dropout stream (torch generator seed / offset; graph-safe)
};
bool attention_supported(int dtype, int D);
hipError_t attention_forward(int dtype, const AttnParams& p, hipStream_t st);
hipError_t attention_backward(int dtype, const AttnBwdParams& p, hipStream_t st);
void attn_set_fwd_narrow(int on);  // 1: one-wave forward workgroups when the default grid is < 128 (A/B)
}  // namespace hyp

namespace hyp {
// ---- cross_entropy.hip -----------------------------------------------------------------------
// In-place softmax-CE fwd+bwd over [rows, V] logits with leading dimension ld (elements).
// loss_rows[r] = lse - z[target] (0 for ignored rows); if write_grad, z <- (softmax - onehot) *
// (*scale_ptr) * scale_mul (rows with an ignored target get 0).  bias (fp32 [V], 16-byte aligned,
// optional): the logits are z + bias (the LM head's bias added here instead of in the GEMM).
hipError_t cross_entropy_fwd_bwd(int dtype, void* logits, int64_t rows, int V, int64_t ld, const int64_t* target,
                                 float* loss_rows, float* lse, const float* scale_ptr, float scale_mul,
                                 int64_t ignore_index, int write_grad, hipStream_t st, const float* bias = nullptr);
}  // namespace hyp

namespace hyp {
// ---- rope_swiglu.hip -------------------------------------------------------------------------
// q [tokens, Hq, D], k [tokens, Hk, D] with token / head strides in elements (unit stride in D);
// pos: int64 [tokens] or null (position = token % S).  inverse=1 rotates by -angle (backward).
hipError_t rope_apply(int dtype, const void* q, const void* k, void* qo, void* ko, int64_t tokens, int S, int Hq,
                      int Hk, int D, int64_t q_tok, int64_t k_tok, int64_t q_head, int64_t k_head, const int64_t* pos,
                      float theta, int inverse, hipStream_t st);
hipError_t swiglu_forward(int dtype, const void* g, const void* u, void* h, int64_t n, hipStream_t st);
hipError_t swiglu_backward(int dtype, const void* dh, const void* g, const void* u, void* dg, void* du, int64_t n,
                           hipStream_t st);
}  // namespace hyp

namespace hyp {
// ---- gemm_mfma.hip ---------------------------------------------------------------------------
// C[M,N] = alpha * A[M,K] · B[N,K]^T ; in bf16/f16, out f32/bf16/f16; 128x128 tiles, BK 32 or 64.
bool gemm_nt_supported(int M, int N, int K, int lda, int ldb, int bk);
hipError_t gemm_nt(int in_dtype, int out_dtype, const void* A, const void* B, void* C, int M, int N, int K, int lda,
                   int ldb, int ldc, float alpha, int bk, hipStream_t st);

// ---- gemm_f32.hip -----------------------------------------------------------------------------
// C = epi(alpha Σ_k A(m,k) B(n,k)) in fp32 on the fp32-input MFMA (exact fp32 products / accumulation).
// A(m,k) at A + m*lda + k (a_tr = 0) or A + k*lda + m (a_tr = 1), B likewise; epi: + beta*C_old,
// + bias[n], ReLU.  Any M, N; row-form operands K % 4, tr-form operands M / N % 4, ld % 4.
// splits / shape (0: 128x128, 1: 256x64, 2: 64x256) < 0: the cost-model plan; split-K needs
// part = fp32 [splits * M * N] (gemm_f32_splits).
bool gemm_f32_supported(int M, int N, int K, bool a_tr, bool b_tr, int lda, int ldb, int ldc);
int gemm_f32_splits(int M, int N, int K, int splits, int shape);
hipError_t gemm_f32(const float* A, const float* B, float* C, float* part, const float* bias, const float* zero,
                    int M, int N, int K, bool a_tr, bool b_tr, int lda, int ldb, int ldc, float alpha, float beta,
                    int relu, int splits, int shape, hipStream_t st);
// NHWC fp32 im2col (cols [Nb*Ho*Wo, Kp], column (r*S + s)*C + c, pad columns zero) and its adjoint
// (a deterministic per-input gather over the taps)
hipError_t im2col_f32(const float* x, float* cols, int Nb, int H, int W, int C, int Ho, int Wo, int R, int S, int sh,
                      int sw, int ph, int pw, int Kp, hipStream_t st);
hipError_t col2im_f32(const float* dcols, float* dx, int Nb, int H, int W, int C, int Ho, int Wo, int R, int S, int sh,
                      int sw, int ph, int pw, int Kp, hipStream_t st);

// ---- gemm_tiles.hip --------------------------------------------------------------------------
// C[M,N] = epi(alpha Σ_k A(m,k) B(n,k)); A(m,k) at A + m*lda + k (a_tr = 0) or A + k*lda + m (a_tr = 1),
// B likewise.  epi: + beta*C_old, + bias[n] (bias_dtype), aux = pre-activation, act (0 none, 1 relu,
// 2 gelu-erf, 3 gelu-tanh), + R[m,n] (ldr), in out_dtype.  tile/splits < 0: automatic plan; split-K
// needs part = fp32 [splits * M * N] (gemm_tiled_splits).  N % 4, K % 8, ld % 8; tr operands: M/N % 8.
struct GemmTiledArgs {
  int in_dtype = kBF16, out_dtype = kBF16, bias_dtype = kF32;
  const void* A = nullptr;
  const void* B = nullptr;
  void* C = nullptr;
  void* aux = nullptr;
  const void* bias = nullptr;
  const void* R = nullptr;
  const void* zero = nullptr;
  float* part = nullptr;
  int M = 0, N = 0, K = 0, lda = 0, ldb = 0, ldc = 0, ldr = 0;
  bool a_tr = false, b_tr = false;
  int act = 0;
  float alpha = 1.f, beta = 0.f;
  int tile = -1, splits = -1;
  // drop_p > 0 (with act): the stored output is dropout(act(z)) with dropout.hip's mask of drng
  // (element index row * ldc + col); aux keeps z
  float drop_p = 0.f;
  RngState drng{};
  // rows of a row-form B operand when fewer than N (0 = N): output columns past them are computed
  // from zeros (the LM head's class padding: N = ceil8(V) columns from V weight rows)
  int b_rows = 0;
};
void gemm_tiled_plan(int M, int N, int K, int* tile, int* splits);
void gemm_tiled_plan_layout(int M, int N, int K, bool a_tr, bool b_tr, int* tile, int* splits);
// split-K reduce in the last-arriving workgroup of each tile (1) or a separate kernel (0, default)
void gemm_set_splitk_inkernel(int on);
int gemm_tiled_splits(const GemmTiledArgs& a);
hipError_t gemm_tiled(const GemmTiledArgs& a, hipStream_t st);
}  // namespace hyp

namespace hyp {
// ---- conv_igemm.hip --------------------------------------------------------------------------
// NHWC implicit-GEMM conv (bf16/f16), optional BN-statistics epilogue: per-channel Σy (psum[K]) and
// Σy² (psq = psum + K; fp64, slots of stride 2K: bn_act.hip layout) of the rounded outputs, ADDED atomically (zero them first); with splits > 1 the
// stats come from the split-K reduce.
bool conv_fwd_supported(int C, int K);
void conv_set_stages(int nb);        // LDS pipeline depth 2..4 (0 = automatic); tuning only
void conv_set_xf_debug(int bits);    // XF diagnostics: 1 skip the transform, 2 the finalize, 4 the side store
void conv_wgrad_set_stages(int nb);
void conv_fwd_tile(int M, int K, int* bm, int* bn);
// addend (optional, splits == 1, no stats): out [M, K] += addend after rounding (fused residual grad).
// dgrad != 0: stride-1 data gradient; "in" is dY [N,H,W,C], "w" the ORIGINAL filter [C][R][S][K]
// (read flipped and transposed in-kernel), (ph, pw) the dgrad padding R-1-p.
// bnb (dgrad only): the BatchNorm-backward epilogue above (any split count).
// Training BatchNorm + ReLU of the conv's INPUT, applied as its A operand is read (forward only):
// the conv reads the producer's raw conv output x and computes with relu(x * scale + shift),
// scale / shift finalized inline from the producer's statistics sums (bn_fin.h arithmetic; the
// workgroup with blockIdx 0 also writes save_mean / save_invstd and the running statistics).
// out (optional): the transformed activation [N, H, W, C] is stored there as a side output —
// by the workgroups of the first output-channel tile, at the filter's centre tap, which covers
// every input pixel exactly once when stride == 1 and the padding is (R-1)/2, (S-1)/2.
struct ConvInXform {
  const double* sums = nullptr;  // [kStatSlots][2][C] Σx, Σx² of the producer
  const float* weight = nullptr;
  const float* bias = nullptr;
  float* running_mean = nullptr;
  float* running_var = nullptr;
  float momentum = 0.1f, eps = 1e-5f;
  float* save_mean = nullptr;
  float* save_invstd = nullptr;
  void* out = nullptr;
};
constexpr int kXfMaxC = 512;  // input channels of a transformed conv (the scale / shift table in LDS)

struct DualWgrad;
hipError_t conv_fwd(int dtype, const void* in, const void* w, void* out, const void* zero, double* psum, double* psq,
                    int N, int H, int W, int C, int K, int P, int Q, int R, int S, int sh, int sw, int ph, int pw,
                    int bm, int bn, int dgrad, int splits, float* part, hipStream_t st, float alpha = 1.f,
                    const struct SplitkEpilogue* ep = nullptr, const void* addend = nullptr,
                    const struct BnBwdEpilogue* bnb = nullptr, int pix = 0, int dgrad_stride = 1, int Hx = 0,
                    int Wx = 0, int nb = 0, const ConvInXform* xf = nullptr, const DualWgrad* dual = nullptr);
// dgrad_stride 2 (dgrad only, no split-K / alpha / rank-r epilogue): the stride-2 data gradient as its
// 4 output-phase sub-convolutions in one launch; (H, W, P, Q) are dY's (H, W) and the phase grid
// (P, Q) = (Hx / 2, Wx / 2) of dX [N, Hx, Wx, K], (ph, pw) the FORWARD padding, w the original filter.
// pix (conv_fwd / conv_wgrad): the input's pixel stride in elements when it differs from the
// 64-multiple reduction slice C (0 = C) — the stem's space-to-depth input (stem.hip): 16-channel
// pixels read as 64-element runs of 4 adjacent pixels.
// Fused linear + cross-entropy epilogues of the implicit-GEMM kernel (linear_ce below).
struct CeEpilogue {
  const float* bias = nullptr;      // [V] fp32 or null, indexed by vocabulary index
  const int64_t* target = nullptr;  // [M]
  int64_t ignore = -100;
  int col_off = 0;                  // vocabulary index of the chunk's first class
  float2* part = nullptr;           // mode 1: [tiles_n][M] (row max, row Σexp)
  float* zt = nullptr;              // mode 1: [M] target logit (written by the tile holding it)
  const float* lse = nullptr;       // mode 2: [M]
  const float* scale = nullptr;     // mode 2: device scalar (1 / non-ignored rows)
};
hipError_t linear_ce(int dtype, int mode, const void* x, const void* w, void* out, const void* zero, int M, int E,
                     int kcols, int kvalid, const CeEpilogue& ce, hipStream_t st, int bn = 64);
// lse[m] = log-sum-exp of the tiles' partials; loss_rows[m] = lse - zt (0 for ignored rows)
hipError_t ce_lse_combine(const float2* part, int tiles, int M, const float* zt, const int64_t* target,
                          int64_t ignore, float* lse, float* loss_rows, hipStream_t st);
// Optional BatchNorm-backward epilogue of a stride-1 data gradient dX whose tensor is the output of a
// fused BN(+residual)(+ReLU) layer: the stored value becomes dz = dX·mask (the BN input's upstream
// gradient), and Σdz, Σdz·x per channel are added into `sums` — bn_backward_dx then needs no reduce
// pass (ops/conv.py BNGradLink).
struct BnBwdEpilogue {
  const void* x = nullptr;  // [M, K] the BN layer's input (its conv output)
  const void* y = nullptr;  // [M, K] the BN layer's output (mode 2 mask source)
  const float* w = nullptr;  // mode 1 mask: x * (w*invstd) + (b - mean*w*invstd) > 0
  const float* b = nullptr;
  const float* mean = nullptr;
  const float* invstd = nullptr;
  int mode = 0;              // 0: no mask (no ReLU); 1: ReLU mask recomputed from x; 2: mask y > 0
  double* sums = nullptr;    // [kStatSlots][2][K] Σdz, Σdz·x (zeroed)
};
// Optional rank-r epilogue of a split-K reduce over an [M, N] output:
//   out[m, n] += beta * (mask ? mask[m, n] : 1) * sum_j U[m, j] * V[j * sv_j + n * sv_n]
// (U, V, mask in the output dtype).  U == nullptr: no epilogue.
struct SplitkEpilogue {
  const void* U = nullptr;
  const void* V = nullptr;
  const void* mask = nullptr;
  int64_t sv_j = 0, sv_n = 0;
  int N = 0, r = 0;
  float beta = 1.f;
  // per-column affine (+ residual) (+ ReLU) — the eval-mode BatchNorm folded into the epilogue:
  // out[m, n] = act(round(acc) * scale[n] + shift[n] (+ residual[m, n]))   (no rank-r term)
  const float* scale = nullptr;
  const float* shift = nullptr;
  const void* residual = nullptr;
  int act = 0;
};
// out (T) = alpha * sum over `splits` fp32 partial slabs of n elements (fixed order; n % 4 == 0)
// [+ the rank-r epilogue]
hipError_t splitk_reduce(int dtype, const float* part, void* out, int64_t n, int splits, hipStream_t st,
                         float alpha = 1.f, const SplitkEpilogue* ep = nullptr);
// Split-K reduce of a conv forward's [splits, M, K] fp32 partials into out [M, K] (T) plus the BN
// statistics of the rounded outputs, added atomically into psum[K] / psq[K] (kStatRows-row blocks).
constexpr int kStatRows = 64;  // (16 when that leaves < 512 blocks)
hipError_t splitk_reduce_stats(int dtype, const float* part, void* out, int M, int K, int splits, double* psum,
                               double* psq, hipStream_t st);
// Split-K reduce of a data gradient [splits, M, K] (+ addend [M, K] in T) with the BN-backward
// epilogue: out = dz = round(round(Σ part) + addend) · mask, Σdz, Σdz·x into bnb.sums.
hipError_t splitk_reduce_bnb(int dtype, const float* part, void* out, const void* addend, int M, int K, int splits,
                             const BnBwdEpilogue& bnb, hipStream_t st);
// Split-K plan for a convolution (forward or stride-1 dgrad) whose bm x bn tiling leaves fewer than
// ~2 workgroups per CU: returns splits >= 1 over the nk = R*S*C/64 reduction steps.
int conv_fwd_splits(int M, int K, int nk, int bm, int bn);
// ---- conv_wgrad.hip --------------------------------------------------------------------------
// NHWC conv weight gradient on MFMA (split-K over pixels; fp32 partials [splits, K, R*S*C] when
// splits > 1, reduced + cast into dw by a second kernel).
bool conv_wgrad_supported(int C, int K);
void conv_wgrad_plan(int M, int K, int C, int R, int S, int* bm, int* bn, int* splits, int* steps_per_split);
// A weight gradient's split-K reduce (out = alpha * Σ_s part[s] in dtype) deferred into the NEXT
// conv_wgrad launch, which runs it in extra workgroups beside its own tiles (one launch less per
// layer; ops/conv.py chains them and flushes the last one at the end of backward).
struct WgradPendingReduce {
  const float* part;
  void* out;
  int64_t n;
  int splits;
  float alpha;
  int dtype;
  int blocks;  // filled by conv_wgrad
};
hipError_t conv_wgrad(int dtype, const void* dy, const void* x, void* dw, float* partials, const void* zero, int N,
                      int H, int W, int C, int K, int P, int Q, int R, int S, int sh, int sw, int ph, int pw, int bm,
                      int bn, int splits, int steps_per_split, hipStream_t st, float alpha,
                      const WgradPendingReduce* pending = nullptr, bool defer_reduce = false, int pix = 0);
// ---- conv_dual.hip ---------------------------------------------------------------------------
// A stride-1 / stride-2 data gradient and a weight gradient of the SAME backward step in ONE launch
// (horizontal fusion): both consume dY, neither consumes the other, and the ResNet backward runs
// them as ~50 latency-bound pairs.  The weight gradient runs 64 x 64 tiles (split-K over pixels,
// its reduce deferred or run by the pending-reduce workgroups as with conv_wgrad).
struct WgradArgs;
struct DualWgrad {
  const void* dy = nullptr;   // [N, P, Q, K] the weight gradient's output gradient (usually the dgrad's dY)
  const void* x = nullptr;    // [N, H, W, C] the conv's input
  void* dw = nullptr;         // [K, R, S, C] in dtype
  float* partials = nullptr;  // [splits, K, R*S*C] when splits > 1
  int N = 0, H = 0, W = 0, C = 0, K = 0, P = 0, Q = 0, R = 0, S = 0, sh = 1, sw = 1, ph = 0, pw = 0;
  int bm = 64, bn = 64;                  // weight-gradient tile (bn_wgrad.hip: 64 / 128 each; conv_dual: 64)
  int splits = 0, steps_per_split = 0;  // pixel split (conv_wgrad_plan's rule)
  const WgradPendingReduce* pending = nullptr;  // an earlier weight gradient's deferred reduce
  bool defer_reduce = false;                    // leave THIS gradient's reduce pending
  int order = 0;  // 0: the two gradients' workgroups interleaved in 8-wide groups; 1: dgrad first
};
// Fill a WgradArgs for the weight gradient d (the checks of conv_wgrad); no launch.
hipError_t conv_wgrad_prepare(WgradArgs* a, int dtype, const DualWgrad& d, const void* zero);
// conv_fwd(..., dual): the data gradient's launch carries the weight gradient `dual` (bf16, a data
// gradient without split-K); any other case launches the two separately (same results).
// A/B: -1 = each DualWgrad's own order, 0 interleaved, 1 data gradient first
void conv_dual_set_order(int order);
// persistent conv launches (conv_persist.h) for the variants they cover: 0 off, 1 on
void conv_set_persist(int on);
void conv_set_group(int mode);  // tile-order group: 0 model, > 0 fixed, -1 x2, -2 x0.5 (A/B)
// BN apply / dx pass grid (bn_act.hip): row-block cap and minimum row iterations per thread
int bn_apply_blocks();
int bn_min_iters();
void bn_set_geom(int apply_blocks, int min_iters);
// bn_wgrad.hip: the BatchNorm backward dx pass of a layer (bn_backward_dx's arguments) and the weight
// gradient d of the conv ABOVE it (whose dY the previous backward step produced) in ONE launch —
// the cheap, memory-bound dx pass runs beside the weight gradient's K loops instead of alone
// between two data gradients.  bf16 only (else hipErrorNotSupported: nothing launched).
hipError_t bn_backward_dx_wgrad(int dtype, const void* dz, const void* x, void* dx, int64_t M, int C,
                                const float* weight, const float* save_mean, const float* save_invstd, int training,
                                const double* sums, float* dweight, float* dbias, const DualWgrad& d,
                                const void* zero, hipStream_t stream);
}  // namespace hyp

namespace hyp {
// ---- reduce.hip ------------------------------------------------------------------------------
// Column sums of a row-major [M, N] matrix (bias gradients): P partial rows (colsum_partials) in
// `part` [P, N] fp32, then combined into out[N] (out_dtype).  N % 8 == 0, 16-byte aligned x.
int colsum_partials(int64_t M, int N);
// the partial count of the one-launch (last-arriver) combine, and its cap (0 = two launches)
int colsum_partials_fused(int64_t M, int N);
int act_colsum_partials(int64_t M, int N);  // act_bwd_colsum's P (more row blocks than colsum_partials)
void colsum_set_act_wgs(int wgs);
void colsum_set_fused(int max_p);
int colsum_fused_max_p();
// loss = mean((x - t)^2) (fp32 scalar) and g = 2 (x - t) / n in x's dtype; one block (small n)
hipError_t mse_fwd_bwd(int dtype, const void* x, const float* t, int64_t n, float* loss, void* g, hipStream_t st);
// classifier head + MSE (linear_mse.hip), M <= 64, K % 8 == 0.  Forward writes the fp32 gradient
// dz [M, N] and the loss; backward writes dX [M, K], dW [N, K] and db [N] (optional) scaled by the
// device scalar go.  ws: linear_mse_workspace(M, N, K) floats (slice partials, combined by their
// own launches in a fixed order: deterministic)
int linear_mse_partials(int N);
int64_t linear_mse_workspace(int M, int N, int K);
hipError_t linear_mse_fwd(int dtype, const void* X, const void* W, const void* b, const float* y, int M, int N, int K,
                          float* dz, float* ws, float* loss, hipStream_t st);
hipError_t linear_mse_bwd(int dtype, const float* dz, const float* go, const void* X, const void* W, int M, int N,
                          int K, void* dX, void* dW, void* db, float* ws, hipStream_t st);
// tickets (non-null): ceil(N / 512) zeroed int32 slots — the combine runs in the same launch (the
// last-arriving block of each column slab; the slots are reset to zero on exit)
hipError_t column_sum(int dtype, const void* x, int64_t M, int N, void* out, int out_dtype, float* part, int P,
                      hipStream_t st, int* tickets = nullptr);
hipError_t colsum_combine(const float* part, int P, int N, void* out, int out_dtype, hipStream_t st);
// columns [0, split) into out (out_dtype), [split, N) into out2 (out2_dtype); split % 4 == 0
hipError_t colsum_combine_split(const float* part, int P, int N, void* out, int out_dtype, int split, void* out2,
                                int out2_dtype, hipStream_t st);
// dy = dh·act'(z) (act 1: ReLU with z = output; 2: exact GELU with z = pre-activation) and its column
// sums into db (out_dtype; null: skip) — the FFN activation backward + bias gradient.
// drop_p > 0: dh is the gradient of dropout(act(z)) (dropout.hip mask of *rs, element index r*N + c)
hipError_t act_bwd_colsum(int dtype, int act, const void* dh, const void* z, void* dy, int64_t M, int N, void* db,
                          int out_dtype, float* part, int P, hipStream_t st, float drop_p = 0.f,
                          const RngState* rs = nullptr, int* tickets = nullptr);
}  // namespace hyp

namespace hyp {
// ---- pool.hip --------------------------------------------------------------------------------
// NHWC max pool (idx: per-element window tap, uint8) and global average pool; C % 8 == 0.
hipError_t maxpool2d_forward(int dtype, const void* x, void* y, uint8_t* idx, int N, int H, int W, int C, int k,
                             int s, int pad, hipStream_t st);
hipError_t maxpool2d_backward(int dtype, const void* dy, const uint8_t* idx, void* dx, int N, int H, int W, int C,
                              int k, int s, int pad, hipStream_t st);
hipError_t global_avgpool_forward(int dtype, const void* x, void* y, int N, int HW, int C, hipStream_t st);
// diagnostic: per-workgroup timeline of the next conv_fwd launches (6 u64 per workgroup; null = off)
void conv_set_stamps(void* buf);
// ---- stem.hip: the 7x7/s2/p3 stem (C <= 4) as a stride-1 R=4 x S=1 conv with pixel stride 16:
// Xs [N, Hs = P + 3, Ws = Q + 3, 16] (space-to-depth) from x [N, H, W, C] (both channels-last)
hipError_t stem_s2d(int dtype, const void* x, void* out, int N, int H, int W, int C, int Hs, int Ws, hipStream_t st);
// W [K, C, 7, 7] (element strides sk, sc, sr, sq) -> W4 channels-last [K, 64, 4, 1]; and back for dW
hipError_t stem_weight4(int dtype, const void* w, void* w4, int K, int C, int64_t sk, int64_t sc, int64_t sr,
                        int64_t sq, hipStream_t st);
hipError_t stem_weight4_grad(int dtype, const void* dw4, void* dw, int K, int C, int64_t sk, int64_t sc, int64_t sr,
                             int64_t sq, hipStream_t st);
// out[N,H,W,C] = addend (optional) + comp[N,P,Q,C] scattered to pixels (p*sh, q*sw), zeros elsewhere
hipError_t upsample_add(int dtype, const void* comp, const void* addend, void* out, int N, int H, int W, int C, int P,
                        int Q, int sh, int sw, hipStream_t st);
hipError_t global_avgpool_backward(int dtype, const void* dy, void* dx, int N, int HW, int C, hipStream_t st);
}  // namespace hyp

namespace hyp {
// ---- embedding.hip ---------------------------------------------------------------------------
hipError_t embedding_forward(int dtype, const int64_t* ids, const void* w, void* out, int64_t n, int E, int64_t V,
                             hipStream_t st);
// dw32: zeroed [V, E] fp32 accumulator (the result for f32 weights); dw: output in the weight dtype
hipError_t embedding_backward(int dtype, const int64_t* ids, const void* dy, float* dw32, void* dw, int64_t n, int E,
                              int64_t V, int64_t pad_idx, hipStream_t st);
}  // namespace hyp

namespace hyp {
// ---- dropout.hip -----------------------------------------------------------------------------
// mode 0: out = keep ? x / (1 - p) : 0 (also the backward on dy with the same state); mode 1: out =
// the scaled keep mask keep / (1 - p).  keep = rng_u32(rng_key(rs), element index) >= p·2^32.
hipError_t dropout_apply(int dtype, int mode, const void* x, void* out, int64_t n, float p, const RngState& rs,
                         hipStream_t st);
}  // namespace hyp

namespace hyp {
// ---- wstream.hip -----------------------------------------------------------------------------
// Weight-streaming GEMM for few-token activations: x slice resident in LDS, W streamed to VGPRs.
// nn = false: y = x Wᵀ (W [N, K]); nn = true: y = x W (W [K, N]).  Writes fp32 partial slabs
// [S][MB*mf][N/16][64][4] (fragment order; sb = 1: bf16 elements); ws_reduce sums them (+ epilogue) into [M, N].
bool ws_supported(int M, int N, int K, bool nn);
void ws_set_depth(int d);  // weight-streaming GEMM: k-steps in flight per wave (4 default, or 8)
void ws_plan(int M, int N, int K, bool nn, int* mf, int* kr, int* G, int* nf);
hipError_t ws_gemm(int dtype, bool nn, const void* x, int64_t ldx, const void* w, int64_t ldw, float* part,
                   const void* zero, int M, int N, int K, int mf, int kr, int G, int nf, hipStream_t st, int sb = 0);
// out[m, n] = alpha Σ_s part + beta addend[m, n] + uscale Σ_r U[m, seg r + rr] V[n, rr] (seg = n / segw)
hipError_t ws_reduce(int dtype, bool nn, const float* part, void* out, int64_t ldo, const void* addend, float alpha,
                     float beta, const float* U, const void* V, int r, int segw, float uscale, int M, int N, int S,
                     int MFtot, hipStream_t st, int sb = 0);
// Fused epilogues of the slabs (see wstream.hip): 0 plain, 1 LoRA up (+ RoPE), 2 SwiGLU fwd,
// 3 SwiGLU bwd (NN), 4 LoRA data gradient (NN).  part == null: the GEMM result is the row-major
// yin [M, N] (a vendor GEMM's output) instead of slabs.
hipError_t ws_epilogue(int dtype, int epi, const float* part, int S, int MFtot, int M, int N, void* out, int64_t ldo,
                       void* out2, int64_t ldo2, const void* aux, int64_t ld_aux, const float* t, int ldt,
                       int64_t t_sstride, int t_splits, const void* const* lw, int P, int r, int segw, float lscale,
                       int rope_segs, int seq, float theta, const RngState* rng, float p_drop, bool nn,
                       const void* yin, int64_t ldy, hipStream_t st, int sb = 0);
}  // namespace hyp

namespace hyp {
// ---- lora_fused.hip --------------------------------------------------------------------------
// rank-r halves of the fused LoRA projections (P projections sharing one input; see the file).
// t and du: fp32 split-partial stacks [splits][M][ld] (slice stride sstride; splits = 1: a plain
// [M, ld] matrix): producers write one slice per split, consumers sum the slices.
// K % 32 == 0 (lora_down), N % 64 == 0 (lora_bwd_t), K % 64 == 0 (lora_bwd_a).
hipError_t lora_down(int dtype, const void* x, int64_t ldx, const void* const* A, int P, int r, float* t, int ldt,
                     int64_t t_sstride, int t_splits, int M, int K, const RngState* rng, float p_drop, hipStream_t st);
hipError_t lora_bwd_t(int dtype, const void* dy, int64_t ldy, int N, const void* const* B, void* const* dB, int P,
                      int r, const float* t, int ldt, int64_t t_sstride, int t_splits, float* du, int ldu,
                      int64_t du_sstride, int du_splits, int M, float c, hipStream_t st);
hipError_t lora_bwd_a(int dtype, const void* x, int64_t ldx, int K, void* const* dA, int P, int r, const float* du,
                      int ldu, int64_t du_sstride, int du_splits, int M, const RngState* rng, float p_drop,
                      hipStream_t st);
}  // namespace hyp

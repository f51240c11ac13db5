// NHWC convolution WEIGHT gradient on gfx950 MFMA (split-K implicit GEMM).
//
// Reference: ResNet-50/18 weight gradients ran through MIOpen's `igemm_wrw` / CK batched-GEMM
// solvers plus their zero-fill and cast kernels (3-4 launches per conv; SURVEY §2.4
// "Convolution + BatchNorm + ReLU" backward, §2.5 ResNet rows).  Here
//
//   dW[k, r, s, c] = Σ_{m = (n,p,q)} dY[m, k] · X[n, p*sh + r - ph, q*sw + s - pw, c]
//
// is a GEMM with rows = output channels k, columns = (r, s, c) in the channels-last filter's own
// order, and a reduction over the N·P·Q output pixels.  BOTH operands have the reduction (pixel)
// dimension strided in memory — dY rows and input pixels are channel-contiguous — so tiles are
// staged pixel-major straight from HBM with 16-byte global_load_lds (a pixel's BM/BN-channel run
// is one contiguous row), and the MFMA operands are read back TRANSPOSED with gfx950's
// ds_read_b64_tr_b16 (guide T10): no register transpose, no ds_permute.
//
// LDS image per operand: [64 pixels][W channels] with W*2-byte rows and an XOR swizzle of the
// 16-byte chunks chosen so every 32-lane half of a transposed read touches 64 distinct banks
// (rows 0..7 of a read half land on disjoint chunk pairs).  The pixel <-> MFMA k-slot mapping is
// free (both operands sum over the same pixels), so each 16-lane group reads 4 consecutive rows.
//
// Work split: tiles BM x BN (k x c) of one filter tap, 4 waves as 2 x 2, 16x16x32 bf16/f16 MFMA;
// the pixel reduction is split over `splits` workgroups (the outputs of a ResNet wgrad are small —
// 64 x 576 for a layer1 3x3 — while the reduction is up to 10^5 pixels long).  splits == 1 stores
// the result in the parameter dtype; otherwise fp32 partials [splits][K][R·S·C] are summed (in a
// fixed order: deterministic) and cast by conv_wgrad_reduce_k.
#include "hyp_common.h"
#include "hyp_kernels.h"
#include "mfma_lds.h"

namespace hyp {
namespace {

using namespace mfl;

constexpr int kBP = 64;  // pixels (reduction) per LDS stage
constexpr int kThreads = 256;

struct WgradArgs {
  const uint16_t* dy;    // [M, K]   (M = N*P*Q output pixels, channels-last)
  const uint16_t* x;     // [N, H, W, C]
  void* out;             // splits == 1: dW [K, R, S, C] in T; else fp32 partials [splits, K, R*S*C]
  const uint16_t* zero;  // >= 1 KiB of zeros
  int N, H, W, C, K, P, Q, R, S, sh, sw, ph, pw;
  int M, splits, steps_per_split;
  uint64_t mq, mpq;  // magic multipliers: floor(m / Q) = (m * mq) >> 36 (same for P*Q)
  float alpha;       // output scale (splits == 1: applied in the store; else in the reduce)
};

// floor(x / d) with magic = ceil(2^36 / d): exact while x * d < 2^36 (host: M < 2^22, P*Q < 2^14)
__device__ __forceinline__ int fdiv(int x, uint64_t magic) { return (int)(((uint64_t)(uint32_t)x * magic) >> 36); }

template <typename T, int BM, int BN, int NB>
__global__ __launch_bounds__(kThreads) void conv_wgrad_k(const WgradArgs a) {
  constexpr int FM = BM / 32, FN = BN / 32;          // 16x16 fragments per wave (wave tile BM/2 x BN/2)
  constexpr int IA = BM / 32, IB = BN / 32;          // glds per wave per stage (8-row blocks)
  constexpr int CA = BM / 8, CB = BN / 8;            // 16-byte chunks per image row
  constexpr int kBuf = (BM + BN) * kBP;
  __shared__ __attribute__((aligned(16))) uint16_t smem[NB * kBuf];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  const int RSC = a.R * a.S * a.C;
  const int tiles_k = (a.K + BM - 1) / BM, tiles_c = RSC / BN, ntiles = tiles_k * tiles_c;
  const int nwg = ntiles * a.splits;
  int bid = blockIdx.x;
  bid = xcd_remap(bid, nwg);  // consecutive logical tiles (same pixel split) share an XCD's L2
  const int split = bid / ntiles, tile = bid - split * ntiles;
  const int tk = tile % tiles_k, tc = tile / tiles_k;
  const int k0 = tk * BM;
  const int col0 = tc * BN;               // column in (r, s, c) order; BN | C so one tap per tile
  const int rs = col0 / a.C, c0 = col0 - rs * a.C;
  const int r = rs / a.S, s = rs - r * a.S;
  const int mbeg = split * a.steps_per_split * kBP;
  const int nsteps = min(a.steps_per_split, (a.M - mbeg + kBP - 1) / kBP);

  // ---- per-lane staging bookkeeping: lane covers image row (i*4 + wave)*8 + lane/CA ... for the
  // A (dY) image, a wave instruction writes 1024 B = 1024 / (2*BM) rows.
  constexpr int RA = 1024 / (2 * BM), RB = 1024 / (2 * BN);  // rows per wave instruction
  int a_row[IA], a_col[IA], b_row[IB], b_col[IB];
#pragma unroll
  for (int i = 0; i < IA; ++i) {
    const int row = (i * 4 + wave) * RA + lane / CA;
    const int slot = lane % CA;
    a_row[i] = row;
    a_col[i] = k0 + ((slot ^ swz_tr<BM>(row)) << 3);
  }
#pragma unroll
  for (int i = 0; i < IB; ++i) {
    const int row = (i * 4 + wave) * RB + lane / CB;
    const int slot = lane % CB;
    b_row[i] = row;
    b_col[i] = c0 + ((slot ^ swz_tr<BN>(row)) << 3);
  }
  const uint16_t* zero = a.zero;

  auto stage = [&](int t, uint16_t* buf) {
    const int mb = mbeg + t * kBP;
#pragma unroll
    for (int i = 0; i < IA; ++i) {
      const int m = mb + a_row[i];
      const bool ok = m < a.M && a_col[i] < a.K;
      glds16(ok ? a.dy + (int64_t)m * a.K + a_col[i] : zero, buf + (i * 4 + wave) * 512);
    }
#pragma unroll
    for (int i = 0; i < IB; ++i) {
      const int m = mb + b_row[i];
      const int n = fdiv(m, a.mpq), pq = m - n * a.P * a.Q;
      const int p = fdiv(pq, a.mq), q = pq - p * a.Q;
      const int h = p * a.sh + r - a.ph, w = q * a.sw + s - a.pw;
      const bool ok = m < a.M && (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W;
      glds16(ok ? a.x + (((int64_t)n * a.H + h) * a.W + w) * a.C + b_col[i] : zero,
             buf + BM * kBP + (i * 4 + wave) * 512);
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // NB-deep ring (see mfma_lds.h wait_stage): stage t+NB-1 is issued after the barrier that
  // retires stage t-1's buffer
#pragma unroll
  for (int i = 0; i < NB - 1; ++i)
    if (i < nsteps) stage(i, smem + i * kBuf);
  for (int t = 0; t < nsteps; ++t) {
    wait_stage<IA + IB, NB>(min(NB - 2, nsteps - 1 - t));
    barrier_keep_vm();
    if (t + NB - 1 < nsteps) stage(t + NB - 1, smem + ((t + NB - 1) % NB) * kBuf);
    const uint16_t* as = smem + (t % NB) * kBuf;
    const uint16_t* bs = as + BM * kBP;
#pragma unroll
    for (int ks = 0; ks < kBP / 32; ++ks) {
      u16x8 fa[FM], fb[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) fa[i] = frag_tr<BM>(as, ks * 32, wm * (BM / 2) + i * 16, lane);
#pragma unroll
      for (int j = 0; j < FN; ++j) fb[j] = frag_tr<BN>(bs, ks * 32, wn * (BN / 2) + j * 16, lane);
      lds_reads_done();  // the asm transposed reads (see mfma_lds.h) have returned
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mma16<T>(fa[i], fb[j], acc[i][j]);
    }
  }

  // ---- epilogue: acc[i][j][e] = dW[k0 + wm*BM/2 + i*16 + (lane>>4)*4 + e][col0 + wn*BN/2 + j*16 + (lane&15)]
  const int r16 = lane & 15, c4 = lane >> 4;
  if (a.splits == 1) {
    T* out = reinterpret_cast<T*>(a.out);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = k0 + wm * (BM / 2) + i * 16 + c4 * 4 + e;
        if (k < a.K) {
#pragma unroll
          for (int j = 0; j < FN; ++j)
            st1<T>(out + (int64_t)k * RSC + col0 + wn * (BN / 2) + j * 16 + r16, a.alpha * acc[i][j][e]);
        }
      }
  } else {
    float* out = reinterpret_cast<float*>(a.out) + (int64_t)split * a.K * RSC;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = k0 + wm * (BM / 2) + i * 16 + c4 * 4 + e;
        if (k < a.K) {
#pragma unroll
          for (int j = 0; j < FN; ++j) out[(int64_t)k * RSC + col0 + wn * (BN / 2) + j * 16 + r16] = acc[i][j][e];
        }
      }
  }
}

// out = alpha * Σ_s part[s] (fixed order: deterministic), cast to T; 4 elements per thread
// (16-byte loads).  Optional rank-r epilogue (the LoRA update fused into the base GEMM's reduce):
//   out[m, n] += beta * (mask ? mask[m, n] : 1) * Σ_j U[m, j] · V[j * sv_j + n * sv_n]
// with U [M, r] and V any 2D view (B of y += t·Bᵀ is V = Bᵀ: sv_j = 1, sv_n = r).
// 64-thread blocks (a wgrad output can be only 37K floats: 256-thread blocks left ~36 workgroups
// on 256 CUs) and 4 independent accumulators, so 4 slab loads are in flight per thread.
constexpr int kRedThreads = 64;

template <typename T, bool LOWRANK, bool AFF>
__global__ __launch_bounds__(kRedThreads) void splitk_reduce_k(const float* __restrict__ part, T* __restrict__ out,
                                                               int64_t n, int splits, float alpha, SplitkEpilogue ep) {
  const int64_t i4 = ((int64_t)blockIdx.x * kRedThreads + threadIdx.x) * 4;
  if (i4 >= n) return;
  const f32x4* src = reinterpret_cast<const f32x4*>(part + i4);
  const int64_t sn = n / 4;  // slab stride in f32x4
  f32x4 a0 = __builtin_nontemporal_load(src), a1 = {0.f, 0.f, 0.f, 0.f}, a2 = a1, a3 = a1;
  int s = 1;
  for (; s + 3 < splits; s += 4) {
    a0 += __builtin_nontemporal_load(src + (int64_t)s * sn);
    a1 += __builtin_nontemporal_load(src + (int64_t)(s + 1) * sn);
    a2 += __builtin_nontemporal_load(src + (int64_t)(s + 2) * sn);
    a3 += __builtin_nontemporal_load(src + (int64_t)(s + 3) * sn);
  }
  for (; s < splits; ++s) a0 += __builtin_nontemporal_load(src + (int64_t)s * sn);
  f32x4 acc = (a0 + a1) + (a2 + a3);
  acc *= alpha;
  if (LOWRANK) {
    // r % 8 == 0, r <= 64: U's row and V's rows / columns are read as 16- / 8-byte vectors
    const int64_t m = i4 / ep.N, n0 = i4 - m * ep.N;  // N % 4 == 0: the 4 elements share a row
    const T* u = reinterpret_cast<const T*>(ep.U) + m * ep.r;
    const T* v = reinterpret_cast<const T*>(ep.V);
    f32x4 lr = {0.f, 0.f, 0.f, 0.f};
    for (int j0 = 0; j0 < ep.r; j0 += 8) {
      float uj[8];
      Vec8<T>::load(u + j0, uj);
      if (ep.sv_n != 1) {  // V = [N, r] (row n holds the r coefficients of output column n)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float vv[8];
          Vec8<T>::load(v + (n0 + e) * ep.sv_n + j0, vv);
#pragma unroll
          for (int q = 0; q < 8; ++q) lr[e] += uj[q] * vv[q];
        }
      } else {  // V = [r, N]: 4 consecutive outputs = one 8-byte run per coefficient row
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const uint2 raw = *reinterpret_cast<const uint2*>(v + (int64_t)(j0 + q) * ep.sv_j + n0);
          const T* h = reinterpret_cast<const T*>(&raw);
#pragma unroll
          for (int e = 0; e < 4; ++e) lr[e] += uj[q] * ld1<T>(h + e);
        }
      }
    }
    if (ep.mask != nullptr) {
      const uint2 raw = *reinterpret_cast<const uint2*>(reinterpret_cast<const T*>(ep.mask) + i4);
      const T* mk = reinterpret_cast<const T*>(&raw);
#pragma unroll
      for (int e = 0; e < 4; ++e) lr[e] *= ld1<T>(mk + e);
    }
    acc += ep.beta * lr;
  }
  if (AFF) {  // eval BN folded in: act(round(acc) * scale + shift (+ residual)), N % 4 == 0
    const int64_t n0 = i4 % ep.N;
    const T* res = static_cast<const T*>(ep.residual);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float v = fmaf(rnd<T>(acc[e]), ep.scale[n0 + e], ep.shift[n0 + e]);
      if (res != nullptr) v += ld1<T>(res + i4 + e);
      acc[e] = ep.act ? fmaxf(v, 0.f) : v;
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) st1<T>(out + i4 + e, acc[e]);
}

template <typename T>
hipError_t reduce_launch(const float* part, T* out, int64_t n, int splits, float alpha, const SplitkEpilogue* ep,
                         hipStream_t st) {
  const int blocks = (int)((n / 4 + kRedThreads - 1) / kRedThreads);
  if (ep != nullptr && ep->U != nullptr)
    hipLaunchKernelGGL((splitk_reduce_k<T, true, false>), dim3(blocks), dim3(kRedThreads), 0, st, part, out, n, splits,
                       alpha, *ep);
  else if (ep != nullptr && ep->scale != nullptr)
    hipLaunchKernelGGL((splitk_reduce_k<T, false, true>), dim3(blocks), dim3(kRedThreads), 0, st, part, out, n, splits,
                       alpha, *ep);
  else
    hipLaunchKernelGGL((splitk_reduce_k<T, false, false>), dim3(blocks), dim3(kRedThreads), 0, st, part, out, n,
                       splits, alpha, SplitkEpilogue{});
  return hipGetLastError();
}

}  // namespace

namespace {
// Split-K reduce of a convolution's [splits, M, K] fp32 partials with the BN-statistics epilogue
// of conv_fwd_k: out = Σ_s part[s] rounded to T, and per-channel Σy, Σy² of the ROUNDED outputs
// over kStatRows-row blocks, added atomically into psum[K] / psq[K] (the sums the BN apply
// finalizes inline).  Used when a forward conv has too few output tiles to fill 256 CUs
// (ResNet-50 layer3/4: 200-392 tiles, 55 us at 0.8 workgroups per CU).  Block = 64 column quads
// (256 channels, 16-byte loads) x 4 row lanes.
template <typename T>
__global__ __launch_bounds__(256) void splitk_reduce_stats_k(const float* __restrict__ part, T* __restrict__ out,
                                                             int M, int K, int splits, int rows,
                                                             double* __restrict__ psum, double* __restrict__ psq) {
  __shared__ float red[2][4][256];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = blockIdx.y * 256 + tx * 4;
  const int r0 = blockIdx.x * rows;
  const int r1 = min(M, r0 + rows);
  const int64_t slab = (int64_t)M * K;
  f32x4 cs = {0.f, 0.f, 0.f, 0.f}, cq = cs;
  if (c < K) {
    for (int r = r0 + ty; r < r1; r += 4) {
      const float* src = part + (int64_t)r * K + c;
      f32x4 a0 = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(src)), a1 = {0.f, 0.f, 0.f, 0.f};
      int s = 1;
      for (; s + 1 < splits; s += 2) {
        a0 += __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(src + (int64_t)s * slab));
        a1 += __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(src + (int64_t)(s + 1) * slab));
      }
      if (s < splits) a0 += __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(src + (int64_t)s * slab));
      const f32x4 acc = a0 + a1;
      T* o = out + (int64_t)r * K + c;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float v = rnd<T>(acc[e]);
        st1<T>(o + e, v);
        cs[e] += v;
        cq[e] += v * v;
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    red[0][ty][tx * 4 + e] = cs[e];
    red[1][ty][tx * 4 + e] = cq[e];
  }
  __syncthreads();
  // one atomic per channel per block: 64 consecutive channels per wave instruction (256-byte runs)
  if (threadIdx.x < 256) {
    const int j = threadIdx.x, ch = blockIdx.y * 256 + j;
    if (ch < K) {
      const int64_t slot = (int64_t)(blockIdx.x % kStatSlots) * 2 * K;
      unsafeAtomicAdd(psum + slot + ch, (double)((red[0][0][j] + red[0][1][j]) + (red[0][2][j] + red[0][3][j])));
      unsafeAtomicAdd(psq + slot + ch, (double)((red[1][0][j] + red[1][1][j]) + (red[1][2][j] + red[1][3][j])));
    }
  }
}
}  // namespace

hipError_t splitk_reduce_stats(int dtype, const float* part, void* out, int M, int K, int splits, double* psum,
                               double* psq, hipStream_t st) {
  if (K % 4 != 0 || splits < 1 || M < 1) return hipErrorInvalidValue;
  // kStatRows-row blocks (fewer atomic adders per channel) unless that leaves < 512 blocks
  const int cb = (K + 255) / 256;
  const int rows = (int64_t)((M + kStatRows - 1) / kStatRows) * cb >= 512 ? kStatRows : 16;
  const dim3 grid((M + rows - 1) / rows, cb);
  if (dtype == kBF16)
    hipLaunchKernelGGL(splitk_reduce_stats_k<bf16_t>, grid, dim3(256), 0, st, part, static_cast<bf16_t*>(out), M, K,
                       splits, rows, psum, psq);
  else if (dtype == kF16)
    hipLaunchKernelGGL(splitk_reduce_stats_k<f16_t>, grid, dim3(256), 0, st, part, static_cast<f16_t*>(out), M, K,
                       splits, rows, psum, psq);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

namespace {
// Split-K reduce of a stride-1 data gradient with the BN-backward epilogue (conv_igemm.hip's BNB
// epilogue for the split case): out = dz = round(round(Σ_s part[s]) + addend) · mask and Σdz,
// Σdz·x per channel into slot blockIdx.x % kStatSlots of bnb.sums.  Same block shape as
// splitk_reduce_stats_k (64 column quads x 4 row lanes, `rows` rows per block).
template <typename T>
__global__ __launch_bounds__(256) void splitk_reduce_bnb_k(const float* __restrict__ part, T* __restrict__ out,
                                                           const T* __restrict__ addend, int M, int K, int splits,
                                                           int rows, BnBwdEpilogue bnb) {
  __shared__ float red[2][4][256];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = blockIdx.y * 256 + tx * 4;
  const int r0 = blockIdx.x * rows;
  const int r1 = min(M, r0 + rows);
  const int64_t slab = (int64_t)M * K;
  const T* xb = static_cast<const T*>(bnb.x);
  const T* yb = static_cast<const T*>(bnb.y);
  float msc[4] = {0.f, 0.f, 0.f, 0.f}, msh[4] = {0.f, 0.f, 0.f, 0.f};
  if (bnb.mode == 1 && c < K) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float sc = (bnb.w ? bnb.w[c + e] : 1.f) * bnb.invstd[c + e];
      msc[e] = sc;
      msh[e] = (bnb.b ? bnb.b[c + e] : 0.f) - bnb.mean[c + e] * sc;
    }
  }
  f32x4 cs = {0.f, 0.f, 0.f, 0.f}, cq = cs;
  if (c < K) {
    for (int r = r0 + ty; r < r1; r += 4) {
      const int64_t off = (int64_t)r * K + c;
      const float* src = part + off;
      f32x4 a0 = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(src)), a1 = {0.f, 0.f, 0.f, 0.f};
      int s = 1;
      for (; s + 1 < splits; s += 2) {
        a0 += __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(src + (int64_t)s * slab));
        a1 += __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(src + (int64_t)(s + 1) * slab));
      }
      if (s < splits) a0 += __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(src + (int64_t)s * slab));
      const f32x4 acc = a0 + a1;
      // 4 channels = one 8-byte run of each 2-byte operand
      const uint2 rx = *reinterpret_cast<const uint2*>(xb + off);
      const uint2 ry = bnb.mode == 2 ? *reinterpret_cast<const uint2*>(yb + off) : uint2{0u, 0u};
      const uint2 rd = addend != nullptr ? *reinterpret_cast<const uint2*>(addend + off) : uint2{0u, 0u};
      const T* hx = reinterpret_cast<const T*>(&rx);
      const T* hy = reinterpret_cast<const T*>(&ry);
      const T* hd = reinterpret_cast<const T*>(&rd);
      T ov[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v = rnd<T>(acc[e]);
        if (addend != nullptr) v = rnd<T>(v + ld1<T>(hd + e));
        const float xv = ld1<T>(hx + e);
        const bool keep = bnb.mode == 0 || (bnb.mode == 1 ? fmaf(xv, msc[e], msh[e]) > 0.f : ld1<T>(hy + e) > 0.f);
        v = keep ? v : 0.f;
        st1<T>(ov + e, v);
        cs[e] += v;
        cq[e] += v * xv;
      }
      *reinterpret_cast<uint2*>(out + off) = *reinterpret_cast<const uint2*>(ov);
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    red[0][ty][tx * 4 + e] = cs[e];
    red[1][ty][tx * 4 + e] = cq[e];
  }
  __syncthreads();
  const int j = threadIdx.x, ch = blockIdx.y * 256 + j;
  if (ch < K) {
    double* slot = bnb.sums + (int64_t)(blockIdx.x % kStatSlots) * 2 * K;
    unsafeAtomicAdd(slot + ch, (double)((red[0][0][j] + red[0][1][j]) + (red[0][2][j] + red[0][3][j])));
    unsafeAtomicAdd(slot + K + ch, (double)((red[1][0][j] + red[1][1][j]) + (red[1][2][j] + red[1][3][j])));
  }
}
}  // namespace

hipError_t splitk_reduce_bnb(int dtype, const float* part, void* out, const void* addend, int M, int K, int splits,
                             const BnBwdEpilogue& bnb, hipStream_t st) {
  if (K % 4 != 0 || splits < 1 || M < 1) return hipErrorInvalidValue;
  const int cb = (K + 255) / 256;
  const int rows = (int64_t)((M + kStatRows - 1) / kStatRows) * cb >= 512 ? kStatRows : 16;
  const dim3 grid((M + rows - 1) / rows, cb);
  if (dtype == kBF16)
    hipLaunchKernelGGL(splitk_reduce_bnb_k<bf16_t>, grid, dim3(256), 0, st, part, static_cast<bf16_t*>(out),
                       static_cast<const bf16_t*>(addend), M, K, splits, rows, bnb);
  else if (dtype == kF16)
    hipLaunchKernelGGL(splitk_reduce_bnb_k<f16_t>, grid, dim3(256), 0, st, part, static_cast<f16_t*>(out),
                       static_cast<const f16_t*>(addend), M, K, splits, rows, bnb);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t splitk_reduce(int dtype, const float* part, void* out, int64_t n, int splits, hipStream_t st, float alpha,
                         const SplitkEpilogue* ep) {
  if (n % 4 != 0 || splits < 1) return hipErrorInvalidValue;
  if (ep != nullptr && ep->U != nullptr && (ep->N % 4 != 0 || ep->r < 8 || ep->r % 8 != 0 || n % ep->N != 0))
    return hipErrorInvalidValue;
  if (ep != nullptr && ep->scale != nullptr && (ep->N % 4 != 0 || n % ep->N != 0 || ep->shift == nullptr))
    return hipErrorInvalidValue;
  if (dtype == kBF16) return reduce_launch<bf16_t>(part, static_cast<bf16_t*>(out), n, splits, alpha, ep, st);
  if (dtype == kF16) return reduce_launch<f16_t>(part, static_cast<f16_t*>(out), n, splits, alpha, ep, st);
  return hipErrorInvalidValue;
}

namespace {

uint64_t magic36(int d) { return ((1ull << 36) + (uint64_t)d - 1) / (uint64_t)d; }

int g_wgrad_stages = 0;  // 0 = automatic (conv_wgrad_set_stages, for tuning sweeps)

template <typename T, int BM, int BN>
hipError_t launch(const WgradArgs& a, hipStream_t st) {
  const int tiles = ((a.K + BM - 1) / BM) * (a.R * a.S * a.C / BN);
  const int nb = g_wgrad_stages > 0 ? g_wgrad_stages : 2;  // deeper rings measured no better (conv_r01)
  if (nb == 2)
    hipLaunchKernelGGL((conv_wgrad_k<T, BM, BN, 2>), dim3(tiles * a.splits), dim3(kThreads), 0, st, a);
  else if (nb == 3)
    hipLaunchKernelGGL((conv_wgrad_k<T, BM, BN, 3>), dim3(tiles * a.splits), dim3(kThreads), 0, st, a);
  else
    hipLaunchKernelGGL((conv_wgrad_k<T, BM, BN, 4>), dim3(tiles * a.splits), dim3(kThreads), 0, st, a);
  return hipGetLastError();
}

}  // namespace

bool conv_wgrad_supported(int C, int K) { return C % 64 == 0 && K % 8 == 0; }

void conv_wgrad_set_stages(int nb) { g_wgrad_stages = (nb >= 2 && nb <= 4) ? nb : 0; }

// Plan (from the per-layer sweep of bench/conv_shapes.py over ResNet-50 at batch 32 on MI355X,
// profiles/conv_r01/conv_shapes_wgrad_sweep.json): 64 x 64 tiles win at every layer (more workgroups in flight;
// the kernel is latency- not MFMA-bound at these sizes), and the best pixel split keeps each
// workgroup at ~16-25 stages of 64 pixels — enough to amortize the prologue/epilogue, short enough
// that the grid fills the chip.  Fewer splits also bound the fp32 partial traffic (splits*K*RSC*8 B).
void conv_wgrad_plan(int M, int K, int C, int R, int S, int* bm, int* bn, int* splits, int* steps_per_split) {
  (void)K, (void)C, (void)R, (void)S;
  *bm = 64;
  *bn = 64;
  const int total_steps = (M + kBP - 1) / kBP;
  const int per = max(16, (total_steps + 63) / 64);
  *steps_per_split = per;
  *splits = (total_steps + per - 1) / per;
}

hipError_t conv_wgrad(int dtype, const void* dy, const void* x, void* dw, float* partials, const void* zero, int N,
                      int H, int W, int C, int K, int P, int Q, int R, int S, int sh, int sw, int ph, int pw, int bm,
                      int bn, int splits, int steps_per_split, hipStream_t st, float alpha) {
  if (!conv_wgrad_supported(C, K) || dtype == kF32) return hipErrorInvalidValue;
  if (C % bn != 0 || (bm != 64 && bm != 128) || (bn != 64 && bn != 128) || splits < 1) return hipErrorInvalidValue;
  const int64_t M64 = (int64_t)N * P * Q;
  // fdiv's 36-bit magic is exact for numerators < 2^22 and divisors < 2^14
  if (M64 <= 0 || M64 >= (1ll << 22) || (int64_t)P * Q >= (1 << 14)) return hipErrorInvalidValue;
  if ((int64_t)splits * steps_per_split * kBP < M64) return hipErrorInvalidValue;
  if (splits > 1 && partials == nullptr) return hipErrorInvalidValue;
  WgradArgs a{static_cast<const uint16_t*>(dy), static_cast<const uint16_t*>(x),
              splits > 1 ? static_cast<void*>(partials) : dw, static_cast<const uint16_t*>(zero), N, H, W, C, K, P, Q,
              R, S, sh, sw, ph, pw, (int)M64, splits, steps_per_split, magic36(Q), magic36(P * Q), alpha};
  hipError_t e;
  if (dtype == kBF16) {
    if (bm == 128 && bn == 128) e = launch<bf16_t, 128, 128>(a, st);
    else if (bm == 128) e = launch<bf16_t, 128, 64>(a, st);
    else if (bn == 128) e = launch<bf16_t, 64, 128>(a, st);
    else e = launch<bf16_t, 64, 64>(a, st);
  } else {
    if (bm == 128 && bn == 128) e = launch<f16_t, 128, 128>(a, st);
    else if (bm == 128) e = launch<f16_t, 128, 64>(a, st);
    else if (bn == 128) e = launch<f16_t, 64, 128>(a, st);
    else e = launch<f16_t, 64, 64>(a, st);
  }
  if (e != hipSuccess || splits == 1) return e;
  return splitk_reduce(dtype, partials, dw, (int64_t)K * R * S * C, splits, st, alpha);  // C % 64 == 0: n % 4 == 0
}

}  // namespace hyp

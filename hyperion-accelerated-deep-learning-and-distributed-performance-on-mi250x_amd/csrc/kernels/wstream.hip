// Weight-streaming GEMM for few-token activations (M <= 128 rows per workgroup): the projections of
// a Llama-2-7B LoRA fine-tune step at batch 1 x 128 tokens, whose runtime is the time to stream
// the frozen 4096-wide weights from HBM (26 GB per step, fwd + dgrad).
//
// Reference: every projection of train_llama_fsdp runs as torch.nn.functional.linear -> hipBLASLt
// (02_development/distributed_utils.py:463-476, 515-524; SURVEY §2.4 "GEMM" / "LoRA", §2.5 Llama
// row), which at M = 128 streams the weight at ~0.6 TB/s on MI355X (profiles/llama_r01).
//
// Design (MI355X-first; guide §5 "Projection GEMM at M = 256" and the M <= 16 GEMV row):
//  * the activation slice x[rows, k0 : k0 + kr] is loaded ONCE into LDS by LDS-DMA (global_load_lds)
//    and stays resident for the workgroup's whole life — no barrier, no LDS write in the main loop;
//  * the weight is streamed straight into VGPRs as MFMA B fragments with D k-steps in flight per
//    wave (16 KB per wave, 64 KB per CU: HBM latency x per-CU share of 6 TB/s), never staged in LDS;
//  * the reduction is split over S slices of kr (fp32 partial slabs); a workgroup is persistent
//    over its share of the output columns of one slice, so x is fetched once per workgroup;
//  * partial slabs are written in MFMA-fragment order: every lane stores one 16-byte float4, a wave
//    instruction one contiguous KiB; ws_reduce sums the slabs in a fixed order (deterministic) and
//    writes the row-major output (+ alpha, + an addend, + a rank-r LoRA term).
//  * NT (y = x Wᵀ, W [N, K]: the forward) loads W rows as fragments directly (lane: row n, 8
//    consecutive k).  NN (y = x W, W [K, N]: the data gradient, reduction over W's ROWS) loads 8
//    consecutive W rows x 4 columns per lane (each row segment 128 B across 16 lanes) and
//    transposes the 8 x 4 block in-lane with v_perm_b32 into four B fragments whose output
//    columns are n0 + 4j + c (c = 0..3) — no transposed weight copy, no LDS round trip.
//
// A fragment LDS image: rows of krp elements (krp % 128 == 0); 16-byte chunk c of row r sits at
// chunk (c & ~15) | ((c ^ r) & 15), which makes every ds_read_b128 A-fragment read (row r = l & 15,
// chunk 4t + (l >> 4)) conflict-free across the instruction's 16-lane service groups.
#include "hyp_common.h"
#include "hyp_kernels.h"
#include "mfma_lds.h"

namespace hyp {
namespace {

using mfl::f32x4;
using mfl::u16x8;

struct WsArgs {
  const uint16_t* x;  // [M, K] row stride ldx
  const uint16_t* w;  // NT: [N, K]; NN: [K, N]; row stride ldw
  float* part;        // [S][MB * MF][N / 16][64][4]
  const uint16_t* zero;
  int64_t ldx, ldw;
  int M, N, K;
  int kr, krp;     // slice length (% 32 == 0) and LDS row pitch (% 128 == 0)
  int S, G, MB;    // slices, workgroups per (slice, m-block), m-blocks
  int chunks;      // column chunks per (slice, m-block)
  int R;           // S * G
  int sb;          // slabs in bf16 (8-byte quads) instead of fp32
};

__device__ __forceinline__ int swz_chunk(int c, int r) { return (c & ~15) | ((c ^ r) & 15); }

// Slab store as inline asm: hipcc's wait pass treats loads and stores pending on the one gfx9
// vector-memory counter as possibly out of order and then waits vmcnt(0) at every later use of a
// load — i.e. the slab stores of one column chunk would drain the weight ring at every k-group of
// the next.  Invisible stores only make its counted waits conservative (they retire the stores
// too), never short.  s_nop 1: the store's data VGPRs may be rewritten right after (acc reset).
__device__ __forceinline__ void store_slab(float* dst, f32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off\n\ts_nop 1" ::"v"(dst), "v"(v) : "memory");
}
// bf16 slabs (half the partial-sum traffic of the split-K GEMM and of its epilogue; each slab is a
// fp32 partial over >= 128 reduction terms rounded once, the slabs are summed in fp32)
__device__ __forceinline__ void store_slab16(uint16_t* dst, f32x4 v) {
  const uint2 q = make_uint2((uint32_t)float_to_bf16(v[0]) | ((uint32_t)float_to_bf16(v[1]) << 16),
                             (uint32_t)float_to_bf16(v[2]) | ((uint32_t)float_to_bf16(v[3]) << 16));
  asm volatile("global_store_dwordx2 %0, %1, off\n\ts_nop 1" ::"v"(dst), "v"(q) : "memory");
}
// one slab quad (4 rows x 1 column) at element offset e of the slab buffer
__device__ __forceinline__ f32x4 load_slab(const float* part, int sb, int64_t e) {
  if (sb) {
    const uint2 q = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(part) + e);
    return f32x4{__uint_as_float(q.x << 16), __uint_as_float(q.x & 0xffff0000u), __uint_as_float(q.y << 16),
                 __uint_as_float(q.y & 0xffff0000u)};
  }
  return *reinterpret_cast<const f32x4*>(part + e);
}

template <typename T, int MF, int NF, bool NN, int D, int WAVES>
__global__ __launch_bounds__(WAVES * 64) void ws_gemm_k(const WsArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint16_t xs[];
  constexpr int NFE = NN ? 4 : NF;  // B fragments per k-step
  constexpr int LPS = NN ? 8 : NF;  // global loads per k-step per lane
  constexpr int Mp = MF * 16;
  typedef uint16_t u16x4 __attribute__((ext_vector_type(4)));
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: scalar branches
  const int l15 = lane & 15, g4 = lane >> 4;

  // ---- block -> (m-block, slice, column group).  M-block siblings sit 8 ids apart (the same XCD
  // under round-robin dispatch) so the second reader of a weight slice hits L2.
  int mb, r;
  {
    const int b = blockIdx.x;
    if (a.MB == 1) {
      mb = 0;
      r = b;
    } else {
      mb = (b >> 3) % a.MB;
      r = (b & 7) + 8 * (b / (8 * a.MB));
    }
  }
  if (r >= a.R) return;
  const int s = r / a.G, g = r - s * a.G;
  const int k0 = s * a.kr;
  const int kn = min(a.kr, a.K - k0);  // this slice's length (% (32 D) == 0)
  const int nkt = kn >> 5;             // 32-deep k-steps per column chunk (% D == 0)

  // this wave's column chunks [c_begin, c_end)
  const int wv = g * WAVES + wave, nwv = a.G * WAVES;
  const int c_begin = (int)((int64_t)wv * a.chunks / nwv), c_end = (int)((int64_t)(wv + 1) * a.chunks / nwv);

  // ---- x slice -> LDS (lane-linear LDS-DMA; chunk-swizzled source addresses; zeros past M / kn)
  {
    const int cpr = a.krp >> 3;                      // 16-byte chunks per LDS row
    const int ninstr = (Mp * cpr) / (64 * WAVES);    // per wave (exact: Mp * cpr % 512 == 0)
    for (int i = 0; i < ninstr; ++i) {
      const int L = (i * WAVES + wave) * 64 + lane;
      const int rr = L / cpr, p = L - rr * cpr;
      const int c = swz_chunk(p, rr);
      const int row = mb * Mp + rr;
      const bool ok = row < a.M && c * 8 < kn;
      const uint16_t* src = ok ? a.x + (int64_t)row * a.ldx + k0 + c * 8 : a.zero;
      mfl::glds16(src, xs + (i * WAVES + wave) * 512);
    }
  }

  // ---- weight stream: a ring of D k-steps in flight per wave.  Past the wave's last step the
  // ring keeps re-issuing that step's (valid) addresses — unused loads instead of branches, so the
  // loop body is straight-line and hipcc's counted waits stay exact.
  // NT: fragment j of chunk ch covers columns ch*16*NF + 16 j .. +15 (rows of W); lane reads row
  //     (that + l15), k = k0 + 32 t + 8 g4 .. +7 (16 B).
  // NN: chunk ch covers columns ch*64 .. +63; lane reads rows k0 + 32 t + 8 g4 + i (i < 8),
  //     columns ch*64 + 4 l15 .. +3 (8 B each).
  u16x8 ringA[D][NN ? 1 : NF];
  u16x4 ringB[D][NN ? 8 : 1];
  int is_ch = c_begin, is_t = 0;  // next step to issue

  auto issue = [&](int d) {
    if (!NN) {
#pragma unroll
      for (int j = 0; j < NF; ++j) {
        int n = (is_ch * NF + j) * 16;
        n = n < a.N ? n : is_ch * NF * 16;  // a partial last chunk re-reads its first fragment
        ringA[d][j] = *reinterpret_cast<const u16x8*>(a.w + (int64_t)(n + l15) * a.ldw + k0 + is_t * 32 + g4 * 8);
      }
    } else {
      const uint16_t* base = a.w + (int64_t)(k0 + is_t * 32 + g4 * 8) * a.ldw + is_ch * 64 + l15 * 4;
#pragma unroll
      for (int i = 0; i < 8; ++i) ringB[d][i] = *reinterpret_cast<const u16x4*>(base + (int64_t)i * a.ldw);
    }
    if (++is_t == nkt) {
      is_t = 0;
      if (++is_ch == c_end) {  // clamp: re-issue the last step
        is_ch = c_end - 1;
        is_t = nkt - 1;
      }
    }
  };

  // x landed everywhere.  (Waiting for the DMA with vmcnt(0) BEFORE the weight prologue keeps
  // hipcc's wait model exact: with an LDS-DMA still pending at the first ds_read it conservatively
  // drains vmcnt(0) inside the main loop, i.e. the whole weight ring every step.)
  mfl::wait_vmcnt<0>();
  mfl::barrier_keep_vm();
  if (c_end <= c_begin) return;
#pragma unroll
  for (int d = 0; d < D; ++d) {
    issue(d);
    __builtin_amdgcn_sched_barrier(0);  // ring slots in order (the main loop's counted waits assume it)
  }

  f32x4 acc[MF][NFE];
#pragma unroll
  for (int i = 0; i < MF; ++i)
#pragma unroll
    for (int j = 0; j < NFE; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int F = a.N >> 4;
  const int MFtot = a.MB * MF;
  // A fragments, double-buffered one k-step ahead (they depend on t only, not on the chunk)
  const uint16_t* xrow = xs + l15 * a.krp;
  u16x8 af[2][MF];
#pragma unroll
  for (int i = 0; i < MF; ++i)
    af[0][i] = *reinterpret_cast<const u16x8*>(xrow + i * 16 * a.krp + swz_chunk(g4, l15) * 8);

  for (int ch = c_begin; ch < c_end; ++ch) {
    for (int t0 = 0; t0 < nkt; t0 += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const int t = t0 + d;
        const int tn = t + 1 == nkt ? 0 : t + 1;
        const int xo = swz_chunk(tn * 4 + g4, l15) * 8;
#pragma unroll
        for (int i = 0; i < MF; ++i)
          af[(d + 1) & 1][i] = *reinterpret_cast<const u16x8*>(xrow + i * 16 * a.krp + xo);
        if (!NN) {
          // MFMAs straight from the ring registers, THEN the refill: no register copy of an
          // in-flight load (a copy would make hipcc wait for it — vmcnt(0) every k-group)
#pragma unroll
          for (int i = 0; i < MF; ++i)
#pragma unroll
            for (int j = 0; j < NF; ++j) acc[i][j] = mfl::mma16<T>(af[d & 1][i], ringA[d][j], acc[i][j]);
          __builtin_amdgcn_sched_barrier(0);
          issue(d);
        } else {
          // rows i (reduction) x columns c -> fragment c: dword q = (row 2q, row 2q+1) of column c
          u16x8 bf[4];
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            uint32_t dw[4];
#pragma unroll
            for (int qd = 0; qd < 4; ++qd)
              dw[qd] = (uint32_t)ringB[d][2 * qd][c] | ((uint32_t)ringB[d][2 * qd + 1][c] << 16);
            bf[c] = __builtin_bit_cast(u16x8, (uint4){dw[0], dw[1], dw[2], dw[3]});
          }
          __builtin_amdgcn_sched_barrier(0);
          issue(d);  // the slot's raw rows are consumed: refill it D steps ahead
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int i = 0; i < MF; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = mfl::mma16<T>(af[d & 1][i], bf[j], acc[i][j]);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // chunk done: fragment-order fp32 slab stores (one contiguous KiB per wave instruction)
    const int fr0 = NN ? ch * 4 : ch * NF;
#pragma unroll
    for (int j = 0; j < NFE; ++j) {
      if (NN || fr0 + j < F) {
#pragma unroll
        for (int i = 0; i < MF; ++i) {
          const int64_t e = ((((int64_t)s * MFtot + mb * MF + i) * F + fr0 + j) * 64 + lane) * 4;
          if (a.sb) store_slab16(reinterpret_cast<uint16_t*>(a.part) + e, acc[i][j]);
          else store_slab(a.part + e, acc[i][j]);
        }
      }
#pragma unroll
      for (int i = 0; i < MF; ++i) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
}

int g_ws_depth = 4;  // k-steps in flight per wave (ws_set_depth): 4, or 8 where the slices allow it

template <typename T, int MF, int NF, bool NN, int D>
hipError_t launch_gemm_d(const WsArgs& a, int grid, hipStream_t st) {
  // two waves per SIMD where the registers allow it (NT with <= 2 fragments per chunk)
  constexpr int WAVES = (!NN && MF * NF <= 16) ? 8 : 4;
  const size_t lds = (size_t)MF * 16 * a.krp * 2;
  auto kfn = ws_gemm_k<T, MF, NF, NN, D, WAVES>;
  static bool attr_set = false;  // per instantiation
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kfn), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL(kfn, dim3(grid), dim3(WAVES * 64), lds, st, a);
  return hipGetLastError();
}

// D = 8 (twice the weight bytes in flight per wave) needs every slice's k-steps to fill whole rings
template <typename T, int MF, int NF, bool NN>
hipError_t launch_gemm(const WsArgs& a, int grid, hipStream_t st) {
  if constexpr (MF == 8) {
    if (g_ws_depth == 8 && a.kr % 256 == 0 && (a.K % a.kr) % 256 == 0) return launch_gemm_d<T, MF, NF, NN, 8>(a, grid, st);
  }
  return launch_gemm_d<T, MF, NF, NN, 4>(a, grid, st);
}

// ---- slab reduction: out[m, n] = alpha * Σ_s part[s] (+ beta * addend) (+ rank-r term) ---------------
struct WsRed {
  const float* part;  // fp32 slabs, or bf16 ones (sb)
  void* out;
  int64_t ldo;
  const void* addend;  // [M, N] (ld ldo) in T, or null
  float alpha, beta;
  // LoRA rank-r term: out += scale * Σ_r U[m, seg * r + rr] V_seg[n - seg * segw, rr]   (V row-major [segw, r])
  const float* U;      // [M, nseg * r] fp32
  const uint16_t* V;   // concatenated [nseg * segw, r] (T)
  int r, segw;
  float uscale;
  int M, N, S, MFtot, NN;
  int sb;  // bf16 slabs
};

// one thread = one (m-fragment, column-fragment, lane) quad: 4 rows x 1 column
template <typename T>
__global__ __launch_bounds__(256) void ws_reduce_k(const WsRed a) {
  const int64_t F = a.N >> 4;
  const int64_t tid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t nquads = (int64_t)a.MFtot * F * 64;
  if (tid >= nquads) return;
  const int lane = (int)(tid & 63);
  const int64_t fr = tid >> 6;
  const int cf = (int)(fr % F), mf = (int)(fr / F);
  const int n = a.NN ? (cf >> 2) * 64 + 4 * (lane & 15) + (cf & 3) : cf * 16 + (lane & 15);
  const int m0 = mf * 16 + 4 * (lane >> 4);
  if (m0 >= a.M) return;
  const int64_t slab = (int64_t)a.MFtot * F * 256;
  f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
  const int64_t e0 = tid * 4;
  {
    f32x4 acc4[4] = {acc, acc, acc, acc};
    int s = 0;
    for (; s + 8 <= a.S; s += 8) {
      f32x4 v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = load_slab(a.part, a.sb, e0 + (s + i) * slab);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc4[i & 3] += v[i];
    }
    for (; s < a.S; ++s) acc4[0] += load_slab(a.part, a.sb, e0 + s * slab);
    acc = (acc4[0] + acc4[1]) + (acc4[2] + acc4[3]);
  }
  float v[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) v[e] = acc[e] * a.alpha;
  if (a.U != nullptr) {
    const int seg = n / a.segw;
    const uint16_t* vr = a.V + (int64_t)n * a.r;
    for (int rr = 0; rr < a.r; ++rr) {
      const float vv = ld1<T>(reinterpret_cast<const T*>(vr + rr));
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + e;
        if (m < a.M) v[e] += a.uscale * a.U[(int64_t)m * (a.r * (a.N / a.segw)) + seg * a.r + rr] * vv;
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int m = m0 + e;
    if (m < a.M) {
      T* o = reinterpret_cast<T*>(a.out) + (int64_t)m * a.ldo + n;
      float y = v[e];
      if (a.addend != nullptr) y += a.beta * ld1<T>(reinterpret_cast<const T*>(a.addend) + (int64_t)m * a.ldo + n);
      st1<T>(o, y);
    }
  }
}

// ---- fused epilogues of the weight-streaming GEMM (ws_epilogue; the Llama LoRA layer) ----------
// One 256-thread block = 16 rows (one m-fragment) x 64 output columns (4 fragments; thread = one
// (fragment, lane) quad of 4 rows x 1 column); "pair" epilogues also own the partner quad 64 (RoPE:
// the other half of the head) or I (SwiGLU: up next to gate) columns away.  The slabs are summed
// in fixed order; LoRA operands of the block's rows / columns are staged in LDS; the outputs go
// out through an LDS tile as 16-byte row chunks.
//   EPI 0  out = Σ
//   EPI 1  out = Σ + c' Σ_rr t[m, seg r + rr] B_seg[n - seg segw, rr]   (the LoRA up term; NT)
//          then RoPE on segments < rope_segs (pairs i, i + 64 of each 128-wide head)
//   EPI 2  SwiGLU forward (NT, N = 2 I): gu = round(Σ) (pre-activations, kept for backward),
//          h[m, n] = silu(g) u
//   EPI 3  SwiGLU backward (NN, N = I): dh = round(Σ); g, u from gu -> dgu[m, n] = dh u silu'(g),
//          dgu[m, n + I] = dh silu(g)
//   EPI 4  LoRA data gradient (NN): out = Σ + Σ_p keep_p(m, n) Σ_rr du[m, p r + rr] A_p[rr, n]
struct WsEpi {
  const float* part;      // fp32 (or bf16: sb) slabs, or null: the GEMM result is the row-major yin (a vendor GEMM's)
  int sb;
  const void* yin;
  int64_t ldy;
  int S, MFtot, M, N;     // GEMM output width N (EPI 2: 2 I; EPI 3: I)
  void* out;
  int64_t ldo;
  void* out2;             // EPI 2: h [M, I]
  int64_t ldo2;
  const void* aux;        // EPI 3: gu [M, 2 I]
  int64_t ld_aux;
  const float* t;         // EPI 1: t' / EPI 4: du'  [t_splits][M][ldt] fp32 split partials (summed here)
  int ldt;
  int64_t t_sstride;
  int t_splits;
  const void* lw[4];      // EPI 1: B_p [segw, r]; EPI 4: A_p [r, N]
  int P, r, segw;
  float lscale;
  int rope_segs, seq;
  float log2_theta;
  RngState rng;
  uint32_t thr;
  int drop;
};

template <typename T, int EPI, bool NN>
__global__ __launch_bounds__(256) void ws_epi_k(const WsEpi a) {
  static_assert(EPI == 0 || (EPI == 3 || EPI == 4) == NN, "slab layout: EPI 1/2 are NT, 3/4 NN, 0 either");
  constexpr bool PAIR = EPI == 1 || EPI == 2;
  __shared__ __attribute__((aligned(16))) float lt[16 * 64];  // t / du rows of the block (P r <= 64)
  __shared__ float lw_s[4 * 16 * 128];    // EPI 1: B rows [128 cols][r]; EPI 4: A_p [r][64 cols] per p
  __shared__ __attribute__((aligned(16))) uint16_t tile[3][16][128 + 8];
  const int tid = threadIdx.x, lane = tid & 63, f = tid >> 6;
  const int F = a.N >> 4;
  const int mf = blockIdx.y;
  // column chunk -> first fragment of the block (and of the partner)
  int cf0, pofs = 0;
  if (EPI == 1) {  // head h: fragments 8h .. 8h+3, partner +4
    cf0 = blockIdx.x * 8;
    pofs = 4;
  } else if (EPI == 2) {
    cf0 = blockIdx.x * 4;
    pofs = F / 2;
  } else {
    cf0 = blockIdx.x * 4;
  }
  const int cf = cf0 + f;
  const int col_of_lane = NN ? 4 * (lane & 15) + (cf & 3) : (lane & 15) + 16 * f;  // within the 64-col chunk
  const int n = NN ? (cf >> 2) * 64 + 4 * (lane & 15) + (cf & 3) : cf * 16 + (lane & 15);
  const int mrow0 = mf * 16;
  const int m0 = mrow0 + 4 * (lane >> 4);

  // ---- stage LoRA operands
  if ((EPI == 1 && a.t != nullptr) || EPI == 4) {
    // 16 rows x P r (<= 64) ranks as float4 cells, one per thread; all slice loads in flight before
    // the sum (the stacks are host-checked to 16-byte alignment)
    const int pr = a.P * a.r, c4 = pr >> 2;
    {
      const int rr = tid / 16, j4 = (tid & 15) * 4, m = mrow0 + rr;
      const bool ok = j4 < pr && m < a.M;
      float4 acc = float4{0.f, 0.f, 0.f, 0.f};
      for (int q0 = 0; q0 < a.t_splits; q0 += 4) {
        float4 v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int q = min(q0 + i, a.t_splits - 1);
          v[i] = ok ? *reinterpret_cast<const float4*>(a.t + q * a.t_sstride + (int64_t)m * a.ldt + j4)
                    : float4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (q0 + i < a.t_splits) {
            acc.x += v[i].x; acc.y += v[i].y; acc.z += v[i].z; acc.w += v[i].w;
          }
      }
      if (j4 < 64) *reinterpret_cast<float4*>(&lt[rr * 64 + j4]) = acc;
      (void)c4;
    }
    // LoRA operand rows with 16-byte loads, every load of a thread issued before any LDS store (a
    // scalar load per element in a loop waited one memory round trip per iteration: ~10 us)
    if (EPI == 1) {  // B rows of the 64 (+64 partner) columns: lw_s[c][rr], c < 128
      const int ncols = 128;
      if (a.r == 16) {  // a column's B row = 32 contiguous bytes: thread = (column, half)
        const int c = tid >> 1, h = tid & 1;
        const int col = c < 64 ? cf0 * 16 + c : (cf0 + pofs) * 16 + (c - 64);
        const int seg = col / a.segw;
        float f[8];
        Vec8<T>::load(static_cast<const T*>(a.lw[seg]) + (int64_t)(col - seg * a.segw) * 16 + h * 8, f);
#pragma unroll
        for (int e = 0; e < 8; ++e) lw_s[c * 16 + h * 8 + e] = f[e];
      } else {
        for (int i = tid; i < ncols * a.r; i += 256) {
          const int c = i / a.r, rr = i - c * a.r;
          const int col = c < 64 ? cf0 * 16 + c : (cf0 + pofs) * 16 + (c - 64);
          const int seg = col / a.segw;
          lw_s[c * 16 + rr] = ld1<T>(static_cast<const T*>(a.lw[seg]) + (int64_t)(col - seg * a.segw) * a.r + rr);
        }
      }
    } else {  // A_p[rr][64 cols of the chunk]: lw_s[(p * 16 + rr) * 64 + c]; 8 16-byte chunks per row
      const int c0 = (cf0 >> 2) * 64;
      const int nch = a.P * a.r * 8;  // <= 512
      float f[2][8];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int chk = tid + 256 * u, prr = chk >> 3, ch = chk & 7;
        if (chk < nch) {
          const int p = prr / a.r, rr = prr - p * a.r;
          Vec8<T>::load(static_cast<const T*>(a.lw[p]) + (int64_t)rr * a.N + c0 + ch * 8, f[u]);
        }
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int chk = tid + 256 * u, prr = chk >> 3, ch = chk & 7;
        if (chk < nch) {
#pragma unroll
          for (int e = 0; e < 8; ++e) lw_s[prr * 64 + ch * 8 + e] = f[u][e];
        }
      }
    }
    __syncthreads();
  }

  // ---- slab sums
  const int64_t slab = (int64_t)a.MFtot * F * 256;
  auto sum_quad = [&](int c) {
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
    if (a.part == nullptr) {  // dense input: the 4 rows of this quad's column
      const int col = NN ? (c >> 2) * 64 + 4 * (lane & 15) + (c & 3) : c * 16 + (lane & 15);
#pragma unroll
      for (int e = 0; e < 4; ++e)
        acc[e] = ld1<T>(static_cast<const T*>(a.yin) + (int64_t)min(m0 + e, a.M - 1) * a.ldy + col);
      return acc;
    }
    // 8 slab loads in flight per step, 4 accumulators (fixed order: deterministic); a one-load
    // loop waited a memory round trip per slab (24-43 slabs on the Llama dgrads)
    const int64_t e0 = (((int64_t)mf * F + c) * 64 + lane) * 4;
    f32x4 acc4[4] = {acc, acc, acc, acc};
    int s = 0;
    if (a.sb) {
      // bf16 slabs: 16 quads (8 bytes each) in flight per round — the 24-43 slabs of a Llama data
      // gradient take 2-3 memory round trips instead of 3-6
      const uint16_t* p16 = reinterpret_cast<const uint16_t*>(a.part) + e0;
      for (; s + 16 <= a.S; s += 16) {
        uint2 q[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) q[i] = *reinterpret_cast<const uint2*>(p16 + (s + i) * slab);
#pragma unroll
        for (int i = 0; i < 16; ++i)
          acc4[i & 3] += f32x4{__uint_as_float(q[i].x << 16), __uint_as_float(q[i].x & 0xffff0000u),
                               __uint_as_float(q[i].y << 16), __uint_as_float(q[i].y & 0xffff0000u)};
      }
    }
    for (; s + 8 <= a.S; s += 8) {
      f32x4 v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = load_slab(a.part, a.sb, e0 + (s + i) * slab);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc4[i & 3] += v[i];
    }
    for (; s < a.S; ++s) acc4[0] += load_slab(a.part, a.sb, e0 + s * slab);
    return (acc4[0] + acc4[1]) + (acc4[2] + acc4[3]);
  };
  f32x4 v = sum_quad(cf);
  f32x4 w = f32x4{0.f, 0.f, 0.f, 0.f};
  if (PAIR) w = sum_quad(cf + pofs);

  if (EPI == 1) {
    const int seg = n / a.segw;
    const int lc = (lane & 15) + 16 * f;  // 0..63
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int rl = 4 * (lane >> 4) + e;
      float s0 = 0.f, s1 = 0.f;
      for (int rr = 0; a.t != nullptr && rr < a.r; ++rr) {
        const float tv = lt[rl * 64 + seg * a.r + rr];
        s0 += tv * lw_s[lc * 16 + rr];
        s1 += tv * lw_s[(64 + lc) * 16 + rr];
      }
      v[e] = rnd<T>(v[e] + a.lscale * s0);
      w[e] = rnd<T>(w[e] + a.lscale * s1);
    }
    if (seg < a.rope_segs) {  // column n is pair index i = n % 128 < 64 of its head
      const int i = n & 127;
      const float inv_freq = exp2f(-(float)(2 * i) / 128.f * a.log2_theta);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float pos = (float)((m0 + e) % a.seq);
        float sn, cs;
        sincosf(pos * inv_freq, &sn, &cs);
        const float x0 = v[e], x1 = w[e];
        v[e] = x0 * cs - x1 * sn;
        w[e] = x1 * cs + x0 * sn;
      }
    }
  } else if (EPI == 2) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[e] = rnd<T>(v[e]);
      w[e] = rnd<T>(w[e]);
    }
  } else if (EPI == 3) {
    const T* gu = static_cast<const T*>(a.aux);
    f32x4 du;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int m = min(m0 + e, a.M - 1);
      const float dd = rnd<T>(v[e]);
      const float g = ld1<T>(gu + (int64_t)m * a.ld_aux + n), u = ld1<T>(gu + (int64_t)m * a.ld_aux + a.N + n);
      const float sg = 1.f / (1.f + __expf(-g));
      v[e] = dd * u * (sg * (1.f + g * (1.f - sg)));
      du[e] = dd * g * sg;
    }
    w = du;
  } else if (EPI == 4) {
    const uint64_t key = a.drop ? rng_key(a.rng) : 0ull;
    const int lc = col_of_lane;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int rl = 4 * (lane >> 4) + e;
      const int m = m0 + e;
      float tot = 0.f;
      for (int p = 0; p < a.P; ++p) {
        float sp = 0.f;
        for (int rr = 0; rr < a.r; ++rr) sp += lt[rl * 64 + p * a.r + rr] * lw_s[(p * a.r + rr) * 64 + lc];
        if (a.drop && !lora_keep(key, (uint32_t)(((int64_t)p * a.M + m) * a.N + n), a.thr)) sp = 0.f;
        tot += sp;
      }
      v[e] += tot;
    }
  }

  // ---- outputs through LDS: tile[o][row][col] (o = 0 main / primary, 1 partner, 2 SwiGLU h)
  const int tc = col_of_lane;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int rl = 4 * (lane >> 4) + e;
    st1<T>(reinterpret_cast<T*>(&tile[0][rl][tc]), v[e]);
    if (PAIR || EPI == 3) st1<T>(reinterpret_cast<T*>(&tile[1][rl][tc]), w[e]);
    if (EPI == 2) {
      const float sg = 1.f / (1.f + __expf(-v[e]));
      st1<T>(reinterpret_cast<T*>(&tile[2][rl][tc]), v[e] * sg * w[e]);
    }
  }
  __syncthreads();
  // 16 rows x 64 columns = 128 16-byte chunks per tile
  const int ntiles = EPI == 2 ? 3 : ((PAIR || EPI == 3) ? 2 : 1);
  const int cbase = NN ? (cf0 >> 2) * 64 : cf0 * 16;
  for (int i = tid; i < ntiles * 128; i += 256) {
    const int o = i >> 7, rl = (i >> 3) & 15, ch = i & 7;
    const int m = mrow0 + rl;
    if (m >= a.M) continue;
    const uint4 val = *reinterpret_cast<const uint4*>(&tile[o][rl][ch * 8]);
    T* dst;
    if (o == 2) {
      dst = static_cast<T*>(a.out2) + (int64_t)m * a.ldo2 + cbase + ch * 8;
    } else {
      int col = cbase + ch * 8;
      if (o == 1) col += EPI == 3 ? a.N : pofs * 16;
      dst = static_cast<T*>(a.out) + (int64_t)m * a.ldo + col;
    }
    *reinterpret_cast<uint4*>(dst) = val;
  }
}

}  // namespace

void ws_set_depth(int d) { g_ws_depth = d == 8 ? 8 : 4; }

bool ws_supported(int M, int N, int K, bool nn) {
  if (M < 1 || K < 128 || K % 128 != 0) return false;
  return nn ? (N % 64 == 0) : (N % 16 == 0);
}

// Plan: m-blocks of <= 128 rows (MF = 8), 64 (MF = 4) or 32 (MF = 2); the slice length kr (% 128:
// the k-steps of a slice fill whole D = 4 rings) as long as the resident x slice fits ~144 KB of
// LDS, and column groups G so that MB * S * G ~ 256 workgroups (one per CU).
void ws_plan(int M, int N, int K, bool nn, int* mf, int* kr, int* G, int* nf) {
  *mf = M <= 32 ? 2 : (M <= 64 ? 4 : 8);
  const int mp = *mf * 16;
  const int mb = (M + 127) / 128;
  // LDS budget ~144 KB for the slice: kr <= 144K / (2 * mp), multiple of 32
  int kmax = (144 * 1024) / (2 * mp);
  kmax = min(kmax, 2048) & ~127;
  int S = (K + kmax - 1) / kmax;
  int krr = ((K + S - 1) / S + 127) & ~127;
  S = (K + krr - 1) / krr;
  int g = max(1, 256 / (S * mb));
  *kr = krr;
  *G = g;
  *nf = nn ? 4 : 2;
}

hipError_t ws_gemm(int dtype, bool nn, const void* x, int64_t ldx, const void* w, int64_t ldw, float* part,
                   const void* zero, int M, int N, int K, int mf, int kr, int G, int nf, hipStream_t st, int sb) {
  if (!ws_supported(M, N, K, nn) || (dtype != kBF16 && dtype != kF16)) return hipErrorInvalidValue;
  if (kr < 128 || kr % 128 != 0 || G < 1 || (mf != 2 && mf != 4 && mf != 8)) return hipErrorInvalidValue;
  if (!nn && nf != 1 && nf != 2 && nf != 4) return hipErrorInvalidValue;
  WsArgs a;
  a.x = static_cast<const uint16_t*>(x);
  a.w = static_cast<const uint16_t*>(w);
  a.part = part;
  a.zero = static_cast<const uint16_t*>(zero);
  a.ldx = ldx;
  a.ldw = ldw;
  a.M = M;
  a.N = N;
  a.K = K;
  a.kr = kr;
  a.krp = (kr + 127) & ~127;
  if ((size_t)mf * 16 * a.krp * 2 > 160 * 1024) return hipErrorInvalidValue;
  a.S = (K + kr - 1) / kr;
  a.G = G;
  a.MB = (M + mf * 16 - 1) / (mf * 16);
  a.chunks = nn ? N / 64 : (N / 16 + nf - 1) / nf;
  a.R = a.S * a.G;
  a.sb = sb;
  const int grid = a.MB == 1 ? a.R : a.MB * ((a.R + 7) / 8) * 8;
#define HYP_WS(TT)                                                              \
  if (nn) {                                                                     \
    if (mf == 8) return launch_gemm<TT, 8, 4, true>(a, grid, st);               \
    if (mf == 4) return launch_gemm<TT, 4, 4, true>(a, grid, st);               \
    return launch_gemm<TT, 2, 4, true>(a, grid, st);                            \
  }                                                                             \
  if (mf == 8) {                                                                \
    if (nf == 4) return launch_gemm<TT, 8, 4, false>(a, grid, st);              \
    if (nf == 2) return launch_gemm<TT, 8, 2, false>(a, grid, st);              \
    return launch_gemm<TT, 8, 1, false>(a, grid, st);                           \
  }                                                                             \
  if (mf == 4) {                                                                \
    if (nf == 4) return launch_gemm<TT, 4, 4, false>(a, grid, st);              \
    if (nf == 2) return launch_gemm<TT, 4, 2, false>(a, grid, st);              \
    return launch_gemm<TT, 4, 1, false>(a, grid, st);                           \
  }                                                                             \
  if (nf == 4) return launch_gemm<TT, 2, 4, false>(a, grid, st);                \
  if (nf == 2) return launch_gemm<TT, 2, 2, false>(a, grid, st);                \
  return launch_gemm<TT, 2, 1, false>(a, grid, st);
  if (dtype == kBF16) {
    HYP_WS(bf16_t)
  } else {
    HYP_WS(f16_t)
  }
#undef HYP_WS
}

hipError_t ws_reduce(int dtype, bool nn, const float* part, void* out, int64_t ldo, const void* addend, float alpha,
                     float beta, const float* U, const void* V, int r, int segw, float uscale, int M, int N, int S,
                     int MFtot, hipStream_t st, int sb) {
  if (dtype != kBF16 && dtype != kF16) return hipErrorInvalidValue;
  if (U != nullptr && (V == nullptr || r < 1 || segw < 1 || N % segw != 0)) return hipErrorInvalidValue;
  WsRed a{part, out, ldo, addend, alpha, beta, U, static_cast<const uint16_t*>(V), r, segw, uscale,
          M, N, S, MFtot, nn ? 1 : 0, sb};
  const int64_t nquads = (int64_t)MFtot * (N / 16) * 64;
  const int blocks = (int)((nquads + 255) / 256);
  if (dtype == kBF16) hipLaunchKernelGGL(ws_reduce_k<bf16_t>, dim3(blocks), dim3(256), 0, st, a);
  else hipLaunchKernelGGL(ws_reduce_k<f16_t>, dim3(blocks), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t ws_epilogue(int dtype, int epi, const float* part, int S, int MFtot, int M, int N, void* out, int64_t ldo,
                       void* out2, int64_t ldo2, const void* aux, int64_t ld_aux, const float* t, int ldt,
                       int64_t t_sstride, int t_splits, const void* const* lw, int P, int r, int segw, float lscale,
                       int rope_segs, int seq, float theta, const RngState* rng, float p_drop, bool nn,
                       const void* yin, int64_t ldy, hipStream_t st, int sb) {
  if (dtype != kBF16 && dtype != kF16) return hipErrorInvalidValue;
  if (part == nullptr && yin == nullptr) return hipErrorInvalidValue;
  if (epi != 0 && nn != (epi == 3 || epi == 4)) return hipErrorInvalidValue;  // the slab layout of that GEMM
  if (MFtot * 16 < M || N % 64 != 0 || epi < 0 || epi > 4) return hipErrorInvalidValue;
  const bool lora = t != nullptr;
  if ((epi == 4 || (epi == 1 && lora)) && (t == nullptr || P < 1 || P > 4 || r < 1 || r > 16 || P * r > 64 || lw == nullptr ||
                                            (P * r) % 4 != 0 || ldt % 4 != 0 || t_sstride % 4 != 0 ||
                                            reinterpret_cast<uintptr_t>(t) % 16 != 0))
    return hipErrorInvalidValue;
  if (epi == 1 && (N % 128 != 0 || segw < 128 || segw % 128 != 0 || (lora && N / segw > P))) return hipErrorInvalidValue;
  if (epi == 2 && (N % 128 != 0 || out2 == nullptr)) return hipErrorInvalidValue;
  if (epi == 3 && aux == nullptr) return hipErrorInvalidValue;
  WsEpi a{};
  a.part = part;
  a.sb = sb;
  a.yin = yin;
  a.ldy = ldy;
  a.S = S;
  a.MFtot = MFtot;
  a.M = M;
  a.N = N;
  a.out = out;
  a.ldo = ldo;
  a.out2 = out2;
  a.ldo2 = ldo2;
  a.aux = aux;
  a.ld_aux = ld_aux;
  a.t = t;
  a.ldt = ldt;
  a.t_sstride = t_sstride;
  a.t_splits = t_splits < 1 ? 1 : t_splits;
  for (int i = 0; i < 4; ++i) a.lw[i] = (lw != nullptr && i < P) ? lw[i] : nullptr;
  a.P = P;
  a.r = r;
  a.segw = segw;
  a.lscale = lscale;
  a.rope_segs = rope_segs;
  a.seq = seq > 0 ? seq : M;
  a.log2_theta = log2f(theta > 0.f ? theta : 10000.f);
  a.drop = (rng != nullptr && p_drop > 0.f) ? 1 : 0;
  if (a.drop) a.rng = *rng;
  a.thr = (uint32_t)fminf(p_drop * 4294967296.f, 4294967295.f);
  const int mfv = (M + 15) / 16;
  dim3 grid(epi == 1 ? N / 128 : (epi == 2 ? N / 128 : N / 64), mfv);
#define HYP_EPI(TT)                                                                            \
  switch (epi) {                                                                               \
    case 0:                                                                                    \
      if (nn) hipLaunchKernelGGL((ws_epi_k<TT, 0, true>), grid, dim3(256), 0, st, a);          \
      else hipLaunchKernelGGL((ws_epi_k<TT, 0, false>), grid, dim3(256), 0, st, a);            \
      break;                                                                                   \
    case 1: hipLaunchKernelGGL((ws_epi_k<TT, 1, false>), grid, dim3(256), 0, st, a); break;   \
    case 2: hipLaunchKernelGGL((ws_epi_k<TT, 2, false>), grid, dim3(256), 0, st, a); break;   \
    case 3: hipLaunchKernelGGL((ws_epi_k<TT, 3, true>), grid, dim3(256), 0, st, a); break;    \
    default: hipLaunchKernelGGL((ws_epi_k<TT, 4, true>), grid, dim3(256), 0, st, a); break;   \
  }
  if (dtype == kBF16) {
    HYP_EPI(bf16_t)
  } else {
    HYP_EPI(f16_t)
  }
#undef HYP_EPI
  return hipGetLastError();
}

}  // namespace hyp

// Persistent implicit-GEMM convolution: each workgroup walks several output tiles and issues the
// NEXT tile's first LDS-DMA stages before it runs the CURRENT tile's epilogue.
//
// Why (MI355X, ResNet-50 batch 32): a conv workgroup's timeline is ~2-3 us of first loads, a 0.5-2 us
// K loop and ~2-3.5 us of epilogue (profiles/r04/conv_timeline_p2.json) at 2-4 resident workgroups
// per CU, so a plain launch spends most of each tile waiting, and rounds of workgroups quantise
// (784 tiles on 768 slots = two rounds).  Here the grid is sized to the resident capacity (a
// multiple of 8, so tile t = blk + i*nblk keeps the XCD of its plain-launch id) with the tiles
// spread evenly, and tile i+1's first stages are in flight while tile i's accumulators are rounded,
// transposed, summed and stored — its prologue latency hides behind the epilogue.
//
// Same numerics as conv_fwd_k (bitwise: the same MFMA order, roundings and statistics partials per
// tile) for the variants the ResNet step runs: forward + BN statistics, plain data gradient and
// data gradient + BN-backward epilogue (LEAN / full), stride-1 or the stride-2 phase split; no
// split-K, XF, DIRECT, CE or timeline stamps (those keep conv_fwd_k).
//
// LDS: the NB-deep ring; the epilogue's transpose tile lives in ring slot NB-1 (free between the
// K loop's final barrier and the next tile's first K step, which is exactly the epilogue) when it
// fits, else in its own region after the ring.
#pragma once
#include "conv_fwd_impl.h"

namespace hyp {
namespace {

template <int BM, int BN, int NB>
struct PersistLds {
  static constexpr int kBuf = (BM + BN) * kBK;
  static constexpr int kEpi = BM * (BN + 8) + 16 * BN;  // transpose tile + reduction scratch
  static constexpr bool kInRing = NB >= 2 && kEpi <= kBuf;
  static constexpr int kElems = kInRing ? NB * kBuf : NB * kBuf + kEpi;
  static constexpr int kEpiOff = kInRing ? (NB - 1) * kBuf : NB * kBuf;
};

template <int IA, int IB>
struct PTile {
  int t, m0, n0, tm, ph_a, ph_b, r0, s0, nr, ns, nk;
  int st_r, st_s, st_c0, st_t;  // reduction position of the next stage to issue
  int64_t a_off[IA];
  int a_h0[IA], a_w0[IA];
  bool a_ok[IA];
  const uint16_t* b_src[IB];
};

template <typename T, int BM, int BN, bool STATS, bool DGRAD, int NB, bool LEAN>
__device__ __forceinline__ void conv_persist_body(const ConvArgs& a, const int blk, const int nblk, uint16_t* smem) {
  constexpr int FM = BM / 32, FN = BN / 32;
  constexpr int IA = BM / 32, IB = BN / 32;
  using L = PersistLds<BM, BN, NB>;
  constexpr int kBuf = L::kBuf;
  uint16_t* epi = smem + L::kEpiOff;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int slot = lane & 7;
  const bool sd2 = DGRAD && a.sd == 2;
  const int tiles_m = (a.M + BM - 1) / BM, tiles_n = (a.K + BN - 1) / BN, nwg = tiles_m * tiles_n;
  const int ntiles = nwg * (sd2 ? 4 : 1);
  const int PQ = a.P * a.Q;
  const int cpb = a.C / kBK;
  const int64_t ldw = (int64_t)a.R * a.S * a.C;
  const uint16_t* zero = a.zero + slot * 8;
  const int kGroup = a.group, group = kGroup * tiles_n;

  // tile coordinates and per-lane row bookkeeping of tile id t (conv_fwd_body's, splits == 1)
  auto setup = [&](PTile<IA, IB>& s, int t) {
    s.t = t;
    int bid, phase = 0;
    if (sd2) {
      const int lb = mfl::xcd_remap(t, nwg * 4);
      phase = lb & 3;
      bid = lb >> 2;
    } else {
      bid = mfl::xcd_remap(t, nwg);
    }
    s.ph_a = phase >> 1;
    s.ph_b = phase & 1;
    s.r0 = sd2 ? ((s.ph_a + a.ph) & 1) : 0;
    s.s0 = sd2 ? ((s.ph_b + a.pw) & 1) : 0;
    s.nr = sd2 ? (a.R - s.r0 + 1) / 2 : a.R;
    s.ns = sd2 ? (a.S - s.s0 + 1) / 2 : a.S;
    const int first_m = (bid / group) * kGroup;
    const int gsize = min(tiles_m - first_m, kGroup);
    s.tm = first_m + (bid % group) % gsize;
    const int tn = (bid % group) / gsize;
    s.m0 = s.tm * BM;
    s.n0 = tn * BN;
#pragma unroll
    for (int i = 0; i < IA; ++i) {
      const int row = (i * 4 + wave) * 8 + (lane >> 3);
      const int m = s.m0 + row;
      const int chunk = slot ^ swz(row);
      s.a_ok[i] = m < a.M;
      const int mm = s.a_ok[i] ? m : 0;
      const int n = fdiv36(mm, a.mpq, PQ), pq = mm - n * PQ, p = fdiv36(pq, a.mq, a.Q), q = pq - p * a.Q;
      s.a_h0[i] = sd2 ? p + (s.ph_a + a.ph - s.r0) / 2 : p * a.sh - a.ph;
      s.a_w0[i] = sd2 ? q + (s.ph_b + a.pw - s.s0) / 2 : q * a.sw - a.pw;
      s.a_off[i] = (((int64_t)n * a.H + s.a_h0[i]) * a.W + s.a_w0[i]) * a.pix + chunk * 8;
    }
#pragma unroll
    for (int i = 0; i < IB; ++i) {
      if (!DGRAD) {
        const int row = (i * 4 + wave) * 8 + (lane >> 3);
        const int k = s.n0 + row;
        const int chunk = slot ^ swz(row);
        s.b_src[i] = k < a.kvalid ? a.w + (int64_t)k * ldw + chunk * 8 : nullptr;
      } else {
        constexpr int RB = 1024 / (2 * BN), CB = BN / 8;
        const int row = (i * 4 + wave) * RB + lane / CB;
        const int col = s.n0 + (((lane % CB) ^ mfl::swz_tr<BN>(row)) << 3);
        s.b_src[i] = col < a.K ? a.w + (int64_t)mfl::tr_row_to_k(row) * a.R * a.S * a.K + col : nullptr;
      }
    }
    s.nk = sd2 ? s.nr * s.ns * cpb : a.R * a.S * cpb;
    s.st_r = s.st_s = s.st_c0 = s.st_t = 0;
  };
  auto stage = [&](PTile<IA, IB>& s, uint16_t* buf) {
    const int r = s.st_r, sx = s.st_s, c0 = s.st_c0;
    const int dh = sd2 ? -r : r, dw = sd2 ? -sx : sx;
    const int64_t tap = ((int64_t)dh * a.W + dw) * a.pix + c0;
#pragma unroll
    for (int i = 0; i < IA; ++i) {
      const int h = s.a_h0[i] + dh, w = s.a_w0[i] + dw;
      const bool ok = s.a_ok[i] & ((unsigned)h < (unsigned)a.H) & ((unsigned)w < (unsigned)a.W);
      glds16(ok ? a.in + s.a_off[i] + tap : zero, buf + (i * 4 + wave) * 8 * kBK);
    }
    const int64_t kofs =
        DGRAD ? ((int64_t)c0 * a.R * a.S +
                 (sd2 ? (s.r0 + 2 * r) * a.S + s.s0 + 2 * sx : (a.R - 1 - r) * a.S + (a.S - 1 - sx))) * a.K
              : (int64_t)s.st_t * kBK;
#pragma unroll
    for (int i = 0; i < IB; ++i) glds16(s.b_src[i] ? s.b_src[i] + kofs : zero, buf + BM * kBK + (i * 4 + wave) * 512);
    ++s.st_t;
    s.st_c0 += kBK;
    if (s.st_c0 == a.C) {
      s.st_c0 = 0;
      if (++s.st_s == s.ns) {
        s.st_s = 0;
        ++s.st_r;
      }
    }
  };
  auto prologue = [&](PTile<IA, IB>& s) {
#pragma unroll
    for (int i = 0; i < (NB > 1 ? NB - 1 : 1); ++i)
      if (i < s.nk) stage(s, smem + i * kBuf);
  };

  constexpr bool FSTATS = STATS && !DGRAD, BNB = STATS && DGRAD;
  constexpr int kChunksPerRow = BN / 8;
  constexpr int kIt = BM * kChunksPerRow / kThreads;
  constexpr int kLd = BN + 8;
  const int r16 = lane & 15, c4 = lane >> 4;

  PTile<IA, IB> cur;
  if (blk >= ntiles) return;
  setup(cur, blk);
  __builtin_amdgcn_sched_barrier(0);
  prologue(cur);
  __builtin_amdgcn_sched_barrier(0);
  for (;;) {
    const int m0 = cur.m0, n0 = cur.n0;
    auto orow = [&](int m) -> int64_t {
      if (!sd2) return m;
      const int n = fdiv36(m, a.mpq, PQ), pq = m - n * PQ, p = fdiv36(pq, a.mq, a.Q), q = pq - p * a.Q;
      return ((int64_t)n * a.Hx + 2 * p + cur.ph_a) * a.Wx + 2 * q + cur.ph_b;
    };
    // epilogue operand prefetch + per-channel constants (conv_fwd_body's, for this tile)
    uint4 pd[kIt], px[kIt], py[kIt];
    const bool has_add = !FSTATS && !LEAN && a.addend != nullptr;
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
      const int idx = it * kThreads + tid;
      const int lr = idx / kChunksPerRow, ch = idx - lr * kChunksPerRow;
      const int m = m0 + lr, k = n0 + ch * 8;
      const bool ok = m < a.M && k < a.K;
      const int64_t off = (ok ? orow(m) : 0) * a.K + k;
      pd[it] = px[it] = py[it] = uint4{0u, 0u, 0u, 0u};
      if (has_add && ok) pd[it] = *reinterpret_cast<const uint4*>(a.addend + off);
      if (BNB && ok) {
        px[it] = *reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(a.bnb.x) + off);
        if (!LEAN && a.bnb.mode == 2) py[it] = *reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(a.bnb.y) + off);
      }
    }
    float asc[8], ash[8];
    {
      const int my_k = n0 + (tid % kChunksPerRow) * 8;
#pragma unroll
      for (int e = 0; e < 8; ++e) asc[e] = ash[e] = 0.f;
      auto ld8 = [](const float* p, float (&v)[8]) {
        const float4 x0 = reinterpret_cast<const float4*>(p)[0], x1 = reinterpret_cast<const float4*>(p)[1];
        v[0] = x0.x; v[1] = x0.y; v[2] = x0.z; v[3] = x0.w; v[4] = x1.x; v[5] = x1.y; v[6] = x1.z; v[7] = x1.w;
      };
      if (BNB && a.bnb.mode == 1 && my_k < a.K) {
        float wv[8], iv[8], bv[8], mv[8];
        ld8(a.bnb.invstd + my_k, iv);
        ld8(a.bnb.mean + my_k, mv);
#pragma unroll
        for (int e = 0; e < 8; ++e) wv[e] = 1.f, bv[e] = 0.f;
        if (a.bnb.w) ld8(a.bnb.w + my_k, wv);
        if (a.bnb.b) ld8(a.bnb.b + my_k, bv);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float sc = wv[e] * iv[e];
          asc[e] = sc;
          ash[e] = bv[e] - mv[e] * sc;
        }
      }
    }

    // ---- K loop (conv_fwd_body's)
    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int nk = cur.nk;
    for (int t = 0; t < nk; ++t) {
      if (NB == 1) {
        if (t > 0) {
          mfl::barrier_keep_vm();
          stage(cur, smem);
        }
        mfl::wait_vmcnt<0>();
        mfl::barrier_keep_vm();
      } else {
        mfl::wait_stage<IA + IB, NB>(min(NB - 2, nk - 1 - t));
        mfl::barrier_keep_vm();
        if (t + NB - 1 < nk) stage(cur, smem + ((t + NB - 1) % NB) * kBuf);
      }
      const uint16_t* as = smem + (t % NB) * kBuf;
      const uint16_t* bs = as + BM * kBK;
#pragma unroll
      for (int ks = 0; ks < kBK / 32; ++ks) {
        u16x8 fa[FM], fb[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) fa[i] = frag(as, wm * (BM / 2) + i * 16 + r16, ks * 4 + c4);
#pragma unroll
        for (int j = 0; j < FN; ++j)
          fb[j] = DGRAD ? mfl::frag_tr<BN>(bs, ks * 32, wn * (BN / 2) + j * 16, lane)
                        : frag(bs, wn * (BN / 2) + j * 16 + r16, ks * 4 + c4);
        if (DGRAD) mfl::lds_reads_done();
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) acc[i][j] = mma<T>(fa[i], fb[j], acc[i][j]);
      }
    }
    __syncthreads();  // every wave is done with the ring

    // ---- the next tile's first stages go out now: their latency overlaps this epilogue
    const int tnext = cur.t + nblk;
    const bool more = tnext < ntiles;
    PTile<IA, IB> nxt;
    if (more) {
      setup(nxt, tnext);
      __builtin_amdgcn_sched_barrier(0);
      prologue(nxt);
      __builtin_amdgcn_sched_barrier(0);
    }

    // ---- epilogue (conv_fwd_body's LDS-transpose path) in the epilogue region
    uint16_t* tile = epi;
    float* red = reinterpret_cast<float*>(epi + BM * kLd);
    float csum[FN], csq[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) csum[j] = csq[j] = 0.f;
    const bool odd = r16 & 1;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int lc = wn * (BN / 2) + j * 16 + (r16 & ~1);
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = rnd<T>(acc[i][j][e]);
          if (FSTATS && m0 + wm * (BM / 2) + i * 16 + c4 * 4 + e < a.M) {
            csum[j] += v[e];
            csq[j] += v[e] * v[e];
          }
        }
#pragma unroll
        for (int ep = 0; ep < 4; ep += 2) {
          const float got = __builtin_bit_cast(
              float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, odd ? v[ep] : v[ep + 1]), 0xB1, 0xF, 0xF, false));
          const int lr = wm * (BM / 2) + i * 16 + c4 * 4 + ep + (odd ? 1 : 0);
          const uint32_t pk = pack2<T>(odd ? got : v[ep], odd ? v[ep + 1] : got);
          *reinterpret_cast<uint32_t*>(reinterpret_cast<T*>(tile) + lr * kLd + lc) = pk;
        }
      }
    }
    if (FSTATS) {
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        csum[j] += __shfl_xor(csum[j], 16, 64);
        csum[j] += __shfl_xor(csum[j], 32, 64);
        csq[j] += __shfl_xor(csq[j], 16, 64);
        csq[j] += __shfl_xor(csq[j], 32, 64);
      }
      if (c4 == 0) {
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int col = wn * (BN / 2) + j * 16 + r16;
          red[(wm * 2 + 0) * BN + col] = csum[j];
          red[(wm * 2 + 1) * BN + col] = csq[j];
        }
      }
    }
    __syncthreads();
    if (FSTATS && tid < BN) {
      const int k = n0 + tid;
      if (k < a.K) {
        const int64_t sl = (int64_t)(cur.tm % kStatSlots) * 2 * a.K;
        unsafeAtomicAdd(a.psum + sl + k, (double)(red[0 * BN + tid] + red[2 * BN + tid]));
        unsafeAtomicAdd(a.psq + sl + k, (double)(red[1 * BN + tid] + red[3 * BN + tid]));
      }
    }
    float bs_[8], bq_[8];
    if (BNB) {
#pragma unroll
      for (int e = 0; e < 8; ++e) bs_[e] = bq_[e] = 0.f;
    }
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
      const int idx = it * kThreads + tid;
      const int lr = idx / kChunksPerRow, ch = idx - lr * kChunksPerRow;
      const int m = m0 + lr, k = n0 + ch * 8;
      if (m < a.M && k < a.K) {
        uint4 v = *reinterpret_cast<const uint4*>(tile + lr * kLd + ch * 8);
        if (BNB) {
          float o[8], xv[8], yv[8] = {};
          Vec8<T>::load(reinterpret_cast<const T*>(&v), o);
          if (has_add) {
            float d[8];
            Vec8<T>::load(reinterpret_cast<const T*>(&pd[it]), d);
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] = rnd<T>(o[e] + d[e]);
          }
          Vec8<T>::load(reinterpret_cast<const T*>(&px[it]), xv);
          if (!LEAN) Vec8<T>::load(reinterpret_cast<const T*>(&py[it]), yv);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const bool keep =
                a.bnb.mode == 0 || ((LEAN || a.bnb.mode == 1) ? fmaf(xv[e], asc[e], ash[e]) > 0.f : yv[e] > 0.f);
            o[e] = keep ? o[e] : 0.f;
            bs_[e] += o[e];
            bq_[e] += o[e] * xv[e];
          }
          Vec8<T>::store(reinterpret_cast<T*>(&v), o);
        } else if (!STATS && has_add) {
          float o[8], d[8];
          Vec8<T>::load(reinterpret_cast<const T*>(&v), o);
          Vec8<T>::load(reinterpret_cast<const T*>(&pd[it]), d);
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] += d[e];
          Vec8<T>::store(reinterpret_cast<T*>(&v), o);
        }
        st16_wt(a.out + orow(m) * a.K + k, v);
      }
    }
    if (BNB) {
      static_assert(64 % kChunksPerRow == 0, "chunk columns repeat within a wave");
#pragma unroll
      for (int o = kChunksPerRow; o < 64; o <<= 1) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          bs_[e] += __shfl_xor(bs_[e], o, 64);
          bq_[e] += __shfl_xor(bq_[e], o, 64);
        }
      }
      float* wred = reinterpret_cast<float*>(epi + BM * kLd);  // (after the tile: no barrier needed)
      if (lane < kChunksPerRow) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          wred[(wave * kChunksPerRow + lane) * 16 + e] = bs_[e];
          wred[(wave * kChunksPerRow + lane) * 16 + 8 + e] = bq_[e];
        }
      }
      __syncthreads();
      if (tid < BN && n0 + tid < a.K) {
        const int chn = tid >> 3, e = tid & 7;
        float sa = 0.f, sb = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          sa += wred[(w * kChunksPerRow + chn) * 16 + e];
          sb += wred[(w * kChunksPerRow + chn) * 16 + 8 + e];
        }
        double* sl = a.bnb.sums + (int64_t)(cur.tm % kStatSlots) * 2 * a.K;
        unsafeAtomicAdd(sl + n0 + tid, (double)sa);
        unsafeAtomicAdd(sl + a.K + n0 + tid, (double)sb);
      }
    }
    if (!more) break;
    cur = nxt;
  }
}

template <typename T, int BM, int BN, bool STATS, bool DGRAD, int NB, bool LEAN>
__global__ __launch_bounds__(kThreads) void conv_persist_k(const ConvArgs a, const int nblk) {
  __shared__ __attribute__((aligned(16))) uint16_t smem[PersistLds<BM, BN, NB>::kElems];
  conv_persist_body<T, BM, BN, STATS, DGRAD, NB, LEAN>(a, blockIdx.x, nblk, smem);
}

}  // namespace
}  // namespace hyp

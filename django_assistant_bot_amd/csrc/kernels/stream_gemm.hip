// Warp-specialised weight-streaming MFMA GEMM for decode batches:  C[M, N] = X[M, K] . W[N, K]^T,
// M <= 256 (decode batches; also the LM head of prefill last tokens and the index scan of 17-128 queries).
//
// Why warp specialisation: at M = 128 a single-queue design (weights and X on the same waves) waits,
// every stage,
// for an X load that sits behind the newest weight loads in the wave's in-order vmcnt queue, so at
// most ~1.5 stages of weights are ever in flight and each 16-33 MB projection runs at 2-3 TB/s
// (profiles/decode_gemm_m128_study.md).  Here the two operands travel on different waves:
//
//   * 4 compute waves stream W straight into VGPRs (MFMA A fragments, 16-B buffer loads) through an
//     NWIN-stage register ring: a slot is reloaded NWIN stages ahead right behind its MFMAs, and
//     since these waves issue nothing but weight loads, the compiler's in-order vmcnt waits only
//     ever wait for the oldest slot (NWIN x 4-8 KB per wave in flight, ~100 KB per CU);
//   * 1 loader wave stages X (L2-resident, shared by the compute waves) into an NB-deep LDS ring
//     with global_load_lds (no VGPRs, source-swizzled so the image is lane-linear), retires each
//     stage with a counted vmcnt and publishes it with the stage barrier (raw s_barrier: every wave
//     passes one barrier per stage, nobody drains a queue at it);
//   * waves = KG k-groups x (4 / KG) row groups of RT 16-row tiles; v_mfma_f32_16x16x32_bf16 with W
//     as A and X as B (one LDS fragment feeds RT MFMAs); partial tiles of the k-groups meet in LDS.
//
// Outputs: S == 1 -> bf16 (optional residual add, or SwiGLU over 16- / 8-row interleaved [gate | up]
// weights); S > 1 -> fp32 K-slice slabs [S][M][N] summed by the consumer's prologue (rmsnorm,
// rope_kv_write) or by slab_reduce below.  Block -> (tile, slice)
// keeps a tile's slices on one XCD (bijective remap, slice-minor).
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "launchers.h"

#define DAB_INLINE __attribute__((always_inline))

namespace dab {

struct StreamParams {
  const bf16* X;
  long ldx;
  const bf16* W;
  long ldw;
  void* out;
  long ldo;
  const bf16* residual;
  long ldr;
  int M, N, K, S, kc;
  int epi;       // 0 none, 2 swiglu (16-row gate | up groups), 4 swiglu (8-row groups), 8 candidates
  // RMSNorm in the consumer (small decode batches): X is the raw residual stream
  // h and the norm gains are folded into W's columns, so RMSNorm(h) W^T = r[m] (h W^T) with
  // r[m] = rsqrt(mean_k h[m][k]^2 + eps).  The epilogue computes r from the X rows (L2-resident,
  // all K even for a K-slice) and scales the accumulators before the slab store / SwiGLU: the
  // separate slab-summing RMSNorm launch disappears (its producer writes h with its residual add).
  int norm;
  float norm_eps;
  int slice_xcd;  // block -> (tile, slice) with the K-slices (not the tiles) grouped per XCD
  int slab_bf16;  // S > 1: bf16 K-slice slabs instead of fp32
  int wgrp;       // SHUF: row blocks per group of the weight copy (shuffle_weights(w, group)), 1 = plain
  // ST_EPI_CAND (index threshold search over W = index rows, X = queries): filtered scores
  // >= thr[m] are appended to query m's list (gemm.hip EPI_CANDIDATES); N need not divide BN
  const int* row_group;  // [N] (<0 = deleted) or null
  const int* q_group;    // [M] (<0 = any) or null
  const float* thr;      // [M]
  int* cnt;              // [M]
  float* cand_val;       // [M, cap]
  int* cand_idx;         // [M, cap]
  int cap;
};

constexpr int ST_EPI_NONE = 0, ST_EPI_SWIGLU = 2, ST_EPI_SWIGLU8 = 4, ST_EPI_CAND = 8;

constexpr int cgcd(int a, int b) { return b == 0 ? a : cgcd(b, a % b); }
constexpr int clcm(int a, int b) { return a / cgcd(a, b) * b; }

// vmcnt(N) with expcnt / lgkmcnt left unconstrained (gfx9 encoding: vmcnt[3:0] | vmcnt[5:4] << 14)
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N <= 63, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x70 | 0xF00);
}
__device__ __forceinline__ void wait_lgkm0() { __builtin_amdgcn_s_waitcnt(0xc07f); }

// f(integral_constant<I>) for I in [B, E) while it returns true
template <int B, int E, typename F>
__device__ __forceinline__ bool static_for(F&& f) {
  if constexpr (B < E) {
    if (!f(std::integral_constant<int, B>{})) return false;
    return static_for<B + 1, E>(f);
  }
  return true;
}

// ABL (benchmark ablations only): 1 no X staging, 2 no MFMA, 3 weight stream only (no X, no LDS
// reads, no MFMA), 4 no split-K slab stores, 5 the weight addressing of a tile-interleaved fragment
// layout (the full kernel on the wrong bytes: what that layout's access pattern would cost); results
// are garbage, timings bound the parts.
//
// NWC compute waves (waves NWC.. are the NL X loaders).  BN = 16 RT NWC / KG need not be a power of
// two: 112 rows (7 waves) tile Llama-3-8B's 28672 gate_up rows onto exactly 256 workgroups, 96 rows
// (6 waves, 4 K-slices) its 6144 qkv rows; the epilogue tile keeps a power-of-two row stride BNP.
template <int MT, int RT, int KG, int KS, int NB, int NWIN, int NL, bool SHUF, bool NT_W, int ABL = 0, int NWC = 4>
__global__ __launch_bounds__(64 * (NWC + NL), 1) void stream_gemm_kernel(StreamParams p) {
  constexpr int RG = NWC / KG;        // row groups
  constexpr int BN = 16 * RT * RG;    // weight rows per workgroup
  constexpr int BNP = BN <= 64 ? 64 : BN <= 128 ? 128 : 256;  // epilogue tile row stride (XOR swizzle range)
  constexpr int MP = 16 * MT;         // padded M
  constexpr int ROWB = KS * 2;        // bytes per staged X row
  constexpr int CPR = KS / 8;         // 16-B chunks per staged row
  constexpr int XBUF = MP * ROWB;     // bytes per X stage
  constexpr int GPS = XBUF / 1024;    // global_load_lds per stage (64 lanes x 16 B), all loaders
  constexpr int GPL = GPS / NL;       // ... per loader wave
  constexpr int KW = KS / KG;         // k per compute wave per stage
  constexpr int CPW = KW / 32;        // 32-deep MFMA chunks per wave per stage
  constexpr int RED = KG * MP * BNP * 4;
  static_assert(BN <= 256 && BN % 16 == 0, "tile rows");
  // + per-row scales of the consumer RMSNorm and each wave's per-row sums of squares (after the ring
  // / reduction area)
  constexpr int SMEM = (NB * XBUF > RED ? NB * XBUF : RED) + MP * 4 * (1 + NWC + NL);
  static_assert(CPR >= 16 && CPW >= 1 && KW % 32 == 0, "stage shape");
  static_assert(NB >= 2 && (NB - 2) * GPL <= 63 && GPS % NL == 0, "loader vmcnt range");
  static_assert(NWC % KG == 0, "k groups");
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tiles = (p.N + BN - 1) / BN;  // partial last tile: candidates only (rows >= N read zeros)
  const int nwg = tiles * p.S;
  const int bid = blockIdx.x;
  const int xcd = bid % 8, q8 = nwg / 8, r8 = nwg % 8;
  const int sid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  // slice_xcd (S a multiple of 8): the workgroups sharing an XCD share K-slices instead of tiles, so
  // each XCD's L2 holds S / 8 slices of X rather than all of it
  const int tile = p.slice_xcd ? bid / p.S : sid / p.S;
  const int slice = p.slice_xcd ? (bid % 8) * (p.S / 8) + (bid / 8) % (p.S / 8) : sid % p.S;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, g = lane >> 4, li = lane & 15;
  const int n0 = tile * BN;
  const int k_begin = slice * p.kc;
  const int nst = p.kc / KS;

  float* red = reinterpret_cast<float*>(smem);  // epilogue partials (after the K loop)
  if (w >= NWC) {
    // ------------------------------------------------------------------ X loader waves
    // loader l issues instructions i = l, l + NL, ... of each stage (1 KB each)
    const int l = w - NWC;
    // stage s image: row r (= m), physical chunk pc holds logical chunk pc ^ (r & 15); rows >= M
    // repeat row M-1 (their outputs are never stored)
    const bf16* xk = p.X + k_begin;
    auto issue = [&](int s) DAB_INLINE {
      char* buf = smem + (s % NB) * XBUF;
#pragma unroll
      for (int j = 0; j < GPL; ++j) {
        const int i = j * NL + l;
        const int e = i * 64 + lane;
        const int r = e / CPR, pc = e % CPR;
        const bf16* src = xk + (size_t)min(r, p.M - 1) * p.ldx + s * KS + (pc ^ (r & 15)) * 8;
        __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(buf + i * 1024),
                                         16, 0, 0);
      }
    };
    // retire everything but the newest `n` stages (n <= NB - 2)
    auto retire = [&](int n) DAB_INLINE {
      static_for<0, NB - 1>([&](auto I) DAB_INLINE {
        constexpr int i = decltype(I)::value;
        if (n == i) wait_vm<i * GPL>();
        return true;
      });
    };
    const int pre = (ABL == 1 || ABL == 3) ? 1 : min(NB - 1, nst);
    for (int s = 0; s < pre; ++s) issue(s);
    retire(pre - 1);
    __builtin_amdgcn_s_barrier();
    for (int st = 0; st < nst; ++st) {
      if (ABL == 1 || ABL == 3) {
        __builtin_amdgcn_s_barrier();
        continue;
      }
      if (st + NB - 1 < nst) issue(st + NB - 1);  // into the buffer read in stage st - 1
      if (st + 1 < nst) retire(min(st + NB - 1, nst - 1) - (st + 1));
      __builtin_amdgcn_s_barrier();
    }
  } else {
    // ------------------------------------------------------------------ compute waves
    const int rg = w / KG, kg = w % KG;
    // SHUF: whole 16-row blocks (a block's rows are interleaved in every 1 KB fragment; the rows
    // past N of a partial block exist in the copy and are dropped by the epilogues)
    const int w_rows = SHUF ? min(BN, (p.N - n0 + 15) / 16 * 16) : min(BN, p.N - n0);
    // grouped fragment layout (p.wgrp = G > 1, shuffle_weights(w, group=G)): the G row blocks of a
    // group are adjacent per 32-deep k chunk, fragment (b, c) at ((b / G) K/32 + c) G + b % G KB;
    // block offsets are then absolute (descriptor over the whole copy) and a k chunk is G KB on
    const bool grp = SHUF && p.wgrp > 1;
    const auto wres = __builtin_amdgcn_make_buffer_rsrc((void*)(p.W + (grp ? 0 : (size_t)n0 * p.ldw)), 0,
                                                        grp ? (int)((long)p.N * p.K * 2) : (int)(w_rows * p.ldw * 2),
                                                        0x00020000);
    const int cstride = SHUF ? (grp ? p.wgrp : 1) * 1024 : 0;  // bytes per 32-deep k chunk (SHUF)
    // row-major W: lane (li, g) reads row li, k 8g..8g+7 of a 16 x 32 chunk (16 rows x 64 B per load);
    // SHUF (shuffle_weights layout [N/16][K/32][64 lanes][8]): every load is 1 KB contiguous
    const int w_voff = SHUF ? lane * 16 + ((k_begin + kg * KW) / 32) * cstride
                            : (int)(((16 * RT * rg + li) * p.ldw + k_begin + kg * KW + 8 * g) * 2);
    const int a_stride = SHUF ? p.K * 32 : 16 * (int)p.ldw * 2;
    const int w_rowtile0 = SHUF ? RT * rg * p.K * 32 : 0;
    // SHUF: byte offset of row block (RT rg + a) of the tile at k chunk 0
    int wblk[RT];
#pragma unroll
    for (int a = 0; a < RT; ++a) {
      if (grp) {
        const int b = n0 / 16 + RT * rg + a;
        wblk[a] = ((b / p.wgrp) * (p.K / 32) * p.wgrp + b % p.wgrp) * 1024;
      } else {
        wblk[a] = a * a_stride + w_rowtile0;
      }
    }
    bf16x8 wr[NWIN][RT][CPW];
    // clamped past the slice end: the ring keeps a branch-free load stream, so the compiler's
    // in-order vmcnt count stays exact (the spare loads re-read the last stage from L2)
    auto load_w = [&](int slot, int st, int a, int c) DAB_INLINE {
      if constexpr (ABL == 5) {
        // the addressing of a tile-interleaved fragment layout (fragment (row block b of the tile,
        // k chunk) at chunk * BN/16 + b): every wave of the workgroup reads next to the others
        // (profiles/decode_stream_layout_r6.md)
        const int chunk = (k_begin + kg * KW) / 32 + min(st, nst - 1) * (KS / 32) + c;
        const int off = (chunk * (BN / 16) + RT * rg + a) * 1024 + lane * 16;
        wr[slot][a][c] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(wres, off, 0, NT_W ? 2 : 0));
      } else if constexpr (SHUF) {
        const int soff = min(st, nst - 1) * (KS / 32) * cstride + wblk[a];
        wr[slot][a][c] = __builtin_bit_cast(
            bf16x8, __builtin_amdgcn_raw_buffer_load_b128(wres, w_voff + cstride * c, soff, NT_W ? 2 : 0));
      } else {
        const int soff = min(st, nst - 1) * KS * 2 + a * a_stride + w_rowtile0;
        wr[slot][a][c] = __builtin_bit_cast(
            bf16x8, __builtin_amdgcn_raw_buffer_load_b128(wres, w_voff + 64 * c, soff, NT_W ? 2 : 0));
      }
    };
    static_for<0, NWIN>([&](auto S_) DAB_INLINE {
      constexpr int s = decltype(S_)::value;
#pragma unroll
      for (int a = 0; a < RT; ++a)
#pragma unroll
        for (int c = 0; c < CPW; ++c) load_w(s, s, a, c);
      return true;
    });
    f32x4 acc[RT][MT];
#pragma unroll
    for (int a = 0; a < RT; ++a)
#pragma unroll
      for (int t = 0; t < MT; ++t) acc[a][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    // one stage: ring slot H (static), LDS buffer st % NB (runtime address only)
    auto stage = [&](auto H_, int st) DAB_INLINE {
      constexpr int h = decltype(H_)::value;
      const char* xb = smem + (st % NB) * XBUF;
#pragma unroll
      for (int c = 0; c < CPW; ++c) {
        const int lc = kg * (KW / 8) + 4 * c + g;  // logical chunk: this lane's 8 k of chunk c
        bf16x8 bx[MT];
#pragma unroll
        for (int t = 0; t < MT; ++t)
          if constexpr (ABL != 3) bx[t] = *reinterpret_cast<const bf16x8*>(xb + (16 * t + li) * ROWB + 16 * (lc ^ li));
#pragma unroll
        for (int a = 0; a < RT; ++a) {
          if constexpr (ABL == 2 || ABL == 3) {
            asm volatile("" ::"v"(wr[h][a][c]));
            if constexpr (ABL == 2) {
#pragma unroll
              for (int t = 0; t < MT; ++t) asm volatile("" ::"v"(bx[t]));
            }
          } else {
#pragma unroll
            for (int t = 0; t < MT; ++t) acc[a][t] = mfma16(wr[h][a][c], bx[t], acc[a][t]);
          }
          load_w(h, st + NWIN, a, c);
          // keep the reload right behind its MFMAs (the scheduler would otherwise sink every
          // reload to the stage end and halve the bytes in flight)
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      wait_lgkm0();
      __builtin_amdgcn_s_barrier();
    };
    __builtin_amdgcn_s_barrier();
    int st0 = 0;
    for (; st0 + NWIN <= nst; st0 += NWIN)
      static_for<0, NWIN>([&](auto J) DAB_INLINE {
        stage(J, st0 + decltype(J)::value);
        return true;
      });
    // tail: the remaining nst % NWIN stages keep their static slots
    const int rem = nst - st0;
    static_for<0, NWIN - 1>([&](auto J) DAB_INLINE {
      if (decltype(J)::value >= rem) return false;
      stage(J, st0 + decltype(J)::value);
      return true;
    });
    // partial tile of k-group kg: red[kg][m][BN], 4-float column groups XOR-swizzled by m (every
    // wave has passed the last stage barrier: the X ring is dead)
#pragma unroll
    for (int a = 0; a < RT; ++a)
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const int m = 16 * t + li;
        const int col = (16 * (RT * rg + a) + 4 * g) ^ (4 * (m & 15));
        *reinterpret_cast<f32x4*>(red + (kg * MP + m) * BNP + col) = acc[a][t];
      }
  }

  // ---------------------------------------------------------------- epilogue (all 5 waves)
  constexpr int NT = 64 * (NWC + NL);
  float* rsq = reinterpret_cast<float*>(smem + (NB * XBUF > RED ? NB * XBUF : RED));
  float* rsq_w = rsq + MP;  // [wave][MP] partial sums of squares
  wait_lgkm0();
  __builtin_amdgcn_s_barrier();
  if (p.norm) {  // (uniform) sums of squares of the X rows: one LDS slot per wave, summed in wave
                 // order (run-to-run reproducible, no LDS atomics)
    const int vpr = p.K / 8;  // 16-B vectors per row
    for (int m = 0; m < p.M; ++m) {
      const bf16* xr = p.X + (size_t)m * p.ldx;
      float ss = 0.f;
      for (int v = tid; v < vpr; v += NT) {
        float f[8];
        unpack8(*reinterpret_cast<const u32x4*>(xr + 8 * v), f);
#pragma unroll
        for (int j = 0; j < 8; ++j) ss = fmaf(f[j], f[j], ss);
      }
      ss = wave_sum(ss);
      if (lane == 0) rsq_w[w * MP + m] = ss;
    }
    wait_lgkm0();
    __builtin_amdgcn_s_barrier();
    for (int m = tid; m < p.M; m += NT) {
      float ss = 0.f;
#pragma unroll
      for (int q = 0; q < NWC + NL; ++q) ss += rsq_w[q * MP + m];
      rsq[m] = rsqrtf(ss / (float)p.K + p.norm_eps);
    }
    wait_lgkm0();
    __builtin_amdgcn_s_barrier();
  }
  auto tile4 = [&](int m, int c4) DAB_INLINE {
    const int col = c4 ^ (4 * (m & 15));
    f32x4 v = *reinterpret_cast<const f32x4*>(red + m * BNP + col);
#pragma unroll
    for (int q = 1; q < KG; ++q) v += *reinterpret_cast<const f32x4*>(red + (q * MP + m) * BNP + col);
    if (p.norm) v *= rsq[m];
    return v;
  };
  if (p.S > 1) {
    if constexpr (ABL == 4) return;
    float* slab = (float*)p.out + (size_t)slice * p.M * p.N;
    // write-through (sc1) 16-B stores: the slab lines leave this XCD's L2 as they are written
    // instead of sitting dirty until the kernel-end write-back, which the next kernel's start
    // would wait for (MI355X_MICROARCH.md price list: +2.8-3.8 us behind 12.6-16.8 MB of fp32
    // partials; o 14.6 -> 13.2 us, qkv 18.0 -> 16.6 us in the decode layer, profiles/decode_round2.md);
    // the consumer reads them once from the Infinity Cache either way
    if (p.slab_bf16) {
      // bf16 slabs (the partial sums rounded to bf16, as the TP path hands them to the all-reduce):
      // half the bytes for the producer's stores and the consumer's reads
      bf16* bslab = (bf16*)p.out + (size_t)slice * p.M * p.N;
      const auto brd = __builtin_amdgcn_make_buffer_rsrc(bslab + n0, 0, (p.M - 1) * p.N * 2 + BN * 2, 0x00020000);
      for (int e = tid; e < MP * (BN / 8); e += NT) {
        const int m = e / (BN / 8), c8 = (e % (BN / 8)) * 8;
        if (m < p.M) {
          const f32x4 lo = tile4(m, c8), hi = tile4(m, c8 + 4);
          float o[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          __builtin_amdgcn_raw_buffer_store_b128(pack8(o), brd, (m * p.N + c8) * 2, 0, 16);
        }
      }
      return;
    }
    const auto srd = __builtin_amdgcn_make_buffer_rsrc(slab + n0, 0, (p.M - 1) * p.N * 4 + BN * 4, 0x00020000);
    for (int e = tid; e < MP * (BN / 4); e += NT) {
      const int m = e / (BN / 4), c4 = (e % (BN / 4)) * 4;
      if (m < p.M)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, tile4(m, c4)), srd, (m * p.N + c4) * 4, 0, 16);
    }
    return;
  }
  if (p.epi == ST_EPI_CAND) {
    for (int e = tid; e < MP * (BN / 4); e += NT) {
      const int m = e / (BN / 4), c4 = (e % (BN / 4)) * 4;
      if (m >= p.M) continue;
      const f32x4 v = tile4(m, c4);
      const float t = p.thr[m];
      const int qg = p.q_group ? p.q_group[m] : -1;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + c4 + j;
        if (n >= p.N || v[j] < t) continue;
        const int rg = p.row_group ? p.row_group[n] : 0;
        if (rg < 0 || (qg >= 0 && rg != qg)) continue;
        const int slot = atomicAdd(p.cnt + m, 1);
        if (slot < p.cap) {
          p.cand_val[(size_t)m * p.cap + slot] = v[j];
          p.cand_idx[(size_t)m * p.cap + slot] = n;
        }
      }
    }
    return;
  }
  bf16* out = (bf16*)p.out;
  if (p.epi == ST_EPI_SWIGLU || p.epi == ST_EPI_SWIGLU8) {
    // hg-row groups: rows [2 hg i, 2 hg i + hg) gate, [2 hg i + hg, 2 hg (i + 1)) up -> output
    // columns n0/2 + hg i + j; each thread makes 4 outputs
    const int hg = p.epi == ST_EPI_SWIGLU ? 16 : 8, pp = hg / 4;
    for (int e = tid; e < MP * (BN / 8); e += NT) {
      const int m = e / (BN / 8), part = e % (BN / 8);
      if (m >= p.M) continue;
      const int i = part / pp, j0 = (part % pp) * 4;
      const f32x4 gt = tile4(m, 2 * hg * i + j0), up = tile4(m, 2 * hg * i + hg + j0);
      float o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = silu_f(gt[j]) * up[j];
      u32x2 v;
      v[0] = pack2bf(o[0], o[1]);
      v[1] = pack2bf(o[2], o[3]);
      *reinterpret_cast<u32x2*>(out + (size_t)m * p.ldo + n0 / 2 + hg * i + j0) = v;
    }
    return;
  }
  for (int e = tid; e < MP * (BN / 8); e += NT) {
    const int m = e / (BN / 8), c8 = (e % (BN / 8)) * 8;
    if (m >= p.M) continue;
    const f32x4 lo = tile4(m, c8), hi = tile4(m, c8 + 4);
    float o[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    if (p.residual) {
      const u32x4 rv = *reinterpret_cast<const u32x4*>(p.residual + (size_t)m * p.ldr + n0 + c8);
      float r[8];
      unpack8(rv, r);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = bf2f(f2bf(o[j])) + r[j];  // round like bf16 GEMM + bf16 add
    }
    *reinterpret_cast<u32x4*>(out + (size_t)m * p.ldo + n0 + c8) = pack8(o);
  }
}

// Configurations (cfg id -> template).  BN = weight rows per workgroup (16 RT 4/KG), KS = 128 k per
// stage, NB = X ring buffers (X issued NB-1 stages ahead), NWIN = weight register-ring stages,
// NL = loader waves.
struct StreamCfg {
  int mt, rt, kg, nb, nwin, nl;
  bool shuf;    // weights in the shuffle_weights layout
  int abl = 0;  // benchmark ablation (see the kernel)
  int nwc = 4;  // compute waves
};
static constexpr StreamCfg kStreamCfgs[] = {
    {8, 2, 2, 3, 3, 1, false},  // 0: M<=128 BN 64
    {8, 2, 1, 3, 3, 1, false},  // 1: M<=128 BN 128
    {8, 2, 2, 4, 4, 2, false},  // 2: M<=128 BN 64, 2 loaders
    {8, 2, 2, 4, 4, 4, false},  // 3: M<=128 BN 64, 4 loaders
    {8, 2, 1, 4, 3, 2, false},  // 4: M<=128 BN 128, 2 loaders
    {8, 2, 1, 4, 3, 4, false},  // 5: M<=128 BN 128, 4 loaders
    {4, 2, 2, 4, 4, 1, false},  // 6: M<=64  BN 64
    {4, 2, 2, 4, 4, 4, false},  // 7: M<=64  BN 64, 4 loaders
    {4, 2, 1, 4, 4, 2, false},  // 8: M<=64  BN 128, 2 loaders
    {8, 2, 2, 4, 4, 2, true},   // 9: = 2, shuffled weights
    {8, 2, 1, 4, 3, 4, true},   // 10: = 5, shuffled weights
    {8, 2, 2, 3, 6, 1, true},   // 11: M<=128 BN 64, 6-stage ring, shuffled
    {4, 2, 2, 4, 4, 4, true},   // 12: = 7, shuffled weights
    {4, 2, 1, 4, 4, 2, true},   // 13: = 8, shuffled weights
    {8, 2, 1, 4, 4, 4, true},   // 14: M<=128 BN 128, 4-stage ring, 4 loaders, shuffled
    {8, 2, 1, 4, 4, 2, true},   // 15: M<=128 BN 128, 4-stage ring, 2 loaders, shuffled
    {4, 2, 1, 4, 6, 4, true},   // 16: M<=64  BN 128, 6-stage ring, 4 loaders, shuffled
    {8, 2, 1, 4, 3, 4, true, 1},  // 17: = 10 without X staging        (ablation, wrong results)
    {8, 2, 1, 4, 3, 4, true, 2},  // 18: = 10 without MFMA             (ablation, wrong results)
    {8, 2, 1, 4, 3, 4, true, 3},  // 19: = 10 weight stream only       (ablation, wrong results)
    // whole-chip tilings at M <= 128: BN = 16 x compute waves (one 16-row tile per wave)
    {8, 1, 1, 4, 4, 2, true, 0, 7},  // 20: BN 112, 7 compute + 2 loader waves (gate_up 28672 -> 256 WGs)
    {8, 1, 1, 4, 4, 2, true, 0, 6},  // 21: BN 96, 6 + 2 waves (qkv 6144 x S4 -> 256 WGs)
    {8, 1, 1, 3, 6, 1, true, 0, 7},  // 22: = 20, 1 loader wave, 6-stage weight ring
    {8, 1, 1, 3, 6, 2, true, 0, 6},  // 23: = 21, 6-stage weight ring
    // M <= 256 (decode batches of 129..256): X stage 64 KB, two-stage X ring
    {16, 1, 1, 2, 3, 1, true, 0, 8},  // 24: BN 128, 8 compute + 1 loader wave
    {16, 1, 1, 2, 3, 2, true, 0, 4},  // 25: BN 64, 4 + 2 waves
    {16, 2, 1, 2, 2, 2, true, 0, 4},  // 26: BN 128, RT 2, 2-stage weight ring
    {16, 1, 2, 2, 4, 2, true, 0, 8},  // 27: BN 64, 2 k-groups x 4 row groups, 8 + 2 waves
    // M <= 128, BN 192 (6 compute waves x RT 2, 2 waves per SIMD): 2/3 of cfg 10's X staging per
    // weight byte (LM head: 128256 = 668 x 192)
    {8, 2, 1, 4, 3, 2, true, 0, 6},  // 28: 6 + 2 waves
    {8, 2, 1, 4, 2, 2, true, 0, 6},  // 29: = 28 with a 2-stage weight ring
    // M <= 16 (interactive decode, batch 1-16): one 16-row X tile per stage, a quarter of cfg 13's X
    // staging and MFMAs
    {1, 2, 1, 4, 4, 2, true},  // 30: BN 128, 2 loaders
    {2, 2, 1, 4, 4, 2, true},  // 31: M <= 32, BN 128, 2 loaders
    // M <= 16, whole-K producers of the residual stream (o / down with the residual add, no split-K
    // slabs, so the consumer can normalise X itself): 16 / 32 weight rows per workgroup, an 8-stage
    // weight ring per compute wave
    {1, 1, 1, 4, 8, 1, true, 0, 1},  // 32: BN 16, 1 compute + 1 loader wave
    {1, 1, 1, 4, 8, 1, true, 0, 2},  // 33: BN 32, 2 compute + 1 loader wave
    // M <= 128 with narrow tiles, so the small projections reach 256 workgroups at 2 K-slices
    // instead of 4-8 (a quarter of the fp32 slab bytes): 8-stage weight ring per compute wave
    {8, 1, 1, 4, 8, 2, true, 0, 2},  // 34: BN 32, 2 compute + 2 loader waves (o / down 4096 x S2)
    {8, 1, 1, 4, 8, 2, true, 0, 3},  // 35: BN 48, 3 + 2 waves (qkv 6144 x S2)
    // M <= 128, two workgroups per CU: a 2-stage X ring (64 KB of LDS) and one row tile per compute
    // wave (~134 registers), so one workgroup's pipeline fill / drain overlaps the other's stream
    {8, 1, 1, 2, 3, 2, true, 0, 4},  // 36: BN 64, 4 compute + 2 loader waves, 3-stage weight ring
    {8, 1, 1, 2, 4, 2, true, 0, 4},  // 37: = 36 with a 4-stage weight ring
    {8, 2, 1, 4, 3, 4, true, 4},     // 38: = 10 without the slab stores (ablation, wrong results)
    {8, 2, 1, 4, 3, 4, true, 5},     // 39: = 10 reading a tile-interleaved layout (ablation, wrong results)
    {8, 1, 1, 4, 4, 2, true, 5, 7},  // 40: = 20 reading a tile-interleaved layout (ablation, wrong results)
    // gate_up on the grouped copy (shuffle_weights(w, 8)): = 20 with deeper weight rings
    {8, 1, 1, 4, 6, 2, true, 0, 7},  // 41: 6-stage weight ring
    {8, 1, 1, 3, 8, 1, true, 0, 7},  // 42: 8-stage weight ring, 1 loader wave
};
constexpr int kNumStreamCfgs = sizeof(kStreamCfgs) / sizeof(kStreamCfgs[0]);

template <int C>
static void launch_cfg(const StreamParams& p, hipStream_t s, bool nt) {
  constexpr StreamCfg c = kStreamCfgs[C];
  const int bn = 16 * c.rt * (c.nwc / c.kg);
  const dim3 grid(((p.N + bn - 1) / bn) * p.S), block(64 * (c.nwc + c.nl));
  if (nt)
    hipLaunchKernelGGL((stream_gemm_kernel<c.mt, c.rt, c.kg, 128, c.nb, c.nwin, c.nl, c.shuf, true, c.abl, c.nwc>), grid,
                       block, 0, s, p);
  else
    hipLaunchKernelGGL((stream_gemm_kernel<c.mt, c.rt, c.kg, 128, c.nb, c.nwin, c.nl, c.shuf, false, c.abl, c.nwc>), grid,
                       block, 0, s, p);
}

int stream_gemm_bn(int cfg) {
  if (cfg < 0 || cfg >= kNumStreamCfgs) return 0;
  return 16 * kStreamCfgs[cfg].rt * (kStreamCfgs[cfg].nwc / kStreamCfgs[cfg].kg);
}

int stream_gemm_max_m(int cfg) { return (cfg < 0 || cfg >= kNumStreamCfgs) ? 0 : 16 * kStreamCfgs[cfg].mt; }

int stream_gemm_shuffled(int cfg) { return (cfg < 0 || cfg >= kNumStreamCfgs) ? 0 : (int)kStreamCfgs[cfg].shuf; }

template <int C = 0>
static void launch_any(int cfg, const StreamParams& p, hipStream_t s, bool nt) {
  if constexpr (C < kNumStreamCfgs) {
    if (cfg == C) return launch_cfg<C>(p, s, nt);
    launch_any<C + 1>(cfg, p, s, nt);
  }
}

// block -> (tile, slice) mapping of split-K launches with S % 8 == 0 (A/B; DAB_STREAM_SLICE_XCD)
static int g_slice_xcd = [] {
  const char* e = std::getenv("DAB_STREAM_SLICE_XCD");
  return e ? std::atoi(e) : 0;
}();
void stream_gemm_set_slice_xcd(int on) { g_slice_xcd = on; }
int stream_gemm_slice_xcd() { return g_slice_xcd; }

int stream_gemm(const void* X, long ldx, const void* W, long ldw, void* out, long ldo, const void* residual, long ldr,
                int M, int N, int K, int S, int epilogue, hipStream_t s, int nt_weights, int cfg, float norm_eps,
                int slab_bf16, int w_group) {
  constexpr int KS = 128;
  if (M <= 0 || N <= 0) return 0;
  const int bn = stream_gemm_bn(cfg);
  if (!bn || M > stream_gemm_max_m(cfg)) return hipErrorInvalidValue;
  if (N % bn || S < 1 || K % (S * KS) || ldx % 8 || ldw % 8 || ldo % 8) return hipErrorInvalidValue;
  if (epilogue != ST_EPI_NONE && epilogue != ST_EPI_SWIGLU && epilogue != ST_EPI_SWIGLU8) return hipErrorInvalidValue;
  if (epilogue == ST_EPI_SWIGLU && bn % 32) return hipErrorInvalidValue;  // whole 16 + 16 row pairs per tile
  if (S > 1 && (epilogue != ST_EPI_NONE || residual)) return hipErrorInvalidValue;
  if (residual && ldr % 8) return hipErrorInvalidValue;
  if ((long)bn * ldw * 2 >= (1L << 31)) return hipErrorInvalidValue;  // buffer descriptor range
  if (kStreamCfgs[cfg].shuf && (ldw != K || K % 32)) return hipErrorInvalidValue;
  StreamParams p{};
  p.X = (const bf16*)X;
  p.ldx = ldx;
  p.W = (const bf16*)W;
  p.ldw = ldw;
  p.out = out;
  p.ldo = ldo;
  p.residual = (const bf16*)residual;
  p.ldr = ldr;
  p.M = M;
  p.N = N;
  p.K = K;
  p.S = S;
  p.kc = K / S;
  p.epi = epilogue;
  // norm_eps > 0: consumer RMSNorm (X = the residual stream h, gains folded into W); not with a
  // residual add (its output is not a normalised product)
  p.norm = norm_eps > 0.f;
  p.norm_eps = norm_eps;
  p.slice_xcd = g_slice_xcd && S % 8 == 0;
  p.slab_bf16 = S > 1 && slab_bf16;
  p.wgrp = w_group < 1 ? 1 : w_group;
  if (p.wgrp > 1 && (!kStreamCfgs[cfg].shuf || N % (16 * p.wgrp) || (long)N * K * 2 >= (1L << 31)))
    return hipErrorInvalidValue;
  if (p.norm && (residual || K % 8 || M > stream_gemm_max_m(cfg))) return hipErrorInvalidValue;
  launch_any(cfg, p, s, nt_weights != 0);
  return hipGetLastError();
}

// Sum S fp32 / bf16 slabs -> bf16 (optionally + residual), rounded like a bf16 GEMM output before the
// add: the TP path hands bf16 partial sums to the all-reduce.
template <typename ST>
__global__ __launch_bounds__(256) void slab_reduce_kernel(bf16* out, long ldo, const ST* slabs, int S, int M, int N,
                                                          const bf16* residual, long ldr) {
  const size_t e = ((size_t)blockIdx.x * 256 + threadIdx.x) * 8;
  const size_t total = (size_t)M * N;
  if (e >= total) return;
  const int m = (int)(e / N), n = (int)(e % N);
  float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < S; ++s) {
    SlabVec8<ST> v;
    v.load(slabs + (size_t)s * total + e);
    v.add_to(o);
  }
  if (residual) {
    float r[8];
    unpack8(*reinterpret_cast<const u32x4*>(residual + (size_t)m * ldr + n), r);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = bf2f(f2bf(o[j])) + r[j];
  }
  *reinterpret_cast<u32x4*>(out + (size_t)m * ldo + n) = pack8(o);
}

int slab_reduce(void* out, long ldo, const void* slabs, int S, int M, int N, const void* residual, long ldr,
                hipStream_t s, int slab_bf16) {
  if (M <= 0 || N <= 0) return 0;
  if (N % 8 || ldo % 8 || (residual && ldr % 8)) return hipErrorInvalidValue;
  const size_t total8 = (size_t)M * N / 8;
  const dim3 grid((unsigned)((total8 + 255) / 256));
  if (slab_bf16)
    hipLaunchKernelGGL(slab_reduce_kernel<bf16>, grid, dim3(256), 0, s, (bf16*)out, ldo, (const bf16*)slabs, S, M, N,
                       (const bf16*)residual, ldr);
  else
    hipLaunchKernelGGL(slab_reduce_kernel<float>, grid, dim3(256), 0, s, (bf16*)out, ldo, (const float*)slabs, S, M,
                       N, (const bf16*)residual, ldr);
  return hipGetLastError();
}

// Index threshold candidates for small query batches (M <= 64): the index rows stream through the
// weight ring like decode weights (row-major, 16 rows x 64 B per load), the queries sit in LDS.
// At M = 1..64 the MFMA tiles of the GEMM kernels are mostly padding and the scan is HBM-bound.
static int stream_candidates_launch(bool shuf, const void* X, long ldx, const void* W, long ldw, int M, int N, int K,
                                    const int* row_group, const int* q_group, const float* thr, int* cnt,
                                    float* cand_val, int* cand_idx, int cap, hipStream_t s) {
  constexpr int KS = 128;
  // M <= 64, BN 64, 4 loader waves: row-major rows (cfg 7) or a shuffle_weights copy (cfg 12);
  // M <= 128 (shuffled copy only): BN 128 (cfg 10, the decode GEMM's)
  const int CFG = shuf ? (M > 64 ? 10 : 12) : 7;
  if (M <= 0 || N <= 0) return 0;
  if (M > stream_gemm_max_m(CFG) || K % KS || ldx % 8 || ldw % 8 || cap <= 0) return hipErrorInvalidValue;
  if ((long)stream_gemm_bn(CFG) * ldw * 2 >= (1L << 31)) return hipErrorInvalidValue;
  if (shuf && (ldw != K || K % 32)) return hipErrorInvalidValue;
  StreamParams p{};
  p.X = (const bf16*)X;
  p.ldx = ldx;
  p.W = (const bf16*)W;
  p.ldw = ldw;
  p.M = M;
  p.N = N;
  p.K = K;
  p.S = 1;
  p.kc = K;
  p.epi = ST_EPI_CAND;
  p.row_group = row_group;
  p.q_group = q_group;
  p.thr = thr;
  p.cnt = cnt;
  p.cand_val = cand_val;
  p.cand_idx = cand_idx;
  p.cap = cap;
  if (CFG == 10)
    launch_cfg<10>(p, s, true);
  else if (CFG == 12)
    launch_cfg<12>(p, s, true);
  else
    launch_cfg<7>(p, s, true);
  return hipGetLastError();
}

int stream_score_candidates(const void* X, long ldx, const void* W, long ldw, int M, int N, int K, const int* row_group,
                            const int* q_group, const float* thr, int* cnt, float* cand_val, int* cand_idx, int cap,
                            hipStream_t s) {
  return stream_candidates_launch(false, X, ldx, W, ldw, M, N, K, row_group, q_group, thr, cnt, cand_val, cand_idx, cap,
                                  s);
}

// W: the rows in the shuffle_weights layout, at least round_up(N, 128) of them (M <= 128)
int stream_score_candidates_shuf(const void* X, long ldx, const void* W, int M, int N, int K, const int* row_group,
                                 const int* q_group, const float* thr, int* cnt, float* cand_val, int* cand_idx,
                                 int cap, hipStream_t s) {
  return stream_candidates_launch(true, X, ldx, W, K, M, N, K, row_group, q_group, thr, cnt, cand_val, cand_idx, cap, s);
}

}  // namespace dab

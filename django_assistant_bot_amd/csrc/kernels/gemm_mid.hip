// Mid-M bf16 GEMM  C[M,N] = A[M,K] . B[N,K]^T  (+ residual, or fused SwiGLU over 8-row [gate | up]
// groups) for M = 256..4096 rows: the token counts of mixed prefill + decode serving steps and of
// request-at-a-time prompts (the reference runs one HF ``generate`` per request:
// ai/providers/transformers.py:57-66, served by gunicorn_conf.py:9 workers).  B is in the
// ops.shuffle_weights fragment layout (the one copy of every projection the decoder keeps).
//
// Why a third GEMM: at these M the 256x256 phased kernel (gemm256.hip) has 12-64 tiles for 256 CUs
// and the 128x128 kernel (gemm.hip) runs at ~20 % of the MFMA rate (profiles/gemm_mid_r5.md).
// Design (cdna_hip_programming.md section 5, "Projection GEMM at M = 256"; stream-K):
//   * tile 128 (rows of A) x 256 (weight rows), K-tile 64; 8 waves = 2 (M) x 4 (N), each wave a
//     64 x 64 piece = 4 x 4 v_mfma_f32_16x16x32_bf16 accumulators, 32 MFMAs per K-tile;
//   * A / B staged by LDS-DMA (buffer_load ... lds, 16 B per lane) into a ring of 3 K-tile stages
//     of 48 KB (A 16 KB | B0 16 KB | B1 16 KB); one phase per K-tile: [fragment reads, DMA of the
//     K-tile two ahead, counted vmcnt] barrier [32 MFMAs] barrier; the two wave groups (wr = 0 / 1)
//     run one barrier apart (one group's MFMAs beside the other's LDS reads), as in gemm256;
//   * work decomposition: the tiles_m workgroups of one "group" (one per 128-row tile of A) march
//     in lockstep through the SAME range of the (weight tile, K-tile) iteration space, so a weight
//     K-tile is fetched from HBM once and served to the group's other workgroups from their XCD's
//     L2 (groups are formed from blocks that share blockIdx % 8).  The iteration space
//     tiles_n x (K / 64) is split evenly over the 8 x floor(32 / tiles_m) groups (stream-K in the
//     N x K plane): every CU gets the same number of MFMAs whatever the tile count;
//   * a tile whose K range spans several groups is combined in-launch by its OWNER, the group
//     holding the tile's first K-steps: that segment ends the owner's range, so in time it finishes
//     last.  The other segments store their fp32 partial (write-through sc1 stores, 1 KB per
//     wave-instruction) and raise a per-slot ready flag two K-steps later, when the pipeline's own
//     counted wait has retired the stores (no drain); the owner keeps its partial in registers,
//     waits for each flag (bounded spin), adds the partials with sc1 loads in segment order (no
//     fence needed: cdna_hip_programming.md section 5 item 2), clears the flags and runs the
//     epilogue.  Only owners wait, on producers that never wait, so there is no deadlock (and the
//     grid is at most one workgroup per CU).  Replaces a last-arriver combine (every segment stored
//     and drained, then an atomic ticket) that cost 5-9 us per launch on the small projections
//     (profiles/gemm_mid_r6.md).
#include "common.h"
#include "launchers.h"

namespace dab {

namespace {

enum { MID_NONE = 0, MID_SWIGLU8 = 4 };

struct GMid {
  const bf16* A;
  const bf16* B;  // shuffle_weights layout, [N][K]
  bf16* C;
  const bf16* residual;
  float* slabs;  // [tiles_m][gn][2] partial tiles of 128 x 256 fp32 (in accumulator order)
  int* cnt;      // [tiles_m][gn][2] ready flags of the stored partial tiles, zero at rest
  int M, N, K;
  long lda, ldc, ldr;
  int tiles_m, tiles_n, kt;
  int spx;  // blocks per XCD label (grid / 8)
  int gpx;  // groups per XCD label
  int gn;   // groups = 8 * gpx
  int q, r;  // tiles_n * kt = q * gn + r iterations: group j owns q (+1 for j < r)
  unsigned b_bytes, slab_bytes;
  int bgrp;  // row blocks per group of the B copy: 1 (plain) or 8 (shuffle_weights(w, 8))
};

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t mk_rsrc(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

template <int VMC>
__device__ __forceinline__ void wait_vmc() {
  static_assert(VMC >= 0 && VMC <= 63, "vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(VMC) : "memory");
}

__device__ __forceinline__ void mbar() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// the barrier after a phase's LDS reads: they are retired first (s_barrier waits for no counter)
__device__ __forceinline__ void mread_bar() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  mbar();
}

// ring geometry per K-step width BK (64: 3 stages of 48 KB, DMA distance 2; 32: 6 stages of 24 KB,
// distance 5 -- the same LDS, two and a half times the latency cover in cycles)
template <int BK>
struct MidGeo {
  static constexpr int kA = 128 * BK * 2;        // A bytes per stage
  static constexpr int kStage = 384 * BK * 2;    // A | B (256 weight rows)
  static constexpr int kStages = BK == 64 ? 3 : 6;
  static constexpr int kDist = kStages - 1;     // stage issued kDist iterations ahead
  static constexpr int kDma = BK == 64 ? 6 : 3;  // LDS-DMA instructions per wave per stage
  static constexpr int kSmem = kStages * kStage;
  static_assert(kSmem <= 163840, "LDS");
};
constexpr int kE = 8;                  // VMEM stores per wave in every epilogue variant
constexpr int kSlabSt = 16;            // VMEM stores per wave of a published partial tile
constexpr int kSlabFloats = 512 * 64;  // one partial tile: 512 threads x 16 f32x4

// group start of the balanced split of the iteration space
__device__ __forceinline__ int grp_start(int j, int q, int r) { return j * q + min(j, r); }
__device__ __forceinline__ int grp_owner(int i, int q, int r) {
  const int big = r * (q + 1);
  return i < big ? i / (q + 1) : r + (i - big) / q;
}

}  // namespace

// BK: K-step width (see MidGeo); DIAG (timing only, benchmarks/gemm_bench.py): 1 = partial tiles
// are stored and counted but never combined (the output of split tiles is left unwritten)
template <int EPI, bool RES, int BK, int DIAG = 0>
__global__ __launch_bounds__(512) void gemm_mid_kernel(GMid p) {
  using Geo = MidGeo<BK>;
  constexpr int kStage = Geo::kStage, kStages = Geo::kStages, kDist = Geo::kDist, kDma = Geo::kDma;
  constexpr int kA = Geo::kA;
  __shared__ __attribute__((aligned(16))) char smem[Geo::kSmem];

  // ---- which group / row tile this block is: blocks b, b + 8, ... share an XCD label
  const int bid = blockIdx.x;
  const int x = bid & 7, slot = bid >> 3;
  const int g = slot / p.tiles_m, mt = slot - g * p.tiles_m;
  if (g >= p.gpx) return;  // whole workgroup (uniform)
  const int j = x * p.gpx + g;
  const int start = grp_start(j, p.q, p.r);
  const int end = start + p.q + (j < p.r ? 1 : 0);
  if (end <= start) return;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 2, wc = w & 3;
  const int li = lane & 15, gq = lane >> 4;
  const int m0 = mt * 128;
  const int kt = p.kt;  // K-steps of BK per tile

  // ---- LDS-DMA staging (per-lane parts in VOFFSET, the K / panel offset in SOFFSET).
  // A: BK = 64: rows of 128 B, 16-B chunk c of row r at c ^ ((r >> 1) & 7), wave w stages rows
  //    8w..8w+7 (+64);  BK = 32: rows of 64 B, chunk c at c ^ ((r >> 2) & 3), wave w rows 16w..16w+15.
  //    (conflict-free for the 4 x 16-lane groups of ds_read_b128; the swizzle goes on the SOURCE
  //    address since LDS-DMA writes lane-linearly)
  // B: the fragment layout: a 16-row x 32-k block is 1 KB in lane order; BK = 64 stages blocks
  //    (rb, 2kk) and (rb, 2kk + 1) back to back (2 KB per row block), BK = 32 block (rb, kk).
  unsigned vA0, vA1 = 0;
  if constexpr (BK == 64) {
    const int sw = (4 * (w & 1) + (lane >> 4)) & 7;
    const int cc = (lane & 7) ^ sw;
    const int srow = 8 * w + (lane >> 3);
    vA0 = (unsigned)((srow * p.lda + 8 * cc) * 2);
    vA1 = vA0 + (unsigned)(64 * p.lda * 2);
  } else {
    const int srow = 16 * w + (lane >> 2);
    const int cc = (lane & 3) ^ ((srow >> 2) & 3);
    vA0 = (unsigned)((srow * p.lda + 8 * cc) * 2);
  }
  const unsigned kblk = (unsigned)(p.K / 32) * 1024u;  // bytes of one 16-row block over all of K
  // grouped copy (p.bgrp = 8, shuffle_weights(w, 8)): the 8 blocks of a 128-row half adjacent per k
  // chunk, so block w of a half is w KB in and a k chunk is 8 KB on (the half itself starts where
  // the plain layout's does)
  const bool bgrp = p.bgrp == 8;
  const unsigned cb = bgrp ? 8192u : 1024u;  // bytes per 32-deep k chunk of a block
  const unsigned vB0 = (unsigned)(lane * 16) + (unsigned)w * (bgrp ? 1024u : kblk), vB2 = vB0 + 8u * kblk;
  const long a_rows = min(128, p.M - m0);
  const __amdgpu_buffer_rsrc_t rA = mk_rsrc(p.A + (size_t)m0 * p.lda, (unsigned)(((a_rows - 1) * p.lda + p.K) * 2));
  const __amdgpu_buffer_rsrc_t rB = mk_rsrc(p.B, p.b_bytes);

  auto stage = [&](int buf, int nt, int kk) {
    char* dst = smem + buf * kStage;
    const unsigned sa = (unsigned)kk * (unsigned)(BK * 2);
    const unsigned sb = (unsigned)nt * 16u * kblk + (unsigned)kk * (unsigned)(BK / 32) * cb;
    if constexpr (BK == 64) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (lds_void*)(dst + w * 1024), 16, vA0, sa, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (lds_void*)(dst + 8192 + w * 1024), 16, vA1, sa, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rB, (lds_void*)(dst + kA + w * 2048), 16, vB0, sb, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rB, (lds_void*)(dst + kA + w * 2048 + 1024), 16, vB0 + cb, sb, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rB, (lds_void*)(dst + kA + 16384 + w * 2048), 16, vB2, sb, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rB, (lds_void*)(dst + kA + 16384 + w * 2048 + 1024), 16, vB2 + cb, sb,
                                               0, 0);
    } else {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (lds_void*)(dst + w * 1024), 16, vA0, sa, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rB, (lds_void*)(dst + kA + w * 1024), 16, vB0, sb, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rB, (lds_void*)(dst + kA + 8192 + w * 1024), 16, vB2, sb, 0, 0);
    }
  };

  // ---- fragment reads: A rows 64 wr + 16 i + li, B row blocks 4 wc + jn
  constexpr int KS = BK / 32;  // MFMA k-steps per stage
  int rdA[KS];
  if constexpr (BK == 64) {
    const int swr = li >> 1;
    rdA[0] = (64 * wr + li) * 128 + 16 * (gq ^ swr);
    rdA[KS - 1] = (64 * wr + li) * 128 + 16 * ((4 + gq) ^ swr);
  } else {
    rdA[0] = (64 * wr + li) * 64 + 16 * (gq ^ ((li >> 2) & 3));
  }
  constexpr int kRowBlk = BK * 32;  // LDS bytes of one 16-row block of A / B in a stage
  const int rdB = kA + wc * 4 * kRowBlk + lane * 16;

  bf16x8 af[4][KS];
  bf16x8 bfr[4][KS];
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int jn = 0; jn < 4; ++jn) acc[i][jn] = f32x4{0.f, 0.f, 0.f, 0.f};

  // staging cursor: the iteration kDist ahead of the one being computed
  int s_nt = start / kt, s_kk = start - s_nt * kt;
  int s_it = start;
  auto advance = [&]() {
    ++s_it;
    if (++s_kk == kt) {
      s_kk = 0;
      ++s_nt;
    }
  };
  // prologue: iterations start .. start + kDist - 1 in flight (buffers 0 ..), the first landed
#pragma unroll
  for (int d = 0; d < kDist; ++d)
    if (s_it < end) {
      stage(d, s_nt, s_kk);
      advance();
    }
  {
    const int beyond = s_it - start - 1;  // issued stages past the first
    if (beyond >= 4) wait_vmc<4 * kDma>();
    else if (beyond == 3) wait_vmc<3 * kDma>();
    else if (beyond == 2) wait_vmc<2 * kDma>();
    else if (beyond == 1) wait_vmc<kDma>();
    else wait_vmc<0>();
  }
  mbar();

  int it = start;
  int b = 0;  // ring buffer of iteration `it`
  // VMEM stores issued since the last phase's wait (younger than the DMA in flight): an epilogue's
  // kE or a published partial's kSlabSt; the next phase's counted wait lets them stay in flight
  int after_st = 0;
  // a partial tile stored by this workgroup whose ready flag is not raised yet: raised at the
  // second phase after the stores, when that phase's vmcnt(kDma) has retired them (no drain)
  int pend_flag = -1, pend_phases = 0;
  const __amdgpu_buffer_rsrc_t rS = mk_rsrc(p.slabs, p.slab_bytes);
  auto slab_off = [&](int jj, int side) { return (unsigned)(((mt * p.gn + jj) * 2 + side) * kSlabFloats) * 4u; };
  auto flag_of = [&](int jj, int side) { return p.cnt + (mt * p.gn + jj) * 2 + side; };
  auto raise_flag = [&]() {  // after every wave's stores retired and a barrier
    if (tid == 0) __hip_atomic_store(p.cnt + pend_flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    pend_flag = -1;
  };
  while (it < end) {
    const int nt = it / kt;
    const int k0 = it - nt * kt;
    const int k1 = min(kt, k0 + (end - it));
    if (wr == 1) mbar();  // group 1 one barrier behind through the K-loop (ping-pong)
    for (int kk = k0; kk < k1; ++kk, ++it) {
      const char* sb = smem + b * kStage;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) af[i][ks] = *reinterpret_cast<const bf16x8*>(sb + i * 16 * (BK * 2) + rdA[ks]);
#pragma unroll
      for (int jn = 0; jn < 4; ++jn)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
          bfr[jn][ks] = *reinterpret_cast<const bf16x8*>(sb + rdB + jn * kRowBlk + ks * 1024);
      // the stage kDist ahead goes into the buffer read one phase ago
      if (s_it < end) {
        stage(b == 0 ? kStages - 1 : b - 1, s_nt, s_kk);
        advance();
        if (after_st == kSlabSt) wait_vmc<(kDist - 1) * kDma + kSlabSt>();
        else if (after_st == kE) wait_vmc<(kDist - 1) * kDma + kE>();
        else wait_vmc<(kDist - 1) * kDma>();
      } else {
        // tail: the stages after `it + 1` that are still in flight may stay so
        const int beyond = after_st ? 0 : s_it - it - 2;
        if (beyond >= 4) wait_vmc<4 * kDma>();
        else if (beyond == 3) wait_vmc<3 * kDma>();
        else if (beyond == 2) wait_vmc<2 * kDma>();
        else if (beyond == 1) wait_vmc<kDma>();
        else wait_vmc<0>();
      }
      after_st = 0;
      mread_bar();
      if (pend_flag >= 0 && ++pend_phases >= 2) raise_flag();  // this phase's wait retired the stores
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int jn = 0; jn < 4; ++jn) acc[i][jn] = mfma16(bfr[jn][ks], af[i][ks], acc[i][jn]);
      __builtin_amdgcn_s_setprio(0);
      mbar();
      b = b == kStages - 1 ? 0 : b + 1;
    }
    if (wr == 0) mbar();  // pairs with group 1's last K-loop barrier
    if (pend_flag >= 0) {  // (a one-phase segment followed: drain and raise now)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      raise_flag();
    }

    // ---- segment end.  A whole tile goes straight to the epilogue.  A split tile's segments are
    // held by groups j_lo .. j_hi in K order; its OWNER is j_lo, whose segment (the tile's first
    // K-steps) ends its own range, so in time it finishes last.  The other segments store their
    // fp32 partial (sc1, write-through) and raise a per-slot ready flag; the owner never stores its
    // own, waits for each flag (bounded spin), adds the partials in segment order (its registers
    // first), clears the flags and runs the epilogue.  Nobody else waits, so the owner's wait
    // cannot deadlock (and the grid is <= one workgroup per CU anyway).
    const int n0 = nt * 256;
    bool write = true;
    if (k0 != 0 || k1 != kt) {
      const int j_lo = grp_owner(nt * kt, p.q, p.r), j_hi = grp_owner(nt * kt + kt - 1, p.q, p.r);
      const int side = start >= nt * kt ? 0 : 1;
      if (j != j_lo) {
        const unsigned own = slab_off(j, side);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int jn = 0; jn < 4; ++jn)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][jn]), rS,
                                                   own + (unsigned)(((i * 4 + jn) * 512 + tid) * 16), 0, 16);
        after_st = kSlabSt;
        if (!DIAG) {  // (DIAG: the owner reads nothing, so no flag may be left raised)
          pend_flag = (int)(flag_of(j, side) - p.cnt);
          pend_phases = 0;
          if (it >= end) {  // nothing left to hide the drain behind
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            raise_flag();
          }
        }
        write = false;
      } else if (DIAG) {
        write = false;
      } else {
        bool ok = true;
        for (int jj = j_lo + 1; jj <= j_hi; ++jj) {
          const int sd = grp_start(jj, p.q, p.r) >= nt * kt ? 0 : 1;
          int* fl = flag_of(jj, sd);
          if (tid == 0) {
            long spins = 0;
            while (__hip_atomic_load(fl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
              if (++spins > (1L << 22)) {
                ok = false;  // a producer never published (cannot happen in a healthy launch)
                break;
              }
              __builtin_amdgcn_s_sleep(2);
            }
            if (ok) __hip_atomic_store(fl, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
          __syncthreads();  // every thread loads only after lane 0 saw the flag
          const unsigned off = slab_off(jj, sd);
          u32x4 v[4][4];
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int jn = 0; jn < 4; ++jn)
              v[i][jn] = __builtin_amdgcn_raw_buffer_load_b128(rS, off + (unsigned)(((i * 4 + jn) * 512 + tid) * 16),
                                                               0, 16);
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int jn = 0; jn < 4; ++jn) acc[i][jn] += __builtin_bit_cast(f32x4, v[i][jn]);
        }
        ok = __builtin_amdgcn_readfirstlane((int)ok) != 0 || tid != 0;
        if (!__syncthreads_and(ok)) {
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int jn = 0; jn < 4; ++jn) {
              const float nan = __builtin_nanf("");
              acc[i][jn] = f32x4{nan, nan, nan, nan};
            }
        }
      }
    }
    if (write) {
      // ---- epilogue: acc[i][jn][r] = C[m0 + 64 wr + 16 i + li][n0 + 64 wc + 16 jn + 4 gq + r];
      // exactly kE stores per wave (rows >= M fall outside the descriptor and are dropped)
      int e_li = li, e_g = gq, e_wc = wc;
      asm volatile("" : "+v"(e_li), "+v"(e_g), "+v"(e_wc));
      const long c_rows = min(128, p.M - m0);
      const __amdgpu_buffer_rsrc_t rC = mk_rsrc(p.C + (size_t)m0 * p.ldc, (unsigned)(c_rows * p.ldc * 2));
      if constexpr (EPI == MID_SWIGLU8) {
        // 8-row [gate | up] groups inside each 16-row block: one permlane32_swap of the (jn, jn + 1)
        // pair gives lanes 0-31 block jn's gate / up rows and lanes 32-63 block jn + 1's
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int mr = 64 * wr + 16 * i + e_li;
#pragma unroll
          for (int pr = 0; pr < 2; ++pr) {
            float o[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const auto s = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc[i][2 * pr][r]),
                                                              __float_as_uint(acc[i][2 * pr + 1][r]), false, false);
              o[r] = silu_f(__uint_as_float(s[0])) * __uint_as_float(s[1]);
            }
            u32x2 v;
            v[0] = pack2bf(o[0], o[1]);
            v[1] = pack2bf(o[2], o[3]);
            const int oc = (n0 + 64 * e_wc + 32 * pr) / 2 + 4 * e_g;
            __builtin_amdgcn_raw_buffer_store_b64(v, rC, (unsigned)((mr * p.ldc + oc) * 2), 0, 0);
          }
        }
      } else {
        // permlane16_swap of the (jn, jn + 1) pair: each lane then holds 8 contiguous columns
        // n0 + 64 wc + 32 pr + cq -> one 16-B store
        const int cq = 16 * (e_g & 1) + 8 * (e_g >> 1);
        u32x4 rv[4][2];
        if constexpr (RES) {
          const __amdgpu_buffer_rsrc_t rR = mk_rsrc(p.residual + (size_t)m0 * p.ldr, (unsigned)(c_rows * p.ldr * 2));
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int pr = 0; pr < 2; ++pr)
              rv[i][pr] = __builtin_amdgcn_raw_buffer_load_b128(
                  rR, (unsigned)(((64 * wr + 16 * i + e_li) * p.ldr + n0 + 64 * e_wc + 32 * pr + cq) * 2), 0, 0);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int mr = 64 * wr + 16 * i + e_li;
#pragma unroll
          for (int pr = 0; pr < 2; ++pr) {
            float o[8];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const auto s = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[i][2 * pr][r]),
                                                              __float_as_uint(acc[i][2 * pr + 1][r]), false, false);
              o[r] = __uint_as_float(s[0]);
              o[4 + r] = __uint_as_float(s[1]);
            }
            if constexpr (RES) {
              const u32x4 rw = rv[i][pr];
#pragma unroll
              for (int qd = 0; qd < 4; ++qd) {  // round like a bf16 GEMM output, then the bf16 add (HF)
                o[2 * qd] = bf2f(f2bf(o[2 * qd])) + __uint_as_float(rw[qd] << 16);
                o[2 * qd + 1] = bf2f(f2bf(o[2 * qd + 1])) + __uint_as_float(rw[qd] & 0xffff0000u);
              }
            }
            u32x4 v;
#pragma unroll
            for (int qd = 0; qd < 4; ++qd) v[qd] = pack2bf(o[2 * qd], o[2 * qd + 1]);
            const int nc = n0 + 64 * e_wc + 32 * pr + cq;
            __builtin_amdgcn_raw_buffer_store_b128(v, rC, (unsigned)((mr * p.ldc + nc) * 2), 0, 0);
          }
        }
      }
      after_st = kE;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int jn = 0; jn < 4; ++jn) acc[i][jn] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
}

namespace {
int cu_count() {
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  return cus;
}
}  // namespace

// Eligible: N % 256 == 0, K % 64 == 0, 16-B aligned A rows, ceil(M / 128) row tiles <= blocks per
// XCD label (32 on MI355X: M <= 4096), 32-bit buffer offsets.
int gemm_mid_ok(int M, int N, int K, long lda) {
  if (M <= 0 || N <= 0 || K <= 0 || N % 256 || K % 64 || lda % 8 || lda < K) return 0;
  const int spx = cu_count() / 8;
  if ((M + 127) / 128 > spx) return 0;
  if ((long)N * K * 2 >= (1L << 32) || (127L * lda + K) * 2 >= (1L << 31)) return 0;
  return 1;
}

// Workspace the launcher needs: partial slabs (bytes) and arrival counters (ints).
long gemm_mid_slab_bytes() { return (long)cu_count() * 2 * kSlabFloats * 4; }
// ready flags of the partial tiles: two per (row tile, group) <= two per workgroup
int gemm_mid_counters(int M, int N) {
  (void)M;
  (void)N;
  return 2 * (cu_count() & ~7);
}

// epilogue 0: C = A B^T (+ residual, bf16 add after rounding); 4: SwiGLU over 8-row [gate | up]
// groups (C has N / 2 columns).  slabs: gemm_mid_slab_bytes() bytes; cnt: >= gemm_mid_counters()
// ints, zero on first use (the launch leaves them zero).  variant (A/B harness only): 0 default
// (BK 64), 32 / 64 force the K-step, + 1000 = DIAG 1 (split tiles not combined: timing only).
// BK 32 (6-stage ring) measured 5-20 % slower than BK 64 on every mid shape, with LDS bank
// conflicts on its 64-B A rows (profiles/gemm_mid_r6.md): kept as an A/B arm only.
int gemm_mid(const void* A, long lda, const void* B, void* C, long ldc, const void* residual, long ldr, int M, int N,
             int K, int epilogue, void* slabs, long slab_bytes, int* cnt, int n_cnt, hipStream_t s, int variant,
             int b_group) {
  if (!gemm_mid_ok(M, N, K, lda)) return hipErrorInvalidValue;
  if (b_group != 1 && b_group != 8) return hipErrorInvalidValue;
  if (epilogue != MID_NONE && epilogue != MID_SWIGLU8) return hipErrorInvalidValue;
  if (epilogue == MID_SWIGLU8 && residual) return hipErrorInvalidValue;
  if (!slabs || !cnt || slab_bytes < gemm_mid_slab_bytes() || n_cnt < gemm_mid_counters(M, N) ||
      slab_bytes >= (1L << 32))
    return hipErrorInvalidValue;
  const bool diag = variant >= 1000;
  const int bk = (variant % 1000) == 32 ? 32 : 64;
  GMid p{};
  p.A = (const bf16*)A;
  p.B = (const bf16*)B;
  p.C = (bf16*)C;
  p.residual = (const bf16*)residual;
  p.slabs = (float*)slabs;
  p.cnt = cnt;
  p.M = M;
  p.N = N;
  p.K = K;
  p.lda = lda;
  p.ldc = ldc;
  p.ldr = ldr;
  p.tiles_m = (M + 127) / 128;
  p.tiles_n = N / 256;
  p.kt = K / bk;
  const int grid = cu_count() & ~7;
  p.spx = grid / 8;
  p.gpx = p.spx / p.tiles_m;
  p.gn = 8 * p.gpx;
  const int iters = p.tiles_n * p.kt;
  p.q = iters / p.gn;
  p.r = iters % p.gn;
  p.b_bytes = (unsigned)((long)N * K * 2);
  p.slab_bytes = (unsigned)slab_bytes;
  p.bgrp = b_group;
#define MID_LAUNCH(E, R, BKV, D) hipLaunchKernelGGL((gemm_mid_kernel<E, R, BKV, D>), dim3(grid), dim3(512), 0, s, p)
#define MID_BK(E, R)                       \
  do {                                     \
    if (diag) {                            \
      if (bk == 64) MID_LAUNCH(E, R, 64, 1); \
      else MID_LAUNCH(E, R, 32, 1);        \
    } else if (bk == 64) {                 \
      MID_LAUNCH(E, R, 64, 0);             \
    } else {                               \
      MID_LAUNCH(E, R, 32, 0);             \
    }                                      \
  } while (0)
  if (epilogue == MID_SWIGLU8) MID_BK(MID_SWIGLU8, false);
  else if (residual) MID_BK(MID_NONE, true);
  else MID_BK(MID_NONE, false);
#undef MID_BK
#undef MID_LAUNCH
  return hipGetLastError();
}

}  // namespace dab

// Large-M bf16 GEMM  C[M,N] = A[M,K] . B[N,K]^T  (+bias, +GELU(erf), +residual, or fused SwiGLU)
// for gfx950: the prefill / encoder projections (Llama-3 qkv / o / gate_up / down at M = 32k tokens,
// bge qkv / o / up / down at M = 64k).  Replaces HF Linear in the reference
// (ai/providers/transformers.py:57-66 generate, ai/embedders/transformers.py:18-22 encoder forward).
//
// Structure: the 256x256 phased schedule of cdna_hip_programming.md section 5 (T1-T5), with two
// quadrants per phase:
//   * 512 threads = 8 waves; per K-tile (BK = 64) the block tile is cut into 2x2 quadrants of
//     128x128 and every wave owns a 64x32 piece of EACH quadrant (waves 2 (M) x 4 (N) per quadrant);
//     one phase = two quadrants = 32 x v_mfma_f32_16x16x32_bf16 per wave, 2 phases per K-tile (the
//     8-phase form's one quadrant per phase spent ~350 of every 2,400 cycles per K-tile at its
//     16 barriers; with 8 barriers per 2 K-tiles a K-tile takes ~2,200 cycles, but the chip then
//     holds a lower clock: profiles/gemm_tile_stamps.md);
//   * the A/B tiles are staged by LDS-DMA (buffer_load ... lds, 16 B per lane) in HALF-TILE pieces
//     (128 rows x 64 k = 16 KB, two instructions per wave), 1 or 3 pieces per phase;
//     2 K-tile buffers = 128 KB of LDS (1 block per CU);
//   * counted waits only: every phase waits `vmcnt(8)` (4 pieces stay in flight ACROSS barriers,
//     each piece has 3 phases ~ 3k cycles to land), raw s_barrier (never __syncthreads, whose
//     fence would drain the DMA), all LDS in ONE __shared__ array;
//   * the two wave groups (wr = 0 / 1, one wave of each per SIMD) are staggered by one barrier so one
//     group's MFMA cluster overlaps the other group's LDS reads + DMA issue (ping-pong), re-made on
//     every tile so the two groups' epilogues overlap;
//     s_setprio(1) around each MFMA cluster keeps hipcc from moving MFMAs across the barriers (T5);
//   * fragment registers: the A rows of the current quadrant row (32 VGPR) and BOTH B halves
//     (2 x 16 VGPR), so a K-tile reads A0+B0+B1 / A1 in its 2 phases (24 ds_read_b128, the
//     minimum), and every staged piece is rewritten one phase after its last read (WAR rule with
//     staggered groups) and waited >= 1 phase before its first read (RAW rule);
//   * LDS rows are 128 B; the 16-B chunk c of row r lives at chunk c ^ ((r >> 1) & 7): conflict-free
//     for the 4 x 16-lane groups of ds_read_b128 (MI355X_MICROARCH.md section LDS).  LDS-DMA writes
//     lane-linearly, so the swizzle is applied to the per-lane SOURCE address (rule 21);
//   * buffer descriptors clamp the tile edges: rows >= M (or >= N) read zeros, no per-lane clamp;
//   * bijective XCD-aware block remap (T1) + grouped tile order so the 32 tiles an XCD runs at once
//     share A / B panels in that XCD's L2;
//   * SHUF: B (the weights) in the ops.shuffle_weights fragment layout [N/16][K/32][64 lanes][8] --
//     the one copy the decode GEMM (stream_gemm.hip) streams too.  A 16-row x 32-k block is one
//     contiguous 1 KB piece in MFMA A-fragment lane order, so each wave's LDS-DMA instruction copies
//     a whole block and the fragment read is lane-linear (ds_read_b128 at lane * 16, no swizzle).
#include "common.h"
#include "launchers.h"

#include <cstdlib>
#include <type_traits>

namespace dab {

namespace {

enum { G_NONE = 0, G_GELU = 1, G_SWIGLU = 2, G_CAND = 3, G_SWIGLU8 = 4 };

struct G256 {
  const bf16* A;
  const bf16* B;
  bf16* C;
  const bf16* bias;
  const bf16* residual;
  int M, N, K;
  long lda, ldb, ldc, ldr;
  int gm;  // tile rows per group of the grouped tile order
  int rows_b;  // SHUF: rows of the B copy (>= N)
  int bgrp;    // SHUF: row blocks per group of the B copy, 1 or 8 (shuffle_weights(w, 8))
  // G_CAND (index threshold search, see gemm.hip EPI_CANDIDATES): filtered scores >= thr[m] are
  // appended to row m's candidate list; no C is written and N need not be a multiple of 256
  const int* row_group;  // [N] (<0 = deleted) or null
  const int* q_group;    // [M] (<0 = any) or null
  const float* thr;      // [M]
  int* cnt;              // [M]
  float* cand_val;       // [M, cap]
  int* cand_idx;         // [M, cap]
  int cap;
  // STAMP (diagnostic instantiations only, benchmarks/gemm_stamps.py): per workgroup and tile,
  // wave 0 records {s_memtime at the tile's first K-iteration (lo, hi), cycles of the K-loop, cycles
  // of the epilogue} as one 16-B vector store; stamp_tiles entries per workgroup
  u32x4* stamps;
  int stamp_tiles;
};

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

template <int VMC>
__device__ __forceinline__ void wait_vm() {
  static_assert(VMC >= 0 && VMC <= 63, "vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(VMC) : "memory");
}

constexpr int kEpiStores = 16;  // VMEM stores per wave in every epilogue variant

__device__ __forceinline__ unsigned lds_off(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

__device__ __forceinline__ void bar() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// The barrier after a phase's LDS reads: those reads are retired first (gfx950's s_barrier does not
// wait for lgkmcnt), so the DMA the other wave group issues one phase later into a piece read here
// is ordered after the reads by the barrier itself, not by load latency.  Nearly free:
// the MFMAs behind the barrier need the data anyway.
__device__ __forceinline__ void read_bar() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  bar();
}

constexpr int kBuf = 65536;   // one K-tile: A0 | A1 | B0 | B1, 16 KB each
constexpr int kHalf = 16384;  // 128 rows x 128 B
// G_CAND, M <= kCandMaxM: after the two K-tile buffers, the thresholds [kCandMaxM] fp32, 8 per-wave
// list counters (64 B) and 8 per-wave candidate lists of kCandW (n, m, score) entries
constexpr int kCandMaxM = 1024;
constexpr int kCandW = 288;
constexpr int kCandExtra = 4 * kCandMaxM + 64 + 8 * kCandW * 12;
static_assert(2 * kBuf + kCandExtra <= 163840, "LDS");

}  // namespace

// grouped tile order: tile id -> (m0, n0), column-major inside groups of GM tile rows
__device__ __forceinline__ void tile_of(int sid, int tiles_m, int tiles_n, int GM, int& m0, int& n0) {
  const int per_group = GM * tiles_n;
  const int grp = sid / per_group, first_m = grp * GM;
  const int gsz = min(GM, tiles_m - first_m);
  const int inner = sid - grp * per_group;
  m0 = (first_m + inner % gsz) << 8;
  n0 = (inner / gsz) << 8;
}

template <int EPI, bool BIAS, bool RES, bool SHUF = false, bool STAMP = false, int SAUX = 0>
__global__ __launch_bounds__(512) void gemm256_kernel(G256 p) {
  __shared__ __attribute__((aligned(16))) char smem[2 * kBuf + (EPI == G_CAND ? kCandExtra : 0)];
  // stores per wave in the epilogue (the next tile's first waits count past them; the candidate
  // epilogue issues none, or drains the queue itself)
  constexpr int kEpi = EPI == G_CAND ? 0 : kEpiStores;

  // Persistent: one workgroup per CU walks a strided list of tiles.  Blocks b and b+8 share an XCD,
  // so the tile ids are split into 8 contiguous chunks (bijective for any count) and the nper
  // workgroups of chunk x take ids cstart + l, cstart + l + nper, ... -> at any time the ~32
  // workgroups of one XCD run consecutive (grouped) tiles that share A / B panels in its L2.
  const int tiles_m = (p.M + 255) >> 8, tiles_n = EPI == G_CAND ? (p.N + 255) >> 8 : p.N >> 8;
  const int nwg = tiles_m * tiles_n;
  const int G = gridDim.x, bid = blockIdx.x;
  const int x = bid & 7, l = bid >> 3;
  const int nper = (G >> 3) + (x < (G & 7) ? 1 : 0);
  const int q8 = nwg >> 3, r8 = nwg & 7;
  const int cstart = x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8;
  const int cend = cstart + q8 + (x < r8 ? 1 : 0);
  int sid = cstart + l;
  if (sid >= cend) return;  // whole workgroup: uniform
  int m0, n0;
  tile_of(sid, tiles_m, tiles_n, p.gm, m0, n0);

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 2, wc = w & 3;
  const int li = lane & 15, g = lane >> 4;

  // ---- G_CAND candidate lists (see the epilogue): a hit is appended to this wave's LDS list
  // (LDS atomic slot); a flush applies the row / query group filters and appends to the global
  // per-query lists.  The list is flushed after a tile that leaves it more than kCandW - 64 entries
  // full; a hit that finds it full is appended to the global list directly.
  float* const thr_s = reinterpret_cast<float*>(smem + 2 * kBuf);
  int* const ccnt = reinterpret_cast<int*>(smem + 2 * kBuf + 4 * kCandMaxM);
  int* const c_n = ccnt + 16 + w * kCandW;
  int* const c_m = ccnt + 16 + 8 * kCandW + w * kCandW;
  float* const c_v = reinterpret_cast<float*>(ccnt + 16 + 16 * kCandW + w * kCandW);
  auto cand_global = [&](int m, int n, float v) {
    const int rg = p.row_group ? p.row_group[n] : 0;
    const int qg = p.q_group ? p.q_group[m] : -1;
    if (rg >= 0 && (qg < 0 || rg == qg)) {
      const int slot = atomicAdd(p.cnt + m, 1);
      if (slot < p.cap) {
        p.cand_val[(size_t)m * p.cap + slot] = v;
        p.cand_idx[(size_t)m * p.cap + slot] = n;
      }
    }
  };
  // The slot claim, the entry writes and the count read are asm: before a compiler-visible LDS
  // atomic or store hipcc waits vmcnt(0) for every LDS-DMA in flight (the next tile's K-tiles),
  // which is the drain these lists exist to avoid.  Each asm waits for its own LDS ops.
  const unsigned a_cnt = lds_off(ccnt + w);
  auto cand_push = [&](int m, int n, float v) {
    int slot;
    asm volatile("ds_add_rtn_u32 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=v"(slot) : "v"(a_cnt), "v"(1) : "memory");
    if (slot < kCandW) {
      asm volatile("ds_write_b32 %0, %1\n\tds_write_b32 %2, %3\n\tds_write_b32 %4, %5" ::"v"(lds_off(c_n + slot)),
                   "v"(n), "v"(lds_off(c_m + slot)), "v"(m), "v"(lds_off(c_v + slot)), "v"(v)
                   : "memory");
    } else {
      cand_global(m, n, v);
    }
  };
  auto cand_count = [&]() {
    int c;
    asm volatile("s_waitcnt lgkmcnt(0)\n\tds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(c) : "v"(a_cnt) : "memory");
    return __builtin_amdgcn_readfirstlane(c);
  };
  auto cand_flush = [&]() {  // wave-uniform call (rare: the list's high-water mark, and the kernel end)
    const int c = min(cand_count(), kCandW);
    for (int e = lane; e < c; e += 64) cand_global(c_m[e], c_n[e], c_v[e]);
    if (lane == 0) asm volatile("ds_write_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" ::"v"(a_cnt), "v"(0) : "memory");
    // retire the flush's memory ops here (the paths the compiler merges after it inherit nothing to
    // wait for); a flush is rare and drains the prefetch queue anyway
    __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
  };
  if constexpr (EPI == G_CAND) {
    if (p.M <= kCandMaxM) {  // before any LDS-DMA is issued: the barrier drains nothing
      for (int e = tid; e < p.M; e += 512) thr_s[e] = p.thr[e];
      if (tid < 8) ccnt[tid] = 0;
      __syncthreads();
    }
  }

  // ---- LDS-DMA staging: piece j (0/1) of wave w = half-tile rows 8(8j + w) .. +7
  const int sw = (4 * (w & 1) + (lane >> 4)) & 7;
  const int cc = (lane & 7) ^ sw;  // global 16-B chunk this lane fetches
  const int srow = 8 * w + (lane >> 3);
  // whole row offsets in VOFFSET (the buffer range check sees them: rows >= M / N read zeros);
  // the K offset goes in SOFFSET
  const unsigned vA0 = (unsigned)((srow * p.lda + 8 * cc) * 2), vA1 = vA0 + (unsigned)(64 * p.lda * 2);
  const unsigned vA2 = vA0 + (unsigned)(128 * p.lda * 2), vA3 = vA0 + (unsigned)(192 * p.lda * 2);
  // SHUF: wave w copies 16-row block w of each 128-row half, both 32-k blocks of the K-tile
  // (1 KB each, lane-linear); block (rb, kb) of a K-tile sits at byte (K / 32 rb + kb) 1 KB
  const unsigned kblk = (unsigned)(p.K / 32) * 1024u;
  // SHUF grouped copy (p.bgrp = 8, shuffle_weights(w, 8)): the 8 blocks of a 128-row half are
  // adjacent per k chunk -- block w of the half w KB in, a k chunk 8 KB on
  const bool bgrp = SHUF && p.bgrp == 8;
  const unsigned cb = bgrp ? 8192u : 1024u;
  const unsigned vB0 = SHUF ? (unsigned)(lane * 16) + (unsigned)w * (bgrp ? 1024u : kblk)
                            : (unsigned)((srow * p.ldb + 8 * cc) * 2);
  const unsigned vB1 = SHUF ? vB0 + cb : vB0 + (unsigned)(64 * p.ldb * 2);
  const unsigned vB2 = SHUF ? vB0 + 8u * kblk : vB0 + (unsigned)(128 * p.ldb * 2);
  const unsigned vB3 = SHUF ? vB2 + cb : vB0 + (unsigned)(192 * p.ldb * 2);
  auto rsrc_a = [&](int mm) {
    const long rows = min(256, p.M - mm);
    return make_rsrc(p.A + (size_t)mm * p.lda, (unsigned)(((rows - 1) * p.lda + p.K) * 2));
  };
  auto rsrc_b = [&](int nn) {
    // SHUF (G_CAND over an index copy): rows past the copy read zeros; they are masked as n >= N
    const long rows = SHUF ? min(256, p.rows_b - nn) : min(256, p.N - nn);
    if (SHUF) return make_rsrc(p.B + (size_t)nn * p.K, (unsigned)(rows > 0 ? rows * p.K * 2 : 0));
    return make_rsrc(p.B + (size_t)nn * p.ldb, (unsigned)(((rows - 1) * p.ldb + p.K) * 2));
  };
  __amdgpu_buffer_rsrc_t rA = rsrc_a(m0), rB = rsrc_b(n0);

  // slot: 0 = A rows 0-127, 1 = A rows 128-255, 2 = B rows 0-127, 3 = B rows 128-255
  auto stage = [&](int buf, int slot, int kt, __amdgpu_buffer_rsrc_t ra, __amdgpu_buffer_rsrc_t rb) {
    const bool shb = SHUF && slot >= 2;  // (slot is a compile-time constant at every call)
    char* dst = smem + buf * kBuf + slot * kHalf + w * (shb ? 2048 : 1024);
    const unsigned so = (unsigned)kt * (shb ? 2u * cb : 128u);
    const __amdgpu_buffer_rsrc_t r = slot < 2 ? ra : rb;
    const unsigned v0 = slot == 0 ? vA0 : slot == 1 ? vA2 : slot == 2 ? vB0 : vB2;
    const unsigned v1 = slot == 0 ? vA1 : slot == 1 ? vA3 : slot == 2 ? vB1 : vB3;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)dst, 16, v0, so, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)(dst + (shb ? 1024 : 8192)), 16, v1, so, 0, 0);
  };

  // ---- fragment reads (per-lane byte offsets inside a half-tile, k-steps 0 / 1)
  const int swr = li >> 1;
  const int rdA0 = (64 * wr + li) * 128 + 16 * (g ^ swr), rdA1 = (64 * wr + li) * 128 + 16 * ((4 + g) ^ swr);
  // SHUF: block (2 wc + j) of the half at 2 KB strides (the j * 2048 below), k-step ks at + 1 KB
  const int rdB0 = SHUF ? wc * 4096 + lane * 16 : (32 * wc + li) * 128 + 16 * (g ^ swr);
  const int rdB1 = SHUF ? rdB0 + 1024 : (32 * wc + li) * 128 + 16 * ((4 + g) ^ swr);

  bf16x8 af[4][2];
  bf16x8 bfr[2][2][2];  // [jh][jn][ks]
  f32x4 acc[2][2][4][2];
  auto zero_acc = [&]() {
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[a][b][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };
  zero_acc();

#define G256_READ_A(BUF, IH)                                                                     \
  _Pragma("unroll") for (int i = 0; i < 4; ++i) {                                                \
    const char* base = smem + (BUF) * kBuf + (IH) * kHalf + i * 2048;                            \
    af[i][0] = *reinterpret_cast<const bf16x8*>(base + rdA0);                                    \
    af[i][1] = *reinterpret_cast<const bf16x8*>(base + rdA1);                                    \
  }
#define G256_READ_B(BUF, JH)                                                                     \
  _Pragma("unroll") for (int j = 0; j < 2; ++j) {                                                \
    const char* base = smem + (BUF) * kBuf + 2 * kHalf + (JH) * kHalf + j * 2048;                \
    bfr[JH][j][0] = *reinterpret_cast<const bf16x8*>(base + rdB0);                               \
    bfr[JH][j][1] = *reinterpret_cast<const bf16x8*>(base + rdB1);                               \
  }
#define G256_MFMA2(IH, JH1, JH2)                                                                 \
  __builtin_amdgcn_s_setprio(1);                                                                 \
  _Pragma("unroll") for (int ks = 0; ks < 2; ++ks)                                               \
  _Pragma("unroll") for (int i = 0; i < 4; ++i)                                                  \
  _Pragma("unroll") for (int j = 0; j < 2; ++j)                                                  \
    acc[IH][JH1][i][j] = mfma16(bfr[JH1][j][ks], af[i][ks], acc[IH][JH1][i][j]);                 \
  _Pragma("unroll") for (int ks = 0; ks < 2; ++ks)                                               \
  _Pragma("unroll") for (int i = 0; i < 4; ++i)                                                  \
  _Pragma("unroll") for (int j = 0; j < 2; ++j)                                                  \
    acc[IH][JH2][i][j] = mfma16(bfr[JH2][j][ks], af[i][ks], acc[IH][JH2][i][j]);                 \
  __builtin_amdgcn_s_setprio(0);

  const int T = p.K >> 6;  // K-tiles (even, >= 2)
  const int iters = T >> 1;

  // prologue (first tile only): K-tile 0 complete, K-tile 1's A0 / B0 / B1 in flight
  stage(0, 0, 0, rA, rB);
  stage(0, 2, 0, rA, rB);
  stage(0, 3, 0, rA, rB);
  stage(0, 1, 0, rA, rB);
  stage(1, 0, 1, rA, rB);
  stage(1, 2, 1, rA, rB);
  stage(1, 3, 1, rA, rB);
  wait_vm<8>();
  bar();

  // One iteration = 4 phases = K-tiles e = 2it (buffer 0) and o = 2it + 1 (buffer 1); a phase is
  // [LDS reads, DMA issue, counted wait] barrier [32 MFMAs: two quadrants] barrier, and the two wave
  // groups run one barrier apart (one group's MFMAs beside the other's reads).
  // phase : reads (quadrants)        stage (buffer, slots, K-tile)   wait (for the next phase's reads)
  //   1   : A0 B0 B1 e ((0,0) (0,1))  (1, A1, o)                     vmcnt(8) -> A1 e
  //   2   : A1 e       ((1,1) (1,0))  (0, A0 B0 B1, e+2)             vmcnt(8) -> A0 B0 B1 o
  //   3   : A0 B0 B1 o ((0,0) (0,1))  (0, A1, e+2)                   vmcnt(8) -> A1 o
  //   4   : A1 o       ((1,1) (1,0))  (1, A0 B0 B1, o+2)             vmcnt(8) -> A0 B0 B1 e+2
  // Every piece is restaged one phase after its last read (a phase is 2 x 32 MFMAs, ~1k cycles:
  // the reads of the other group's previous phase have long returned when the DMA lands) and read
  // three phases later.  In the last iteration of a tile the phase 2-4 pieces are the NEXT tile's
  // K-tiles 0 / 1 (same buffers as e+2 / o+2), so the next tile starts without a prologue; after
  // the last tile nothing is staged and the phase-2 wait drains everything.  Half the barriers of
  // the 8-phase form (one quadrant per phase), same registers (the B fragments of both halves
  // stay live across a phase pair as before).  One copy of the body: the variants differ only in
  // uniform (SGPR) values, which keeps hipcc's register allocation of the loop intact.
  bool after_epi = false;
  int tile_no = 0;
  unsigned long long st_t0 = 0, st_t1 = 0;
  for (;;) {
    if constexpr (STAMP) st_t0 = __builtin_amdgcn_s_memtime();
    // group 1 runs one barrier behind group 0 through the K-loop (ping-pong: one group's MFMAs beside
    // the other's LDS reads and DMA issue); the pairing is re-made for every tile and undone before
    // the epilogue (below), so the two groups' epilogues run side by side.  Kept across the tile
    // boundary instead, each group's epilogue paired with one MFMA phase of the other and the
    // epilogues ran one after the other.
    if (wr == 1) bar();
    const int nsid = sid + nper;
    const bool more = nsid < cend;
    int nm0 = m0, nn0 = n0;
    if (more) tile_of(nsid, tiles_m, tiles_n, p.gm, nm0, nn0);
    const __amdgpu_buffer_rsrc_t nA = rsrc_a(nm0), nB = rsrc_b(nn0);
    // G_CAND: a tile whose rows 128-255 are all past M (97-128 queries, or the last row tile of a
    // larger batch) skips their MFMAs (the accumulators stay zero; their thresholds are +inf).
    // Uniform per tile; the LDS reads, barriers and DMA schedule are unchanged.
    const bool h2 = EPI != G_CAND || m0 + 128 < p.M;
    for (int it = 0; it < iters; ++it) {
      const bool last = it == iters - 1;
      const bool st = !last || more;  // stage phases 2-4
      // first iteration after an epilogue: kEpi younger stores sit in the VM queue
      const bool fe = after_epi && it == 0;
      const int e = 2 * it, o = e + 1;
      const int ke = last ? 0 : e + 2, ko = last ? 1 : o + 2;
      const __amdgpu_buffer_rsrc_t sa = last ? nA : rA, sb = last ? nB : rB;
      // phase 1
      G256_READ_A(0, 0)
      G256_READ_B(0, 0)
      G256_READ_B(0, 1)
      stage(1, 1, o, rA, rB);
      if (fe) wait_vm<8 + kEpi>();
      else wait_vm<8>();
      read_bar();
      G256_MFMA2(0, 0, 1)
      bar();
      // phase 2
      G256_READ_A(0, 1)
      if (st) {
        stage(0, 0, ke, sa, sb);
        stage(0, 2, ke, sa, sb);
        stage(0, 3, ke, sa, sb);
        if (fe) wait_vm<8 + kEpi>();
        else wait_vm<8>();
      } else {
        wait_vm<0>();
      }
      read_bar();
      if (h2) {
        G256_MFMA2(1, 1, 0)
      }
      bar();
      // phase 3
      G256_READ_A(1, 0)
      G256_READ_B(1, 0)
      G256_READ_B(1, 1)
      if (st) {
        stage(0, 1, ke, sa, sb);
        wait_vm<8>();
      }
      read_bar();
      G256_MFMA2(0, 0, 1)
      bar();
      // phase 4
      G256_READ_A(1, 1)
      if (st) {
        stage(1, 0, ko, sa, sb);
        stage(1, 2, ko, sa, sb);
        stage(1, 3, ko, sa, sb);
        wait_vm<8>();
      }
      read_bar();
      if (h2) {
        G256_MFMA2(1, 1, 0)
      }
      bar();
    }

    if constexpr (STAMP) st_t1 = __builtin_amdgcn_s_memtime();
    if (wr == 0) bar();  // pairs with group 1's last K-loop barrier
    // ---- epilogue: acc[ih][jh][i][jn][r] = C[m0 + 128 ih + 64 wr + 16 i + li][n0 + 128 jh + 32 wc + 16 jn + 4 g + r]
    // The next tile's first K-tiles are already in flight; the stores overlap them.  Exactly
    // kEpiStores buffer stores per wave, unconditional (rows >= M fall outside the descriptor and
    // are dropped), so the next tile's first waits can count past them (vmcnt(8 + kEpiStores)).
    // The lane offsets go through an opaque asm so hipcc cannot hoist the epilogue's address
    // arithmetic out of the tile loop (it would stay live across the K-loop and spill).
    int e_li = li, e_g = g, e_wc = wc;
    asm volatile("" : "+v"(e_li), "+v"(e_g), "+v"(e_wc));
    const long c_rows = min(256, p.M - m0);
    const __amdgpu_buffer_rsrc_t rC = make_rsrc(p.C + (size_t)m0 * p.ldc, (unsigned)(c_rows * p.ldc * 2));
    if constexpr (EPI == G_CAND) {
      // acc[ih][jh][i][jn][r] = score of query m0 + 128 ih + 64 wr + 16 i + li against index row
      // n0 + 128 jh + 32 wc + 16 jn + 4 g + r.  M <= kCandMaxM: the thresholds sit in LDS and a hit
      // (rare: ~105 per 256x256 tile at k = 250 under the 1/64 sample's bound) goes to this wave's
      // LDS list; the group filters and the global appends run when the list is flushed.  The
      // epilogue then issues no vector-memory
      // op, so the next tile's prefetched K-tiles stay in flight (a vmcnt(0) here drained them on
      // every tile).  Larger M: per-tile threshold / group loads, waited here.
      if (p.M <= kCandMaxM) {
        const float* thr_s = reinterpret_cast<const float*>(smem + 2 * kBuf);
        // Pass 1, branch-free: bit b = 64 ih + 16 i + 8 jh + 4 jn + r of hb[b / 32] marks a score >= the
        // query's threshold.  Pass 2, a runtime loop over the wave's hits (as many trips as the
        // busiest lane has hits, ~1-2): the lowest set bit is decoded, its score picked out of the
        // accumulators by a select tree, and appended.  One copy of the append code instead of 128
        // inlined ones: the unrolled form was ~60 KB of epilogue code whose fetch evicted the K-loop
        // from the instruction cache (the next tile's K-loop ran ~8k cycles slower, with no hits).
        unsigned hb[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int ih = 0; ih < 2; ++ih)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int m = m0 + 128 * ih + 64 * wr + 16 * i + e_li;
            const float t = m < p.M ? thr_s[m] : __builtin_huge_valf();
#pragma unroll
            for (int jh = 0; jh < 2; ++jh)
#pragma unroll
              for (int jn = 0; jn < 2; ++jn)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                  const int b = 64 * ih + 16 * i + 8 * jh + 4 * jn + r;
                  hb[b >> 5] |= acc[ih][jh][i][jn][r] >= t ? 1u << (b & 31) : 0u;
                }
          }
        for (;;) {
          const bool has = (hb[0] | hb[1] | hb[2] | hb[3]) != 0u;
          if (__builtin_amdgcn_ballot_w64(has) == 0) break;  // wave-uniform
          if (has) {
            const int wd = hb[0] ? 0 : hb[1] ? 1 : hb[2] ? 2 : 3;
            const unsigned wb = wd == 0 ? hb[0] : wd == 1 ? hb[1] : wd == 2 ? hb[2] : hb[3];
            const int b = 32 * wd + __builtin_ctz(wb);
            const unsigned clr = wb & (wb - 1u);
            hb[0] = wd == 0 ? clr : hb[0];
            hb[1] = wd == 1 ? clr : hb[1];
            hb[2] = wd == 2 ? clr : hb[2];
            hb[3] = wd == 3 ? clr : hb[3];
            // score: for each of the 16 (jh, jn, r) positions pick the (ih, i) row by bits 4-6, then
            // the position by bits 0-3
            float col[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) {
              const int jh = q >> 3, jn = (q >> 2) & 1, r = q & 3;
              float x[8];
#pragma unroll
              for (int u = 0; u < 8; ++u) x[u] = acc[u >> 2][jh][u & 3][jn][r];
#pragma unroll
              for (int L = 0; L < 3; ++L)
#pragma unroll
                for (int u = 0; u < (4 >> L); ++u) x[u] = (b >> (4 + L)) & 1 ? x[2 * u + 1] : x[2 * u];
              col[q] = x[0];
            }
#pragma unroll
            for (int L = 0; L < 4; ++L)
#pragma unroll
              for (int u = 0; u < (8 >> L); ++u) col[u] = (b >> L) & 1 ? col[2 * u + 1] : col[2 * u];
            const int m = m0 + 128 * (b >> 6) + 64 * wr + 16 * ((b >> 4) & 3) + e_li;
            const int n = n0 + 128 * ((b >> 3) & 1) + 32 * e_wc + 16 * ((b >> 2) & 1) + 4 * e_g + (b & 3);
            if (n < p.N) cand_push(m, n, col[0]);
          }
        }
        // (a per-step capacity check inside this fully unrolled loop made hipcc keep the loop and
        // move the accumulators to scratch: the list is checked once per tile, and a step that
        // finds it full appends directly)
        if (cand_count() > kCandW - 64) cand_flush();
      } else {
        const int cq = 16 * (e_g & 1) + 8 * (e_g >> 1);
        float thr_r[2][4];
        int qg_r[2][4];
        int rg[2][8];
#pragma unroll
        for (int ih = 0; ih < 2; ++ih)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int m = min(m0 + 128 * ih + 64 * wr + 16 * i + e_li, p.M - 1);
            thr_r[ih][i] = p.thr[m];
            qg_r[ih][i] = p.q_group ? p.q_group[m] : -1;
          }
#pragma unroll
        for (int jh = 0; jh < 2; ++jh)
#pragma unroll
          for (int r = 0; r < 8; ++r) {
            const int n = n0 + 128 * jh + 32 * e_wc + cq + r;
            rg[jh][r] = n >= p.N ? -1 : p.row_group ? p.row_group[n] : 0;
          }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int ih = 0; ih < 2; ++ih)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int m = m0 + 128 * ih + 64 * wr + 16 * i + e_li;
#pragma unroll
            for (int jh = 0; jh < 2; ++jh) {
              float o[8];
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[ih][jh][i][0][r]),
                                                           __float_as_uint(acc[ih][jh][i][1][r]), false, false);
                o[r] = __uint_as_float(sw[0]);
                o[4 + r] = __uint_as_float(sw[1]);
              }
              if (m >= p.M) continue;
              const int nb = n0 + 128 * jh + 32 * e_wc + cq;
              const int qg = qg_r[ih][i];
#pragma unroll
              for (int r = 0; r < 8; ++r) {
                const bool ok = rg[jh][r] >= 0 && (qg < 0 || rg[jh][r] == qg);
                if (ok && o[r] >= thr_r[ih][i]) {
                  const int slot = atomicAdd(p.cnt + m, 1);
                  if (slot < p.cap) {
                    p.cand_val[(size_t)m * p.cap + slot] = o[r];
                    p.cand_idx[(size_t)m * p.cap + slot] = nb + r;
                  }
                }
              }
            }
          }
      }
    } else if constexpr (EPI == G_SWIGLU || EPI == G_SWIGLU8) {
      // G_SWIGLU: weight rows interleaved in 16-row groups [gate 16 | up 16]: jn = 0 gate, jn = 1 up.
      // G_SWIGLU8: 8-row groups [gate 8 | up 8] inside every 16-row MFMA block (the decode layout:
      // any 16-row multiple tiles it): lane g holds rows 4g..4g+3 of both blocks, so one
      // v_permlane32_swap of the (jn 0, jn 1) pair gives lanes 0-31 block 0's gate / up rows and
      // lanes 32-63 block 1's -- the same output column 16 wc + 4 g as the 16-row form.
      float bg[2][4], bu[2][4];
      if constexpr (BIAS) {
#pragma unroll
        for (int jh = 0; jh < 2; ++jh) {
          const bf16* bp = p.bias + n0 + 128 * jh + 32 * e_wc + 4 * e_g;
          const u32x2 gv = *reinterpret_cast<const u32x2*>(bp), uv = *reinterpret_cast<const u32x2*>(bp + 16);
          bg[jh][0] = __uint_as_float(gv[0] << 16), bg[jh][1] = __uint_as_float(gv[0] & 0xffff0000u);
          bg[jh][2] = __uint_as_float(gv[1] << 16), bg[jh][3] = __uint_as_float(gv[1] & 0xffff0000u);
          bu[jh][0] = __uint_as_float(uv[0] << 16), bu[jh][1] = __uint_as_float(uv[0] & 0xffff0000u);
          bu[jh][2] = __uint_as_float(uv[1] << 16), bu[jh][3] = __uint_as_float(uv[1] & 0xffff0000u);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
#pragma unroll
      for (int ih = 0; ih < 2; ++ih)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int mr = 128 * ih + 64 * wr + 16 * i + e_li;
#pragma unroll
          for (int jh = 0; jh < 2; ++jh) {
            float o[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              float gt = acc[ih][jh][i][0][r], up = acc[ih][jh][i][1][r];
              if constexpr (EPI == G_SWIGLU8) {
                const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(gt), __float_as_uint(up), false, false);
                gt = __uint_as_float(sw[0]);
                up = __uint_as_float(sw[1]);
              }
              if constexpr (BIAS) {
                gt += bg[jh][r];
                up += bu[jh][r];
              }
              o[r] = silu_f(gt) * up;
            }
            u32x2 v;
            v[0] = pack2bf(o[0], o[1]);
            v[1] = pack2bf(o[2], o[3]);
            const int oc = (n0 + 128 * jh) / 2 + 16 * e_wc + 4 * e_g;
            __builtin_amdgcn_raw_buffer_store_b64(v, rC, (unsigned)((mr * p.ldc + oc) * 2), 0, SAUX);
          }
        }
    } else {
      // v_permlane16_swap between the jn = 0 / 1 fragments: afterwards each lane holds 8 contiguous
      // columns n0 + 128 jh + 32 wc + cq, cq = 16 (g & 1) + 8 (g >> 1) -> one 16-B store (T21 idea
      // for the 16x16 layout: half the store instructions at equal bytes)
      const int cq = 16 * (e_g & 1) + 8 * (e_g >> 1);
      float bv[2][8];
      if constexpr (BIAS) {
#pragma unroll
        for (int jh = 0; jh < 2; ++jh) {
          const u32x4 b4 = *reinterpret_cast<const u32x4*>(p.bias + n0 + 128 * jh + 32 * e_wc + cq);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            bv[jh][2 * q] = __uint_as_float(b4[q] << 16);
            bv[jh][2 * q + 1] = __uint_as_float(b4[q] & 0xffff0000u);
          }
        }
      }
      __amdgpu_buffer_rsrc_t rR = rC;
      if constexpr (RES) {
        rR = make_rsrc(p.residual + (size_t)m0 * p.ldr, (unsigned)(c_rows * p.ldr * 2));
      }
      // RES: all 16 residual vectors of the wave are requested before the first store (64 VGPRs,
      // the dead fragment registers), so one vmcnt(0) per tile instead of one per 128-row half
      // (the second also waited for the first half's stores: gfx9 counts stores in vmcnt).  Within
      // noise of the per-half form (profiles/gemm_epilogue_probe.md): what the residual costs at
      // short K (+25-35 % at K = 768) is the chip-wide burst of residual reads when every CU reaches
      // its epilogue at the same time, not the round trips.
      u32x4 rvv[2][4][2];
      if constexpr (RES) {
#pragma unroll
        for (int ih = 0; ih < 2; ++ih)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int jh = 0; jh < 2; ++jh)
              rvv[ih][i][jh] = __builtin_amdgcn_raw_buffer_load_b128(
                  rR, (unsigned)(((128 * ih + 64 * wr + 16 * i + e_li) * p.ldr + n0 + 128 * jh + 32 * e_wc + cq) * 2), 0,
                  0);
      }
#pragma unroll
      for (int ih = 0; ih < 2; ++ih) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int mr = 128 * ih + 64 * wr + 16 * i + e_li;
#pragma unroll
          for (int jh = 0; jh < 2; ++jh) {
            float o[8];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[ih][jh][i][0][r]),
                                                         __float_as_uint(acc[ih][jh][i][1][r]), false, false);
              o[r] = __uint_as_float(sw[0]);
              o[4 + r] = __uint_as_float(sw[1]);
            }
            const int nc = n0 + 128 * jh + 32 * e_wc + cq;
            if constexpr (BIAS) {
#pragma unroll
              for (int r = 0; r < 8; ++r) o[r] += bv[jh][r];
            }
            if constexpr (EPI == G_GELU) {
#pragma unroll
              for (int r = 0; r < 8; ++r) o[r] = gelu_erf(o[r]);
            }
            if constexpr (RES) {
              const u32x4 rv = rvv[ih][i][jh];
#pragma unroll
              for (int q = 0; q < 4; ++q) {  // round like a bf16 GEMM output, then the bf16 add (HF)
                o[2 * q] = bf2f(f2bf(o[2 * q])) + __uint_as_float(rv[q] << 16);
                o[2 * q + 1] = bf2f(f2bf(o[2 * q + 1])) + __uint_as_float(rv[q] & 0xffff0000u);
              }
            }
            u32x4 v;
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = pack2bf(o[2 * q], o[2 * q + 1]);
            if constexpr (BIAS || RES) {
              if (i == 0 && jh == 0 && ih == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            __builtin_amdgcn_raw_buffer_store_b128(v, rC, (unsigned)((mr * p.ldc + nc) * 2), 0, SAUX);
          }
        }
      }
    }
    if constexpr (STAMP) {
      // one vector store by lane 0 of wave 0 (its next counted waits only get stricter by it)
      const unsigned long long t2 = __builtin_amdgcn_s_memtime();
      if (w == 0 && lane == 0 && tile_no < p.stamp_tiles) {
        u32x4 v;
        v[0] = (unsigned)st_t0;
        v[1] = (unsigned)(st_t0 >> 32);
        v[2] = (unsigned)(st_t1 - st_t0);
        v[3] = (unsigned)(t2 - st_t1);
        p.stamps[(size_t)blockIdx.x * p.stamp_tiles + tile_no] = v;
      }
      ++tile_no;
    }
    after_epi = true;
    if (!more) break;
    sid = nsid;
    m0 = nm0;
    n0 = nn0;
    rA = nA;
    rB = nB;
    zero_acc();
  }
  if constexpr (EPI == G_CAND) {
    if (p.M <= kCandMaxM) cand_flush();
  }
#undef G256_READ_A
#undef G256_READ_B
#undef G256_MFMA2
}

// Threshold candidates of the index search (see gemm.hip gemm_score_candidates): queries A [M, K] x
// index rows B [N, K], any N; K % 128 == 0.
// b_rows > 0: B is a shuffle_weights copy of b_rows >= N rows (b_rows % 16 == 0, ldb == K).
int gemm256_candidates(const void* A, long lda, const void* B, long ldb, int M, int N, int K, const int* row_group,
                       const int* q_group, const float* thr, int* cnt, float* cand_val, int* cand_idx, int cap,
                       hipStream_t s, int b_rows) {
  if (M <= 0 || N <= 0) return 0;
  if (K % 128 || K <= 0 || lda % 8 || ldb % 8 || cap <= 0) return hipErrorInvalidValue;
  if ((255L * lda + K) * 2 >= (1L << 31) || (255L * ldb + K) * 2 >= (1L << 31)) return hipErrorInvalidValue;
  if (b_rows > 0 && (b_rows < N || b_rows % 16 || ldb != K)) return hipErrorInvalidValue;
  G256 p{};
  p.A = (const bf16*)A;
  p.B = (const bf16*)B;
  p.M = M;
  p.N = N;
  p.K = K;
  p.lda = lda;
  p.ldb = ldb;
  p.gm = 4;
  p.row_group = row_group;
  p.q_group = q_group;
  p.thr = thr;
  p.cnt = cnt;
  p.cand_val = cand_val;
  p.cand_idx = cand_idx;
  p.cap = cap;
  p.rows_b = b_rows;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const long tiles = (long)((M + 255) / 256) * ((N + 255) / 256);
  const int nwg = tiles > cus ? cus : (int)tiles;
  if (b_rows > 0) hipLaunchKernelGGL((gemm256_kernel<G_CAND, false, false, true>), dim3(nwg), dim3(512), 0, s, p);
  else hipLaunchKernelGGL((gemm256_kernel<G_CAND, false, false>), dim3(nwg), dim3(512), 0, s, p);
  return hipGetLastError();
}

// Diagnostic: the candidate GEMM over a shuffled index copy (b_rows >= N rows) with per-tile stamps
// (layout as gemm256_stamped).  No group filters.  Returns the grid.
int gemm256_candidates_stamped(const void* A, long lda, const void* B, int M, int N, int K, int b_rows,
                               const float* thr, int* cnt, float* cand_val, int* cand_idx, int cap, void* stamps,
                               int stamp_tiles, hipStream_t s) {
  if (M <= 0 || N <= 0 || M > kCandMaxM || K % 128 || lda % 8 || cap <= 0 || b_rows < N || b_rows % 16)
    return -hipErrorInvalidValue;
  G256 p{};
  p.A = (const bf16*)A;
  p.B = (const bf16*)B;
  p.M = M;
  p.N = N;
  p.K = K;
  p.lda = lda;
  p.ldb = K;
  p.gm = 4;
  p.thr = thr;
  p.cnt = cnt;
  p.cand_val = cand_val;
  p.cand_idx = cand_idx;
  p.cap = cap;
  p.rows_b = b_rows;
  p.stamps = (u32x4*)stamps;
  p.stamp_tiles = stamp_tiles;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const long tiles = (long)((M + 255) / 256) * ((N + 255) / 256);
  const int nwg = tiles > cus ? cus : (int)tiles;
  hipLaunchKernelGGL((gemm256_kernel<G_CAND, false, false, true, true>), dim3(nwg), dim3(512), 0, s, p);
  const int rc = hipGetLastError();
  return rc ? -rc : nwg;
}

// Diagnostic: gemm256 with per-tile s_memtime stamps (epilogues 0 / 1 with optional bias / residual).
// stamps: [grid][stamp_tiles] u32x4 {t0 lo, t0 hi, K-loop cycles, epilogue cycles}; returns the grid.
int gemm256_stamped(const void* A, long lda, const void* B, void* C, const void* bias, const void* residual, int M,
                    int N, int K, int epilogue, int b_shuf, void* stamps, int stamp_tiles, hipStream_t s, int store_aux) {
  if (!gemm256_ok(M, N, K, lda, K) || (epilogue != G_NONE && epilogue != G_GELU) || (epilogue == G_GELU && residual))
    return -hipErrorInvalidValue;
  G256 p{};
  p.A = (const bf16*)A;
  p.B = (const bf16*)B;
  p.C = (bf16*)C;
  p.bias = (const bf16*)bias;
  p.residual = (const bf16*)residual;
  p.M = M;
  p.N = N;
  p.K = K;
  p.lda = lda;
  p.ldb = K;
  p.ldc = N;
  p.ldr = N;
  p.rows_b = N;
  p.gm = 4;
  p.stamps = (u32x4*)stamps;
  p.stamp_tiles = stamp_tiles;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int tiles = ((M + 255) / 256) * (N / 256);
  const int nwg = tiles > cus ? cus : tiles;
  const bool hb = bias != nullptr, hr = residual != nullptr;
  // store_aux: cache policy of the epilogue stores (0 default, 2 nt, 16 sc1, 18 sc1 + nt) -- A/B only
#define G256_STAMPED_AUX(E, BI, R, AX)                                                                            \
  do {                                                                                                            \
    if (b_shuf) hipLaunchKernelGGL((gemm256_kernel<E, BI, R, true, true, AX>), dim3(nwg), dim3(512), 0, s, p);   \
    else hipLaunchKernelGGL((gemm256_kernel<E, BI, R, false, true, AX>), dim3(nwg), dim3(512), 0, s, p);         \
  } while (0)
#define G256_STAMPED(E, BI, R)                          \
  do {                                                  \
    if (store_aux == 2) G256_STAMPED_AUX(E, BI, R, 2);   \
    else if (store_aux == 16) G256_STAMPED_AUX(E, BI, R, 16); \
    else if (store_aux == 18) G256_STAMPED_AUX(E, BI, R, 18); \
    else G256_STAMPED_AUX(E, BI, R, 0);                  \
  } while (0)
  if (epilogue == G_GELU) G256_STAMPED(G_GELU, true, false);
  else if (hb && hr) G256_STAMPED(G_NONE, true, true);
  else if (hr) G256_STAMPED(G_NONE, false, true);
  else if (hb) G256_STAMPED(G_NONE, true, false);
  else G256_STAMPED(G_NONE, false, false);
#undef G256_STAMPED
#undef G256_STAMPED_AUX
  const int rc = hipGetLastError();
  return rc ? -rc : nwg;
}

// Eligible shapes: N % 256 == 0, K % 128 == 0, 16-B aligned rows, 32-bit buffer offsets.
int gemm256_ok(int M, int N, int K, long lda, long ldb) {
  if (M <= 0 || N <= 0 || N % 256 || K % 128 || K <= 0 || lda % 8 || ldb % 8) return 0;
  if ((255L * lda + K) * 2 >= (1L << 31) || (255L * ldb + K) * 2 >= (1L << 31)) return 0;
  if ((128L * lda) * 2 + (long)K * 2 >= (1L << 31) || (128L * ldb) * 2 + (long)K * 2 >= (1L << 31)) return 0;
  return 1;
}

// b_shuf: B is in the shuffle_weights layout (ldb == K).  Epilogues: 0 none, 1 GELU, 2 SwiGLU over
// 16-row [gate | up] groups, 4 SwiGLU over 8-row groups (no bias); bias / residual optional.
int gemm256(const void* A, long lda, const void* B, long ldb, void* C, long ldc, const void* bias,
            const void* residual, long ldr, int M, int N, int K, int epilogue, hipStream_t s, int b_shuf,
            int b_group) {
  if (!gemm256_ok(M, N, K, lda, ldb)) return hipErrorInvalidValue;
  if (b_group != 1 && !(b_group == 8 && b_shuf)) return hipErrorInvalidValue;  // (N % 256: whole groups)
  if ((epilogue == G_SWIGLU || epilogue == G_SWIGLU8) && residual) return hipErrorInvalidValue;
  if (epilogue == G_SWIGLU8 && bias) return hipErrorInvalidValue;
  if (b_shuf && ldb != K) return hipErrorInvalidValue;
  G256 p{};
  p.A = (const bf16*)A;
  p.B = (const bf16*)B;
  p.C = (bf16*)C;
  p.bias = (const bf16*)bias;
  p.residual = (const bf16*)residual;
  p.M = M;
  p.N = N;
  p.K = K;
  p.lda = lda;
  p.ldb = ldb;
  p.ldc = ldc;
  p.ldr = ldr;
  p.rows_b = N;
  p.bgrp = b_group;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int tiles = ((M + 255) / 256) * (N / 256);
  p.gm = 4;  // grouped tile order: 4 tile rows per group
  // persistent: one workgroup (128 KB of LDS) per CU walks a strided tile list
  const int nwg = tiles > cus ? cus : tiles;
  const bool hb = bias != nullptr, hr = residual != nullptr;
#define G256_LAUNCH_AUX(E, B, R, AX)                                                                          \
  do {                                                                                                         \
    if (b_shuf) hipLaunchKernelGGL((gemm256_kernel<E, B, R, true, false, AX>), dim3(nwg), dim3(512), 0, s, p); \
    else hipLaunchKernelGGL((gemm256_kernel<E, B, R, false, false, AX>), dim3(nwg), dim3(512), 0, s, p);       \
  } while (0)
  // C stores: write-through + non-temporal (sc1 nt) for the short-K bias / GELU projections of the
  // encoder -- their epilogue burst then retires before the next tile's third K-tile is waited for
  // (bge qkv 217 -> 203 us, up 338 -> 326 us); the default policy everywhere else, where it measured
  // faster (residual epilogues, Llama prefill: profiles/gemm_tile_stamps.md)
  const bool nt_out = K <= 1024 && !residual && !b_shuf;
#define G256_LAUNCH(E, B, R)                         \
  do {                                               \
    if (nt_out) G256_LAUNCH_AUX(E, B, R, 18);        \
    else G256_LAUNCH_AUX(E, B, R, 0);                \
  } while (0)
  switch (epilogue) {
    case G_NONE:
      if (hb && hr) G256_LAUNCH(G_NONE, true, true);
      else if (hb) G256_LAUNCH(G_NONE, true, false);
      else if (hr) G256_LAUNCH(G_NONE, false, true);
      else G256_LAUNCH(G_NONE, false, false);
      break;
    case G_GELU:
      if (hr) return hipErrorInvalidValue;
      if (hb) G256_LAUNCH(G_GELU, true, false);
      else G256_LAUNCH(G_GELU, false, false);
      break;
    case G_SWIGLU:
      if (hb) G256_LAUNCH(G_SWIGLU, true, false);
      else G256_LAUNCH(G_SWIGLU, false, false);
      break;
    case G_SWIGLU8:
      G256_LAUNCH(G_SWIGLU8, false, false);
      break;
    default: return hipErrorInvalidValue;
  }
#undef G256_LAUNCH
#undef G256_LAUNCH_AUX
  return hipGetLastError();
}

}  // namespace dab

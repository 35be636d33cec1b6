// bf16 MFMA GEMM  C[M,N] = A[M,K] . B[N,K]^T  with fused epilogues, for gfx950.
//
// Used for (a) the encoder projections with their bias / GELU / residual epilogues fused (BERT/bge),
// (b) the Llama MLP gate|up projection with SwiGLU fused into the epilogue, and (c) the in-HBM
// cosine index scan (queries x index rows -> fp32 scores with the row-validity / per-query group /
// allow-bitmask filter applied in the epilogue), which replaces pgvector's CosineDistance ORDER BY
// (reference rag/services/search_service.py:185-196, storage/models.py:32-58).
//
// Structure ("2-phase" of cdna_hip_programming.md section 5.5 T3/T4 minimum form):
//   * 128x128 block tile, BK = 64, 256 threads = 2x2 waves, 64x64 per wave = 4x4 MFMA 16x16x32 tiles;
//   * A/B tiles staged global->LDS with global_load_lds_dwordx4 (no VGPR round trip), double-buffered,
//     next K tile issued before the current tile's MFMAs, one barrier per K step;
//   * 128-B LDS rows XOR-swizzled on the SOURCE address (LDS-DMA writes lane-linear), the same
//     involution applied on the ds_read_b128 side -> conflict-free fragment reads;
//   * operands swapped in the MFMA (B rows feed the A slot) so each lane ends with 4 consecutive
//     output columns of one row -> 8-B / 16-B epilogue stores;
//   * bijective XCD-aware block remap (T1) so neighbouring tiles share an XCD's L2;
//   * SHUF: B in the ops.shuffle_weights fragment layout (the one weight copy the decode GEMM also
//     streams): each 1 KB staging piece is one 16-row x 32-k block, read back lane-linearly.
#include <cstdlib>

#include "common.h"
#include "launchers.h"

namespace dab {

// EPI_SWIGLU8 = ops EPI_SWIGLU8 (4); EPI_CANDIDATES is internal (gemm_score_candidates)
enum EpiMode { EPI_NONE = 0, EPI_GELU = 1, EPI_SWIGLU = 2, EPI_SCORES = 3, EPI_SWIGLU8 = 4, EPI_CANDIDATES = 5 };

struct GemmParams {
  const bf16* A;
  const bf16* B;
  void* C;
  const bf16* bias;
  const bf16* residual;
  const int* row_group;   // scores: [N] group id of each index row (<0 = deleted)
  const int* q_group;     // scores: [M] group each query may see (<0 = any)
  const uint32_t* allow;  // scores: [M, ceil(N/32)] allow bitmask (optional)
  int M, N, K;
  long lda, ldb, ldc, ldr;
  int allow_words;
  int out_f32;
  // EPI_CANDIDATES: filtered scores >= thr[m] are appended to query m's candidate list instead of
  // writing the [M, N] score matrix (exact threshold top-k, see VectorIndex.search)
  const float* thr;  // [M]
  int* cnt;          // [M] appended count (may exceed cap: overflow, caller falls back)
  float* cand_val;   // [M, cap]
  int* cand_idx;     // [M, cap] column n
  int cap;
  int rows_b;  // SHUF: rows of the B copy (>= N, multiple of 16)
  int bgrp;    // SHUF: row blocks per group of the copy (shuffle_weights(w, group)), 1 = plain
};

__device__ __forceinline__ int gsw(int r) { return 2 * ((r >> 1) & 3); }

template <int EPI, int BM, int BN, int WGM, int WGN, bool SHUF = false>
__global__ __launch_bounds__(64 * WGM * WGN) void gemm_bt_kernel(GemmParams p) {
  constexpr int BK = 64;
  constexpr int NW = WGM * WGN;            // waves
  constexpr int TM = BM / WGM, TN = BN / WGN;  // per-wave tile
  constexpr int MI = TM / 16, NI = TN / 16;    // MFMA tiles per wave
  constexpr int TILE_A = BM * BK * 2, TILE_B = BN * BK * 2;
  __shared__ __attribute__((aligned(16))) char smem[2 * (TILE_A + TILE_B)];  // [buf][A|B]

  const int tiles_m = (p.M + BM - 1) / BM;
  const int tiles_n = (p.N + BN - 1) / BN;
  const int nwg = tiles_m * tiles_n;
  // bijective XCD remap: blocks b and b+8 share an XCD; give each XCD a contiguous id range
  const int bid = blockIdx.x;
  const int xcd = bid % 8, q8 = nwg / 8, r8 = nwg % 8;
  const int swz_id = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  const int tm = swz_id % tiles_m, tn = swz_id / tiles_m;
  const int m0 = tm * BM, n0 = tn * BN;

  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, g = lane >> 4, li = lane & 15;
  const int wm = w / WGN, wn = w % WGN;

  // staging: instruction c of wave w writes LDS bytes [(c*NW+w)*1024, +1024) of a tile = rows 8(c*NW+w)..+7
  auto stage = [&](int buf, int k0) {
    char* As = smem + buf * (TILE_A + TILE_B);
    char* Bs = As + TILE_A;
#pragma unroll
    for (int c = 0; c < BM / (8 * NW); ++c) {
      const int e = (c * NW + w) * 64 + lane;
      const int r = e >> 3, pos = e & 7;
      const int ra = min(m0 + r, p.M - 1);
      const bf16* ga = p.A + (size_t)ra * p.lda + k0 + (pos ^ gsw(r)) * 8;
      __builtin_amdgcn_global_load_lds((const void*)ga,
                                       (__attribute__((address_space(3))) void*)(As + (c * NW + w) * 1024), 16, 0, 0);
    }
#pragma unroll
    for (int c = 0; c < BN / (8 * NW); ++c) {
      const int idx = c * NW + w;
      const bf16* gb;
      if constexpr (SHUF) {  // piece idx = 16-row block idx / 2, 32-k block idx % 2 (clamped past the copy)
        const int blk = min(n0 / 16 + (idx >> 1), p.rows_b / 16 - 1);
        const int G = p.bgrp;  // fragment (blk, chunk) at ((blk / G) K/32 + chunk) G + blk % G
        gb = p.B + (((size_t)(blk / G) * (p.K / 32) + k0 / 32 + (idx & 1)) * G + blk % G) * 512 + lane * 8;
      } else {
        const int e = idx * 64 + lane;
        const int r = e >> 3, pos = e & 7;
        const int rb = min(n0 + r, p.N - 1);
        gb = p.B + (size_t)rb * p.ldb + k0 + (pos ^ gsw(r)) * 8;
      }
      __builtin_amdgcn_global_load_lds((const void*)gb,
                                       (__attribute__((address_space(3))) void*)(Bs + idx * 1024), 16, 0, 0);
    }
  };

  f32x4 acc[NI][MI];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < MI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = p.K / BK;
  stage(0, 0);
  for (int kt = 0; kt < nk; ++kt) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (kt + 1 < nk) stage((kt + 1) & 1, (kt + 1) * BK);
    const char* As = smem + (kt & 1) * (TILE_A + TILE_B);
    const char* Bs = As + TILE_A;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[MI], bfr[NI];
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int ra = wm * TM + 16 * i + li;
        af[i] = *reinterpret_cast<const bf16x8*>(As + ra * 128 + 16 * ((4 * ks + g) ^ gsw(ra)));
      }
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        if constexpr (SHUF) {
          bfr[i] = *reinterpret_cast<const bf16x8*>(Bs + (2 * ((wn * TN) / 16 + i) + ks) * 1024 + lane * 16);
        } else {
          const int rb = wn * TN + 16 * i + li;
          bfr[i] = *reinterpret_cast<const bf16x8*>(Bs + rb * 128 + 16 * ((4 * ks + g) ^ gsw(rb)));
        }
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ni = 0; ni < NI; ++ni)
#pragma unroll
        for (int mi = 0; mi < MI; ++mi) acc[ni][mi] = mfma16(bfr[ni], af[mi], acc[ni][mi]);
      __builtin_amdgcn_s_setprio(0);
    }
  }

  // epilogue: acc[ni][mi][r] = C[m = m0 + wm*TM + 16 mi + li][n = n0 + wn*TN + 16 ni + 4 g + r]
  if constexpr (EPI == EPI_SWIGLU8) {
    // 8-row [gate | up] groups inside each 16-row block: v_permlane32_swap of blocks (2 pi, 2 pi + 1)
    // hands lanes 0-31 block 2 pi's gate / up rows and lanes 32-63 block 2 pi + 1's (gemm256.hip);
    // the swap runs with every lane active, the row / column bounds only guard the stores
#pragma unroll
    for (int mi = 0; mi < MI; ++mi) {
      const int m = m0 + wm * TM + 16 * mi + li;
#pragma unroll
      for (int pi = 0; pi < NI / 2; ++pi) {
        float o[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc[2 * pi][mi][r]),
                                                           __float_as_uint(acc[2 * pi + 1][mi][r]), false, false);
          o[r] = silu_f(__uint_as_float(sw[0])) * __uint_as_float(sw[1]);
        }
        const int oc = (n0 + wn * TN) / 2 + 16 * pi + 4 * g;
        if (m < p.M && 2 * oc < p.N) {
          u32x2 v;
          v[0] = pack2bf(o[0], o[1]);
          v[1] = pack2bf(o[2], o[3]);
          *reinterpret_cast<u32x2*>((bf16*)p.C + (size_t)m * p.ldc + oc) = v;
        }
      }
    }
    return;
  }
#pragma unroll
  for (int mi = 0; mi < MI; ++mi) {
    const int m = m0 + wm * TM + 16 * mi + li;
    if (m >= p.M) continue;
    if (EPI == EPI_SWIGLU) {
      // weight rows interleaved in 16-row groups [gate 16 | up 16]: ni even = gate, ni odd = up
#pragma unroll
      for (int pi = 0; pi < NI / 2; ++pi) {
        const int ng = n0 + wn * TN + 32 * pi + 4 * g;  // gate column in the interleaved space
        if (ng >= p.N) continue;
        const int oc = (n0 + wn * TN) / 2 + 16 * pi + 4 * g;
        float o[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float gt = acc[2 * pi][mi][r], up = acc[2 * pi + 1][mi][r];
          if (p.bias) {
            gt += bf2f(p.bias[ng + r]);
            up += bf2f(p.bias[ng + 16 + r]);
          }
          o[r] = silu_f(gt) * up;
        }
        u32x2 v;
        v[0] = pack2bf(o[0], o[1]);
        v[1] = pack2bf(o[2], o[3]);
        *reinterpret_cast<u32x2*>((bf16*)p.C + (size_t)m * p.ldc + oc) = v;
      }
      continue;
    }
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
      const int n = n0 + wn * TN + 16 * ni + 4 * g;
      if (n >= p.N) continue;  // N % 4 == 0 is required by the launcher
      float o[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = acc[ni][mi][r];
      if (EPI == EPI_SCORES || EPI == EPI_CANDIDATES) {
        const int qg = p.q_group ? p.q_group[m] : -1;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          bool ok = true;
          if (p.row_group) {
            const int rg = p.row_group[n + r];
            ok = rg >= 0 && (qg < 0 || rg == qg);
          }
          if (p.allow) ok = ok && ((p.allow[(size_t)m * p.allow_words + ((n + r) >> 5)] >> ((n + r) & 31)) & 1u);
          if (!ok) o[r] = -__builtin_huge_valf();
        }
        if (EPI == EPI_CANDIDATES) {
          const float t = p.thr[m];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            if (o[r] >= t && o[r] != -__builtin_huge_valf()) {
              const int slot = atomicAdd(p.cnt + m, 1);
              if (slot < p.cap) {
                p.cand_val[(size_t)m * p.cap + slot] = o[r];
                p.cand_idx[(size_t)m * p.cap + slot] = n + r;
              }
            }
          }
          continue;  // no score matrix
        }
      } else {
        if (p.bias) {
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] += bf2f(p.bias[n + r]);
        }
        if (EPI == EPI_GELU) {
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = gelu_erf(o[r]);
        }
        if (p.residual) {
          const bf16* rr = p.residual + (size_t)m * p.ldr + n;
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = (p.out_f32 ? o[r] : bf2f(f2bf(o[r]))) + bf2f(rr[r]);  // bf16 GEMM + add
        }
      }
      if (p.out_f32) {
        *reinterpret_cast<f32x4*>((float*)p.C + (size_t)m * p.ldc + n) = f32x4{o[0], o[1], o[2], o[3]};
      } else {
        u32x2 v;
        v[0] = pack2bf(o[0], o[1]);
        v[1] = pack2bf(o[2], o[3]);
        *reinterpret_cast<u32x2*>((bf16*)p.C + (size_t)m * p.ldc + n) = v;
      }
    }
  }
}

template <int EPI, bool SHUF>
static int launch_gemm(const GemmParams& p, bool big, hipStream_t s) {
  if (big) {
    const int nwg = ((p.M + 255) / 256) * ((p.N + 255) / 256);
    hipLaunchKernelGGL((gemm_bt_kernel<EPI, 256, 256, 2, 4, SHUF>), dim3(nwg), dim3(512), 0, s, p);
  } else {
    const int nwg = ((p.M + 127) / 128) * ((p.N + 127) / 128);
    hipLaunchKernelGGL((gemm_bt_kernel<EPI, 128, 128, 2, 2, SHUF>), dim3(nwg), dim3(256), 0, s, p);
  }
  return hipGetLastError();
}

template <int EPI>
static int launch_gemm(const GemmParams& p, bool big, hipStream_t s, bool shuf) {
  return shuf ? launch_gemm<EPI, true>(p, big, s) : launch_gemm<EPI, false>(p, big, s);
}

int gemm_bt(const void* A, long lda, const void* B, long ldb, void* C, long ldc, const void* bias, const void* residual,
            long ldr, int M, int N, int K, int epilogue, int out_f32, const int* row_group, const int* q_group,
            const uint32_t* allow, int allow_words, hipStream_t s, int b_rows, int b_group) {
  if (M <= 0 || N <= 0) return 0;
  if (K % 64 || N % 4 || lda % 8 || ldb % 8) return hipErrorInvalidValue;
  if (b_group < 1 || (b_group > 1 && (b_rows <= 0 || b_rows % (16 * b_group)))) return hipErrorInvalidValue;
  if (epilogue == EPI_SWIGLU && (N % 32 || out_f32)) return hipErrorInvalidValue;
  if (epilogue == EPI_SWIGLU8 && (N % 32 || out_f32 || bias || residual)) return hipErrorInvalidValue;
  if (b_rows > 0 && (b_rows < N || b_rows % 16 || ldb != K)) return hipErrorInvalidValue;
  GemmParams p;
  p.A = (const bf16*)A;
  p.B = (const bf16*)B;
  p.C = C;
  p.bias = (const bf16*)bias;
  p.residual = (const bf16*)residual;
  p.row_group = row_group;
  p.q_group = q_group;
  p.allow = allow;
  p.M = M;
  p.N = N;
  p.K = K;
  p.lda = lda;
  p.ldb = ldb;
  p.ldc = ldc;
  p.ldr = ldr;
  p.allow_words = allow_words;
  p.out_f32 = out_f32;
  p.rows_b = b_rows;
  p.bgrp = b_group;
  const bool sh = b_rows > 0;
  // large problems: 256x256 tiles, 8 waves of 128x64 (half the LDS fragment traffic per MFMA of the
  // 64x64 wave tile); small M or N: 128x128 tiles, 4 waves (less padding, more workgroups)
  const bool big = M >= 2048 && N >= 512 && ((long)((M + 255) / 256) * ((N + 255) / 256)) >= 160;
  switch (epilogue) {
    case EPI_NONE: return launch_gemm<EPI_NONE>(p, big, s, sh);
    case EPI_GELU: return launch_gemm<EPI_GELU>(p, big, s, sh);
    case EPI_SWIGLU: return launch_gemm<EPI_SWIGLU>(p, big, s, sh);
    case EPI_SCORES: return launch_gemm<EPI_SCORES>(p, big, s, sh);
    case EPI_SWIGLU8: return launch_gemm<EPI_SWIGLU8>(p, big, s, sh);
    default: return hipErrorInvalidValue;
  }
}

// b_rows > 0: B is a shuffle_weights copy of b_rows >= N rows (the index's one row layout).
int gemm_score_candidates(const void* A, long lda, const void* B, long ldb, int M, int N, int K, const int* row_group,
                          const int* q_group, const float* thr, int* cnt, float* cand_val, int* cand_idx, int cap,
                          hipStream_t s, int b_rows) {
  if (M <= 0 || N <= 0) return 0;
  if (K % 64 || N % 4 || lda % 8 || ldb % 8 || cap <= 0 || !thr || !cnt || !cand_val || !cand_idx)
    return hipErrorInvalidValue;
  if (b_rows > 0 && (b_rows < N || b_rows % 16 || ldb != K)) return hipErrorInvalidValue;
  // 65+ query batches past the scan's limits (and every batch of 128+): the persistent gemm256 kernel
  // (a 10M-row scan at K 768 is 39k short-K tiles per 256 queries; the one-tile-per-workgroup kernel
  // below pays its prologue and epilogue on every one of them)
  const bool scan_ok = b_rows == 0 && K % 256 == 0 && ((M <= 64 && K <= 1024) || (M <= 96 && K <= 768));
  if (K % 128 == 0 && (M >= 128 || (M > 64 && !scan_ok)))
    return gemm256_candidates(A, lda, B, ldb, M, N, K, row_group, q_group, thr, cnt, cand_val, cand_idx, cap, s,
                              b_rows);
  // 1..64 queries (K <= 1024) or 65..96 (K <= 768): the persistent scan with the queries in LDS once
  // per workgroup (K % 256 == 0); 32..64 at other widths: the index streams through the decode GEMM's weight ring.
  // Row-major copies only here; shuffled copies go through score_candidates_shuf (VectorIndex picks).
  if (scan_ok)
    return index_scan_candidates(A, lda, B, ldb, M, N, K, row_group, q_group, thr, cnt, cand_val, cand_idx, cap, s);
  if (b_rows == 0 && M >= 32 && M <= 64 && K % 128 == 0)
    return stream_score_candidates(A, lda, B, ldb, M, N, K, row_group, q_group, thr, cnt, cand_val, cand_idx, cap, s);
  GemmParams p{};
  p.bgrp = 1;
  p.A = (const bf16*)A;
  p.B = (const bf16*)B;
  p.row_group = row_group;
  p.q_group = q_group;
  p.M = M;
  p.N = N;
  p.K = K;
  p.lda = lda;
  p.ldb = ldb;
  p.thr = thr;
  p.cnt = cnt;
  p.cand_val = cand_val;
  p.cand_idx = cand_idx;
  p.cap = cap;
  p.rows_b = b_rows;
  const bool big = M >= 2048 && N >= 512 && ((long)((M + 255) / 256) * ((N + 255) / 256)) >= 160;
  return launch_gemm<EPI_CANDIDATES>(p, big, s, b_rows > 0);
}

}  // namespace dab

// Attention kernels on MFMA (v_mfma_f32_16x16x32_bf16) for gfx950.
//
//  flash_fwd   : variable-length, flash-style forward (online softmax) used for
//                  - the BERT/bge encoder (bidirectional, K/V read from the packed QKV rows)   (N5)
//                  - Llama prefill (causal, GQA, K/V read from the paged KV cache, so chunked
//                    prefill and shared prefixes need no special path)                         (N10)
//  paged_decode: single-token decode over the paged KV cache, split over key partitions
//                (flash-decoding); the last workgroup to finish a (sequence, kv head) combines
//                its partitions in the same launch                                              (N9)
//
// Both compute S^T = K Q^T so that the MFMA C layout leaves the QUERY on the lane and the keys in
// the registers; the probabilities P are then already the B operand of O^T = V^T P^T (no LDS round
// trip for P), and V^T is fed from a row-major LDS V tile with ds_read_b64_tr_b16 (hardware
// transpose).  K and V tiles are XOR-swizzled in LDS so that both the ds_read_b128 row reads of K
// and the transposed reads of V are bank-conflict free (derivation in docs/kernels.md).
//
// Reference behaviour replaced: HF BertSelfAttention (ai/embedders/transformers.py:18-22) and the
// HF Llama attention inside model.generate (ai/providers/transformers.py:57-66).
#include <cstdlib>

#include "common.h"
#include "launchers.h"

#include <type_traits>

#define DAB_ALWAYS_INLINE __attribute__((always_inline))

namespace dab {

constexpr float kNegInf = -__builtin_huge_valf();

// Byte offset of 16-byte chunk c of row r in a [rows][D] bf16 LDS tile.  The XOR keeps chunk
// pairs (2j, 2j+1) together so that the 32-byte row pieces of a transposed read also spread.
template <int D>
__device__ __forceinline__ int swz(int r, int c) {
  constexpr int RB = D * 2;
  constexpr int CPR = D / 8;
  constexpr int RPB = (256 / RB) > 0 ? (256 / RB) : 1;
  return r * RB + 16 * (c ^ ((2 * (r / RPB)) & (CPR - 1)));
}

struct FlashParams {
  const bf16* q;
  long q_stride_tok, q_stride_head;
  const bf16* k;
  const bf16* v;
  long kv_stride_tok, kv_stride_head;
  const bf16* k_cache;
  const bf16* v_cache;
  const int* block_tables;
  int max_blocks, block_size;
  bf16* out;
  long o_stride_tok, o_stride_head;
  const int* cu_q;
  const int* cu_k;
  const int* ctx_k;
  int Hq, Hkv;
  float scale_log2;
  // flash_d128 only: rotate Q by RoPE on load (positions of the packed query tokens, [max_pos, 64]
  // float2 cos/sin table), when the RoPE/KV-write kernel wrote only K / V
  const int* rope_pos;
  const float2* rope_cs;
  int pairs_per_wg;  // flash_d128 PAIR: causal query-block pairs walked by one workgroup (>= 1)
  // flash_d128 PAIR: heaviest-first walk -- each XCD runs the first pair group (the longest blocks)
  // of all its (sequence, head) units before any later group (lighter), instead of alternating
  int lpt;
};

// One workgroup = 16 QT NW queries (NW waves x QT 16-query sub-tiles) of one (sequence, head);
// 64-key tiles staged through LDS with register prefetch of the next tile during compute (issue
// early / write late).  Each K / V fragment read from LDS feeds QT MFMAs (QT = 2 halves the LDS
// reads per MFMA but needs 294 registers, one wave per SIMD, and measured 45 % slower than QT = 1
// with 8 waves; see the launcher).
// The K/V tiles of a (sequence, kv head) are re-read by every query block of its GQA heads, so the
// grid is walked XCD-major: a (sequence, kv head)'s workgroups get ids that share blockIdx % 8 and
// land on one XCD, whose L2 then serves the re-reads (round-robin dispatch puts block i on XCD i % 8).
// Deferred online-softmax rescale (cdna_hip_programming.md T13): the running maximum is kept until a
// row maximum grows by more than 2^kDeferLog2, so P stays <= 2^8 and the O / l rescale is skipped on
// most tiles; decided before the tile's P is exponentiated (nothing is scaled twice).
constexpr float kDeferLog2 = 8.f;

// (QT = 2 with 4 waves is held to 256 registers -- 2 waves per SIMD, no spills -- by the
// launch bound; unbounded it took 294 and ran at 1 wave per SIMD.)  MINW > 0 overrides the bound:
// the encoder (D 64, one or two key tiles per ~50-token sequence) is a short latency chain per
// workgroup, so resident workgroups are its throughput; MINW 5 holds it to 88 registers (5 waves per
// SIMD, no spills) instead of 112 (4).
template <int D, bool CAUSAL, bool PAGED, int NW, int QT, int MINW = 0>
__global__ __launch_bounds__(64 * NW, MINW ? MINW : ((QT == 2 && NW == 4) ? 2 : 1)) void flash_fwd_kernel(FlashParams p) {
  constexpr int KT = 64;
  constexpr int NT = 64 * NW;
  constexpr int QB = 16 * QT * NW;
  constexpr int NKK = D / 32;
  constexpr int NTD = D / 16;
  constexpr int CPR = D / 8;
  constexpr int TILE_BYTES = KT * D * 2;
  constexpr int CH = KT * CPR / NT;
  static_assert(CH >= 1, "tile too small for the workgroup");
  __shared__ __attribute__((aligned(16))) char smem[2 * TILE_BYTES];
  char* ks = smem;
  char* vs = smem + TILE_BYTES;

  // linear block id -> XCD-major id (bijective for any grid size) -> (query block, head, sequence)
  // with query blocks fastest and the heads of one GQA group adjacent
  const int nqb = gridDim.x;
  const int nwg = nqb * gridDim.y * gridDim.z;
  const int lin = blockIdx.x + nqb * (blockIdx.y + gridDim.y * blockIdx.z);
  const int xcd = lin % 8, q8 = nwg / 8, r8 = nwg % 8;
  const int sid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + lin / 8;
  const int h = (sid / nqb) % gridDim.y;
  const int b = sid / (nqb * gridDim.y);
  const int q_start = p.cu_q[b];
  const int seqlen_q = p.cu_q[b + 1] - q_start;
  // causal: a sequence's last query block (the most key tiles) starts first, so the short blocks
  // fill the end of each XCD's walk instead of a long one trailing alone
  const int nqb_b = div_up(seqlen_q, QB);
  const int qb = CAUSAL && sid % nqb < nqb_b ? nqb_b - 1 - sid % nqb : sid % nqb;
  const int q0 = qb * QB;
  if (q0 >= seqlen_q) return;
  int kv_len, k_start = 0;
  if (PAGED) {
    kv_len = p.ctx_k[b];
  } else {
    k_start = p.cu_k[b];
    kv_len = p.cu_k[b + 1] - k_start;
  }
  const int hk = h / (p.Hq / p.Hkv);
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, g = lane >> 4, li = lane & 15;
  // this lane's query in sub-tile qt: row q0 + 16 (QT w + qt) + li
  int my_q[QT], q_pos[QT];
  bool q_valid[QT];
  bf16x8 qf[QT][NKK];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    my_q[qt] = q0 + 16 * (QT * w + qt) + li;
    q_valid[qt] = my_q[qt] < seqlen_q;
    q_pos[qt] = kv_len - seqlen_q + my_q[qt];
    const bf16* qrow =
        p.q + (size_t)(q_start + (q_valid[qt] ? my_q[qt] : 0)) * p.q_stride_tok + (size_t)h * p.q_stride_head;
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk) {
      bf16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
      qf[qt][kk] = q_valid[qt] ? *reinterpret_cast<const bf16x8*>(qrow + 32 * kk + 8 * g) : z;
    }
  }

  int n_keys = kv_len;
  if (CAUSAL) {
    const int last_q = min(q0 + QB - 1, seqlen_q - 1);
    n_keys = min(kv_len, kv_len - seqlen_q + last_q + 1);
  }
  const int n_tiles = div_up(n_keys, KT);

  u32x4 kreg[CH], vreg[CH];
  // Branch-free staging: rows past the end are clamped to the last valid key (finite data, masked
  // to -inf in the scores), and the paged block id is looked up once per tile (wave-uniform) --
  // per-lane lookups behind a branch made the compiler drain vmcnt(0) per 16-B chunk.
  auto load_tile = [&](int kt) {
    const int k0 = kt * KT;
    const int last = kv_len - 1 - k0;
    size_t base;
    if (PAGED) {
      const int blk = p.block_tables[(size_t)b * p.max_blocks + k0 / p.block_size];
      base = (((size_t)blk * p.Hkv + hk) * p.block_size + (k0 % p.block_size)) * D;
    } else {
      base = (size_t)(k_start + k0) * p.kv_stride_tok + (size_t)hk * p.kv_stride_head;
    }
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int idx = tid + c * NT;
      const int row = min(idx / CPR, last), ch = idx % CPR;
      const size_t off = base + (PAGED ? (size_t)row * D : (size_t)row * p.kv_stride_tok) + ch * 8;
      kreg[c] = *reinterpret_cast<const u32x4*>((PAGED ? p.k_cache : p.k) + off);
      vreg[c] = *reinterpret_cast<const u32x4*>((PAGED ? p.v_cache : p.v) + off);
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int idx = tid + c * NT;
      const int row = idx / CPR, ch = idx % CPR;
      *reinterpret_cast<u32x4*>(ks + swz<D>(row, ch)) = kreg[c];
      *reinterpret_cast<u32x4*>(vs + swz<D>(row, ch)) = vreg[c];
    }
  };

  f32x4 o[QT][NTD];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt)
#pragma unroll
    for (int t = 0; t < NTD; ++t) o[qt][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run[QT], l_run[QT];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    m_run[qt] = -1e30f;
    l_run[qt] = 0.f;
  }

  if (n_tiles > 0) {
    load_tile(0);
    store_tile();
  }
  for (int kt = 0; kt < n_tiles; ++kt) {
    __syncthreads();
    if (kt + 1 < n_tiles) load_tile(kt + 1);
    // S^T = K Q^T: each K fragment feeds QT MFMAs
    f32x4 s[QT][4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) s[qt][m] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < NKK; ++kk) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(ks + swz<D>(16 * m + li, 4 * kk + g));
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) s[qt][m] = mfma16(a, qf[qt][kk], s[qt][m]);
      }
    }
    // online softmax per query sub-tile; only the tail / diagonal tiles need the mask
    const bool need_mask = (kt + 1) * KT > kv_len || (CAUSAL && (kt + 1) * KT - 1 > kv_len - seqlen_q + q0);
    bf16x8 pb[QT][2];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
      float mx = kNegInf;
#pragma unroll
      for (int m = 0; m < 4; ++m) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = s[qt][m][r] * p.scale_log2;
          if (need_mask) {
            const int key = kt * KT + 16 * m + 4 * g + r;
            if (key >= kv_len || (CAUSAL && key > q_pos[qt])) v = kNegInf;
          }
          s[qt][m][r] = v;
          mx = fmaxf(mx, v);
        }
      }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      // deferred rescale as in flash_d128 (kDeferLog2); raw v_exp_f32 (results below 2^-126 do not
      // matter next to the row maximum's 1)
      const bool keep = __all(mx - m_run[qt] <= kDeferLog2);
      const float m_new = keep ? m_run[qt] : fmaxf(m_run[qt], mx);
      const float alpha = __builtin_amdgcn_exp2f(m_run[qt] - m_new);
      float ls = 0.f;
#pragma unroll
      for (int m = 0; m < 4; ++m) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = __builtin_amdgcn_exp2f(s[qt][m][r] - m_new);
          s[qt][m][r] = e;
          ls += e;
        }
      }
      l_run[qt] = l_run[qt] * alpha + ls;
      m_run[qt] = m_new;
#pragma unroll
      for (int ss = 0; ss < 2; ++ss)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pb[qt][ss][j] = (short)f2bf(s[qt][2 * ss][j]);
          pb[qt][ss][j + 4] = (short)f2bf(s[qt][2 * ss + 1][j]);
        }
      if (!keep) {
#pragma unroll
        for (int t = 0; t < NTD; ++t) o[qt][t] *= alpha;
      }
    }
    // O^T += V^T P^T: each transposed V fragment feeds QT MFMAs
    const int qq = li >> 2, pp = li & 3;
#pragma unroll
    for (int ss = 0; ss < 2; ++ss) {
#pragma unroll
      for (int t = 0; t < NTD; ++t) {
        const int ch = 2 * t + (pp >> 1);
        const int boff = 8 * (pp & 1);
        const bf16x4 lo = ds_read_tr16(vs + swz<D>(32 * ss + 4 * g + qq, ch) + boff);
        const bf16x4 hi = ds_read_tr16(vs + swz<D>(32 * ss + 16 + 4 * g + qq, ch) + boff);
        const bf16x8 a = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) o[qt][t] = mfma16(a, pb[qt][ss], o[qt][t]);
      }
    }
    __syncthreads();
    if (kt + 1 < n_tiles) store_tile();
  }

#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    float l_tot = l_run[qt];
    l_tot += __shfl_xor(l_tot, 16, 64);
    l_tot += __shfl_xor(l_tot, 32, 64);
    if (!q_valid[qt]) continue;
    const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
    bf16* orow = p.out + (size_t)(q_start + my_q[qt]) * p.o_stride_tok + (size_t)h * p.o_stride_head;
#pragma unroll
    for (int t = 0; t < NTD; ++t) {
      u32x2 v;
      v[0] = pack2bf(o[qt][t][0] * inv, o[qt][t][1] * inv);
      v[1] = pack2bf(o[qt][t][2] * inv, o[qt][t][3] * inv);
      *reinterpret_cast<u32x2*>(orow + 16 * t + 4 * g) = v;
    }
  }
}

// -----------------------------------------------------------------------------------------------
// Llama prefill attention (D = 128, paged KV cache, GQA): 32x32x16 MFMA tiles.
//
// The 16x16 kernel above feeds every K / V fragment it reads from LDS to ONE MFMA for 16 queries;
// at D = 128 that made its LDS traffic (reads + register-staged tile writes) larger than its MFMA
// time.  Here a wave owns 32 queries and every fragment feeds a 32x32x16 MFMA (half the LDS bytes
// per FLOP, cdna_hip_programming.md Appendix B "Fused attention prefill"):
//   * workgroup = 4 waves x 32 queries of one (sequence, head); 64-key K / V tiles arrive by LDS-DMA
//     (buffer_load ... lds, no VGPR round trip) into a 2-deep ring (64 KB: 2 workgroups per CU); the
//     descriptor range stops at the last valid key, so rows past it are zeros (finite under the mask);
//   * S^T = K Q^T (K rows as the A operand, Q^T fragments held in registers): lane (q, hi) ends with
//     32 of the 64 scores of query q; row max / sum combine with the partner lane q ^ 32;
//   * P^T is the B operand of O^T += V^T P^T straight from the S accumulators (cvt_pk only, the k
//     order permuted to match), V^T fragments by ds_read_b64_tr_b16 (hardware transpose);
//   * LDS rows are 256 B; the 16-B chunk c of row r lives at c ^ f(r), f(r) = (r & 3) << 2 | (r >> 2) & 3:
//     conflict-free for the 16-row ds_read_b128 lane groups of the K reads AND for the 4-row x 64-B
//     pieces of the transposed V reads (each row of a 4-row group lands in its own 64-B bank range).
// (f32x16 / mfma32: common.h)

// f(integral_constant<I>) for I in [B, E)
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

__device__ __forceinline__ int f128(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }

// The 8 transposed V reads of one k-step (ds_read_b64_tr_b16) as ONE asm statement that also waits
// for them: the intrinsic form makes hipcc drain every LDS-DMA still in flight (vmcnt(0)) before the
// first transposed read, i.e. the next tile's copy that should stream in under this tile's P.V, and
// separate asm reads would let hipcc copy an output register before the data has landed.  The
// per-lane addresses are loop invariants; OFF (tile buffer, key block) is the instruction offset.
template <int OFF>
__device__ __forceinline__ void ds_tr16_x8(const unsigned (&a)[8], u32x2 (&r)[8]) {
  asm volatile(
      "ds_read_b64_tr_b16 %0, %8 offset:%16\n\t"
      "ds_read_b64_tr_b16 %1, %9 offset:%16\n\t"
      "ds_read_b64_tr_b16 %2, %10 offset:%16\n\t"
      "ds_read_b64_tr_b16 %3, %11 offset:%16\n\t"
      "ds_read_b64_tr_b16 %4, %12 offset:%16\n\t"
      "ds_read_b64_tr_b16 %5, %13 offset:%16\n\t"
      "ds_read_b64_tr_b16 %6, %14 offset:%16\n\t"
      "ds_read_b64_tr_b16 %7, %15 offset:%16\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]), "=&v"(r[4]), "=&v"(r[5]), "=&v"(r[6]), "=&v"(r[7])
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7]), "i"(OFF)
      : "memory");
}

// The same 8 transposed reads without the wait (VPIPE): the next k-step's V fragments are requested
// before the current k-step's MFMAs and retired by a counted lgkmcnt (lgkm_wait) right before their
// use, so the LDS latency hides under the MFMAs instead of stalling the wave four times per tile.
template <int OFF>
__device__ __forceinline__ void ds_tr16_issue(const unsigned (&a)[8], u32x2 (&r)[8]) {
  asm volatile(
      "ds_read_b64_tr_b16 %0, %8 offset:%16\n\t"
      "ds_read_b64_tr_b16 %1, %9 offset:%16\n\t"
      "ds_read_b64_tr_b16 %2, %10 offset:%16\n\t"
      "ds_read_b64_tr_b16 %3, %11 offset:%16\n\t"
      "ds_read_b64_tr_b16 %4, %12 offset:%16\n\t"
      "ds_read_b64_tr_b16 %5, %13 offset:%16\n\t"
      "ds_read_b64_tr_b16 %6, %14 offset:%16\n\t"
      "ds_read_b64_tr_b16 %7, %15 offset:%16"
      : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]), "=&v"(r[4]), "=&v"(r[5]), "=&v"(r[6]), "=&v"(r[7])
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7]), "i"(OFF)
      : "memory");
}

// s_waitcnt lgkmcnt(N) + a scheduling fence: hipcc would otherwise hoist the register-only MFMAs
// that consume the asm reads above the wait (cdna_hip_programming.md rule 18)
template <int N>
__device__ __forceinline__ void lgkm_wait() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(N) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// the value of lane l ^ 32 (v_permlane32_swap: VALU, no LDS round trip on the lgkm counter)
__device__ __forceinline__ float xor32(float v) {
  const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float((threadIdx.x & 32) ? sw[0] : sw[1]);
}

__device__ __forceinline__ unsigned lds_addr(const char* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

// NW = 8 (W8): 8 waves x 32 queries share each K / V tile (half the DMA per query) and the ring is 3
// tiles deep (96 KB: one workgroup per CU, still 2 waves per SIMD): tile t + 2 is requested right
// after the one barrier of tile t, so each tile has two tiles' compute to land in, and the
// per-tile wait is a counted vmcnt (tile t + 1's pieces stay in flight).
//
// STAG (8 waves, 4-deep ring): the two wave groups (waves 0-3 / 4-7, one of each per SIMD) are half a
// tile apart.  Group 0 runs S(t), softmax(t), PV(t); group 1 runs PV(t-1), S(t), softmax(t), holding
// P(t-1) in registers across the barrier, so on every SIMD one group's softmax VALU runs beside the
// other group's MFMAs instead of both groups hitting the same pipe at once.  PV(t-1) finishes before
// softmax(t) may rescale O (cdna_hip_programming.md T13 hazard).  Tile t-1's buffer stays live through
// iteration t, hence the 4th buffer (128 KB).
//
// PAIR (causal, 4 waves): one workgroup runs query block nqb-1-i and then block i of its (sequence,
// head), so every workgroup has 2 (nqb + 1) key tiles of work, and block i's first K / V tile and the
// rest of its stream continue from block nqb-1-i's last tile on without a cold start (same keys).
//
// ONEBAR (4 waves): one barrier per tile instead of two.  Each wave waits for its own pieces of tile
// t, then the barrier says both "every piece of tile t landed" and "every wave is past tile t - 1",
// so tile t + 1's DMA goes into t - 1's buffer right after it.
//
// SMS (with VPIPE): the softmax split across the PV k-steps -- the row maximum first, then the
// exponentials of k-step ks + 1's 16 keys issued behind k-step ks's MFMAs, so the transcendental
// work of one slice runs beside the matrix cores instead of all of it before them (the
// 'sm-split' of cdna_hip_programming.md Appendix B).  The row sum accumulates slice by slice (a
// different fp32 summation order than the unsplit kernel: equal to within a bf16 rounding).
//
// SGB (A/B): the S^T phase's 16 K-fragment LDS reads and 16 MFMAs interleaved by
// sched_group_barrier (4 reads ahead, then one MFMA per read) instead of hipcc's own order; same
// instructions and accumulation order (bit-identical).
template <bool CAUSAL, bool VPIPE = false, int NW = 4, bool STAG = false, bool PAIR = false, bool ONEBAR = false,
          bool SMS = false, bool SGB = false>
__global__ __launch_bounds__(64 * NW, NW == 4 ? 2 : 1) void flash_d128_kernel(FlashParams p) {
  static_assert(NW == 4 || NW == 8, "4 or 8 waves");
  static_assert(!STAG || NW == 8, "staggered groups: 8 waves");
  static_assert(!PAIR || (NW == 4 && CAUSAL), "paired blocks: 4 waves, causal");
  constexpr int D = 128, KT = 64, QB = 32 * NW;
  constexpr int TILE = KT * D * 2;  // 16 KB
  constexpr int BUF = 2 * TILE;     // K | V
  constexpr int NBUF = STAG ? 4 : (NW == 8 ? 3 : 2);
  constexpr int PPW = 16 / NW;      // 1-KB K (and V) pieces per wave per tile
  __shared__ __attribute__((aligned(16))) char smem[NBUF * BUF];

  // same XCD-major (query block, head, sequence) walk as flash_fwd_kernel
  const int nqb = gridDim.x;
  const int nwg = nqb * gridDim.y * gridDim.z;
  const int lin = blockIdx.x + nqb * (blockIdx.y + gridDim.y * blockIdx.z);
  const int xcd = lin % 8, q8 = nwg / 8, r8 = nwg % 8;
  int sid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + lin / 8;
  if (PAIR && p.lpt) {
    // the (sequence, head) units split evenly over the XCDs (units % 8 == 0, checked by the host);
    // on each XCD, pair group 0 of every unit, then group 1, ...: the mixed-duration workgroups of
    // a ragged pair split no longer alternate, so greedy dispatch cannot strand a long one at the end
    const int nu = gridDim.y * gridDim.z / 8, k = lin / 8;
    sid = (xcd * nu + k % nu) * nqb + k / nu;
  }
  const int h = (sid / nqb) % gridDim.y;
  const int b = sid / (nqb * gridDim.y);
  // the sequence's block ids are requested first: they depend on b alone, so their round trip runs
  // beside the cu_q / ctx_k loads instead of after them (in-bounds for any row: lane / tpb < max_blocks)
  const int* bt = p.block_tables + (size_t)b * p.max_blocks;
  const int tpb = p.block_size / KT;  // tiles per cache block
  const int bl = (int)(threadIdx.x & 63);
  const int bt_a = bl / tpb < p.max_blocks ? bt[bl / tpb] : 0;
  const int bt_b = (64 + bl) / tpb < p.max_blocks ? bt[(64 + bl) / tpb] : 0;
  const int q_start = p.cu_q[b];
  const int seqlen_q = p.cu_q[b + 1] - q_start;
  // causal: a sequence's last query block (the most key tiles) starts first, so the short blocks
  // fill the end of each XCD's walk instead of a long one trailing alone
  const int nqb_b = div_up(seqlen_q, QB);
  // PAIR: this workgroup's blocks are, for its pairs pp = p_first .. p_first + G - 1, the long block
  // nqb_b - 1 - pp then the short block pp (absent for the middle block of an odd count)
  const int G = PAIR ? p.pairs_per_wg : 1;
  const int p_first = (sid % nqb) * G;
  const int npairs = div_up(nqb_b, 2);
  auto blk_qb = [&](const int j) DAB_ALWAYS_INLINE {
    const int pp = p_first + (j >> 1);
    if (j >= 2 * G || pp >= npairs) return -1;
    const int lng = nqb_b - 1 - pp;
    return (j & 1) ? (pp < lng ? pp : -1) : lng;
  };
  auto next_blk = [&](const int j) DAB_ALWAYS_INLINE {
    if (blk_qb(j + 1) >= 0) return j + 1;
    return blk_qb(j + 2) >= 0 ? j + 2 : -1;  // (only a missing short block is skipped)
  };
  int qb;
  if constexpr (PAIR) {
    if (p_first >= npairs) return;  // whole workgroup
    qb = blk_qb(0);
  } else {
    qb = CAUSAL && sid % nqb < nqb_b ? nqb_b - 1 - sid % nqb : sid % nqb;
  }
  int q0 = qb * QB;
  if (q0 >= seqlen_q) return;  // whole workgroup
  const int kv_len = p.ctx_k[b];
  const int hk = h / (p.Hq / p.Hkv);
  const int tid = threadIdx.x, lane = tid & 63, lq = lane & 31, hi = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  int my_q, q_pos, w_kmax;
  bool q_valid, w_any;
  auto set_block = [&](const int q0_) DAB_ALWAYS_INLINE {
    q0 = q0_;
    my_q = q0 + 32 * w + lq;
    q_valid = my_q < seqlen_q;
    q_pos = kv_len - seqlen_q + my_q;
    // highest key position any valid query of this wave attends to (wave-uniform)
    const int w_last_q = min(q0 + 32 * w + 31, seqlen_q - 1);
    w_kmax = CAUSAL ? kv_len - seqlen_q + w_last_q : kv_len - 1;
    w_any = q0 + 32 * w < seqlen_q;
  };
  set_block(q0);

  // Q^T fragments (B operand): lane (q, hi) holds Q[q][16 s + 8 hi .. + 8], s = 0..7
  bf16x8 qf[8];
  auto load_q = [&]() DAB_ALWAYS_INLINE {
    const bf16* qrow = p.q + (size_t)(q_start + (q_valid ? my_q : 0)) * p.q_stride_tok + (size_t)h * p.q_stride_head;
#pragma unroll
    for (int st = 0; st < 8; ++st) {
      const bf16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
      qf[st] = q_valid ? *reinterpret_cast<const bf16x8*>(qrow + 16 * st + 8 * hi) : z;
    }
  };
  load_q();
  // RoPE of Q on load (rope_cs): dims 16 st + 8 hi + j (st < 4) pair with the same lane's dims + 64
  // (st + 4).  Applied after the first K/V tile's DMA is issued, so its loads and math overlap it.
  bool rope_q = p.rope_cs && q_valid;
  // cos/sin rows through a wave-uniform buffer descriptor (empty range without RoPE: the loads
  // return zeros and touch nothing), so the loads are unconditional and hipcc's wait counting stays
  // exact across them (a conditional load made it drain the first tile's DMA)
  int cs_row = p.rope_cs ? p.rope_pos[q_start + (q_valid ? my_q : 0)] : 0;
  const auto cs_rs = __builtin_amdgcn_make_buffer_rsrc((void*)(p.rope_cs ? (const void*)p.rope_cs : (const void*)p.q),
                                                       (short)0, p.rope_cs ? 0x7ffffff0 : 0, 0x00020000);
  float4 c4[4][4];
  auto apply_rope = [&]() DAB_ALWAYS_INLINE {
    if (!rope_q) return;
#pragma unroll
    for (int st = 0; st < 4; ++st) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float4 cc = c4[st][j >> 1];
        const float2 cs = (j & 1) ? make_float2(cc.z, cc.w) : make_float2(cc.x, cc.y);
        float x1 = bf2f((uint16_t)qf[st][j]), x2 = bf2f((uint16_t)qf[st + 4][j]);
        rope_rot(x1, x2, cs);
        qf[st][j] = (short)f2bf(x1);
        qf[st + 4][j] = (short)f2bf(x2);
      }
    }
  };

  auto tiles_of = [&](const int q0_) DAB_ALWAYS_INLINE {
    int n_keys = kv_len;
    if (CAUSAL) {
      const int last_q = min(q0_ + QB - 1, seqlen_q - 1);
      n_keys = min(kv_len, kv_len - seqlen_q + last_q + 1);
    }
    return div_up(n_keys, KT);
  };
  const int n_tiles = tiles_of(q0);  // (PAIR: of the long block; the short one's are a prefix)

  // LDS-DMA staging (buffer_load ... lds): wave w issues K / V pieces i = 4 w .. 4 w + 3 (1 KB =
  // 4 rows each); LDS slot (row 4 i + lane / 16, physical chunk lane % 16) receives logical chunk
  // (lane % 16) ^ f(row).  The descriptor range ends at the last valid key: rows past it read zeros.
  const int st_row = lane >> 4, st_pc = lane & 15;
  // block ids of the first 128 tiles (8192 keys) in two registers per lane, read once; per tile a
  // readlane (no memory round trip in the loop: a block-id load there exposed a full global-memory
  // latency per tile, because the DMA request that needs it waits for it)
  auto blk_of = [&](int t) {
    if (t < 64) return __builtin_amdgcn_readlane(bt_a, t);
    if (t < 128) return __builtin_amdgcn_readlane(bt_b, t - 64);
    // past 8192 keys (volatile: never speculated; readfirstlane: the block id, and with it the
    // DMA descriptor, stays wave-uniform, so hipcc builds no waterfall loop around the DMA)
    return __builtin_amdgcn_readfirstlane(((volatile const int*)bt)[t / tpb]);
  };
  auto issue = [&](int t, int buf, int blk) {
    const int k0 = t * KT;
    const int nvalid = min(KT, kv_len - k0);
    const size_t base = (((size_t)blk * p.Hkv + hk) * p.block_size + (k0 % p.block_size)) * D;
    const auto rk = __builtin_amdgcn_make_buffer_rsrc((void*)(p.k_cache + base), (short)0, nvalid * D * 2, 0x00020000);
    const auto rv = __builtin_amdgcn_make_buffer_rsrc((void*)(p.v_cache + base), (short)0, nvalid * D * 2, 0x00020000);
    char* kdst = smem + buf * BUF;
#pragma unroll
    for (int j = 0; j < PPW; ++j) {
      const int i = PPW * w + j;
      const int row = 4 * i + st_row;
      const unsigned off = (unsigned)(row * D + 8 * (st_pc ^ f128(row))) * 2u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rk, (__attribute__((address_space(3))) void*)(kdst + i * 1024), 16, off,
                                               0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rv, (__attribute__((address_space(3))) void*)(kdst + TILE + i * 1024),
                                               16, off, 0, 0, 0);
    }
  };

  f32x16 o[4];
#pragma unroll
  for (int db = 0; db < 4; ++db)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[db][r] = 0.f;
  float m_run = -1e30f, l_run = 0.f;  // running max in log2 units (scores x scale_log2)
  const float sc = p.scale_log2;

  // Loop-invariant LDS addresses (the tile buffer and the key block go in the instruction offset).
  // K reads of k-step st: row lq (and 32 + lq: +8 KB), logical chunk 2 st + hi at (2 st + hi) ^ f(lq).
  const unsigned smem0 = lds_addr(smem);
  unsigned kadr[8];
  {
    const int fr = f128(lq);
#pragma unroll
    for (int st = 0; st < 8; ++st) kadr[st] = smem0 + lq * 256 + 16 * ((2 * st + hi) ^ fr);
  }
  // Transposed V reads: 16-lane group G = lane / 16 covers d 32 db + 16 (G & 1) + (0..15); lane
  // 4 qq + pp supplies row k + qq, d 4 pp .. 4 pp + 3.  For k-step (kb, ss) the first read's rows are
  // 32 kb + 16 ss + 4 (G >> 1) + qq, whose f is (qq << 2) | (G >> 1) for every kb, ss (and
  // | ((G >> 1) + 2) for the second read, 8 rows on), so only the offset changes with (kb, ss).
  unsigned vadr[8];
  {
    const int G = lane >> 4, gi = lane & 15, qq = gi >> 2, pp = gi & 3;
    const int r0 = 4 * (G >> 1) + qq;
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      const int c = 4 * db + 2 * (G & 1) + (pp >> 1);
      const int boff = 8 * (pp & 1);
      vadr[2 * db] = smem0 + TILE + r0 * 256 + 16 * (c ^ f128(r0)) + boff;
      vadr[2 * db + 1] = smem0 + TILE + (r0 + 8) * 256 + 16 * (c ^ f128(r0 + 8)) + boff;
    }
  }

  // kadr / vadr point into the buffer of the tile being computed: toggled (xor BUF) after every tile
  // (one body for both buffers: a body per buffer made hipcc move the 64 O registers at the join)
  auto compute = [&](const int k0) DAB_ALWAYS_INLINE {
    constexpr int B0 = 0;
    // ---- S^T = K Q^T: K fragments in two batches of 8 reads
    f32x16 s0, s1;
#pragma unroll
    for (int r = 0; r < 16; ++r) s0[r] = s1[r] = 0.f;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      bf16x8 ka[4], kb2[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const auto* kp = (const __attribute__((address_space(3))) bf16x8*)(uintptr_t)(kadr[4 * half + i] + B0);
        ka[i] = kp[0];
        kb2[i] = kp[8192 / 16];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        s0 = mfma32(ka[i], qf[4 * half + i], s0);
        s1 = mfma32(kb2[i], qf[4 * half + i], s1);
      }
    }
    if constexpr (SGB) {  // masks: MFMA 0x8, DS_READ 0x100
      __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
      for (int i = 0; i < 12; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x8, 4, 0);
    }
    // ---- online softmax on the raw scores (scale folded into the exponent's FMA): lane (q, hi)
    // holds keys k0 + crow(r, hi) (s0) and + 32 (s1)
    const bool need_mask = k0 + KT > kv_len || (CAUSAL && k0 + KT - 1 > kv_len - seqlen_q + q0);
    if (need_mask) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = k0 + (r & 3) + 8 * (r >> 2) + 4 * hi;
        if (key >= kv_len || (CAUSAL && key > q_pos)) s0[r] = kNegInf;
        if (key + 32 >= kv_len || (CAUSAL && key + 32 > q_pos)) s1[r] = kNegInf;
      }
    }
    // VPIPE: the first k-step's V fragments are requested now and land under the softmax
    u32x2 trA[8], trB[8];
    if constexpr (VPIPE) ds_tr16_issue<B0>(vadr, trA);
    float mx = kNegInf;
#pragma unroll
    for (int r = 0; r < 16; ++r) mx = fmaxf(mx, fmaxf(s0[r], s1[r]));
    mx = fmaxf(mx, VPIPE ? xor32(mx) : __shfl_xor(mx, 32, 64));
    // Deferred rescale (cdna_hip_programming.md T13): while no query of the wave sees its maximum
    // grow by more than kDeferLog2 (log2 units) the running maximum stays, P reaches at most
    // 2^kDeferLog2 (exact in bf16 up to the usual 8-bit mantissa) and the O / l rescale is skipped;
    // the decision is taken before this tile's P is exponentiated, so nothing is scaled twice.
    const float mxs = mx * sc;
    const bool keep = __all(mxs - m_run <= kDeferLog2);
    const float m_new = keep ? m_run : fmaxf(m_run, mxs);
    // raw v_exp_f32 (exp2f adds a denormal-range fix-up around each one; results below 2^-126 are
    // irrelevant next to the row maximum's 1)
    const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
    // exponentials of k-step ks (registers 8 ss .. 8 ss + 7 of S block kb)
    float ls_sms = 0.f;  // SMS: the row sum, slice by slice
    auto exp_slice = [&](const int ks) DAB_ALWAYS_INLINE {
      f32x16& sv = (ks >> 1) ? s1 : s0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sv[8 * (ks & 1) + j] = __builtin_amdgcn_exp2f(fmaf(sv[8 * (ks & 1) + j], sc, -m_new));
        ls_sms += sv[8 * (ks & 1) + j];
      }
    };
    if constexpr (!(SMS && VPIPE)) {
      float ls = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        s0[r] = __builtin_amdgcn_exp2f(fmaf(s0[r], sc, -m_new));
        s1[r] = __builtin_amdgcn_exp2f(fmaf(s1[r], sc, -m_new));
        ls += s0[r] + s1[r];
      }
      l_run = l_run * alpha + ls;
      m_run = m_new;
    } else {
      exp_slice(0);  // the rest go out one k-step ahead inside the PV loop
    }
    if (!keep && __any(alpha < 1.f)) {  // the running max moved for some query of the wave
#pragma unroll
      for (int db = 0; db < 4; ++db) o[db] *= alpha;
    }
    // ---- O^T += V^T P^T.  P^T needs no lane movement (cdna_hip_programming.md section 3, "an
    // accumulator tile as the next MFMA's operand"): registers 8 ss .. 8 ss + 7 of S block kb,
    // packed to bf16, are the B fragment of k-step (kb, ss), element j of lane half hi holding key
    // 32 kb + 16 ss + 8 (j >> 2) + 4 hi + (j & 3); the V^T A fragment takes its elements from the
    // same keys: two transposed reads of 4 keys at 32 kb + 16 ss + 4 hi (+ 8).
    static_for<0, 4>([&](auto KS_) DAB_ALWAYS_INLINE {
      constexpr int ks = decltype(KS_)::value;
      constexpr int kb = ks >> 1, ss = ks & 1;
      const f32x16& sv = kb ? s1 : s0;
      u32x4 pu;
#pragma unroll
      for (int e = 0; e < 4; ++e) pu[e] = pack2bf(sv[8 * ss + 2 * e], sv[8 * ss + 2 * e + 1]);
      const bf16x8 pf = __builtin_bit_cast(bf16x8, pu);
      u32x2 tr[8];
      if constexpr (VPIPE) {
        // k-step ks + 1's reads go out behind k-step ks's, then ks's are retired (in-order counter)
        u32x2(&cur)[8] = (ks & 1) ? trB : trA;
        u32x2(&nxt)[8] = (ks & 1) ? trA : trB;
        if constexpr (ks < 3) {
          ds_tr16_issue<B0 + ((ks + 1) >> 1) * 8192 + ((ks + 1) & 1) * 4096>(vadr, nxt);
          lgkm_wait<8>();
        } else {
          lgkm_wait<0>();
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) tr[i] = cur[i];
      } else {
        ds_tr16_x8<B0 + kb * 8192 + ss * 4096>(vadr, tr);
      }
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        u32x4 u;
        u[0] = tr[2 * db][0];
        u[1] = tr[2 * db][1];
        u[2] = tr[2 * db + 1][0];
        u[3] = tr[2 * db + 1][1];
        o[db] = mfma32(__builtin_bit_cast(bf16x8, u), pf, o[db]);
      }
      if constexpr (SMS && VPIPE && ks < 3) exp_slice(ks + 1);  // beside this k-step's MFMAs
      return true;
    });
    if constexpr (SMS && VPIPE) {
      l_run = l_run * alpha + ls_sms;  // (summed in slice order: l differs from the unsplit form in
      m_run = m_new;                    // its last fp32 bits, the output by at most a bf16 rounding)
    }
  };

  // ---- epilogue: O[q][d], d = 32 db + (r & 3) + 8 (r >> 2) + 4 hi
  auto epilogue = [&]() DAB_ALWAYS_INLINE {
    const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
    if (q_valid) {
      const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
      bf16* orow = p.out + (size_t)(q_start + my_q) * p.o_stride_tok + (size_t)h * p.o_stride_head;
#pragma unroll
      for (int db = 0; db < 4; ++db)
#pragma unroll
        for (int rg = 0; rg < 4; ++rg) {
          u32x2 v;
          v[0] = pack2bf(o[db][4 * rg] * inv, o[db][4 * rg + 1] * inv);
          v[1] = pack2bf(o[db][4 * rg + 2] * inv, o[db][4 * rg + 3] * inv);
          *reinterpret_cast<u32x2*>(orow + 32 * db + 8 * rg + 4 * hi) = v;
        }
    }
  };

  // STAG group 1: the two halves of compute() on their own.  ssm: S^T, mask, online softmax (O / l
  // rescaled here), P packed to the 4 bf16 B fragments of the PV k-steps.  pv: O^T += V^T P^T from the
  // tile buffer whose V addresses are va.
  auto ssm = [&](const int k0, bf16x8 (&pf)[4]) DAB_ALWAYS_INLINE {
    f32x16 s0, s1;
#pragma unroll
    for (int r = 0; r < 16; ++r) s0[r] = s1[r] = 0.f;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      bf16x8 ka[4], kb2[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const auto* kp = (const __attribute__((address_space(3))) bf16x8*)(uintptr_t)(kadr[4 * half + i]);
        ka[i] = kp[0];
        kb2[i] = kp[8192 / 16];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        s0 = mfma32(ka[i], qf[4 * half + i], s0);
        s1 = mfma32(kb2[i], qf[4 * half + i], s1);
      }
    }
    const bool need_mask = k0 + KT > kv_len || (CAUSAL && k0 + KT - 1 > kv_len - seqlen_q + q0);
    if (need_mask) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = k0 + (r & 3) + 8 * (r >> 2) + 4 * hi;
        if (key >= kv_len || (CAUSAL && key > q_pos)) s0[r] = kNegInf;
        if (key + 32 >= kv_len || (CAUSAL && key + 32 > q_pos)) s1[r] = kNegInf;
      }
    }
    float mx = kNegInf;
#pragma unroll
    for (int r = 0; r < 16; ++r) mx = fmaxf(mx, fmaxf(s0[r], s1[r]));
    mx = fmaxf(mx, xor32(mx));
    const float mxs = mx * sc;
    const bool keep = __all(mxs - m_run <= kDeferLog2);
    const float m_new = keep ? m_run : fmaxf(m_run, mxs);
    const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
    float ls = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      s0[r] = __builtin_amdgcn_exp2f(fmaf(s0[r], sc, -m_new));
      s1[r] = __builtin_amdgcn_exp2f(fmaf(s1[r], sc, -m_new));
      ls += s0[r] + s1[r];
    }
    l_run = l_run * alpha + ls;
    m_run = m_new;
    if (!keep && __any(alpha < 1.f)) {
#pragma unroll
      for (int db = 0; db < 4; ++db) o[db] *= alpha;
    }
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const f32x16& sv = (ks >> 1) ? s1 : s0;
      const int ss = ks & 1;
      u32x4 pu;
#pragma unroll
      for (int e = 0; e < 4; ++e) pu[e] = pack2bf(sv[8 * ss + 2 * e], sv[8 * ss + 2 * e + 1]);
      pf[ks] = __builtin_bit_cast(bf16x8, pu);
    }
  };
  auto pv = [&](const int delta, const bf16x8 (&pf)[4]) DAB_ALWAYS_INLINE {
    unsigned va[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) va[i] = vadr[i] + delta;
    static_for<0, 4>([&](auto KS_) DAB_ALWAYS_INLINE {
      constexpr int ks = decltype(KS_)::value;
      u32x2 tr[8];
      ds_tr16_x8<(ks >> 1) * 8192 + (ks & 1) * 4096>(va, tr);
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        u32x4 u;
        u[0] = tr[2 * db][0];
        u[1] = tr[2 * db][1];
        u[2] = tr[2 * db + 1][0];
        u[3] = tr[2 * db + 1][1];
        o[db] = mfma32(__builtin_bit_cast(bf16x8, u), pf[ks], o[db]);
      }
      return true;
    });
  };

  // One tile in flight: tile t + 1 is requested once tile t has landed and streams in under tile
  // t's math.
  // the cos/sin loads go out after the block-table loads and before the first DMA, so the waits
  // for them neither drain the DMA nor wait behind it
  auto load_cs = [&]() DAB_ALWAYS_INLINE {
#pragma unroll
    for (int st = 0; st < 4; ++st)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        c4[st][e] = __builtin_bit_cast(
            float4, __builtin_amdgcn_raw_buffer_load_b128(cs_rs, cs_row * 512 + ((16 * st + 8 * hi) / 2 + e) * 16, 0, 0));
  };
  load_cs();
  if (n_tiles > 0) issue(0, 0, blk_of(0));
  // PAIR: the next block's Q is loaded one block ahead into qfB (raw; RoPE is applied when it
  // becomes the current block's, at the seam).  Loading qf itself at the seam made hipcc wait for the
  // in-flight DMA before every step's MFMAs.
  bf16x8 qfB[8];
  auto load_qB = [&](const int qbn) DAB_ALWAYS_INLINE {
    const int myB = qbn * QB + 32 * w + lq;
    const bool vB = myB < seqlen_q;
    const bf16* qrow = p.q + (size_t)(q_start + (vB ? myB : 0)) * p.q_stride_tok + (size_t)h * p.q_stride_head;
#pragma unroll
    for (int st = 0; st < 8; ++st) {
      const bf16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
      qfB[st] = vB ? *reinterpret_cast<const bf16x8*>(qrow + 16 * st + 8 * hi) : z;
    }
  };
  if constexpr (PAIR) {
    if (next_blk(0) >= 0) load_qB(blk_qb(next_blk(0)));
  }
  if constexpr (NBUF >= 3) {
    if (n_tiles > 1) issue(1, 1, blk_of(1));
  }
  apply_rope();
  if constexpr (NBUF >= 3) {
    const bool g1 = STAG && w >= 4;  // wave-uniform
    bf16x8 pp[4];                    // STAG group 1: P of the pending tile (in the previous buffer)
    bool pend = false;
    for (int t = 0; t < n_tiles; ++t) {
      // this wave's pieces of tile t (tile t + 1's 2 PPW stay in flight), then every wave's -- and
      // every wave is past its reads of tile t - 2 (t - 1 without STAG), whose buffer takes tile t + 2
      if (t + 1 < n_tiles) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(2 * PPW) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (t + 2 < n_tiles) {
        const int nb = (t + 2) % NBUF;
        issue(t + 2, nb, blk_of(t + 2));
      }
      const int k0 = t * KT;
      if constexpr (STAG) {
        if (g1) {
          if (pend) pv(t % NBUF == 0 ? (NBUF - 1) * BUF : -BUF, pp);  // tile t - 1's buffer
          pend = w_any && k0 <= w_kmax;
          if (pend) ssm(k0, pp);
        } else if (w_any && k0 <= w_kmax) {
          compute(k0);
        }
      } else {
        if (w_any && k0 <= w_kmax) compute(k0);
      }
      const int adv = (t % NBUF == NBUF - 1) ? -(NBUF - 1) * BUF : BUF;  // next tile's buffer
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        kadr[i] += adv;
        vadr[i] += adv;
      }
    }
    if constexpr (STAG) {
      if (pend) pv(n_tiles % NBUF == 0 ? (NBUF - 1) * BUF : -BUF, pp);  // the last tile's buffer
    }
  } else {
    // PAIR: the steps walk the tiles of the workgroup's blocks one after the other (tile t of block
    // j); the DMA of the next step's tile, the next block's tile 0 at a seam, always goes out under
    // the current step's MFMAs
    int j = 0, t = 0, nt = n_tiles;
    int jn = PAIR ? next_blk(0) : -1;
    int ntn = jn >= 0 ? tiles_of(blk_qb(jn) * QB) : 0;
    for (int s = 0; nt > 0; ++s) {
      const int buf = s & 1;
      if constexpr (ONEBAR) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pieces of tile t
        __builtin_amdgcn_s_barrier();  // every wave's pieces of t; every wave past step s - 1
        if (t + 1 < nt || jn >= 0) {
          const int tn = t + 1 < nt ? t + 1 : 0;
          issue(tn, buf ^ 1, blk_of(tn));
        }
      } else {
        if (t + 1 < nt || jn >= 0) {
          const int tn = t + 1 < nt ? t + 1 : 0;
          __builtin_amdgcn_s_barrier();  // every wave is done reading buffer (s + 1) & 1 (step s - 1)
          const int blk = blk_of(tn);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pieces of tile t
          issue(tn, buf ^ 1, blk);
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_s_barrier();  // ... and every other wave's pieces of tile t
      }
      const int k0 = t * KT;
      if (w_any && k0 <= w_kmax) compute(k0);  // else this wave's queries see no key of the tile
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        kadr[i] ^= BUF;
        vadr[i] ^= BUF;
      }
      if (t + 1 < nt) {
        ++t;
        continue;
      }
      if (!PAIR || jn < 0) break;
      // seam: the block's rows out, the next block's state in
      epilogue();
      set_block(blk_qb(jn) * QB);
#pragma unroll
      for (int db = 0; db < 4; ++db)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[db][r] = 0.f;
      m_run = -1e30f;
      l_run = 0.f;
#pragma unroll
      for (int st = 0; st < 8; ++st) qf[st] = qfB[st];
      rope_q = p.rope_cs && q_valid;
      if (rope_q) {
        // RoPE of the new block's Q, one cos / sin row group at a time (16 registers, not the
        // prologue's 64); its loads are waited here, next to the next tile's DMA wait
        cs_row = p.rope_pos[q_start + my_q];
#pragma unroll
        for (int st = 0; st < 4; ++st) {
          float4 cr[4];
#pragma unroll
          for (int e = 0; e < 4; ++e)
            cr[e] = __builtin_bit_cast(
                float4, __builtin_amdgcn_raw_buffer_load_b128(cs_rs, cs_row * 512 + ((16 * st + 8 * hi) / 2 + e) * 16, 0, 0));
#pragma unroll
          for (int jj = 0; jj < 8; ++jj) {
            const float4 cc = cr[jj >> 1];
            const float2 cs = (jj & 1) ? make_float2(cc.z, cc.w) : make_float2(cc.x, cc.y);
            float x1 = bf2f((uint16_t)qf[st][jj]), x2 = bf2f((uint16_t)qf[st + 4][jj]);
            rope_rot(x1, x2, cs);
            qf[st][jj] = (short)f2bf(x1);
            qf[st + 4][jj] = (short)f2bf(x2);
          }
        }
      }
      j = jn;
      t = 0;
      nt = ntn;
      jn = next_blk(j);
      ntn = jn >= 0 ? tiles_of(blk_qb(jn) * QB) : 0;
      if (jn >= 0) load_qB(blk_qb(jn));
    }
  }
  epilogue();
}

// -----------------------------------------------------------------------------------------------
// Prefill attention with 64 queries per wave (Q64; A/B arm DAB_FLASH_Q64=1).  The 32-query kernel
// above reads each wave's whole K / V tile from LDS for 32 queries: 8 waves per CU x 32 KB per tile
// is as many LDS cycles (128 B / clk) as the tile's MFMA cycles, so LDS bandwidth and the matrix
// cores bind together (MFMA busy ~40 % on long sequences).  Here each wave owns two 32-query halves
// u = 0 / 1 and feeds every K / V fragment it reads to both: half the LDS bytes per FLOP.  The cost
// is registers -- O 128, Q 64, S 64 -- so one wave per SIMD (4 waves, 256 queries per workgroup, one
// workgroup per CU) with the whole 512-entry register file, and a 3-deep K / V ring (96 KB): tile
// t + 2 is requested after tile t's barrier, each wave waits only for its own pieces of tile t.
// Causal blocks are taken heavy-first.  Same math per query as flash_d128_kernel (bit-identical).
template <bool CAUSAL>
__global__ __launch_bounds__(256, 1) void flash_q64_kernel(FlashParams p) {
  constexpr int D = 128, KT = 64, QB = 256;
  constexpr int TILE = KT * D * 2;  // 16 KB
  constexpr int BUF = 2 * TILE;     // K | V
  constexpr int NBUF = 3;
  constexpr int PPW = 4;            // 1-KB K (and V) pieces per wave per tile
  __shared__ __attribute__((aligned(16))) char smem[NBUF * BUF];

  const int nqb = gridDim.x;
  const int nwg = nqb * gridDim.y * gridDim.z;
  const int lin = blockIdx.x + nqb * (blockIdx.y + gridDim.y * blockIdx.z);
  const int xcd = lin % 8, q8 = nwg / 8, r8 = nwg % 8;
  const int sid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + lin / 8;
  const int h = (sid / nqb) % gridDim.y;
  const int b = sid / (nqb * gridDim.y);
  const int* bt = p.block_tables + (size_t)b * p.max_blocks;
  const int tpb = p.block_size / KT;
  const int bl = (int)(threadIdx.x & 63);
  const int bt_a = bl / tpb < p.max_blocks ? bt[bl / tpb] : 0;
  const int bt_b = (64 + bl) / tpb < p.max_blocks ? bt[(64 + bl) / tpb] : 0;
  const int q_start = p.cu_q[b];
  const int seqlen_q = p.cu_q[b + 1] - q_start;
  const int nqb_b = div_up(seqlen_q, QB);
  const int qb = CAUSAL && sid % nqb < nqb_b ? nqb_b - 1 - sid % nqb : sid % nqb;
  const int q0 = qb * QB;
  if (q0 >= seqlen_q) return;  // whole workgroup
  const int kv_len = p.ctx_k[b];
  const int hk = h / (p.Hq / p.Hkv);
  const int tid = threadIdx.x, lane = tid & 63, lq = lane & 31, hi = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  int my_q[2], q_pos[2];
  bool q_valid[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    my_q[u] = q0 + 64 * w + 32 * u + lq;
    q_valid[u] = my_q[u] < seqlen_q;
    q_pos[u] = kv_len - seqlen_q + my_q[u];
  }
  const int w_last_q = min(q0 + 64 * w + 63, seqlen_q - 1);
  const int w_kmax = CAUSAL ? kv_len - seqlen_q + w_last_q : kv_len - 1;
  const bool w_any = q0 + 64 * w < seqlen_q;

  bf16x8 qf[2][8];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const bf16* qrow =
        p.q + (size_t)(q_start + (q_valid[u] ? my_q[u] : 0)) * p.q_stride_tok + (size_t)h * p.q_stride_head;
#pragma unroll
    for (int st = 0; st < 8; ++st) {
      const bf16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
      qf[u][st] = q_valid[u] ? *reinterpret_cast<const bf16x8*>(qrow + 16 * st + 8 * hi) : z;
    }
  }
  if (p.rope_cs) {  // RoPE of Q on load, one cos / sin row group at a time
    const auto cs_rs = __builtin_amdgcn_make_buffer_rsrc((void*)p.rope_cs, (short)0, 0x7ffffff0, 0x00020000);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (!q_valid[u]) continue;
      const int row = p.rope_pos[q_start + my_q[u]];
#pragma unroll
      for (int st = 0; st < 4; ++st) {
        float4 cr[4];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          cr[e] = __builtin_bit_cast(
              float4, __builtin_amdgcn_raw_buffer_load_b128(cs_rs, row * 512 + ((16 * st + 8 * hi) / 2 + e) * 16, 0, 0));
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float4 cc = cr[j >> 1];
          const float2 cs = (j & 1) ? make_float2(cc.z, cc.w) : make_float2(cc.x, cc.y);
          float x1 = bf2f((uint16_t)qf[u][st][j]), x2 = bf2f((uint16_t)qf[u][st + 4][j]);
          rope_rot(x1, x2, cs);
          qf[u][st][j] = (short)f2bf(x1);
          qf[u][st + 4][j] = (short)f2bf(x2);
        }
      }
    }
  }

  int n_keys = kv_len;
  if (CAUSAL) {
    const int last_q = min(q0 + QB - 1, seqlen_q - 1);
    n_keys = min(kv_len, kv_len - seqlen_q + last_q + 1);
  }
  const int n_tiles = div_up(n_keys, KT);

  const int st_row = lane >> 4, st_pc = lane & 15;
  auto blk_of = [&](int t) {
    if (t < 64) return __builtin_amdgcn_readlane(bt_a, t);
    if (t < 128) return __builtin_amdgcn_readlane(bt_b, t - 64);
    return __builtin_amdgcn_readfirstlane(((volatile const int*)bt)[t / tpb]);
  };
  auto issue = [&](int t, int buf, int blk) {
    const int k0 = t * KT;
    const int nvalid = min(KT, kv_len - k0);
    const size_t base = (((size_t)blk * p.Hkv + hk) * p.block_size + (k0 % p.block_size)) * D;
    const auto rk = __builtin_amdgcn_make_buffer_rsrc((void*)(p.k_cache + base), (short)0, nvalid * D * 2, 0x00020000);
    const auto rv = __builtin_amdgcn_make_buffer_rsrc((void*)(p.v_cache + base), (short)0, nvalid * D * 2, 0x00020000);
    char* kdst = smem + buf * BUF;
#pragma unroll
    for (int j = 0; j < PPW; ++j) {
      const int i = PPW * w + j;
      const int row = 4 * i + st_row;
      const unsigned off = (unsigned)(row * D + 8 * (st_pc ^ f128(row))) * 2u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rk, (__attribute__((address_space(3))) void*)(kdst + i * 1024), 16, off,
                                               0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rv, (__attribute__((address_space(3))) void*)(kdst + TILE + i * 1024),
                                               16, off, 0, 0, 0);
    }
  };

  f32x16 o[2][4];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
      for (int r = 0; r < 16; ++r) o[u][db][r] = 0.f;
  float m_run[2] = {-1e30f, -1e30f}, l_run[2] = {0.f, 0.f};
  const float sc = p.scale_log2;

  const unsigned smem0 = lds_addr(smem);
  unsigned kadr[8];
  {
    const int fr = f128(lq);
#pragma unroll
    for (int st = 0; st < 8; ++st) kadr[st] = smem0 + lq * 256 + 16 * ((2 * st + hi) ^ fr);
  }
  unsigned vadr[8];
  {
    const int G = lane >> 4, gi = lane & 15, qq = gi >> 2, pp = gi & 3;
    const int r0 = 4 * (G >> 1) + qq;
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      const int c = 4 * db + 2 * (G & 1) + (pp >> 1);
      const int boff = 8 * (pp & 1);
      vadr[2 * db] = smem0 + TILE + r0 * 256 + 16 * (c ^ f128(r0)) + boff;
      vadr[2 * db + 1] = smem0 + TILE + (r0 + 8) * 256 + 16 * (c ^ f128(r0 + 8)) + boff;
    }
  }

  auto compute = [&](const int k0) DAB_ALWAYS_INLINE {
    // ---- S^T = K Q^T for both halves: each K fragment feeds two MFMAs
    f32x16 s0[2], s1[2];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) s0[u][r] = s1[u][r] = 0.f;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      bf16x8 ka[4], kb2[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const auto* kp = (const __attribute__((address_space(3))) bf16x8*)(uintptr_t)(kadr[4 * half + i]);
        ka[i] = kp[0];
        kb2[i] = kp[8192 / 16];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          s0[u] = mfma32(ka[i], qf[u][4 * half + i], s0[u]);
          s1[u] = mfma32(kb2[i], qf[u][4 * half + i], s1[u]);
        }
    }
    const bool need_mask = k0 + KT > kv_len || (CAUSAL && k0 + KT - 1 > kv_len - seqlen_q + q0);
    bf16x8 pf[2][4];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (need_mask) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = k0 + (r & 3) + 8 * (r >> 2) + 4 * hi;
          if (key >= kv_len || (CAUSAL && key > q_pos[u])) s0[u][r] = kNegInf;
          if (key + 32 >= kv_len || (CAUSAL && key + 32 > q_pos[u])) s1[u][r] = kNegInf;
        }
      }
      float mx = kNegInf;
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, fmaxf(s0[u][r], s1[u][r]));
      mx = fmaxf(mx, xor32(mx));
      const float mxs = mx * sc;
      const bool keep = __all(mxs - m_run[u] <= kDeferLog2);
      const float m_new = keep ? m_run[u] : fmaxf(m_run[u], mxs);
      const float alpha = __builtin_amdgcn_exp2f(m_run[u] - m_new);
      float ls = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        s0[u][r] = __builtin_amdgcn_exp2f(fmaf(s0[u][r], sc, -m_new));
        s1[u][r] = __builtin_amdgcn_exp2f(fmaf(s1[u][r], sc, -m_new));
        ls += s0[u][r] + s1[u][r];
      }
      l_run[u] = l_run[u] * alpha + ls;
      m_run[u] = m_new;
      if (!keep && __any(alpha < 1.f)) {
#pragma unroll
        for (int db = 0; db < 4; ++db) o[u][db] *= alpha;
      }
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const f32x16& sv = (ks >> 1) ? s1[u] : s0[u];
        const int ss = ks & 1;
        u32x4 pu;
#pragma unroll
        for (int e = 0; e < 4; ++e) pu[e] = pack2bf(sv[8 * ss + 2 * e], sv[8 * ss + 2 * e + 1]);
        pf[u][ks] = __builtin_bit_cast(bf16x8, pu);
      }
    }
    // ---- O^T += V^T P^T for both halves: each transposed V fragment feeds two MFMAs
    static_for<0, 4>([&](auto KS_) DAB_ALWAYS_INLINE {
      constexpr int ks = decltype(KS_)::value;
      u32x2 tr[8];
      ds_tr16_x8<(ks >> 1) * 8192 + (ks & 1) * 4096>(vadr, tr);
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        u32x4 uu;
        uu[0] = tr[2 * db][0];
        uu[1] = tr[2 * db][1];
        uu[2] = tr[2 * db + 1][0];
        uu[3] = tr[2 * db + 1][1];
        const bf16x8 va = __builtin_bit_cast(bf16x8, uu);
#pragma unroll
        for (int u = 0; u < 2; ++u) o[u][db] = mfma32(va, pf[u][ks], o[u][db]);
      }
      return true;
    });
  };

  if (n_tiles > 0) issue(0, 0, blk_of(0));
  if (n_tiles > 1) issue(1, 1, blk_of(1));
  // Q is consumed here, behind the first two tiles' DMA (a counted wait hipcc computes in this
  // straight-line prologue): with its first use inside the loop, hipcc put a vmcnt(0) there that
  // drained the in-flight tile on every step
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int st = 0; st < 8; ++st) asm volatile("" ::"v"(qf[u][st]));
  for (int t = 0; t < n_tiles; ++t) {
    if (t + 1 < n_tiles) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(2 * PPW) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (t + 2 < n_tiles) issue(t + 2, (t + 2) % NBUF, blk_of(t + 2));
    const int k0 = t * KT;
    if (w_any && k0 <= w_kmax) compute(k0);
    const int adv = (t % NBUF == NBUF - 1) ? -(NBUF - 1) * BUF : BUF;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      kadr[i] += adv;
      vadr[i] += adv;
    }
  }

#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const float l_tot = l_run[u] + __shfl_xor(l_run[u], 32, 64);
    if (!q_valid[u]) continue;
    const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
    bf16* orow = p.out + (size_t)(q_start + my_q[u]) * p.o_stride_tok + (size_t)h * p.o_stride_head;
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {
        u32x2 v;
        v[0] = pack2bf(o[u][db][4 * rg] * inv, o[u][db][4 * rg + 1] * inv);
        v[1] = pack2bf(o[u][db][4 * rg + 2] * inv, o[u][db][4 * rg + 3] * inv);
        *reinterpret_cast<u32x2*>(orow + 32 * db + 8 * rg + 4 * hi) = v;
      }
  }
}

// -----------------------------------------------------------------------------------------------
// Persistent encoder attention (ENC_P; A/B arm DAB_ENC_PERSIST=1): D 64, packed varlen,
// bidirectional, the embed path's ~50-token chunks.  flash_fwd_kernel runs one workgroup per
// (query block, head, sequence): at ~50 tokens that is a single tile, and each workgroup's life is one
// dependent chain (sequence bounds -> Q / K / V loads -> LDS -> MFMAs -> stores) with nothing to
// overlap it.  Here a workgroup walks (sequence, head) items with a grid stride, and the next step's
// K / V tile and Q (the next item's, at an item seam) are loaded into registers while the current
// step computes, so the load round trip hides under the previous item's math and stores.
// Same per-query math as flash_fwd_kernel<64, false, false, 4, 1> (bit-identical).
__global__ __launch_bounds__(256, 5) void flash_enc_kernel(FlashParams p, int n_items) {
  constexpr int D = 64, KT = 64, NT = 256, QB = 64;
  constexpr int NKK = D / 32, NTD = D / 16, CPR = D / 8;
  constexpr int TILE_BYTES = KT * D * 2;
  constexpr int CH = KT * CPR / NT;
  __shared__ __attribute__((aligned(16))) char smem[2 * TILE_BYTES];
  char* ks = smem;
  char* vs = smem + TILE_BYTES;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, g = lane >> 4, li = lane & 15;
  const int H = p.Hq;

  // the item / step being computed (c_*) and the one being loaded (n_*)
  struct Step {
    int it, qb, kt;
    int b, h, q_start, seqlen_q, k_start, kv_len, nqb, nkt;
  };
  auto item_of = [&](Step& s, const int it) DAB_ALWAYS_INLINE {
    s.it = it;
    s.b = it / H;
    s.h = it - s.b * H;
    s.q_start = p.cu_q[s.b];
    s.seqlen_q = p.cu_q[s.b + 1] - s.q_start;
    s.k_start = p.cu_k[s.b];
    s.kv_len = p.cu_k[s.b + 1] - s.k_start;
    s.nqb = div_up(s.seqlen_q, QB);
    s.nkt = div_up(s.kv_len, KT);
    s.qb = 0;
    s.kt = 0;
  };
  u32x4 kreg[CH], vreg[CH];
  auto load_tile = [&](const Step& s) DAB_ALWAYS_INLINE {
    const int k0 = s.kt * KT;
    const int last = s.kv_len - 1 - k0;
    const int hk = s.h / (p.Hq / p.Hkv);
    const size_t base = (size_t)(s.k_start + k0) * p.kv_stride_tok + (size_t)hk * p.kv_stride_head;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int idx = tid + c * NT;
      const int row = min(idx / CPR, last), ch = idx % CPR;
      const size_t off = base + (size_t)row * p.kv_stride_tok + ch * 8;
      kreg[c] = *reinterpret_cast<const u32x4*>(p.k + off);
      vreg[c] = *reinterpret_cast<const u32x4*>(p.v + off);
    }
  };
  auto store_tile = [&]() DAB_ALWAYS_INLINE {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int idx = tid + c * NT;
      const int row = idx / CPR, ch = idx % CPR;
      *reinterpret_cast<u32x4*>(ks + swz<D>(row, ch)) = kreg[c];
      *reinterpret_cast<u32x4*>(vs + swz<D>(row, ch)) = vreg[c];
    }
  };
  bf16x8 qf[NKK], qn[NKK];
  auto load_q = [&](const Step& s, bf16x8 (&dst)[NKK]) DAB_ALWAYS_INLINE {
    const int mq = s.qb * QB + 16 * w + li;
    const bool v = mq < s.seqlen_q;
    const bf16* qrow = p.q + (size_t)(s.q_start + (v ? mq : 0)) * p.q_stride_tok + (size_t)s.h * p.q_stride_head;
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk) {
      const bf16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
      dst[kk] = v ? *reinterpret_cast<const bf16x8*>(qrow + 32 * kk + 8 * g) : z;
    }
  };
  // the step after s (same item: next tile / next query block; else the next item), or it = -1
  auto advance = [&](Step& s) DAB_ALWAYS_INLINE {
    if (s.kt + 1 < s.nkt) {
      ++s.kt;
    } else if (s.qb + 1 < s.nqb) {
      ++s.qb;
      s.kt = 0;
    } else {
      const int nit = s.it + (int)gridDim.x;
      if (nit < n_items) item_of(s, nit);
      else s.it = -1;
    }
  };

  if ((int)blockIdx.x >= n_items) return;
  Step c;
  item_of(c, blockIdx.x);
  load_q(c, qf);
  load_tile(c);
  f32x4 o[NTD];
#pragma unroll
  for (int t = 0; t < NTD; ++t) o[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run = -1e30f, l_run = 0.f;
  for (;;) {
    __syncthreads();  // every wave is past the previous step's LDS reads
    store_tile();
    __syncthreads();
    Step n = c;
    advance(n);
    const bool new_q = n.it >= 0 && n.kt == 0;  // the next step starts a query block
    if (n.it >= 0) load_tile(n);
    if (new_q) load_q(n, qn);
    // ---- compute tile c.kt of query block c.qb (flash_fwd_kernel's math, QT = 1)
    {
      const int kt = c.kt;
      const int my_q = c.qb * QB + 16 * w + li;
      f32x4 s[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        s[m] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < NKK; ++kk) {
          const bf16x8 a = *reinterpret_cast<const bf16x8*>(ks + swz<D>(16 * m + li, 4 * kk + g));
          s[m] = mfma16(a, qf[kk], s[m]);
        }
      }
      const bool need_mask = (kt + 1) * KT > c.kv_len;
      float mx = kNegInf;
#pragma unroll
      for (int m = 0; m < 4; ++m) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = s[m][r] * p.scale_log2;
          if (need_mask && kt * KT + 16 * m + 4 * g + r >= c.kv_len) v = kNegInf;
          s[m][r] = v;
          mx = fmaxf(mx, v);
        }
      }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const bool keep = __all(mx - m_run <= kDeferLog2);
      const float m_new = keep ? m_run : fmaxf(m_run, mx);
      const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
      float ls = 0.f;
#pragma unroll
      for (int m = 0; m < 4; ++m) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = __builtin_amdgcn_exp2f(s[m][r] - m_new);
          s[m][r] = e;
          ls += e;
        }
      }
      l_run = l_run * alpha + ls;
      m_run = m_new;
      bf16x8 pb[2];
#pragma unroll
      for (int ss = 0; ss < 2; ++ss)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pb[ss][j] = (short)f2bf(s[2 * ss][j]);
          pb[ss][j + 4] = (short)f2bf(s[2 * ss + 1][j]);
        }
      if (!keep) {
#pragma unroll
        for (int t = 0; t < NTD; ++t) o[t] *= alpha;
      }
      const int qq = li >> 2, pp = li & 3;
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
#pragma unroll
        for (int t = 0; t < NTD; ++t) {
          const int ch = 2 * t + (pp >> 1);
          const int boff = 8 * (pp & 1);
          const bf16x4 lo = ds_read_tr16(vs + swz<D>(32 * ss + 4 * g + qq, ch) + boff);
          const bf16x4 hi = ds_read_tr16(vs + swz<D>(32 * ss + 16 + 4 * g + qq, ch) + boff);
          const bf16x8 a = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          o[t] = mfma16(a, pb[ss], o[t]);
        }
      }
      if (kt + 1 == c.nkt) {  // the query block is complete: its rows out, the state reset
        float l_tot = l_run;
        l_tot += __shfl_xor(l_tot, 16, 64);
        l_tot += __shfl_xor(l_tot, 32, 64);
        if (my_q < c.seqlen_q) {
          const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
          bf16* orow = p.out + (size_t)(c.q_start + my_q) * p.o_stride_tok + (size_t)c.h * p.o_stride_head;
#pragma unroll
          for (int t = 0; t < NTD; ++t) {
            u32x2 v;
            v[0] = pack2bf(o[t][0] * inv, o[t][1] * inv);
            v[1] = pack2bf(o[t][2] * inv, o[t][3] * inv);
            *reinterpret_cast<u32x2*>(orow + 16 * t + 4 * g) = v;
          }
        }
#pragma unroll
        for (int t = 0; t < NTD; ++t) o[t] = f32x4{0.f, 0.f, 0.f, 0.f};
        m_run = -1e30f;
        l_run = 0.f;
      }
    }
    if (n.it < 0) break;
    if (new_q) {
#pragma unroll
      for (int kk = 0; kk < NKK; ++kk) qf[kk] = qn[kk];
    }
    c = n;
  }
}

// -----------------------------------------------------------------------------------------------
// Paged decode.  grid = (max_parts, Hkv, B); one workgroup reduces keys [part*part_size, +part_size)
// of one (sequence, kv head) for all G = Hq/Hkv query heads of the GQA group (the MFMA N dimension,
// padded to 16).  Each wave streams 32-key sub-tiles through a private LDS slot (no block barriers in
// the loop), with the next sub-tile's global loads in flight during compute.

struct DecodeParams {
  const bf16* q;
  const bf16* k_cache;
  const bf16* v_cache;
  const int* block_tables;
  int max_blocks, block_size;
  const int* ctx_lens;
  bf16* out;
  float* part_o;
  float* part_m;
  float* part_l;
  int* counters;  // [B * Hkv] partition arrivals (zero between launches; the last arriver resets)
  const int* order;  // optional [B] sequence visit order (longest first: see paged_decode_attention)
  int Hq, Hkv, part_size, max_parts;
  float scale_log2;
  L3Warm warm;  // optional: the next projections' weights, warmed into L3 by appended workgroups
};

// DMA (D = 128): each wave streams its 32-key K / V sub-tiles straight into its LDS slot by LDS-DMA
// (buffer_load ... lds, non-temporal: MI355X_MICROARCH.md rows ldsdma-fill / nt-weights put the
// LDS-DMA stream at 6.5-6.8 TB/s chip-wide against 5.7-5.8 for register gathers) instead of through
// a register double buffer + ds_write; one slot per wave, the 8 waves of a CU's two workgroups keep
// ~128 KB in flight.  The next sub-tile's block id is fetched under the current sub-tile's DMA.
//
// NSLOT 2 (small batches, DMA): two LDS slots per wave, so sub-tile i + 1's copy is in
// flight while sub-tile i computes, and the wave's block ids are fetched once, one per lane, before
// the first copy.  At batch 1 - 8 a workgroup's waves walk their sub-tiles back to back with the
// whole GPU otherwise idle: one copy round trip per sub-tile was the critical path.  128 KB of LDS:
// one workgroup per CU, which small batches never fill anyway.
template <int D, bool KV_NT, bool DMA = false, int NSLOT = 1>
__global__ __launch_bounds__(256, NSLOT == 1 ? 2 : 1) void paged_decode_kernel(DecodeParams p, int total_items) {
  static_assert(NSLOT == 1 || (NSLOT == 2 && DMA), "two slots: DMA staging only");
  // appended workgroups (small batches leave most CUs idle during this latency-bound launch): warm
  // the following projections' weights into the Infinity Cache and leave
  const int attn_blocks = gridDim.x - p.warm.blocks;
  if ((int)blockIdx.x >= attn_blocks) {
    l3_warm(p.warm, blockIdx.x - attn_blocks);
    return;
  }
  constexpr int KT = 32;
  constexpr int NKK = D / 32;
  constexpr int NTD = D / 16;
  constexpr int CPR = D / 8;
  constexpr int SUB_BYTES = KT * D * 2;
  constexpr int CH = KT * CPR / 64;  // 16-B chunks per lane per sub-tile (K and V each)
  constexpr int RED_BYTES = 4 * 16 * D * 4 + 2 * 4 * 16 * 4;
  constexpr int STAGE_BYTES = 4 * 2 * SUB_BYTES * NSLOT;
  // one LDS array (a second __shared__ object can cost vmcnt(0) waits); the last-arriver flag
  // lives right after the reduction area
  constexpr int AREA_BYTES = STAGE_BYTES > RED_BYTES + 16 ? STAGE_BYTES : RED_BYTES + 16;
  __shared__ __attribute__((aligned(16))) char smem[AREA_BYTES];
  int* last_flag = reinterpret_cast<int*>(smem + RED_BYTES);

  const int G = p.Hq / p.Hkv;
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, li = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  char* ks = smem + w * 2 * SUB_BYTES * NSLOT;
  char* vs = ks + SUB_BYTES;

  // persistent walk over (key partition, sequence, kv head) items.  The partition is the SLOWEST
  // index so the live partitions (low part ids) form a dense prefix spread over every workgroup of
  // the grid-stride loop; with part fastest, a power-of-two max_parts pinned all live work onto the
  // few workgroups with blockIdx % max_parts == live part (measured 3-10x slower).
  const int BH = total_items / p.max_parts;
  // partitions past the longest context are empty: the walk stops there instead of visiting every
  // partition the workspace could hold (max_parts covers max_model_len at the finest partition).
  // The longest context is a wave max over ctx_lens (B <= a few hundred ints, L2-resident), so the
  // bound holds for any visit order; the longest-first order is only a load-balancing hint.
  int maxc = 0;
  for (int i = lane; i < BH / p.Hkv; i += 64) maxc = max(maxc, p.ctx_lens[i]);
#pragma unroll
  for (int off = 32; off; off >>= 1) maxc = max(maxc, __shfl_xor(maxc, off));
  maxc = __builtin_amdgcn_readfirstlane(maxc);
  const int live_items = min(p.max_parts, (maxc + p.part_size - 1) / p.part_size) * BH;
  for (int item = blockIdx.x; item < live_items; item += attn_blocks) {
    const int part = item / BH;
    const int bh = item - part * BH;
    const int hk = bh % p.Hkv, b = p.order ? p.order[bh / p.Hkv] : bh / p.Hkv;
    const int ctx = p.ctx_lens[b];
    const int k_begin = part * p.part_size;
    if (k_begin >= ctx) continue;
    const int k_end = min(ctx, k_begin + p.part_size);

    bf16x8 qf[NKK];
    {
      const bool qv = li < G;
      const bf16* qrow = p.q + ((size_t)b * p.Hq + hk * G + (qv ? li : 0)) * D;
#pragma unroll
      for (int kk = 0; kk < NKK; ++kk) {
        bf16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
        qf[kk] = qv ? *reinterpret_cast<const bf16x8*>(qrow + 32 * kk + 8 * g) : z;
      }
    }

    // Two register buffers of one 32-key sub-tile (K and V) per wave: the sub-tile two steps ahead
    // is in flight while one computes.  Buffer loads with the sub-tile's uniform base in the
    // descriptor and lane offsets lane*16 + c*1024 (no per-chunk 64-bit address registers); rows
    // past the partition end, and whole sub-tiles past it, read as zeros without memory traffic
    // (descriptor range), and are masked to -inf below.
    u32x4 kA[CH], vA[CH], kB[CH], vB[CH];
    const int k_last = ((k_end - 1) / KT) * KT;
    auto load_sub = [&](u32x4(&kr)[CH], u32x4(&vr)[CH], int k0) {
      const int kc = min(k0, k_last);
      const int blk = p.block_tables[(size_t)b * p.max_blocks + kc / p.block_size];
      const size_t base = (((size_t)blk * p.Hkv + hk) * p.block_size + (kc % p.block_size)) * D;
      const int bytes = k0 > k_last ? 0 : min(KT, k_end - k0) * D * 2;
      const auto kd = __builtin_amdgcn_make_buffer_rsrc((void*)(p.k_cache + base), 0, bytes, 0x00020000);
      const auto vd = __builtin_amdgcn_make_buffer_rsrc((void*)(p.v_cache + base), 0, bytes, 0x00020000);
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        kr[c] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(kd, lane * 16, c * 1024, KV_NT ? 2 : 0));
        vr[c] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(vd, lane * 16, c * 1024, KV_NT ? 2 : 0));
      }
    };
    auto stage = [&](const u32x4(&kr)[CH], const u32x4(&vr)[CH]) {
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        const int idx = lane + c * 64;
        const int row = idx / CPR, ch = idx % CPR;
        *reinterpret_cast<u32x4*>(ks + swz<D>(row, ch)) = kr[c];
        *reinterpret_cast<u32x4*>(vs + swz<D>(row, ch)) = vr[c];
      }
    };

    f32x4 o[NTD];
#pragma unroll
    for (int t = 0; t < NTD; ++t) o[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m_run = -1e30f, l_run = 0.f;

    auto compute = [&](const int k0) {
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes landed
      __builtin_amdgcn_wave_barrier();
      f32x4 s[2];
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        s[m] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < NKK; ++kk) {
          const bf16x8 a = *reinterpret_cast<const bf16x8*>(ks + swz<D>(16 * m + li, 4 * kk + g));
          s[m] = mfma16(a, qf[kk], s[m]);
        }
      }
      float mx = kNegInf;
#pragma unroll
      for (int m = 0; m < 2; ++m) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = k0 + 16 * m + 4 * g + r;
          float v = s[m][r] * p.scale_log2;
          if (key >= k_end) v = kNegInf;
          s[m][r] = v;
          mx = fmaxf(mx, v);
        }
      }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float m_new = fmaxf(m_run, mx);
      const float alpha = exp2f(m_run - m_new);
      float ls = 0.f;
#pragma unroll
      for (int m = 0; m < 2; ++m) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = exp2f(s[m][r] - m_new);
          s[m][r] = e;
          ls += e;
        }
      }
      l_run = l_run * alpha + ls;
      m_run = m_new;
      bf16x8 pb;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pb[j] = (short)f2bf(s[0][j]);
        pb[j + 4] = (short)f2bf(s[1][j]);
      }
      const int qq = li >> 2, pp = li & 3;
#pragma unroll
      for (int t = 0; t < NTD; ++t) {
        o[t] *= alpha;
        const int ch = 2 * t + (pp >> 1);
        const int boff = 8 * (pp & 1);
        const bf16x4 lo = ds_read_tr16(vs + swz<D>(4 * g + qq, ch) + boff);
        const bf16x4 hi = ds_read_tr16(vs + swz<D>(16 + 4 * g + qq, ch) + boff);
        const bf16x8 a = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        o[t] = mfma16(a, pb, o[t]);
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
    };
    const int kw = k_begin + w * KT;
    if constexpr (DMA) {
      static_assert(D == 128, "DMA staging assumes 256-B rows (4 rows per 1 KB piece)");
      // LDS slot (row 4 i + lane / 16, physical chunk lane % 16) of piece i holds logical chunk
      // (lane % 16) ^ (2 row & 15): the swz<128> image compute() reads
      const int drow = lane >> 4;
      auto blk_at = [&](int k0) {
        return p.block_tables[(size_t)b * p.max_blocks + min(k0, k_last) / p.block_size];
      };
      auto dma = [&](int k0, int blk) {
        const int kc = min(k0, k_last);
        const size_t base = (((size_t)blk * p.Hkv + hk) * p.block_size + (kc % p.block_size)) * D;
        const int bytes = k0 > k_last ? 0 : min(KT, k_end - k0) * D * 2;
        const auto kd = __builtin_amdgcn_make_buffer_rsrc((void*)(p.k_cache + base), 0, bytes, 0x00020000);
        const auto vd = __builtin_amdgcn_make_buffer_rsrc((void*)(p.v_cache + base), 0, bytes, 0x00020000);
#pragma unroll
        for (int i = 0; i < KT / 4; ++i) {
          const int row = 4 * i + drow;
          const unsigned off = (unsigned)(row * 256 + 16 * ((lane & 15) ^ ((2 * row) & 15)));
          __builtin_amdgcn_raw_ptr_buffer_load_lds(kd, (__attribute__((address_space(3))) void*)(ks + i * 1024), 16, off,
                                                   0, 0, KV_NT ? 2 : 0);
          __builtin_amdgcn_raw_ptr_buffer_load_lds(vd, (__attribute__((address_space(3))) void*)(vs + i * 1024), 16, off,
                                                   0, 0, KV_NT ? 2 : 0);
        }
      };
      if constexpr (NSLOT == 2) {
        char* const slot0 = smem + w * 2 * SUB_BYTES * NSLOT;
        const int n_sub = kw < k_end ? (k_end - kw + 4 * KT - 1) / (4 * KT) : 0;  // <= 64 (launcher)
        const int myblk = lane < n_sub ? blk_at(kw + lane * 4 * KT) : 0;  // lane i: sub-tile i's block
        auto issue = [&](int i) {
          ks = slot0 + (i & 1) * 2 * SUB_BYTES;
          vs = ks + SUB_BYTES;
          dma(kw + i * 4 * KT, __builtin_amdgcn_readlane(myblk, i));
        };
        if (n_sub > 0) issue(0);
        for (int i = 0; i < n_sub; ++i) {
          if (i + 1 < n_sub) {
            issue(i + 1);  // into the slot sub-tile i - 1 was read from (its MFMAs consumed it)
            asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // sub-tile i's 16 pieces landed
          } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          }
          ks = slot0 + (i & 1) * 2 * SUB_BYTES;
          vs = ks + SUB_BYTES;
          compute(kw + i * 4 * KT);
        }
      } else {
      int blk = __builtin_amdgcn_readfirstlane(blk_at(kw));
      for (int k0 = kw; k0 < k_end; k0 += 4 * KT) {
        dma(k0, blk);
        blk = blk_at(k0 + 4 * KT);  // in flight under this sub-tile's copy and math
        asm volatile("s_waitcnt vmcnt(1)" ::: "memory");  // this sub-tile's 16 pieces landed
        compute(k0);
        blk = __builtin_amdgcn_readfirstlane(blk);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    } else {
      load_sub(kA, vA, kw);
      load_sub(kB, vB, kw + 4 * KT);
      for (int k0 = kw; k0 < k_end; k0 += 8 * KT) {
        stage(kA, vA);
        load_sub(kA, vA, k0 + 8 * KT);
        compute(k0);
        if (k0 + 4 * KT >= k_end) break;
        stage(kB, vB);
        load_sub(kB, vB, k0 + 12 * KT);
        compute(k0 + 4 * KT);
      }
    }

    // combine the 4 waves of the workgroup through LDS
    l_run += __shfl_xor(l_run, 16, 64);
    l_run += __shfl_xor(l_run, 32, 64);
    __syncthreads();
    float* ored = reinterpret_cast<float*>(smem);  // [4][16][D]
    float* mred = ored + 4 * 16 * D;               // [4][16]
    float* lred = mred + 4 * 16;                   // [4][16]
#pragma unroll
    for (int t = 0; t < NTD; ++t) *reinterpret_cast<f32x4*>(ored + (w * 16 + li) * D + 16 * t + 4 * g) = o[t];
    if (g == 0) {
      mred[w * 16 + li] = m_run;
      lred[w * 16 + li] = l_run;
    }
    __syncthreads();
    const int np = min(p.max_parts, div_up(ctx, p.part_size));
    const bool direct = np == 1;
    for (int e = tid; e < G * D; e += 256) {
      const int qh = e / D, d = e % D;
      float M = -1e30f;
#pragma unroll
      for (int ww = 0; ww < 4; ++ww) M = fmaxf(M, mred[ww * 16 + qh]);
      float L = 0.f, O = 0.f;
#pragma unroll
      for (int ww = 0; ww < 4; ++ww) {
        const float f = exp2f(mred[ww * 16 + qh] - M);
        L += f * lred[ww * 16 + qh];
        O += f * ored[(ww * 16 + qh) * D + d];
      }
      const size_t hq = (size_t)b * p.Hq + hk * G + qh;
      if (direct) {
        p.out[hq * D + d] = f2bf(L > 0.f ? O / L : 0.f);
      } else {
        const size_t pi = hq * p.max_parts + part;
        // write-through (sc1) stores: visible to the combining workgroup on any XCD without a
        // release fence (cdna_hip_programming.md Guideline 16, R1)
        __hip_atomic_store(p.part_o + pi * D + d, O, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (d == 0) {
          __hip_atomic_store(p.part_m + pi, M, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(p.part_l + pi, L, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
    if (!direct) {
      // partition combine by the last arriving workgroup of this (sequence, kv head), in the same
      // launch (Guideline 16, R1): every storing wave drains its sc1 partial stores, barrier, one
      // lane takes an agent-scope arrival ticket; the last arriver reads the partials with sc1
      // loads (no acquire fence: nothing it reads can sit stale in its L1)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        const int ci = b * p.Hkv + hk;
        const int prev = __hip_atomic_fetch_add(p.counters + ci, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = prev == np - 1;
        if (last) __hip_atomic_store(p.counters + ci, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *last_flag = last;
      }
      __syncthreads();
      if (*last_flag) {
        auto ld = [](const float* a) { return __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
        for (int e = tid; e < G * D; e += 256) {
          const int qh = e / D, d = e % D;
          const size_t hq = (size_t)b * p.Hq + hk * G + qh;
          const size_t base = hq * p.max_parts;
          float M = -1e30f;
          for (int i = 0; i < np; ++i) M = fmaxf(M, ld(p.part_m + base + i));
          float L = 0.f, O = 0.f;
          for (int i = 0; i < np; ++i) {
            const float f = exp2f(ld(p.part_m + base + i) - M);
            L += f * ld(p.part_l + base + i);
            O += f * ld(p.part_o + (base + i) * D + d);
          }
          p.out[hq * D + d] = f2bf(L > 0.f ? O / L : 0.f);
        }
      }
    }
    __syncthreads();  // LDS is restaged by the next item
  }
}

// -----------------------------------------------------------------------------------------------

int flash_attention(const void* q, long q_stride_tok, long q_stride_head, const void* k, const void* v,
                    long kv_stride_tok, long kv_stride_head, const void* k_cache, const void* v_cache,
                    const int* block_tables, int max_blocks, int block_size, void* out, long o_stride_tok,
                    long o_stride_head, const int* cu_q, const int* cu_k, const int* ctx_k, int batch,
                    int max_seqlen_q, int Hq, int Hkv, int D, int causal, int paged, float scale, hipStream_t s,
                    const int* rope_pos, const void* rope_cs) {
  if (batch <= 0 || max_seqlen_q <= 0) return 0;
  if (Hq % Hkv || (paged && block_size % 64)) return hipErrorInvalidValue;
  FlashParams prm{};
  prm.rope_pos = rope_pos;
  prm.rope_cs = (const float2*)rope_cs;
  prm.q = (const bf16*)q;
  prm.q_stride_tok = q_stride_tok;
  prm.q_stride_head = q_stride_head;
  prm.k = (const bf16*)k;
  prm.v = (const bf16*)v;
  prm.kv_stride_tok = kv_stride_tok;
  prm.kv_stride_head = kv_stride_head;
  prm.k_cache = (const bf16*)k_cache;
  prm.v_cache = (const bf16*)v_cache;
  prm.block_tables = block_tables;
  prm.max_blocks = max_blocks;
  prm.block_size = block_size;
  prm.out = (bf16*)out;
  prm.o_stride_tok = o_stride_tok;
  prm.o_stride_head = o_stride_head;
  prm.cu_q = cu_q;
  prm.cu_k = cu_k;
  prm.ctx_k = ctx_k;
  prm.Hq = Hq;
  prm.Hkv = Hkv;
  prm.scale_log2 = scale * 1.4426950408889634f;
  prm.pairs_per_wg = 1;
  // Llama prefill (D = 128 over the paged cache): the 32x32 kernel below
  if (D == 128 && paged && block_size % 64 == 0) {
    // software-pipelined V reads by default (3% faster, bit-identical: profiles/attn_vpipe_r5.md);
    // DAB_FLASH_VPIPE=0 selects the unpipelined kernel (A/B: benchmarks/kernel_bench.py attn)
    const char* vp = std::getenv("DAB_FLASH_VPIPE");
    const bool vpipe = !(vp && vp[0] == '0');
    // DAB_FLASH_W8=1: 8 waves per workgroup sharing a 3-deep K / V ring (A/B)
    const char* w8e = std::getenv("DAB_FLASH_W8");
    if (w8e && (w8e[0] == '1' || w8e[0] == '2')) {  // 2: with the staggered wave groups
      dim3 g8((max_seqlen_q + 255) / 256, Hq, batch);
      const bool stag = w8e[0] == '2';
      if (causal && stag) hipLaunchKernelGGL((flash_d128_kernel<true, false, 8, true>), g8, dim3(512), 0, s, prm);
      else if (causal) hipLaunchKernelGGL((flash_d128_kernel<true, true, 8>), g8, dim3(512), 0, s, prm);
      else if (stag) hipLaunchKernelGGL((flash_d128_kernel<false, false, 8, true>), g8, dim3(512), 0, s, prm);
      else hipLaunchKernelGGL((flash_d128_kernel<false, true, 8>), g8, dim3(512), 0, s, prm);
      return hipGetLastError();
    }
    dim3 g32((max_seqlen_q + 127) / 128, Hq, batch);
    // DAB_FLASH_Q64=1: 64 queries per wave, one wave per SIMD (A/B)
    const char* q64 = std::getenv("DAB_FLASH_Q64");
    if (q64 && q64[0] == '1') {
      dim3 gq((max_seqlen_q + 255) / 256, Hq, batch);
      if (causal) hipLaunchKernelGGL((flash_q64_kernel<true>), gq, dim3(256), 0, s, prm);
      else hipLaunchKernelGGL((flash_q64_kernel<false>), gq, dim3(256), 0, s, prm);
      return hipGetLastError();
    }
    // causal: one workgroup per (long, short) query-block pair by default (+8 % on 16 x 1024,
    // bit-identical: profiles/attn_vpipe_r5.md), unless the pairs would leave CUs idle (a single
    // prompt of <= 1k tokens: 1 x 1024 37.2 vs 42.8 us one block per workgroup,
    // profiles/attn_prefill_shape_r6.md); DAB_FLASH_PAIR=0 / 1 forces either
    const char* pe = std::getenv("DAB_FLASH_PAIR");
    const long pair_wgs = (long)(((max_seqlen_q + 127) / 128 + 1) / 2) * Hq * batch;
    const bool pair = pe && pe[0] == '1' ? true : !(pe && pe[0] == '0') && pair_wgs >= 256;
    if (causal && vpipe && pair) {
      // G = 2 pairs per workgroup (1 when that leaves < 1024 workgroups), walked heaviest-first
      // (lpt).  Large G made the workgroups few and long: the headline's prefill step (33 prompts of
      // ~1.03k queries, G = 5 = all pairs) ran 1056 workgroups of equal work on 512 slots, i.e.
      // three rounds where the third held 32 -- 770 us against ~520 (profiles/attn_prefill_shape_r6.md).
      // With G < pairs the groups of a (sequence, head) differ in work (9 query blocks = 5 pairs), and
      // dispatching them alternately stranded long ones at the end: heaviest-first walks all first
      // groups, then all second groups.  DAB_FLASH_G / DAB_FLASH_LPT=0 override (A/B)
      const int npairs = ((max_seqlen_q + 127) / 128 + 1) / 2;
      int G = (long)npairs * Hq * batch >= 2048 ? 2 : 1;
      if (const char* ge = std::getenv("DAB_FLASH_G")) G = std::atoi(ge);
      G = G < 1 ? 1 : (G > npairs ? npairs : G);
      prm.pairs_per_wg = G;
      dim3 gp((npairs + G - 1) / G, Hq, batch);
      const char* lp = std::getenv("DAB_FLASH_LPT");
      prm.lpt = !(lp && lp[0] == '0') && ((long)Hq * batch) % 8 == 0;
      const char* ob = std::getenv("DAB_FLASH_1BAR");  // A/B: one barrier per tile
      const char* sm = std::getenv("DAB_FLASH_SMS");   // A/B: softmax split across the PV k-steps
      const char* sg = std::getenv("DAB_FLASH_SGB");   // A/B: sched_group_barrier S^T interleave
      if (sg && sg[0] == '1')
        hipLaunchKernelGGL((flash_d128_kernel<true, true, 4, false, true, false, false, true>), gp, dim3(256), 0, s,
                           prm);
      else if (sm && sm[0] == '1')
        hipLaunchKernelGGL((flash_d128_kernel<true, true, 4, false, true, false, true>), gp, dim3(256), 0, s, prm);
      else if (ob && ob[0] == '1')
        hipLaunchKernelGGL((flash_d128_kernel<true, true, 4, false, true, true>), gp, dim3(256), 0, s, prm);
      else
        hipLaunchKernelGGL((flash_d128_kernel<true, true, 4, false, true>), gp, dim3(256), 0, s, prm);
      return hipGetLastError();
    }
    if (causal && vpipe) hipLaunchKernelGGL((flash_d128_kernel<true, true>), g32, dim3(256), 0, s, prm);
    else if (causal) hipLaunchKernelGGL((flash_d128_kernel<true>), g32, dim3(256), 0, s, prm);
    else if (vpipe) hipLaunchKernelGGL((flash_d128_kernel<false, true>), g32, dim3(256), 0, s, prm);
    else hipLaunchKernelGGL((flash_d128_kernel<false>), g32, dim3(256), 0, s, prm);
    return hipGetLastError();
  }
  if (rope_cs) return hipErrorInvalidValue;  // Q RoPE lives only in the D = 128 paged kernel above
  // Long D = 128 sequences: 128-query blocks of 8 waves x 16 queries halve the K/V tile traffic per
  // query (16x1024 causal: 298 -> 355 TFLOP/s); the encoder (D <= 64) runs 64-query blocks of 4
  // waves (8 waves measured 5 % slower there; a 4-wave x 2-sub-tile form was no faster either)
  // DAB_ENC_PERSIST=1: the persistent encoder kernel (D 64, packed, bidirectional; A/B)
  if (const char* ep = std::getenv("DAB_ENC_PERSIST")) {
    if (ep[0] == '1' && D == 64 && !paged && !causal && !rope_cs) {
      const int items = batch * Hq;
      const int grid = items < 256 * 5 ? items : 256 * 5;
      hipLaunchKernelGGL(flash_enc_kernel, dim3(grid), dim3(256), 0, s, prm, items);
      return hipGetLastError();
    }
  }
  const bool wide = D == 128 && max_seqlen_q > 64;
  // the 5-waves-per-SIMD encoder variant by default (3 % faster on the embed bench's packed batch,
  // bit-identical: profiles/embed_r5.md); DAB_ENC_W5=0 selects the unbounded-register kernel
  const char* e5 = std::getenv("DAB_ENC_W5");
  const bool enc5 = !(e5 && e5[0] == '0');
  const int qb = wide ? 128 : 64;
  dim3 grid((max_seqlen_q + qb - 1) / qb, Hq, batch);
#define DAB_FLASH(DD, C, P)                                                                          \
  do {                                                                                              \
    if (wide)                                                                                       \
      hipLaunchKernelGGL((flash_fwd_kernel<DD, C, P, (DD == 128 ? 8 : 4), 1>), grid,              \
                         dim3(DD == 128 ? 512 : 256), 0, s, prm);                                   \
    else if (DD == 64 && enc5)                                                                      \
      hipLaunchKernelGGL((flash_fwd_kernel<DD, C, P, 4, 1, DD == 64 ? 5 : 0>), grid, dim3(256), 0, s, prm); \
    else                                                                                            \
      hipLaunchKernelGGL((flash_fwd_kernel<DD, C, P, 4, 1>), grid, dim3(256), 0, s, prm);           \
  } while (0)
#define DAB_FLASH_D(DD)                    \
  if (paged) {                             \
    if (causal) DAB_FLASH(DD, true, true); \
    else DAB_FLASH(DD, false, true);       \
  } else {                                 \
    if (causal) DAB_FLASH(DD, true, false); \
    else DAB_FLASH(DD, false, false);      \
  }
  if (D == 128) {
    DAB_FLASH_D(128)
  } else if (D == 64) {
    DAB_FLASH_D(64)
  } else if (D == 32) {
    DAB_FLASH_D(32)
  } else {
    return hipErrorInvalidValue;
  }
#undef DAB_FLASH_D
#undef DAB_FLASH
  return hipGetLastError();
}

// The workgroups of a launch are dispatched in blockIdx order as CU slots free up; at RAG batch sizes
// every CU runs about two (sequence, kv head) items one after the other, so with sequences of mixed
// length the launch ends when the unluckiest slot has run two long ones.  ``order`` (optional, a
// permutation of the batch, longest context first, built on the host with the step's inputs) makes
// the dispatch longest-processing-time-first: the long items start in the first round, the short
// ones fill in behind them.
int paged_decode_attention(const void* q, const void* k_cache, const void* v_cache, const int* block_tables,
                           int max_blocks, int block_size, const int* ctx_lens, void* out, float* part_o,
                           float* part_m, float* part_l, int* counters, int batch, int Hq, int Hkv, int D,
                           int part_size, int max_parts, float scale, hipStream_t s, const int* order,
                           const L3Warm* warm) {
  if (batch <= 0) return 0;
  if (Hq % Hkv || Hq / Hkv > 16 || part_size % 128 || max_parts < 1 || block_size % 32) return hipErrorInvalidValue;
  if (max_parts > 1 && !counters) return hipErrorInvalidValue;
  if (!q) return hipErrorInvalidValue;
  DecodeParams prm;
  prm.q = (const bf16*)q;
  prm.k_cache = (const bf16*)k_cache;
  prm.v_cache = (const bf16*)v_cache;
  prm.block_tables = block_tables;
  prm.max_blocks = max_blocks;
  prm.block_size = block_size;
  prm.ctx_lens = ctx_lens;
  prm.out = (bf16*)out;
  prm.part_o = part_o;
  prm.part_m = part_m;
  prm.part_l = part_l;
  prm.counters = counters;
  prm.order = order;
  prm.Hq = Hq;
  prm.Hkv = Hkv;
  prm.part_size = part_size;
  prm.max_parts = max_parts;
  prm.scale_log2 = scale * 1.4426950408889634f;
  prm.warm = warm ? *warm : L3Warm{{nullptr, nullptr}, {0, 0}, 0};
  if (prm.warm.blocks < 0 || prm.warm.blocks > 1024 || ((prm.warm.bytes[0] | prm.warm.bytes[1]) & 15) ||
      (prm.warm.blocks && prm.warm.bytes[0] + prm.warm.bytes[1] <= 0))
    return hipErrorInvalidValue;
  const int total_items = max_parts * Hkv * batch;
  dim3 grid((total_items < 2048 ? total_items : 2048) + prm.warm.blocks);
  // K/V are read exactly once per step: non-temporal loads (aux = 2) -- in the Llama-3-8B decode step
  // at batch 128 this took the attention from 127 to 111 us per layer (5.1 -> 5.8 TB/s;
  // profiles/decode_round2.md).  D = 128 stages K / V by LDS-DMA (100.7 vs 102.6 us isolated, same
  // section); D = 64 (small test models) keeps the register path.
  if (D == 128) {
    // small batches: two LDS slots per wave (at batch 128 the one-slot kernel's two workgroups per CU
    // are 2.8 % faster per step: 7.44 vs 7.65 ms, profiles/low_load_latency.md)
    if (batch * Hkv <= 64 && part_size <= 64 * 4 * 32)
      hipLaunchKernelGGL((paged_decode_kernel<128, true, true, 2>), grid, dim3(256), 0, s, prm, total_items);
    else hipLaunchKernelGGL((paged_decode_kernel<128, true, true>), grid, dim3(256), 0, s, prm, total_items);
  } else if (D == 64) {
    hipLaunchKernelGGL((paged_decode_kernel<64, true>), grid, dim3(256), 0, s, prm, total_items);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace dab

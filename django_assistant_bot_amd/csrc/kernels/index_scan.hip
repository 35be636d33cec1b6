// Persistent exact-cosine scan of the in-HBM index for small query batches (M <= 96): the
// threshold-candidate pass of VectorIndex search (the pgvector CosineDistance ORDER BY it replaces:
// reference rag/services/search_service.py:185-196) at 1-96 queries.
//
// At M <= 96 the scan is an HBM stream (15 GB for 10M x 768 rows; 1 TFLOP at 64 queries, a sixth
// of the stream time on the matrix cores).  The GEMM kernels stage the queries again for every
// output tile (as many L2 bytes as the rows they scan); here they are staged into LDS ONCE per
// workgroup and every wave streams index rows through a VGPR ring for the whole launch:
//   * MT 16-query tiles (M <= 16 MT): MT 1-2 -> 4-wave workgroups, 2 per CU; MT 3-6 -> 8-wave
//     workgroups, 1 per CU (up to 144 KB of queries in LDS: MT 5-6 need K <= 768);
//   * persistent grid, tile = 32 rows per wave (two 16-row MFMA A tiles),
//     row-major 16-B loads (lane = row li, k 8g..8g+7 of a 32-k chunk) with the tile's base in the
//     buffer descriptor, whose range clamps the last partial tile to zeros;
//   * the ring runs across tile boundaries (a flat stream of 32-k chunks), so the next tile's loads
//     are in flight under the current tile's epilogue;
//   * queries [16 MT, K] in LDS with chunk c of row r at c ^ (r & 15): conflict-free ds_read_b128
//     B fragments (one fragment feeds both A tiles' MFMAs; one A fragment feeds MT MFMAs);
//   * epilogue straight from the accumulators: a score >= thr[query] (rare) takes a slot in the
//     wave's LDS list; flushing the list applies the row / query group filters and appends to the
//     query's global list with one returning atomic per hit (gemm.hip EPI_CANDIDATES) -- a wait
//     that in the tile loop would drain the wave's whole load ring;
//   * SHUF: the rows come from a copy in the decode-stream layout [rows/16][K/32][64 lanes][8]
//     (ops.shuffle_weights), where each 16-row x 32-k A fragment is 1 KB contiguous in lane order:
//     every load is one fully coalesced 1 KB read instead of 16 rows x 64 B.
#include "common.h"
#include "launchers.h"

namespace dab {

namespace {

struct ScanParams {
  const bf16* X;  // queries [M, K]
  long ldx;
  const bf16* W;  // index rows [N, K]
  long ldw;
  int M, N, K;
  const int* row_group;
  const int* q_group;
  const float* thr;
  int* cnt;
  float* cand_val;
  int* cand_idx;
  int cap;
};

constexpr int kScanKMax = 1024;
constexpr int kScanMaxM = 96;
// widest rows the queries of MT 16-query tiles may have (LDS: 16 MT KMax 2 B <= 144 KB)
constexpr int scan_kmax(int mt) { return mt <= 4 ? kScanKMax : 768; }
constexpr int kScanRT = 2;     // 16-row A tiles per wave
constexpr int kScanNWIN = 8;   // chunks (of 32 k) in flight per wave
constexpr int kScanListW = 160;  // candidate list entries per wave (12 B each)

}  // namespace

template <bool SHUF, int MT, int NW>
__global__ __launch_bounds__(64 * NW, 8 / NW) void index_scan_kernel(ScanParams p) {
  constexpr int RT = kScanRT, NWIN = kScanNWIN, TR = 32 * NW;  // rows per workgroup tile
  constexpr int XS = 16 * MT * scan_kmax(MT) * 2;
  __shared__ __attribute__((aligned(16))) char xs[XS + 64 + NW * kScanListW * 12];
  const int tid = threadIdx.x, lane = tid & 63, li = lane & 15, g = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cpr = p.K / 8;  // 16-B chunks per query row
  const int RB = p.K * 2;

  // ---- per-wave candidate lists (after the queries): a hit takes an LDS slot; the group filters
  // and the global append (a returning atomic, whose wait would drain this wave's whole load ring)
  // run when the list is flushed -- at a high-water mark and at the end
  int* const lcnt = reinterpret_cast<int*>(xs + XS);
  int* const l_n = lcnt + 16 + w * kScanListW;
  int* const l_m = lcnt + 16 + NW * kScanListW + w * kScanListW;
  float* const l_v = reinterpret_cast<float*>(lcnt + 16 + 2 * NW * kScanListW + w * kScanListW);
  auto cand_global = [&](int m, int n, float v) {
    const int rg = p.row_group ? p.row_group[n] : 0;
    const int qgm = p.q_group ? p.q_group[m] : -1;
    if (rg >= 0 && (qgm < 0 || rg == qgm)) {
      const int slot = atomicAdd(p.cnt + m, 1);
      if (slot < p.cap) {
        p.cand_val[(size_t)m * p.cap + slot] = v;
        p.cand_idx[(size_t)m * p.cap + slot] = n;
      }
    }
  };
  auto list_count = [&]() {
    return __builtin_amdgcn_readfirstlane(__hip_atomic_load(lcnt + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
  };
  auto cand_flush = [&]() {  // wave-uniform
    const int c = list_count();
    for (int e = lane; e < c; e += 64) cand_global(l_m[e], l_n[e], l_v[e]);
    if (lane == 0) __hip_atomic_store(lcnt + w, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    // retire the flush's own memory ops here, so the code after it (and the hit test of every tile,
    // which the compiler merges with this path) inherits no pending store or load to wait for
    __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
  };
  if (tid < NW) lcnt[tid] = 0;

  // ---- queries -> LDS once (rows >= M repeat row M - 1; their scores are never appended)
  for (int e = tid; e < 16 * MT * cpr; e += 64 * NW) {
    const int r = e / cpr, c = e % cpr;
    const u32x4 v = *reinterpret_cast<const u32x4*>(p.X + (size_t)min(r, p.M - 1) * p.ldx + 8 * c);
    *reinterpret_cast<u32x4*>(xs + r * RB + 16 * (c ^ (r & 15))) = v;
  }
  float thr[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) {
    const int m = 16 * t + li;
    thr[t] = m < p.M ? p.thr[m] : __builtin_huge_valf();
  }
  __syncthreads();

  // ---- flat chunk stream over this wave's tiles: tile i of the wave = rows
  // (blockIdx.x + i * gridDim.x) * TR + 32 w .. + 31; chunk = 32 k of both 16-row A tiles
  const int nck = p.K / 32;  // chunks per tile (a multiple of NWIN: checked by the launcher)
  const int tiles = (p.N + TR - 1) / TR;
  const int my_tiles = blockIdx.x < tiles ? (tiles - 1 - blockIdx.x) / gridDim.x + 1 : 0;
  if (my_tiles == 0) return;
  auto tile_row0 = [&](int i) { return (blockIdx.x + i * gridDim.x) * TR + 32 * w; };
  // descriptor of tile i (rows past N read zeros); past the wave's last tile or wholly past N: empty
  // range (the ring's loads return zeros without memory traffic)
  // SHUF: a tile's two 16-row blocks are whole in the copy (round_up(N, 128) rows) when it starts
  // below N; rows >= N there score like any row and are dropped by the epilogue's n < N test
  auto rsrc_of = [&](int i) {
    const int r0 = tile_row0(i);
    const bool live = i < my_tiles && r0 < p.N;
    if constexpr (SHUF) {
      return __builtin_amdgcn_make_buffer_rsrc((void*)(p.W + (size_t)(min(r0, p.N - 1) / 16) * nck * 512), (short)0,
                                               live ? 2 * nck * 1024 : 0, 0x00020000);
    } else {
      const int rows = live ? min(32, p.N - r0) : 0;
      return __builtin_amdgcn_make_buffer_rsrc((void*)(p.W + (size_t)min(r0, p.N - 1) * p.ldw), (short)0,
                                               (int)(rows * p.ldw * 2), 0x00020000);
    }
  };
  const int voff = SHUF ? lane * 16 : (int)((li * p.ldw + 8 * g) * 2);
  const int astr = SHUF ? nck * 1024 : (int)(16 * p.ldw * 2);  // next 16-row block
  constexpr int CSTR = SHUF ? 1024 : 64;                         // next 32-k chunk

  bf16x8 wr[NWIN][RT];
  int ld_tile = 0, ld_c = 0;  // next chunk to load (wave-uniform)
  auto ld_rs = rsrc_of(0);
  auto load = [&](int slot) __attribute__((always_inline)) {
#pragma unroll
    for (int a = 0; a < RT; ++a)
      wr[slot][a] = __builtin_bit_cast(
          bf16x8, __builtin_amdgcn_raw_buffer_load_b128(ld_rs, voff + a * astr, ld_c * CSTR, 2));  // nt: read once
    if (++ld_c == nck) {
      ld_c = 0;
      ld_rs = rsrc_of(++ld_tile);
    }
  };
#pragma unroll
  for (int s = 0; s < NWIN; ++s) load(s);

  f32x4 acc[RT][MT];
  for (int i = 0; i < my_tiles; ++i) {
#pragma unroll
    for (int a = 0; a < RT; ++a)
#pragma unroll
      for (int t = 0; t < MT; ++t) acc[a][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int c0 = 0; c0 < nck; c0 += NWIN) {
#pragma unroll
      for (int s = 0; s < NWIN; ++s) {
        const int c = c0 + s;
        bf16x8 bx[MT];
#pragma unroll
        for (int t = 0; t < MT; ++t)
          bx[t] = *reinterpret_cast<const bf16x8*>(xs + (16 * t + li) * RB + 16 * ((4 * c + g) ^ li));
#pragma unroll
        for (int a = 0; a < RT; ++a)
#pragma unroll
          for (int t = 0; t < MT; ++t) acc[a][t] = mfma16(wr[s][a], bx[t], acc[a][t]);
        load(s);  // refill the slot right behind its MFMAs (NWIN chunks ahead)
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // ---- candidates: acc[a][t] lane (li, g) = scores of query 16 t + li against rows 16 a + 4 g + r
    const int r0 = tile_row0(i);
    if (r0 >= p.N) continue;  // wave-uniform
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
      for (int a = 0; a < RT; ++a)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = r0 + 16 * a + 4 * g + r;
          const float v = acc[a][t][r];
          const bool hit = v >= thr[t] && n < p.N;
          // the list holds <= kScanListW - 64 entries here, so the <= 64 hits of one step fit
          if (__builtin_amdgcn_ballot_w64(hit)) {
            if (hit) {
              const int slot = __hip_atomic_fetch_add(lcnt + w, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
              l_n[slot] = n;
              l_m[slot] = 16 * t + li;
              l_v[slot] = v;
            }
            if (list_count() > kScanListW - 64) cand_flush();
          }
        }
  }
  cand_flush();
}

static int index_scan_launch(bool shuf, const void* X, long ldx, const void* W, long ldw, int M, int N, int K,
                             const int* row_group, const int* q_group, const float* thr, int* cnt, float* cand_val,
                             int* cand_idx, int cap, hipStream_t s) {
  ScanParams p;
  p.X = (const bf16*)X;
  p.ldx = ldx;
  p.W = (const bf16*)W;
  p.ldw = ldw;
  p.M = M;
  p.N = N;
  p.K = K;
  p.row_group = row_group;
  p.q_group = q_group;
  p.thr = thr;
  p.cnt = cnt;
  p.cand_val = cand_val;
  p.cand_idx = cand_idx;
  p.cap = cap;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int mt = (M + 15) / 16;
  const int nw = mt <= 2 ? 4 : 8, per_cu = 8 / nw;
  const long tiles = (N + 32L * nw - 1) / (32L * nw);
  const int grid = (int)(tiles < (long)per_cu * cus ? tiles : (long)per_cu * cus);
#define SCAN_LAUNCH(MT_, NW_)                                                                        \
  do {                                                                                               \
    if (shuf) hipLaunchKernelGGL((index_scan_kernel<true, MT_, NW_>), dim3(grid), dim3(64 * NW_), 0, s, p); \
    else hipLaunchKernelGGL((index_scan_kernel<false, MT_, NW_>), dim3(grid), dim3(64 * NW_), 0, s, p);     \
  } while (0)
  switch (mt) {
    case 1: SCAN_LAUNCH(1, 4); break;
    case 2: SCAN_LAUNCH(2, 4); break;
    case 3: SCAN_LAUNCH(3, 8); break;
    case 4: SCAN_LAUNCH(4, 8); break;
    case 5: SCAN_LAUNCH(5, 8); break;
    default: SCAN_LAUNCH(6, 8); break;
  }
#undef SCAN_LAUNCH
  return hipGetLastError();
}

int index_scan_candidates(const void* X, long ldx, const void* W, long ldw, int M, int N, int K, const int* row_group,
                          const int* q_group, const float* thr, int* cnt, float* cand_val, int* cand_idx, int cap,
                          hipStream_t s) {
  if (M <= 0 || N <= 0) return 0;
  if (M > kScanMaxM || K > scan_kmax((M + 15) / 16) || K % (32 * kScanNWIN) || ldx % 8 || ldw % 8 || cap <= 0)
    return hipErrorInvalidValue;
  if (32L * ldw * 2 >= (1L << 31)) return hipErrorInvalidValue;
  return index_scan_launch(false, X, ldx, W, ldw, M, N, K, row_group, q_group, thr, cnt, cand_val, cand_idx, cap, s);
}

// W: the rows in the shuffle_weights layout, with at least round_up(N, 32) rows
int index_scan_candidates_shuf(const void* X, long ldx, const void* W, int M, int N, int K, const int* row_group,
                               const int* q_group, const float* thr, int* cnt, float* cand_val, int* cand_idx,
                               int cap, hipStream_t s) {
  if (M <= 0 || N <= 0) return 0;
  if (M > kScanMaxM || K > scan_kmax((M + 15) / 16) || K % (32 * kScanNWIN) || ldx % 8 || cap <= 0)
    return hipErrorInvalidValue;
  return index_scan_launch(true, X, ldx, W, K, M, N, K, row_group, q_group, thr, cnt, cand_val, cand_idx, cap, s);
}

}  // namespace dab

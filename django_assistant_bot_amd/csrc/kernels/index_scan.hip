// Persistent exact-cosine scan of the in-HBM index for small query batches (M <= 16): the
// threshold-candidate pass of VectorIndex search (the pgvector CosineDistance ORDER BY it replaces:
// reference rag/services/search_service.py:185-196) at 1-16 queries.
//
// At M <= 16 a GEMM tile is mostly padding and the scan is a pure HBM stream (15 GB for 10M x 768
// rows).  The GEMM kernels stage the queries again for every output tile (as many L2 bytes as the
// rows they scan at M = 1); here they are staged into LDS ONCE per workgroup and every wave streams
// index rows through a VGPR ring for the whole launch:
//   * persistent grid (2 workgroups per CU), tile = 32 rows per wave (two 16-row MFMA A tiles),
//     row-major 16-B loads (lane = row li, k 8g..8g+7 of a 32-k chunk) with the tile's base in the
//     buffer descriptor, whose range clamps the last partial tile to zeros;
//   * the ring runs across tile boundaries (a flat stream of 32-k chunks), so the next tile's loads
//     are in flight under the current tile's epilogue;
//   * queries [16, K] in LDS with chunk c of row r at c ^ (r & 15): conflict-free ds_read_b128
//     B fragments (one fragment feeds both A tiles' MFMAs);
//   * epilogue straight from the accumulators: a score >= thr[query] (rare) loads its row's group
//     and appends (score, row) to the query's list with one atomic (gemm.hip EPI_CANDIDATES);
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
constexpr int kScanRT = 2;     // 16-row A tiles per wave
constexpr int kScanNWIN = 8;   // chunks (of 32 k) in flight per wave

}  // namespace

template <bool SHUF>
__global__ __launch_bounds__(256, 2) void index_scan_kernel(ScanParams p) {
  constexpr int RT = kScanRT, NWIN = kScanNWIN;
  __shared__ __attribute__((aligned(16))) char xs[16 * kScanKMax * 2];
  const int tid = threadIdx.x, lane = tid & 63, li = lane & 15, g = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cpr = p.K / 8;  // 16-B chunks per query row
  const int RB = p.K * 2;

  // ---- queries -> LDS once (rows >= M repeat row M - 1; their scores are never appended)
  for (int e = tid; e < 16 * cpr; e += 256) {
    const int r = e / cpr, c = e % cpr;
    const u32x4 v = *reinterpret_cast<const u32x4*>(p.X + (size_t)min(r, p.M - 1) * p.ldx + 8 * c);
    *reinterpret_cast<u32x4*>(xs + r * RB + 16 * (c ^ (r & 15))) = v;
  }
  const bool q_ok = li < p.M;
  const float thr = q_ok ? p.thr[li] : __builtin_huge_valf();
  const int qg = (q_ok && p.q_group) ? p.q_group[li] : -1;
  __syncthreads();

  // ---- flat chunk stream over this wave's tiles: tile i of the wave = rows
  // (blockIdx.x + i * gridDim.x) * 128 + 32 w .. + 31; chunk = 32 k of both 16-row A tiles
  const int nck = p.K / 32;  // chunks per tile (a multiple of NWIN: checked by the launcher)
  const int tiles = (p.N + 127) / 128;
  const int my_tiles = blockIdx.x < tiles ? (tiles - 1 - blockIdx.x) / gridDim.x + 1 : 0;
  if (my_tiles == 0) return;
  auto tile_row0 = [&](int i) { return (blockIdx.x + i * gridDim.x) * 128 + 32 * w; };
  // descriptor of tile i (rows past N read zeros); past the wave's last tile: empty range (the ring's
  // run-out loads return zeros without memory traffic)
  // SHUF: the tile's two 16-row blocks are whole in the copy (its row count is a multiple of 32);
  // rows >= N there score like any row and are dropped by the epilogue's n < N test
  auto rsrc_of = [&](int i) {
    const int r0 = tile_row0(i);
    if constexpr (SHUF) {
      const int bytes = i < my_tiles ? 2 * nck * 1024 : 0;
      return __builtin_amdgcn_make_buffer_rsrc((void*)(p.W + (size_t)(min(r0, p.N - 1) / 16) * nck * 512), (short)0,
                                               bytes, 0x00020000);
    } else {
      const int rows = i < my_tiles ? max(0, min(32, p.N - r0)) : 0;
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

  f32x4 acc[RT];
  for (int i = 0; i < my_tiles; ++i) {
#pragma unroll
    for (int a = 0; a < RT; ++a) acc[a] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int c0 = 0; c0 < nck; c0 += NWIN) {
#pragma unroll
      for (int s = 0; s < NWIN; ++s) {
        const int c = c0 + s;
        const bf16x8 bx = *reinterpret_cast<const bf16x8*>(xs + li * RB + 16 * ((4 * c + g) ^ li));
#pragma unroll
        for (int a = 0; a < RT; ++a) acc[a] = mfma16(wr[s][a], bx, acc[a]);
        load(s);  // refill the slot right behind its MFMAs (NWIN chunks ahead)
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // ---- candidates: acc[a] lane (li, g) = scores of query li against rows 16 a + 4 g + r
    const int r0 = tile_row0(i);
#pragma unroll
    for (int a = 0; a < RT; ++a)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = r0 + 16 * a + 4 * g + r;
        const float v = acc[a][r];
        if (v >= thr && n < p.N) {
          const int rg = p.row_group ? p.row_group[n] : 0;
          if (rg >= 0 && (qg < 0 || rg == qg)) {
            const int slot = atomicAdd(p.cnt + li, 1);
            if (slot < p.cap) {
              p.cand_val[(size_t)li * p.cap + slot] = v;
              p.cand_idx[(size_t)li * p.cap + slot] = n;
            }
          }
        }
      }
  }
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
  const int tiles = (N + 127) / 128;
  const int grid = tiles < 2 * cus ? tiles : 2 * cus;
  if (shuf)
    hipLaunchKernelGGL(index_scan_kernel<true>, dim3(grid), dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL(index_scan_kernel<false>, dim3(grid), dim3(256), 0, s, p);
  return hipGetLastError();
}

int index_scan_candidates(const void* X, long ldx, const void* W, long ldw, int M, int N, int K, const int* row_group,
                          const int* q_group, const float* thr, int* cnt, float* cand_val, int* cand_idx, int cap,
                          hipStream_t s) {
  if (M <= 0 || N <= 0) return 0;
  if (M > 16 || K > kScanKMax || K % (32 * kScanNWIN) || ldx % 8 || ldw % 8 || cap <= 0) return hipErrorInvalidValue;
  if (32L * ldw * 2 >= (1L << 31)) return hipErrorInvalidValue;
  return index_scan_launch(false, X, ldx, W, ldw, M, N, K, row_group, q_group, thr, cnt, cand_val, cand_idx, cap, s);
}

// W: the rows in the shuffle_weights layout, with at least round_up(N, 32) rows
int index_scan_candidates_shuf(const void* X, long ldx, const void* W, int M, int N, int K, const int* row_group,
                               const int* q_group, const float* thr, int* cnt, float* cand_val, int* cand_idx,
                               int cap, hipStream_t s) {
  if (M <= 0 || N <= 0) return 0;
  if (M > 16 || K > kScanKMax || K % (32 * kScanNWIN) || ldx % 8 || cap <= 0) return hipErrorInvalidValue;
  return index_scan_launch(true, X, ldx, W, K, M, N, K, row_group, q_group, thr, cnt, cand_val, cand_idx, cap, s);
}

}  // namespace dab

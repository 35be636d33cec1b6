// Weight-streaming MFMA GEMM for decode-sized M:  C[M, N] = X[M, K] . W[N, K]^T,  M <= 128.
//
// Decode projections are HBM-bound on the weight stream (Llama-3-8B: 436 MB per layer against
// <= 1.8 MB of activations), so the kernel is organised around reading W exactly once at full rate:
//
//   * grid = (N / 64 row tiles) x S K-slices; a 256-thread workgroup owns 64 weight rows and one
//     K-slice; inside it the 4 waves split every 256-deep stage four ways (each wave: all 64 rows x
//     64 k), so one X fragment read from LDS feeds four MFMAs; partial tiles meet through LDS once.  The block -> (tile, slice) map keeps a tile's slices on one XCD
//     (bijective XCD remap, then slice-minor) so their slabs meet in one L2.
//   * W goes straight to VGPRs (MI355X guide: "GEMV / M <= 16 decode weights ... load straight to
//     VGPRs, deep unroll, late vmcnt"): each lane issues 16-B loads that form the MFMA A fragment
//     directly (lane l: row l&15, k 8(l>>4)..+8 of a 32-deep chunk); every chunk's registers are
//     reloaded two stages ahead right after its MFMAs, keeping a 512-deep window (16 KB per wave)
//     in flight; buffer loads with SGPR offsets; optional non-temporal policy for once-read weights.
//   * X (shared by the 4 waves) is staged through registers into an XOR-swizzled LDS double buffer,
//     full 512-B rows per stage (guide: "x operand ... through LDS in full lines"); B fragments are
//     conflict-free ds_read_b128.  (LDS-DMA staging was tried: the compiler cannot separate its
//     LDS writes from the fragment reads and drains vmcnt before every read.)
//   * v_mfma_f32_16x16x32_bf16 with W as A and X as B, so a lane ends with 4 consecutive output
//     columns n of one row m.
//   * S == 1: epilogue in-kernel through LDS (bf16, optional residual add, or SwiGLU on weights
//     interleaved in 16-row [gate | up] groups) with 16-B row-contiguous stores.
//     S > 1: fp32 slabs [S][M][N] (plain 16-B stores).  The reduction is fused into the CONSUMER's
//     prologue (rmsnorm / rope+KV-write read the slabs) -- the guide's launch-boundary reduce -- or
//     done by skinny_reduce for library use.
#include "common.h"
#include "launchers.h"

namespace dab {

struct SkinnyParams {
  const bf16* X;
  long ldx;
  const bf16* W;
  long ldw;
  void* out;  // bf16 [M, ldo] (S == 1) or fp32 slabs [S][M][N] (S > 1)
  long ldo;
  const bf16* residual;  // optional, S == 1 and EPI_NONE only
  long ldr;
  int M, N, K, S, kc;
  int epi;  // 0 none, 2 swiglu (same codes as gemm.hip)
};

constexpr int SK_KSTAGE = 256;  // k per pipeline stage
constexpr int SK_EPI_NONE = 0, SK_EPI_SWIGLU = 2;

// MT <= 4: 2 workgroups per CU (<= 64 KB of X stages each).  MT == 8 (M <= 128): the 128 KB X double
// buffer allows one workgroup per CU, which in turn gives each wave the whole 512-VGPR budget.
template <int MT, int RT, bool NT_W>
__global__ __launch_bounds__(256, (MT >= 8 ? 1 : 2)) void skinny_gemm_kernel(SkinnyParams p) {
  // waves = (4 / RT row groups of RT 16-row tiles) x (RT k-groups splitting every stage)
  constexpr int NKG = RT;            // k groups
  constexpr int CPW = 8 / RT;        // 32-deep chunks per wave per stage
  constexpr int MP = 16 * MT;                       // padded M
  constexpr int ROWB = SK_KSTAGE * 2;               // bytes per staged X row (512)
  constexpr int XBUF = MP * ROWB;                   // bytes per X stage buffer
  // X stage double buffer (two objects so the unrolled stages address them statically); after the
  // K loop the pair holds the 4 waves' partial tiles (4 x MP x 64 fp32 == 2 x XBUF).
  __shared__ __attribute__((aligned(16))) char xs0[XBUF];
  __shared__ __attribute__((aligned(16))) char xs1[XBUF];

  const int tiles = p.N / 64;
  const int nwg = tiles * p.S;
  const int bid = blockIdx.x;
  const int xcd = bid % 8, q8 = nwg / 8, r8 = nwg % 8;
  const int sid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  const int tile = sid / p.S, slice = sid % p.S;

  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, g = lane >> 4, li = lane & 15;
  const int n0 = tile * 64;
  const int k_begin = slice * p.kc;
  const int nst = p.kc / SK_KSTAGE;

  // Buffer loads: 32-bit per-lane voffset + wave-uniform (SGPR) soffset, so per-stage offsets and
  // the end-of-slice clamp cost scalar ALU only.
  const auto wres = __builtin_amdgcn_make_buffer_rsrc((void*)(p.W + (size_t)n0 * p.ldw), 0,
                                                      (int)(64 * p.ldw * 2), 0x00020000);
  // X rows >= M fall outside the descriptor's range and read as zeros
  const auto xres = __builtin_amdgcn_make_buffer_rsrc((void*)p.X, 0, (int)(p.M * p.ldx * 2), 0x00020000);
  // wave w = (row group rg, k group kg): RT row tiles x the kg-th 1/RT of every stage (intra-workgroup
  // split-K), so each X fragment read from LDS feeds RT MFMAs
  const int rg = w / NKG, kg = w % NKG;
  const int w_voff = (int)(((16 * RT * rg + li) * p.ldw + k_begin + kg * (SK_KSTAGE / NKG) + 8 * g) * 2);
  const int a_stride = 16 * (int)p.ldw * 2;  // bytes between 16-row W tiles (uniform)

  // X stage through registers: thread tid moves chunks e = tid + 256 c (c < 2 MT) of the stage image
  // (row e >> 5, physical 16-B chunk e & 31, holding logical chunk (e & 31) ^ (row & 15)).  Plain
  // loads keep every wait exact in the compiler's in-order vmcnt accounting; an LDS-DMA would make
  // each fragment read wait for vmcnt(0), draining the weight prefetch.
  constexpr int XC = MP / 8;  // 16-B chunks per thread per stage
  int x_voff[XC];
#pragma unroll
  for (int c = 0; c < XC; ++c) {
    const int e = tid + 256 * c;
    const int r = e >> 5, lc = (e & 31) ^ (r & 15);
    x_voff[c] = (int)((r * p.ldx + lc * 8) * 2);
  }
  u32x4 xr[XC];
  auto load_x = [&](int st) {
    const int soff = (k_begin + min(st, nst - 1) * SK_KSTAGE) * 2;  // clamped: branch-free body
#pragma unroll
    for (int c = 0; c < XC; ++c)
      xr[c] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(xres, x_voff[c], soff, 0));
  };
  auto store_x = [&](char* xs) {
#pragma unroll
    for (int c = 0; c < XC; ++c) *reinterpret_cast<u32x4*>(xs + (tid + 256 * c) * 16) = xr[c];
  };

  // W window: two stages x RT row tiles x CPW chunks of 32 k.  A chunk's registers are reloaded with
  // the same chunk two stages ahead right after its MFMAs issue (a 512-deep window in flight).
  bf16x8 wr[2][RT][CPW];
  auto load_w = [&](int slot, int st, int a, int c) {
    const int soff = min(st, nst - 1) * SK_KSTAGE * 2 + a * a_stride;
    wr[slot][a][c] = __builtin_bit_cast(
        bf16x8, __builtin_amdgcn_raw_buffer_load_b128(wres, w_voff + 64 * c, soff, NT_W ? 2 : 0));
  };

  f32x4 acc[RT][MT];
#pragma unroll
  for (int a = 0; a < RT; ++a)
#pragma unroll
    for (int t = 0; t < MT; ++t) acc[a][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Stage st: per 32-deep chunk, fragments from LDS -> RT x MT MFMAs -> reload that chunk's W
  // registers with stage st+2; then X(st+1) (loaded a stage ago) goes to the other LDS buffer and
  // X(st+2) is loaded.  Every wait is then on data issued at least a stage earlier.
  auto stage = [&](const int h, char* xcur, char* xnext, int st) {
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
      const int lc = kg * (4 * CPW) + 4 * c + g;  // logical 16-B chunk holding this lane's 8 k values
      bf16x8 b[MT];
#pragma unroll
      for (int t = 0; t < MT; ++t)
        b[t] = *reinterpret_cast<const bf16x8*>(xcur + (16 * t + li) * ROWB + 16 * (lc ^ li));
#pragma unroll
      for (int a = 0; a < RT; ++a) {
#pragma unroll
        for (int t = 0; t < MT; ++t) acc[a][t] = mfma16(wr[h][a][c], b[t], acc[a][t]);
        load_w(h, st + 2, a, c);
        // pin the reload right behind its MFMAs: left alone the scheduler sinks all reloads to the
        // end of the stage, halving the bytes in flight
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    store_x(xnext);
    load_x(st + 2);
    __syncthreads();
  };

  // Prologue issue order W(0) X(0) W(1) X(1), pinned: the compiler's vmcnt for the loop is the
  // merge of this order and the steady state, so W(0) must be as old here as a slot is there.
#pragma unroll
  for (int a = 0; a < RT; ++a)
#pragma unroll
    for (int c = 0; c < CPW; ++c) load_w(0, 0, a, c);
  __builtin_amdgcn_sched_barrier(0);
  load_x(0);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int a = 0; a < RT; ++a)
#pragma unroll
    for (int c = 0; c < CPW; ++c) load_w(1, 1, a, c);
  __builtin_amdgcn_sched_barrier(0);
  store_x(xs0);
  load_x(1);
  __syncthreads();
  for (int st = 0; st < nst; st += 2) {
    stage(0, xs0, xs1, st);
    if (st + 1 >= nst) break;
    stage(1, xs1, xs0, st + 1);
  }

  // ---- cross-wave reduction.  acc[a][t][r] = partial C[m = 16t + li][n = 16 (RT rg + a) + 4g + r];
  // wave w's partial goes to red_w[m][64] (xs0 holds waves 0-1, xs1 waves 2-3) with the 4-float
  // column groups XOR-swizzled by m so the 16 lanes of a row group hit distinct banks.
  auto red = [&](int q) -> float* {
    return (q < 2 ? reinterpret_cast<float*>(xs0) : reinterpret_cast<float*>(xs1)) + (q & 1) * MP * 64;
  };
  {
    float* mine = red(w);
#pragma unroll
    for (int a = 0; a < RT; ++a)
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const int m = 16 * t + li;
        const int col = (16 * (RT * rg + a) + 4 * g) ^ (4 * (m & 15));
        *reinterpret_cast<f32x4*>(mine + m * 64 + col) = acc[a][t];
      }
  }
  __syncthreads();
  // sum over the k groups for 4 consecutive columns [c4, c4+4) of row m
  auto tile4 = [&](int m, int c4) {
    const int col = c4 ^ (4 * (m & 15));
    const int w0 = (c4 / (16 * RT)) * NKG;  // first wave of the column's row group
    f32x4 v = *reinterpret_cast<const f32x4*>(red(w0) + m * 64 + col);
#pragma unroll
    for (int q = 1; q < NKG; ++q) {
      const f32x4 u = *reinterpret_cast<const f32x4*>(red(w0 + q) + m * 64 + col);
      v += u;
    }
    return v;
  };

  if (p.S > 1) {
    float* slab = (float*)p.out + (size_t)slice * p.M * p.N;
    for (int e = tid; e < MP * 16; e += 256) {
      const int m = e >> 4, c4 = (e & 15) * 4;
      if (m < p.M) *reinterpret_cast<f32x4*>(slab + (size_t)m * p.N + n0 + c4) = tile4(m, c4);
    }
    return;
  }
  bf16* out = (bf16*)p.out;
  if (p.epi == SK_EPI_SWIGLU) {
    // rows [32i, 32i+16) gate, [32i+16, 32i+32) up -> output columns n0/2 + 16i + j
    for (int e = tid; e < MP * 8; e += 256) {
      const int m = e >> 3, part = e & 7;  // part: 4 output columns
      if (m >= p.M) continue;
      const int i = part >> 2, j0 = (part & 3) * 4;
      const f32x4 gt = tile4(m, 32 * i + j0), up = tile4(m, 32 * i + 16 + j0);
      float o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = silu_f(gt[j]) * up[j];
      u32x2 v;
      v[0] = pack2bf(o[0], o[1]);
      v[1] = pack2bf(o[2], o[3]);
      *reinterpret_cast<u32x2*>(out + (size_t)m * p.ldo + n0 / 2 + 16 * i + j0) = v;
    }
    return;
  }
  for (int e = tid; e < MP * 8; e += 256) {
    const int m = e >> 3, c8 = (e & 7) * 8;
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

// Sum S fp32 slabs -> bf16 (optionally + residual).  Matches a bf16 GEMM: the sum is rounded to
// bf16 before the residual add.
__global__ __launch_bounds__(256) void skinny_reduce_kernel(bf16* out, long ldo, const float* slabs, int S, int M,
                                                            int N, const bf16* residual, long ldr) {
  const size_t e = ((size_t)blockIdx.x * 256 + threadIdx.x) * 8;
  const size_t total = (size_t)M * N;
  if (e >= total) return;
  const int m = (int)(e / N), n = (int)(e % N);
  float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < S; ++s) {
    const f32x4* src = reinterpret_cast<const f32x4*>(slabs + (size_t)s * total + e);
    const f32x4 a = src[0], b = src[1];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      o[j] += a[j];
      o[4 + j] += b[j];
    }
  }
  if (residual) {
    float r[8];
    unpack8(*reinterpret_cast<const u32x4*>(residual + (size_t)m * ldr + n), r);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = bf2f(f2bf(o[j])) + r[j];
  }
  *reinterpret_cast<u32x4*>(out + (size_t)m * ldo + n) = pack8(o);
}

template <bool NT_W>
static void launch_skinny(const SkinnyParams& p, hipStream_t s) {
  const dim3 grid((p.N / 64) * p.S);
  // RT (row tiles per wave) trades accumulator VGPRs for fewer LDS fragment reads
  if (p.M <= 16)
    hipLaunchKernelGGL((skinny_gemm_kernel<1, 4, NT_W>), grid, dim3(256), 0, s, p);
  else if (p.M <= 32)
    hipLaunchKernelGGL((skinny_gemm_kernel<2, 4, NT_W>), grid, dim3(256), 0, s, p);
  else if (p.M <= 64)
    hipLaunchKernelGGL((skinny_gemm_kernel<4, 2, NT_W>), grid, dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL((skinny_gemm_kernel<8, 2, NT_W>), grid, dim3(256), 0, s, p);
}

int skinny_gemm(const void* X, long ldx, const void* W, long ldw, void* out, long ldo, const void* residual, long ldr,
                int M, int N, int K, int S, int epilogue, hipStream_t s, int nt_weights) {
  if (M <= 0 || N <= 0) return 0;
  if (M > 128 || N % 64 || S < 1 || K % (S * SK_KSTAGE) || ldx % 8 || ldw % 8 || ldo % 8) return hipErrorInvalidValue;
  if (epilogue != SK_EPI_NONE && epilogue != SK_EPI_SWIGLU) return hipErrorInvalidValue;
  if (S > 1 && (epilogue != SK_EPI_NONE || residual)) return hipErrorInvalidValue;
  if (residual && ldr % 8) return hipErrorInvalidValue;
  SkinnyParams p;
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
  if (nt_weights)
    launch_skinny<true>(p, s);
  else
    launch_skinny<false>(p, s);
  return hipGetLastError();
}

int skinny_reduce(void* out, long ldo, const float* slabs, int S, int M, int N, const void* residual, long ldr,
                  hipStream_t s) {
  if (M <= 0 || N <= 0) return 0;
  if (N % 8 || ldo % 8 || (residual && ldr % 8)) return hipErrorInvalidValue;
  const size_t total8 = (size_t)M * N / 8;
  hipLaunchKernelGGL(skinny_reduce_kernel, dim3((unsigned)((total8 + 255) / 256)), dim3(256), 0, s, (bf16*)out, ldo,
                     slabs, S, M, N, (const bf16*)residual, ldr);
  return hipGetLastError();
}

}  // namespace dab

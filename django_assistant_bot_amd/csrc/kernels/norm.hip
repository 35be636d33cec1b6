// Row-wise normalisation, embedding and pooling kernels (memory-bound; 16-B vectorised rows).
//
// Replaces the implicit HF ops of the reference encoder / generator:
//   * Llama RMSNorm with the residual add fused in           (N7)
//   * BERT post-LN: residual add + LayerNorm fused          (N3)
//   * BERT embedding gather + sum + LayerNorm fused          (N2)
//   * masked mean-pool (+ optional L2 normalise)             (N6; reference embedders/transformers.py:25)
#include "common.h"
#include "launchers.h"

namespace dab {

// One block per row; each thread owns VPT 8-element vectors kept in registers between the
// reduction and the scaling pass, so the row is read from HBM exactly once.
template <int NT, int VPT>
__global__ __launch_bounds__(NT) void rmsnorm_kernel(bf16* __restrict__ out, bf16* __restrict__ res_out,
                                                     const bf16* __restrict__ x, const bf16* __restrict__ res_in,
                                                     const bf16* __restrict__ w, int cols, float eps) {
  __shared__ float red[NT / 64];
  const size_t row = blockIdx.x;
  const int nvec = cols >> 3;
  const u32x4* xr = reinterpret_cast<const u32x4*>(x + row * cols);
  const u32x4* rr = reinterpret_cast<const u32x4*>(res_in + row * cols);
  float v[VPT][8];
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int i = threadIdx.x + k * NT;
    if (i < nvec) {
      unpack8(xr[i], v[k]);
      if (res_in) {
        float r[8];
        unpack8(rr[i], r);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[k][j] = bf2f(f2bf(v[k][j] + r[j]));  // residual kept in bf16 like HF
        reinterpret_cast<u32x4*>(res_out + row * cols)[i] = pack8(v[k]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[k][j] * v[k][j];
    }
  }
  const float tot = block_sum<NT>(ss, red);
  const float inv = rsqrtf(tot / (float)cols + eps);
  const u32x4* wr = reinterpret_cast<const u32x4*>(w);
  u32x4* orow = reinterpret_cast<u32x4*>(out + row * cols);
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int i = threadIdx.x + k * NT;
    if (i < nvec) {
      float g[8], o[8];
      unpack8(wr[i], g);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = v[k][j] * inv * g[j];
      orow[i] = pack8(o);
    }
  }
}

// Same as rmsnorm_kernel but x arrives as S fp32 split-K slabs of the producing projection:
// x = bf16(sum_s slabs[s]) (the rounding a bf16 GEMM output would have had).
// Latency-bound at decode sizes (one row per workgroup, 128-256 rows): everything a thread reads --
// residual, gain and the slab chunks of KG vectors at once -- is issued before the first add, so the
// kernel waits out one memory round trip instead of one per slab group plus one for the gain after
// the row reduction.  Out-of-range vectors load a clamped (valid) address and are masked.
template <int NT, int VPT, typename ST = float>
__global__ __launch_bounds__(NT) void rmsnorm_slab_kernel(bf16* __restrict__ out, bf16* __restrict__ res_out,
                                                          const ST* __restrict__ slabs, int S, long slab_stride,
                                                          const bf16* __restrict__ res_in, const bf16* __restrict__ w,
                                                          int cols, float eps) {
  constexpr int KG = VPT < 2 ? VPT : 2;  // vectors whose slab loads are in flight together
  __shared__ float red[NT / 64];
  const size_t row = blockIdx.x;
  const int nvec = cols >> 3;
  const u32x4* rr = reinterpret_cast<const u32x4*>(res_in + row * cols);
  const u32x4* wr = reinterpret_cast<const u32x4*>(w);
  int iv[VPT];
  bool ok[VPT];
  u32x4 graw[VPT], rraw[VPT];
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int i = threadIdx.x + k * NT;
    ok[k] = i < nvec;
    iv[k] = ok[k] ? i : nvec - 1;
    graw[k] = wr[iv[k]];
    if (res_in) rraw[k] = rr[iv[k]];
  }
  float v[VPT][8];
#pragma unroll
  for (int k = 0; k < VPT; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) v[k][j] = 0.f;
  const ST* base = slabs + row * cols;
#pragma unroll
  for (int k0 = 0; k0 < VPT; k0 += KG) {
    int sl = 0;
    for (; sl + 8 <= S; sl += 8) {
      SlabVec8<ST> a[KG][8];
#pragma unroll
      for (int kk = 0; kk < KG; ++kk)
#pragma unroll
        for (int q = 0; q < 8; ++q) a[kk][q].load(base + (size_t)(sl + q) * slab_stride + (size_t)iv[k0 + kk] * 8);
      __builtin_amdgcn_sched_barrier(0);  // keep every load of the round ahead of the adds
#pragma unroll
      for (int kk = 0; kk < KG; ++kk)
#pragma unroll
        for (int q = 0; q < 8; ++q) a[kk][q].add_to(v[k0 + kk]);
    }
    for (; sl + 4 <= S; sl += 4) {
      SlabVec8<ST> a[KG][4];
#pragma unroll
      for (int kk = 0; kk < KG; ++kk)
#pragma unroll
        for (int q = 0; q < 4; ++q) a[kk][q].load(base + (size_t)(sl + q) * slab_stride + (size_t)iv[k0 + kk] * 8);
      __builtin_amdgcn_sched_barrier(0);  // keep every load of the round ahead of the adds
#pragma unroll
      for (int kk = 0; kk < KG; ++kk)
#pragma unroll
        for (int q = 0; q < 4; ++q) a[kk][q].add_to(v[k0 + kk]);
    }
    for (; sl < S; ++sl) {
      SlabVec8<ST> a[KG];
#pragma unroll
      for (int kk = 0; kk < KG; ++kk) a[kk].load(base + (size_t)sl * slab_stride + (size_t)iv[k0 + kk] * 8);
#pragma unroll
      for (int kk = 0; kk < KG; ++kk) a[kk].add_to(v[k0 + kk]);
    }
  }
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[k][j] = bf2f(f2bf(v[k][j]));
    if (res_in) {
      float r[8];
      unpack8(rraw[k], r);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[k][j] = bf2f(f2bf(v[k][j] + r[j]));
      if (ok[k]) reinterpret_cast<u32x4*>(res_out + row * cols)[iv[k]] = pack8(v[k]);
    }
    if (ok[k]) {
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[k][j] * v[k][j];
    }
  }
  const float tot = block_sum<NT>(ss, red);
  const float inv = rsqrtf(tot / (float)cols + eps);
  u32x4* orow = reinterpret_cast<u32x4*>(out + row * cols);
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    if (ok[k]) {
      float g[8], o[8];
      unpack8(graw[k], g);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = v[k][j] * inv * g[j];
      orow[iv[k]] = pack8(o);
    }
  }
}

// out = LayerNorm(x + res) * gamma + beta   (BERT post-LN; two-pass mean/var in registers)
template <int NT, int VPT>
__global__ __launch_bounds__(NT) void layernorm_kernel(bf16* __restrict__ out, const bf16* __restrict__ x,
                                                       const bf16* __restrict__ res_in, const bf16* __restrict__ gamma,
                                                       const bf16* __restrict__ beta, int cols, float eps) {
  __shared__ float red[NT / 64];
  const size_t row = blockIdx.x;
  const int nvec = cols >> 3;
  const u32x4* xr = reinterpret_cast<const u32x4*>(x + row * cols);
  const u32x4* rr = reinterpret_cast<const u32x4*>(res_in + row * cols);
  float v[VPT][8];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int i = threadIdx.x + k * NT;
    if (i < nvec) {
      unpack8(xr[i], v[k]);
      if (res_in) {
        float r[8];
        unpack8(rr[i], r);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[k][j] += r[j];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[k][j];
    }
  }
  const float mean = block_sum<NT>(s, red) / (float)cols;
  float sq = 0.f;
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int i = threadIdx.x + k * NT;
    if (i < nvec) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[k][j] - mean;
        sq += d * d;
      }
    }
  }
  const float inv = rsqrtf(block_sum<NT>(sq, red) / (float)cols + eps);
  const u32x4* gr = reinterpret_cast<const u32x4*>(gamma);
  const u32x4* br = reinterpret_cast<const u32x4*>(beta);
  u32x4* orow = reinterpret_cast<u32x4*>(out + row * cols);
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int i = threadIdx.x + k * NT;
    if (i < nvec) {
      float g[8], b[8], o[8];
      unpack8(gr[i], g);
      unpack8(br[i], b);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (v[k][j] - mean) * inv * g[j] + b[j];
      orow[i] = pack8(o);
    }
  }
}

// Same LayerNorm, one WAVE per row for encoder widths (cols = 256 CPL: bge-base 768, bge-large
// 1024): every lane holds CPL 4-element chunks (lane-strided, so each load instruction is one
// coalesced 512-B run), the two row sums are wave shuffles (no LDS, no barrier), a wave takes RPW
// rows with all their loads in flight at once and a 256-thread workgroup 4 RPW rows.  Per 64k x 768
// LN in the bge encoder (rocprof, profiles/embed_study.md): row-per-workgroup kernel 45.2 us, RPW 1
// 41.0, RPW 2 34.1 (5.9 TB/s), RPW 4 34.0.  The row-per-workgroup kernel above left a quarter of its 128 lanes
// idle at 768 columns and waited on two workgroup barriers per row.
template <int CPL, int RPW>
__global__ __launch_bounds__(256) void layernorm_rows_kernel(bf16* __restrict__ out, const bf16* __restrict__ x,
                                                            const bf16* __restrict__ res_in,
                                                            const bf16* __restrict__ gamma,
                                                            const bf16* __restrict__ beta, int rows, float eps) {
  constexpr int cols = 256 * CPL;
  const int lane = threadIdx.x & 63;
  const size_t row0 = ((size_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW;
  if (row0 >= (size_t)rows) return;  // whole wave
  // every row's loads are issued before the first reduction (RPW rows of one wave in flight)
  u32x2 xv[RPW][CPL], rv[RPW][CPL];
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    const size_t row = min(row0 + r, (size_t)rows - 1);
    const u32x2* xr = reinterpret_cast<const u32x2*>(x + row * cols);
    const u32x2* rr = reinterpret_cast<const u32x2*>(res_in + row * cols);
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      xv[r][c] = xr[c * 64 + lane];
      if (res_in) rv[r][c] = rr[c * 64 + lane];
    }
  }
  const u32x2* gr = reinterpret_cast<const u32x2*>(gamma);
  const u32x2* br = reinterpret_cast<const u32x2*>(beta);
  u32x2 gv[CPL], bv[CPL];
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    gv[c] = gr[c * 64 + lane];
    bv[c] = br[c * 64 + lane];
  }
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    if (row0 + r >= (size_t)rows) break;  // wave-uniform
    float v[CPL][4];
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        v[c][2 * j] = __uint_as_float(xv[r][c][j] << 16);
        v[c][2 * j + 1] = __uint_as_float(xv[r][c][j] & 0xffff0000u);
        if (res_in) {
          v[c][2 * j] += __uint_as_float(rv[r][c][j] << 16);
          v[c][2 * j + 1] += __uint_as_float(rv[r][c][j] & 0xffff0000u);
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) s += v[c][j];
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d, 64);
    const float mean = s / (float)cols;
    float sq = 0.f;
#pragma unroll
    for (int c = 0; c < CPL; ++c)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float d = v[c][j] - mean;
        sq += d * d;
      }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) sq += __shfl_xor(sq, d, 64);
    const float inv = rsqrtf(sq / (float)cols + eps);
    u32x2* orow = reinterpret_cast<u32x2*>(out + (row0 + r) * cols);
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      float o[4];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        o[2 * j] = (v[c][2 * j] - mean) * inv * __uint_as_float(gv[c][j] << 16) + __uint_as_float(bv[c][j] << 16);
        o[2 * j + 1] = (v[c][2 * j + 1] - mean) * inv * __uint_as_float(gv[c][j] & 0xffff0000u) +
                       __uint_as_float(bv[c][j] & 0xffff0000u);
      }
      orow[c * 64 + lane] = u32x2{pack2bf(o[0], o[1]), pack2bf(o[2], o[3])};
    }
  }
}

// BERT embeddings: LN(word[id] + pos[pos_id] + type[type_id]) fused; type ids default to 0.
template <int NT, int VPT>
__global__ __launch_bounds__(NT) void bert_embed_kernel(bf16* __restrict__ out, const int* __restrict__ ids,
                                                        const int* __restrict__ pos_ids, const int* __restrict__ type_ids,
                                                        const bf16* __restrict__ word, const bf16* __restrict__ pos,
                                                        const bf16* __restrict__ type, const bf16* __restrict__ gamma,
                                                        const bf16* __restrict__ beta, int cols, float eps) {
  __shared__ float red[NT / 64];
  const size_t row = blockIdx.x;
  const int nvec = cols >> 3;
  const size_t id = (size_t)ids[row];
  const size_t pid = (size_t)pos_ids[row];
  const size_t tid = type_ids ? (size_t)type_ids[row] : 0;
  const u32x4* wr = reinterpret_cast<const u32x4*>(word + id * cols);
  const u32x4* pr = reinterpret_cast<const u32x4*>(pos + pid * cols);
  const u32x4* tr = reinterpret_cast<const u32x4*>(type + tid * cols);
  float v[VPT][8];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int i = threadIdx.x + k * NT;
    if (i < nvec) {
      float a[8], b[8];
      unpack8(wr[i], v[k]);
      unpack8(pr[i], a);
      unpack8(tr[i], b);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[k][j] += a[j] + b[j];
        s += v[k][j];
      }
    }
  }
  const float mean = block_sum<NT>(s, red) / (float)cols;
  float sq = 0.f;
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int i = threadIdx.x + k * NT;
    if (i < nvec) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[k][j] - mean;
        sq += d * d;
      }
    }
  }
  const float inv = rsqrtf(block_sum<NT>(sq, red) / (float)cols + eps);
  const u32x4* gr = reinterpret_cast<const u32x4*>(gamma);
  const u32x4* br = reinterpret_cast<const u32x4*>(beta);
  u32x4* orow = reinterpret_cast<u32x4*>(out + row * cols);
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int i = threadIdx.x + k * NT;
    if (i < nvec) {
      float g[8], b[8], o[8];
      unpack8(gr[i], g);
      unpack8(br[i], b);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (v[k][j] - mean) * inv * g[j] + b[j];
      orow[i] = pack8(o);
    }
  }
}

// Row gather (token embedding lookup for the decoder).
__global__ __launch_bounds__(256) void embed_gather_kernel(bf16* __restrict__ out, const int* __restrict__ ids,
                                                           const bf16* __restrict__ table, int cols) {
  const size_t row = blockIdx.y;
  const int nvec = cols >> 3;
  const u32x4* src = reinterpret_cast<const u32x4*>(table + (size_t)ids[row] * cols);
  u32x4* dst = reinterpret_cast<u32x4*>(out + row * cols);
  for (int i = blockIdx.x * 256 + threadIdx.x; i < nvec; i += gridDim.x * 256) dst[i] = src[i];
}

// Mean over the tokens of each packed sequence [cu[b], cu[b+1]) (all tokens incl. [CLS]/[SEP], as the
// reference does), optional L2 normalisation; fp32 output [B, cols] and optional bf16 copy.
__global__ __launch_bounds__(256) void mean_pool_kernel(float* __restrict__ out, bf16* __restrict__ out_bf16,
                                                        const bf16* __restrict__ hidden, const int* __restrict__ cu,
                                                        int cols, int normalize) {
  __shared__ float red[4];
  const int b = blockIdx.x;
  const int start = cu[b], end = cu[b + 1];
  const int nvec = cols >> 3;
  const float inv_n = end > start ? 1.f / (float)(end - start) : 0.f;
  float acc[2][8];
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int i = threadIdx.x + k * 256;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[k][j] = 0.f;
    if (i < nvec) {
      for (int t = start; t < end; ++t) {
        float v[8];
        unpack8(reinterpret_cast<const u32x4*>(hidden + (size_t)t * cols)[i], v);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[k][j] += v[j];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        acc[k][j] *= inv_n;
        ss += acc[k][j] * acc[k][j];
      }
    }
  }
  float scale = 1.f;
  if (normalize) {
    const float tot = block_sum<256>(ss, red);
    scale = tot > 0.f ? rsqrtf(tot) : 0.f;
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int i = threadIdx.x + k * 256;
    if (i < nvec) {
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        o[j] = acc[k][j] * scale;
        out[(size_t)b * cols + i * 8 + j] = o[j];
      }
      if (out_bf16) reinterpret_cast<u32x4*>(out_bf16 + (size_t)b * cols)[i] = pack8(o);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// launchers

#define DAB_ROW_DISPATCH(KERNEL, ROWS, COLS, STREAM, ...)                                        \
  do {                                                                                          \
    const int nvec_ = (COLS) / 8;                                                               \
    if (nvec_ <= 64)                                                                            \
      hipLaunchKernelGGL((KERNEL<64, 1>), dim3(ROWS), dim3(64), 0, STREAM, __VA_ARGS__);        \
    else if (nvec_ <= 128)                                                                      \
      hipLaunchKernelGGL((KERNEL<128, 1>), dim3(ROWS), dim3(128), 0, STREAM, __VA_ARGS__);      \
    else if (nvec_ <= 256)                                                                      \
      hipLaunchKernelGGL((KERNEL<256, 1>), dim3(ROWS), dim3(256), 0, STREAM, __VA_ARGS__);      \
    else if (nvec_ <= 512)                                                                      \
      hipLaunchKernelGGL((KERNEL<256, 2>), dim3(ROWS), dim3(256), 0, STREAM, __VA_ARGS__);      \
    else if (nvec_ <= 1024)                                                                     \
      hipLaunchKernelGGL((KERNEL<256, 4>), dim3(ROWS), dim3(256), 0, STREAM, __VA_ARGS__);      \
    else                                                                                        \
      hipLaunchKernelGGL((KERNEL<256, 8>), dim3(ROWS), dim3(256), 0, STREAM, __VA_ARGS__);      \
  } while (0)

int rmsnorm(void* out, void* res_out, const void* x, const void* res_in, const void* w, int rows, int cols, float eps,
            hipStream_t s) {
  if (rows <= 0) return 0;
  if (cols % 8 || cols > 16384) return hipErrorInvalidValue;
  DAB_ROW_DISPATCH(rmsnorm_kernel, rows, cols, s, (bf16*)out, (bf16*)res_out, (const bf16*)x, (const bf16*)res_in,
                   (const bf16*)w, cols, eps);
  return hipGetLastError();
}

// DAB_ROW_DISPATCH for a kernel templated <NT, VPT, T>
#define DAB_ROW_DISPATCH_T(KERNEL, T, ROWS, COLS, STREAM, ...)                                   \
  do {                                                                                          \
    const int nvec_ = (COLS) / 8;                                                               \
    if (nvec_ <= 64)                                                                            \
      hipLaunchKernelGGL((KERNEL<64, 1, T>), dim3(ROWS), dim3(64), 0, STREAM, __VA_ARGS__);     \
    else if (nvec_ <= 128)                                                                      \
      hipLaunchKernelGGL((KERNEL<128, 1, T>), dim3(ROWS), dim3(128), 0, STREAM, __VA_ARGS__);   \
    else if (nvec_ <= 256)                                                                      \
      hipLaunchKernelGGL((KERNEL<256, 1, T>), dim3(ROWS), dim3(256), 0, STREAM, __VA_ARGS__);   \
    else if (nvec_ <= 512)                                                                      \
      hipLaunchKernelGGL((KERNEL<256, 2, T>), dim3(ROWS), dim3(256), 0, STREAM, __VA_ARGS__);   \
    else if (nvec_ <= 1024)                                                                     \
      hipLaunchKernelGGL((KERNEL<256, 4, T>), dim3(ROWS), dim3(256), 0, STREAM, __VA_ARGS__);   \
    else                                                                                        \
      hipLaunchKernelGGL((KERNEL<256, 8, T>), dim3(ROWS), dim3(256), 0, STREAM, __VA_ARGS__);   \
  } while (0)

template <typename ST>
static int rmsnorm_slabs_t(void* out, void* res_out, const ST* slabs, int S, long slab_stride, const void* res_in,
                           const void* w, int rows, int cols, float eps, hipStream_t s) {
  // 4096-wide rows (Llama-3-8B decode, 8 slabs): 512 threads x 1 vector instead of 256 x 2 -- twice
  // the waves issuing the slab loads: 4.97 vs 5.52 us per call at 128 rows (benchmarks/slab_norm_bench.py)
  if (cols / 8 > 256 && cols / 8 <= 512) {
    hipLaunchKernelGGL((rmsnorm_slab_kernel<512, 1, ST>), dim3(rows), dim3(512), 0, s, (bf16*)out, (bf16*)res_out,
                       slabs, S, slab_stride, (const bf16*)res_in, (const bf16*)w, cols, eps);
    return hipGetLastError();
  }
  DAB_ROW_DISPATCH_T(rmsnorm_slab_kernel, ST, rows, cols, s, (bf16*)out, (bf16*)res_out, slabs, S, slab_stride,
                     (const bf16*)res_in, (const bf16*)w, cols, eps);
  return hipGetLastError();
}

// slab_bf16: bf16 slabs (stream_gemm(..., slab_bf16)), else fp32
int rmsnorm_slabs(void* out, void* res_out, const void* slabs, int S, long slab_stride, const void* res_in,
                  const void* w, int rows, int cols, float eps, hipStream_t s, int slab_bf16) {
  if (rows <= 0) return 0;
  if (cols % 8 || cols > 16384 || S < 1 || slab_stride % 8) return hipErrorInvalidValue;
  if (slab_bf16)
    return rmsnorm_slabs_t(out, res_out, (const bf16*)slabs, S, slab_stride, res_in, w, rows, cols, eps, s);
  return rmsnorm_slabs_t(out, res_out, (const float*)slabs, S, slab_stride, res_in, w, rows, cols, eps, s);
}

int layernorm(void* out, const void* x, const void* res_in, const void* gamma, const void* beta, int rows, int cols,
              float eps, hipStream_t s) {
  if (rows <= 0) return 0;
  if (cols % 8 || cols > 16384) return hipErrorInvalidValue;
  // encoder widths: one wave per LN_RPW rows, 4 waves per workgroup
  constexpr int LN_RPW = 2;  // 4 measured the same (34.0 us)
  const dim3 g4((rows + 4 * LN_RPW - 1) / (4 * LN_RPW));
  if (cols == 768) {
    hipLaunchKernelGGL((layernorm_rows_kernel<3, LN_RPW>), g4, dim3(256), 0, s, (bf16*)out, (const bf16*)x,
                       (const bf16*)res_in, (const bf16*)gamma, (const bf16*)beta, rows, eps);
    return hipGetLastError();
  }
  if (cols == 1024) {
    hipLaunchKernelGGL((layernorm_rows_kernel<4, LN_RPW>), g4, dim3(256), 0, s, (bf16*)out, (const bf16*)x,
                       (const bf16*)res_in, (const bf16*)gamma, (const bf16*)beta, rows, eps);
    return hipGetLastError();
  }
  DAB_ROW_DISPATCH(layernorm_kernel, rows, cols, s, (bf16*)out, (const bf16*)x, (const bf16*)res_in,
                   (const bf16*)gamma, (const bf16*)beta, cols, eps);
  return hipGetLastError();
}

int bert_embed(void* out, const int* ids, const int* pos_ids, const int* type_ids, const void* word, const void* pos,
               const void* type, const void* gamma, const void* beta, int rows, int cols, float eps, hipStream_t s) {
  if (rows <= 0) return 0;
  if (cols % 8 || cols > 16384) return hipErrorInvalidValue;
  DAB_ROW_DISPATCH(bert_embed_kernel, rows, cols, s, (bf16*)out, ids, pos_ids, type_ids, (const bf16*)word,
                   (const bf16*)pos, (const bf16*)type, (const bf16*)gamma, (const bf16*)beta, cols, eps);
  return hipGetLastError();
}

int embed_gather(void* out, const int* ids, const void* table, int rows, int cols, hipStream_t s) {
  if (rows <= 0) return 0;
  if (cols % 8) return hipErrorInvalidValue;
  const int nvec = cols / 8;
  dim3 grid(div_up_host(nvec, 256), rows);
  hipLaunchKernelGGL(embed_gather_kernel, grid, dim3(256), 0, s, (bf16*)out, ids, (const bf16*)table, cols);
  return hipGetLastError();
}

int mean_pool(float* out, void* out_bf16, const void* hidden, const int* cu_seqlens, int batch, int cols,
              int normalize, hipStream_t s) {
  if (batch <= 0) return 0;
  if (cols % 8 || cols > 4096) return hipErrorInvalidValue;
  hipLaunchKernelGGL(mean_pool_kernel, dim3(batch), dim3(256), 0, s, out, (bf16*)out_bf16, (const bf16*)hidden,
                     cu_seqlens, cols, normalize);
  return hipGetLastError();
}

}  // namespace dab

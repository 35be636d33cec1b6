// Element-wise kernels of the encoder / decoder layers (memory-bound, 16 B per lane):
//   * erf-GELU with optional fused bias (BERT FFN, N4)
//   * SwiGLU  silu(gate) * up (Llama MLP, N11)
//   * RoPE on q/k fused with the paged KV-cache write (N8 + N9 write half)
#include "common.h"
#include "launchers.h"

namespace dab {

__global__ __launch_bounds__(256) void gelu_kernel(bf16* __restrict__ out, const bf16* __restrict__ x,
                                                   const bf16* __restrict__ bias, size_t nvec, int cols) {
  const int cvec = cols >> 3;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < nvec; i += (size_t)gridDim.x * 256) {
    float v[8];
    unpack8(reinterpret_cast<const u32x4*>(x)[i], v);
    if (bias) {
      float b[8];
      unpack8(reinterpret_cast<const u32x4*>(bias)[i % cvec], b);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += b[j];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = gelu_erf(v[j]);
    reinterpret_cast<u32x4*>(out)[i] = pack8(v);
  }
}

// x: [rows, 2F] = [gate | up] (or, interleaved, 16-column groups [g16 | u16 | g16 | ...]); out: [rows, F]
__global__ __launch_bounds__(256) void silu_mul_kernel(bf16* __restrict__ out, const bf16* __restrict__ x,
                                                       size_t rows, int F, int interleaved) {
  const int fvec = F >> 3;
  const size_t nvec = rows * fvec;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < nvec; i += (size_t)gridDim.x * 256) {
    const size_t r = i / fvec;
    const int c = (int)(i - r * fvec);
    const u32x4* xr = reinterpret_cast<const u32x4*>(x + r * 2 * F);
    float g[8], u[8], o[8];
    if (interleaved) {
      const int gc = 4 * (c >> 1) + (c & 1);  // 8-col chunk c of the output -> gate chunk in [g16|u16] pairs
      unpack8(xr[gc], g);
      unpack8(xr[gc + 2], u);
    } else {
      unpack8(xr[c], g);
      unpack8(xr[c + fvec], u);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = silu_f(g[j]) * u[j];
    reinterpret_cast<u32x4*>(out + r * F)[c] = pack8(o);
  }
}

// qkv: [T, (Hq + 2*Hkv) * D] rows (row stride `ld` elements). Each thread handles 8 rotation pairs
// (elements i..i+7 and i+D/2..i+D/2+7) of one (token, head). q heads go to q_out [T, Hq, D] rotated,
// k heads are rotated and written to the paged cache, v heads copied to the paged cache.
// cos_sin: [max_pos, D/2] float2 (cos, sin); slots[t] = block * block_size + offset (or < 0: skip).
// Cache layout: [num_blocks, Hkv, block_size, D].
template <typename ST>
__global__ __launch_bounds__(256) void rope_kv_kernel(const bf16* __restrict__ qkv, int ld,
                                                      const int* __restrict__ positions,
                                                      const float2* __restrict__ cos_sin, bf16* __restrict__ q_out,
                                                      bf16* __restrict__ k_cache, bf16* __restrict__ v_cache,
                                                      const int64_t* __restrict__ slots, int T, int Hq, int Hkv, int D,
                                                      int block_size, const ST* __restrict__ slabs, int S,
                                                      long slab_stride) {
  const int per_head = D >> 4;  // threads per head
  const int heads = Hq + 2 * Hkv;
  const int h0 = q_out ? 0 : Hq;  // no q output: k / v heads only (the attention rotates q itself)
  const int hrun = heads - h0;
  const size_t total = (size_t)T * hrun * per_head;
  const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  const int c = (int)(idx % per_head);
  const size_t th = idx / per_head;
  const int h = h0 + (int)(th % hrun);
  const int t = (int)(th / hrun);
  const int half = D >> 1;
  const int i0 = c * 8;
  // rotation and cache slot first (pos -> cos/sin is a dependent chain): their round trips overlap
  // the slab loads instead of following them
  float2 cs[8];
  rope_cs(cos_sin, positions[t], half, i0, cs);
  const int64_t slot = h >= Hq ? slots[t] : 0;
  float x1[8], x2[8];
  rope_chunk(qkv, slabs, S, slab_stride, ld, t, h, D, i0, cs, h < Hq + Hkv, x1, x2);
  bf16* dst;
  if (h < Hq) {
    dst = q_out + ((size_t)t * Hq + h) * D;
  } else {
    if (slot < 0) return;
    const int64_t blk = slot / block_size, off = slot - blk * block_size;
    const int kh = (h < Hq + Hkv) ? h - Hq : h - Hq - Hkv;
    bf16* cache = (h < Hq + Hkv) ? k_cache : v_cache;
    dst = cache + (((size_t)blk * Hkv + kh) * block_size + off) * D;
  }
  *reinterpret_cast<u32x4*>(dst + i0) = pack8(x1);
  *reinterpret_cast<u32x4*>(dst + i0 + half) = pack8(x2);
}

static inline int grid_for(size_t nvec) {
  size_t g = (nvec + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (int)g;
}

int gelu(void* out, const void* x, const void* bias, size_t rows, int cols, hipStream_t s) {
  if (cols % 8) return hipErrorInvalidValue;
  const size_t nvec = rows * (size_t)(cols / 8);
  if (!nvec) return 0;
  hipLaunchKernelGGL(gelu_kernel, dim3(grid_for(nvec)), dim3(256), 0, s, (bf16*)out, (const bf16*)x,
                     (const bf16*)bias, nvec, cols);
  return hipGetLastError();
}

int silu_mul(void* out, const void* x, size_t rows, int F, hipStream_t s, int interleaved) {
  if (F % 8 || (interleaved && F % 16)) return hipErrorInvalidValue;
  const size_t nvec = rows * (size_t)(F / 8);
  if (!nvec) return 0;
  hipLaunchKernelGGL(silu_mul_kernel, dim3(grid_for(nvec)), dim3(256), 0, s, (bf16*)out, (const bf16*)x, rows, F,
                     interleaved);
  return hipGetLastError();
}

int rope_kv_write(const void* qkv, int ld, const int* positions, const void* cos_sin, void* q_out, void* k_cache,
                  void* v_cache, const int64_t* slots, int T, int Hq, int Hkv, int D, int block_size, hipStream_t s,
                  const void* slabs, int S, long slab_stride, int slab_bf16) {
  if (T <= 0) return 0;
  if (D % 16 || ld % 8 || (slabs && (S < 1 || slab_stride % 8))) return hipErrorInvalidValue;
  const size_t total = (size_t)T * (q_out ? Hq + 2 * Hkv : 2 * Hkv) * (D / 16);
  const dim3 grid((unsigned)((total + 255) / 256));
  if (slabs && slab_bf16)
    hipLaunchKernelGGL(rope_kv_kernel<bf16>, grid, dim3(256), 0, s, (const bf16*)qkv, ld, positions,
                       (const float2*)cos_sin, (bf16*)q_out, (bf16*)k_cache, (bf16*)v_cache, slots, T, Hq, Hkv, D,
                       block_size, (const bf16*)slabs, S, slab_stride);
  else
    hipLaunchKernelGGL(rope_kv_kernel<float>, grid, dim3(256), 0, s, (const bf16*)qkv, ld, positions,
                       (const float2*)cos_sin, (bf16*)q_out, (bf16*)k_cache, (bf16*)v_cache, slots, T, Hq, Hkv, D,
                       block_size, (const float*)slabs, S, slab_stride);
  return hipGetLastError();
}

}  // namespace dab

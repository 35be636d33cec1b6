// Shared device helpers for the gfx950 (MI355X / CDNA4) kernel library.
//
// Conventions used by every kernel in this directory:
//   * activations / weights are bf16 stored as raw uint16 bits, accumulation is fp32;
//   * a wavefront is 64 lanes (never 32) and blocks are multiples of 64 threads;
//   * global loads/stores of bf16 are vectorised to 16 B per lane (8 x bf16);
//   * MFMA tiles use v_mfma_f32_16x16x32_bf16 whose lane maps are
//       A: lane l holds A[row l&15][k 8(l>>4)+j], j=0..7
//       B: lane l holds B[k 8(l>>4)+j][col l&15]
//       C: lane l holds C[row 4(l>>4)+r][col l&15], r=0..3
//     (cdna_hip_programming.md section 3).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "launchers.h"  // L3Warm

namespace dab {

typedef uint16_t bf16;
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

constexpr int kWave = 64;

__device__ __forceinline__ float bf2f(uint16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

// Round-to-nearest-even through the compiler's native conversion (v_cvt_pk_bf16_f32 on gfx950),
// which keeps NaN a NaN (MI355X_MICROARCH.md, correctness boundaries).
__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 h = (__bf16)f;
  return __builtin_bit_cast(uint16_t, h);
}

// One v_cvt_pk_bf16_f32 (a <2 x float> -> <2 x bfloat> truncation), not two converts and an OR.
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack2bf(float lo, float hi) {
  const f32x2_t v = {lo, hi};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}

__device__ __forceinline__ void unpack8(const u32x4& v, float* f) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(v[i] << 16);
    f[2 * i + 1] = __uint_as_float(v[i] & 0xffff0000u);
  }
}

__device__ __forceinline__ u32x4 pack8(const float* f) {
  u32x4 v;
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = pack2bf(f[2 * i], f[2 * i + 1]);
  return v;
}

// Exact-erf GELU, 0.5 x (1 + erf(x / sqrt 2)), without the library erff (a long piecewise routine
// that, in a GEMM epilogue, costs more VALU time than the tile's bf16 stores): erfc by Abramowitz &
// Stegun 7.1.26 (|error| <= 1.5e-7 in erf), one v_rcp + one v_exp + 7 FMAs.  For x < 0 the result is
// 0.5 x erfc(|x| / sqrt 2) directly (no cancellation), for x >= 0 it is x - 0.5 x erfc(x / sqrt 2).
__device__ __forceinline__ float gelu_erf(float x) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.f));
  float q = fmaf(1.061405429f, t, -1.453152027f);
  q = fmaf(q, t, 1.421413741f);
  q = fmaf(q, t, -0.284496736f);
  q = fmaf(q, t, 0.254829592f);
  q *= t;
  const float c = 0.5f * x * q * __builtin_amdgcn_exp2f(z * z * -1.4426950408889634f);  // 0.5 x erfc(z)
  return x >= 0.f ? x - c : c;
}

// SiLU x / (1 + e^-x) with one v_rcp_f32 instead of the IEEE division (a ~10-instruction
// div_scale / div_fmas / div_fixup sequence per element in the SwiGLU epilogues); the reciprocal's
// 1-ulp error is far below the bf16 rounding of the result.  x -> -inf: rcp(inf) = 0 -> -0.
__device__ __forceinline__ float silu_f(float x) { return x * __builtin_amdgcn_rcpf(1.f + __expf(-x)); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x == NT (multiple of 64). `red` must hold NT/64 floats.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) t += red[i];
  __syncthreads();
  return t;
}

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// v_mfma_f32_32x32x16_bf16: lane l (r = l & 31, h = l >> 5) holds A[r][8h..8h+7] / B[8h..8h+7][r];
// C[row][col = l & 31] with row = (reg & 3) + 8 (reg >> 2) + 4 h
typedef float f32x16 __attribute__((ext_vector_type(16)));
__device__ __forceinline__ f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

// ds_read_b64_tr_b16: per 16-lane group, lane 4q+p supplies the address of row q, columns 4p..4p+3
// of a 4x16 bf16 block; lane i receives column i of the 4 rows (row q in element q).
__device__ __forceinline__ bf16x4 ds_read_tr16(const void* lds_ptr) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(lds_ptr));
}

__device__ __forceinline__ int div_up(int a, int b) { return (a + b - 1) / b; }

// Infinity-Cache (L3) warm-up of up to two byte ranges, read as one concatenated range: workgroup
// ``part`` of ``nparts`` reads its share with plain (allocating) 16-B loads, 8 per lane in flight,
// so a later kernel's read of the same bytes is served on-die (MI355X_MICROARCH.md § Infinity
// Cache: 256 MiB, resident while the bytes between two uses fit).  Nothing is written: the loaded
// words feed an empty asm statement, which keeps the loads.  Ranges must be 16-B multiples.
__device__ __forceinline__ void l3_warm_range(const char* base, long lo, long hi) {
  const u32x4* p = reinterpret_cast<const u32x4*>(base);
  const long step = blockDim.x;
  uint32_t acc = 0;
  for (long i = (lo >> 4) + threadIdx.x; i < (hi >> 4); i += 8 * step) {
    u32x4 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const long k = i + j * step;
      v[j] = k < (hi >> 4) ? p[k] : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) acc ^= v[j].x ^ v[j].w;
  }
  asm volatile("" ::"v"(acc));
}

__device__ __forceinline__ void l3_warm(const L3Warm& w, int part) {
  const long total = w.bytes[0] + w.bytes[1];
  const long per = ((total + w.blocks - 1) / w.blocks + 4095) & ~4095L;
  const long lo = part * per, hi = lo + per < total ? lo + per : total;
  if (lo < w.bytes[0]) l3_warm_range(w.ptr[0], lo, hi < w.bytes[0] ? hi : w.bytes[0]);
  if (hi > w.bytes[0]) l3_warm_range(w.ptr[1], (lo > w.bytes[0] ? lo : w.bytes[0]) - w.bytes[0], hi - w.bytes[0]);
}

// Orderable unsigned key of a float: larger float -> larger key (used by radix selects).
__device__ __forceinline__ uint32_t float_key(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key_float(uint32_t k) {
  uint32_t u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
  return __uint_as_float(u);
}

// Rotate-half RoPE of the pair (x1 = dim i, x2 = dim i + D/2) by (cos, sin): explicit FMAs, so the
// RoPE/KV-write kernel and the prefill attention's Q prologue round identically.
__device__ __forceinline__ void rope_rot(float& x1, float& x2, const float2 cs) {
  const float o1 = fmaf(x1, cs.x, -(x2 * cs.y));
  const float o2 = fmaf(x2, cs.x, x1 * cs.y);
  x1 = o1;
  x2 = o2;
}

// 8 consecutive elements of one split-K slab, loaded raw (fp32: two 16-B loads; bf16: one) so every
// load of a round can be issued before the first add, then added in fp32 to an accumulator.
template <typename ST>
struct SlabVec8;
template <>
struct SlabVec8<float> {
  f32x4 a, b;
  __device__ __forceinline__ void load(const float* p) {
    a = *reinterpret_cast<const f32x4*>(p);
    b = *reinterpret_cast<const f32x4*>(p + 4);
  }
  __device__ __forceinline__ void add_to(float (&v)[8]) const {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[j] += a[j];
      v[4 + j] += b[j];
    }
  }
};
template <>
struct SlabVec8<bf16> {
  u32x4 r;
  __device__ __forceinline__ void load(const bf16* p) { r = *reinterpret_cast<const u32x4*>(p); }
  __device__ __forceinline__ void add_to(float (&v)[8]) const {
    float f[8];
    unpack8(r, f);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] += f[j];
  }
};

// One 8-dim chunk pair (dims i0..i0+7 and i0+D/2..) of head `h` of token `t` of a QKV projection,
// with rotate-half RoPE applied when `rotate`: the shared body of rope_kv_kernel and of the fused
// decode-attention prologue (bitwise the same result in both).  The projection is either bf16 rows
// (`qkv`, row stride `ld`) or S fp32 / bf16 split-K slabs (`slabs`, row stride `ld`, slab stride
// `slab_stride`) summed in slab order and rounded like a bf16 GEMM output.  `cs` holds the 8
// (cos, sin) pairs of the token's position for dims i0..i0+7.  U slabs' loads are in flight per
// round (the per-element add order is slab order for any U).
template <int U = 4, typename ST = float>
__device__ __forceinline__ void rope_chunk(const bf16* __restrict__ qkv, const ST* __restrict__ slabs, int S,
                                           long slab_stride, int ld, int t, int h, int D, int i0,
                                           const float2 (&cs)[8], bool rotate, float (&x1)[8], float (&x2)[8]) {
  const int half = D >> 1;
  if (slabs) {
    const ST* src = slabs + (size_t)t * ld + (size_t)h * D;
#pragma unroll
    for (int j = 0; j < 8; ++j) x1[j] = x2[j] = 0.f;
    int sl = 0;
    for (; sl + U <= S; sl += U, src += U * slab_stride) {
      SlabVec8<ST> a[U], b[U];
#pragma unroll
      for (int q = 0; q < U; ++q) {
        const ST* sq = src + q * slab_stride;
        a[q].load(sq + i0);
        b[q].load(sq + i0 + half);
      }
#pragma unroll
      for (int q = 0; q < U; ++q) {
        a[q].add_to(x1);
        b[q].add_to(x2);
      }
    }
    for (; sl < S; ++sl, src += slab_stride) {
      SlabVec8<ST> a, b;
      a.load(src + i0);
      b.load(src + i0 + half);
      a.add_to(x1);
      b.add_to(x2);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      x1[j] = bf2f(f2bf(x1[j]));
      x2[j] = bf2f(f2bf(x2[j]));
    }
  } else {
    const bf16* src = qkv + (size_t)t * ld + (size_t)h * D;
    unpack8(*reinterpret_cast<const u32x4*>(src + i0), x1);
    unpack8(*reinterpret_cast<const u32x4*>(src + i0 + half), x2);
  }
  if (rotate) {
#pragma unroll
    for (int j = 0; j < 8; ++j) rope_rot(x1[j], x2[j], cs[j]);
  }
}

// The 8 (cos, sin) pairs of dims i0..i0+7 at position `pos` ([max_pos, D/2] float2 table).
__device__ __forceinline__ void rope_cs(const float2* __restrict__ cos_sin, int pos, int half, int i0, float2 (&cs)[8]) {
  const float4* csp = reinterpret_cast<const float4*>(cos_sin + (size_t)pos * half + i0);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float4 v = csp[j];
    cs[2 * j] = make_float2(v.x, v.y);
    cs[2 * j + 1] = make_float2(v.z, v.w);
  }
}

}  // namespace dab

#define DAB_CHECK_LAUNCH() (hipGetLastError())

// One-shot all-reduce over IPC-mapped peer buffers, for tensor-parallel decode on one xGMI node.
//
// A TP decode step all-reduces a [batch, hidden] bf16 activation twice per layer.  That is 16 KB to
// 2 MB, which is latency-bound.  RCCL's ring moves it in 2(W-1) serial hops over 2 of the 7 links.
// Here every rank reads all W-1 peers directly, one xGMI hop each and all links at once
// (SURVEY.md 5.8, 7.4 #5).
//
//   * Rank r owns one IPC allocation: a signal area, then two staging halves of `half_bytes`.
//   * The grid size is fixed (AR_BLOCKS).  Block b owns a contiguous segment of the vector.  Per
//     call, block b:
//       1. copies its segment of the local input into staging[e & 1];
//       2. writes system-scope release flags into every peer's signal area;
//       3. waits for the W flags addressed to it;
//       4. reads that segment from all W staging buffers;
//       5. sums in fp32 in rank order 0..W-1, so every rank produces bitwise the same result;
//       6. writes the result over the local input (in place).
//   * The epoch e lives in device memory (one counter per block, advanced by the kernel).  A
//     captured HIP graph replays correctly.
//   * Parity double-buffers the staging.  A peer that is one call ahead writes the other half.  It
//     cannot get two calls ahead, because its next barrier needs our flag.  One barrier per call
//     is therefore enough.
//   * Spins are bounded.  A missing peer sets `error` and the block gives up, so a broken group
//     cannot hang the GPU.  A block that gave up writes NaN over its output segment and does NOT
//     advance its epoch; the error word is sticky (until the host clears it), and every later call
//     on this rank only poisons its output.  The engine copies the word to the host behind every
//     TP step and fails the step's requests when it is set (engine/llm_engine.py
//     ``_tp_fault_check``); the group is then restarted.
#include <cstring>
#include <string>
#include <vector>

#include "common.h"
#include "launchers.h"

namespace dab {

constexpr int AR_MAX_RANKS = 8;
constexpr int AR_BLOCKS = 64;
constexpr int AR_THREADS = 512;

struct ArSignal {
  uint32_t flag[AR_BLOCKS][AR_MAX_RANKS];  // flag[b][src]: latest epoch rank src reached in block b
  uint32_t epoch[AR_BLOCKS];              // this rank's per-block call counter
  uint32_t error;
  uint32_t pad[63];
};

struct ArParams {
  char* base[AR_MAX_RANKS];  // each rank's IPC allocation (signal area, then 2 staging halves)
  bf16* data;                // local in/out
  long n16;                  // 16-B vectors
  long half_bytes;
  int rank;
  long spin_limit;
};

size_t allreduce_signal_bytes() { return (sizeof(ArSignal) + 4095) / 4096 * 4096; }

template <int W>
__global__ __launch_bounds__(AR_THREADS) void allreduce_kernel(ArParams p) {
  const int b = blockIdx.x, tid = threadIdx.x;
  const size_t sig_bytes = (sizeof(ArSignal) + 4095) / 4096 * 4096;
  ArSignal* me = reinterpret_cast<ArSignal*>(p.base[p.rank]);
  __shared__ uint32_t e_sh, bad_sh;
  if (tid == 0) {
    e_sh = me->epoch[b] + 1;
    bad_sh = __hip_atomic_load(&me->error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __syncthreads();
  const uint32_t e = e_sh;
  const size_t stage_off = sig_bytes + (size_t)(e & 1) * p.half_bytes;

  const long per = (p.n16 + AR_BLOCKS - 1) / AR_BLOCKS;
  const long s0 = min(p.n16, (long)b * per), s1 = min(p.n16, s0 + per);
  u32x4* dst = reinterpret_cast<u32x4*>(p.data);
  auto poison = [&]() {  // bf16 quiet NaN over this block's segment
    const u32x4 nan4 = {0x7fc07fc0u, 0x7fc07fc0u, 0x7fc07fc0u, 0x7fc07fc0u};
    for (long i = s0 + tid; i < s1; i += AR_THREADS) dst[i] = nan4;
  };
  if (bad_sh) {  // this rank's group already broke: no flags, no epoch, NaN out (uniform)
    poison();
    return;
  }
  u32x4* mine = reinterpret_cast<u32x4*>(p.base[p.rank] + stage_off);
  const u32x4* src = reinterpret_cast<const u32x4*>(p.data);
  for (long i = s0 + tid; i < s1; i += AR_THREADS) mine[i] = src[i];
  __threadfence_system();  // staging visible to every peer before the flag
  __syncthreads();
  if (tid < W) {
    ArSignal* peer = reinterpret_cast<ArSignal*>(p.base[tid]);
    __hip_atomic_store(&peer->flag[b][p.rank], e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    long spins = 0;
    // >= : a peer already one call ahead has overwritten the flag with e + 1
    while ((int)(__hip_atomic_load(&me->flag[b][tid], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - e) < 0) {
      if (++spins > p.spin_limit) {
        __hip_atomic_store(&me->error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        bad_sh = 1u;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  if (bad_sh) {  // a peer never arrived: this block's sum would mix stale staging (uniform)
    poison();
    return;
  }

  const u32x4* stage[W];
#pragma unroll
  for (int r = 0; r < W; ++r) stage[r] = reinterpret_cast<const u32x4*>(p.base[r] + stage_off);
  for (long i = s0 + tid; i < s1; i += AR_THREADS) {
    u32x4 v[W];
#pragma unroll
    for (int r = 0; r < W; ++r) v[r] = __builtin_nontemporal_load(stage[r] + i);
    float acc[8], t[8];
    unpack8(v[0], acc);
#pragma unroll
    for (int r = 1; r < W; ++r) {
      unpack8(v[r], t);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += t[j];
    }
    dst[i] = pack8(acc);
  }
  __syncthreads();
  if (tid == 0) me->epoch[b] = e;
}

// ---- all-reduce fused with the split-K slab sum, the residual add and the RMSNorm ---------------
// One TP decode all-reduce site was three launches: slab_reduce (this rank's fp32 split-K slabs ->
// bf16 partial) -> allreduce_kernel -> rmsnorm (+ residual).  Here one launch does all three with
// the same arithmetic, so at W = 1 the result is bitwise that of the sequence:
//   1. block b sums, for each of its rows (b, b + 64, ...), the S slabs in slab order and rounds to
//      bf16 (slab_reduce), into this rank's staging half (or copies a bf16 partial when S == 0);
//   2. the flag exchange of allreduce_kernel (same signal area, epochs, parity, bounded spins,
//      sticky error + NaN poisoning);
//   3. the row is summed over the W staging buffers in rank order and rounded to bf16 (the
//      all-reduce's output), the residual is added in bf16, and the RMSNorm runs with the thread
//      mapping and block reduction of rmsnorm_kernel<NT, VPT> (the launcher picks NT / VPT exactly as
//      rmsnorm's DAB_ROW_DISPATCH does).
// Every launch runs all AR_BLOCKS blocks (rowless blocks still exchange flags), so every block's
// epoch -- and the staging parity -- stays in step with allreduce_kernel's calls.
struct ArNormParams {
  char* base[AR_MAX_RANKS];
  int rank;
  long half_bytes;
  long spin_limit;
  const float* slabs;  // [S][rows][cols] fp32 partials (S > 0) ...
  int S;
  long slab_stride;
  const bf16* x;       // ... or this rank's bf16 partial [rows][cols] (S == 0)
  const bf16* res_in;  // [rows][cols] residual stream in (may be null)
  bf16* res_out;       // x + residual (when res_in)
  bf16* out;           // RMSNorm output
  const bf16* w;       // gains [cols]
  int rows, cols;
  float eps;
};

template <int W, int NT, int VPT>
__global__ __launch_bounds__(NT) void allreduce_rmsnorm_kernel(ArNormParams p) {
  const int b = blockIdx.x, tid = threadIdx.x;
  const size_t sig_bytes = (sizeof(ArSignal) + 4095) / 4096 * 4096;
  ArSignal* me = reinterpret_cast<ArSignal*>(p.base[p.rank]);
  __shared__ uint32_t e_sh, bad_sh;
  __shared__ float red[NT / 64];
  if (tid == 0) {
    e_sh = me->epoch[b] + 1;
    bad_sh = __hip_atomic_load(&me->error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __syncthreads();
  const uint32_t e = e_sh;
  const size_t stage_off = sig_bytes + (size_t)(e & 1) * p.half_bytes;
  const int nvec = p.cols >> 3;
  auto poison = [&]() {
    const u32x4 nan4 = {0x7fc07fc0u, 0x7fc07fc0u, 0x7fc07fc0u, 0x7fc07fc0u};
    for (int row = b; row < p.rows; row += AR_BLOCKS)
      for (int i = tid; i < nvec; i += NT) {
        reinterpret_cast<u32x4*>(p.out + (size_t)row * p.cols)[i] = nan4;
        if (p.res_in) reinterpret_cast<u32x4*>(p.res_out + (size_t)row * p.cols)[i] = nan4;
      }
  };
  if (bad_sh) {
    poison();
    return;
  }
  // 1. this rank's partial rows -> staging
  u32x4* mine = reinterpret_cast<u32x4*>(p.base[p.rank] + stage_off);
  for (int row = b; row < p.rows; row += AR_BLOCKS) {
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      const int i = tid + k * NT;
      if (i >= nvec) continue;
      const size_t v16 = (size_t)row * nvec + i;
      if (p.S > 0) {
        float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        for (int sl = 0; sl < p.S; ++sl) {
          const f32x4* src = reinterpret_cast<const f32x4*>(p.slabs + (size_t)sl * p.slab_stride + v16 * 8);
          const f32x4 a = src[0], c = src[1];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            o[j] += a[j];
            o[4 + j] += c[j];
          }
        }
        mine[v16] = pack8(o);
      } else {
        mine[v16] = reinterpret_cast<const u32x4*>(p.x)[v16];
      }
    }
  }
  __threadfence_system();
  __syncthreads();
  // 2. flags (as allreduce_kernel)
  if (tid < W) {
    ArSignal* peer = reinterpret_cast<ArSignal*>(p.base[tid]);
    __hip_atomic_store(&peer->flag[b][p.rank], e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    long spins = 0;
    while ((int)(__hip_atomic_load(&me->flag[b][tid], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - e) < 0) {
      if (++spins > p.spin_limit) {
        __hip_atomic_store(&me->error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        bad_sh = 1u;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  if (bad_sh) {
    poison();
    return;
  }
  // 3. sum over ranks, residual, RMSNorm (rmsnorm_kernel's arithmetic and reduction order)
  const u32x4* stage[W];
#pragma unroll
  for (int r = 0; r < W; ++r) stage[r] = reinterpret_cast<const u32x4*>(p.base[r] + stage_off);
  const u32x4* wr = reinterpret_cast<const u32x4*>(p.w);
  for (int row = b; row < p.rows; row += AR_BLOCKS) {
    float v[VPT][8];
    float ss = 0.f;
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      const int i = tid + k * NT;
      if (i < nvec) {
        const size_t v16 = (size_t)row * nvec + i;
        u32x4 sv[W];
#pragma unroll
        for (int r = 0; r < W; ++r) sv[r] = __builtin_nontemporal_load(stage[r] + v16);
        float acc[8], t[8];
        unpack8(sv[0], acc);
#pragma unroll
        for (int r = 1; r < W; ++r) {
          unpack8(sv[r], t);
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] += t[j];
        }
        unpack8(pack8(acc), v[k]);  // the all-reduce's bf16 output
        if (p.res_in) {
          float rr[8];
          unpack8(reinterpret_cast<const u32x4*>(p.res_in + (size_t)row * p.cols)[i], rr);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[k][j] = bf2f(f2bf(v[k][j] + rr[j]));  // residual kept in bf16 like HF
          reinterpret_cast<u32x4*>(p.res_out + (size_t)row * p.cols)[i] = pack8(v[k]);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) ss += v[k][j] * v[k][j];
      }
    }
    const float tot = block_sum<NT>(ss, red);
    const float inv = rsqrtf(tot / (float)p.cols + p.eps);
    u32x4* orow = reinterpret_cast<u32x4*>(p.out + (size_t)row * p.cols);
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      const int i = tid + k * NT;
      if (i < nvec) {
        float g[8], o[8];
        unpack8(wr[i], g);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = v[k][j] * inv * g[j];
        orow[i] = pack8(o);
      }
    }
  }
  __syncthreads();
  if (tid == 0) me->epoch[b] = e;
}

template <int W>
static void launch_ar_norm(const ArNormParams& p, hipStream_t s) {
  const int nvec = p.cols / 8;
  const dim3 grid(AR_BLOCKS);
  if (nvec <= 64) hipLaunchKernelGGL((allreduce_rmsnorm_kernel<W, 64, 1>), grid, dim3(64), 0, s, p);
  else if (nvec <= 128) hipLaunchKernelGGL((allreduce_rmsnorm_kernel<W, 128, 1>), grid, dim3(128), 0, s, p);
  else if (nvec <= 256) hipLaunchKernelGGL((allreduce_rmsnorm_kernel<W, 256, 1>), grid, dim3(256), 0, s, p);
  else if (nvec <= 512) hipLaunchKernelGGL((allreduce_rmsnorm_kernel<W, 256, 2>), grid, dim3(256), 0, s, p);
  else if (nvec <= 1024) hipLaunchKernelGGL((allreduce_rmsnorm_kernel<W, 256, 4>), grid, dim3(256), 0, s, p);
  else hipLaunchKernelGGL((allreduce_rmsnorm_kernel<W, 256, 8>), grid, dim3(256), 0, s, p);
}

int custom_allreduce_rmsnorm(const std::vector<uintptr_t>& bases, int rank, const float* slabs, int S,
                             long slab_stride, const void* x, const void* res_in, void* res_out, void* out,
                             const void* w, int rows, int cols, float eps, long half_bytes, long spin_limit,
                             hipStream_t s) {
  const int W = (int)bases.size();
  if (W < 1 || W > AR_MAX_RANKS || rank < 0 || rank >= W) return hipErrorInvalidValue;
  if (rows <= 0) return 0;
  if (cols % 8 || cols > 16384 || (long)rows * cols * 2 > half_bytes) return hipErrorInvalidValue;
  if ((S > 0 && (!slabs || slab_stride % 4 || slab_stride < (long)rows * cols)) || (S == 0 && !x) || S < 0)
    return hipErrorInvalidValue;
  if (res_in && !res_out) return hipErrorInvalidValue;
  ArNormParams p;
  for (int r = 0; r < AR_MAX_RANKS; ++r) p.base[r] = r < W ? reinterpret_cast<char*>(bases[r]) : nullptr;
  p.rank = rank;
  p.half_bytes = half_bytes;
  p.spin_limit = spin_limit;
  p.slabs = slabs;
  p.S = S;
  p.slab_stride = slab_stride;
  p.x = (const bf16*)x;
  p.res_in = (const bf16*)res_in;
  p.res_out = (bf16*)res_out;
  p.out = (bf16*)out;
  p.w = (const bf16*)w;
  p.rows = rows;
  p.cols = cols;
  p.eps = eps;
  switch (W) {
    case 1: launch_ar_norm<1>(p, s); break;
    case 2: launch_ar_norm<2>(p, s); break;
    case 3: launch_ar_norm<3>(p, s); break;
    case 4: launch_ar_norm<4>(p, s); break;
    case 5: launch_ar_norm<5>(p, s); break;
    case 6: launch_ar_norm<6>(p, s); break;
    case 7: launch_ar_norm<7>(p, s); break;
    default: launch_ar_norm<8>(p, s); break;
  }
  return hipGetLastError();
}

int custom_allreduce(const std::vector<uintptr_t>& bases, int rank, void* data, long nbytes, long half_bytes,
                     long spin_limit, hipStream_t s) {
  const int W = (int)bases.size();
  if (W < 1 || W > AR_MAX_RANKS || rank < 0 || rank >= W) return hipErrorInvalidValue;
  if (nbytes % 16 || nbytes > half_bytes || ((uintptr_t)data & 15)) return hipErrorInvalidValue;
  if (nbytes == 0) return 0;
  ArParams p;
  for (int r = 0; r < AR_MAX_RANKS; ++r) p.base[r] = r < W ? reinterpret_cast<char*>(bases[r]) : nullptr;
  p.data = (bf16*)data;
  p.n16 = nbytes / 16;
  p.half_bytes = half_bytes;
  p.rank = rank;
  p.spin_limit = spin_limit;
  const dim3 grid(AR_BLOCKS), block(AR_THREADS);
  switch (W) {
    case 1: hipLaunchKernelGGL(allreduce_kernel<1>, grid, block, 0, s, p); break;
    case 2: hipLaunchKernelGGL(allreduce_kernel<2>, grid, block, 0, s, p); break;
    case 3: hipLaunchKernelGGL(allreduce_kernel<3>, grid, block, 0, s, p); break;
    case 4: hipLaunchKernelGGL(allreduce_kernel<4>, grid, block, 0, s, p); break;
    case 5: hipLaunchKernelGGL(allreduce_kernel<5>, grid, block, 0, s, p); break;
    case 6: hipLaunchKernelGGL(allreduce_kernel<6>, grid, block, 0, s, p); break;
    case 7: hipLaunchKernelGGL(allreduce_kernel<7>, grid, block, 0, s, p); break;
    default: hipLaunchKernelGGL(allreduce_kernel<8>, grid, block, 0, s, p); break;
  }
  return hipGetLastError();
}

// ---- IPC buffer management (host) ------------------------------------------------------------

// uncached = fine-grained, uncached device memory (hipDeviceMallocUncached): every load and store of
// the signal flags and staging halves goes to HBM, never to a (remote) L2 line that a peer on another
// GPU could leave stale.  The release/acquire system-scope atomics and __threadfence_system order the
// accesses; uncached memory is what makes them coherent ACROSS xGMI (coarse-grained hipMalloc memory
// is coherent only at kernel boundaries for peer accesses).  Peers read it over xGMI either way, so
// the cost is the local staging write, which is tiny.
int allreduce_buffer_alloc(long bytes, int uncached, uintptr_t* out) {
  void* ptr = nullptr;
  hipError_t err = uncached ? hipExtMallocWithFlags(&ptr, (size_t)bytes, hipDeviceMallocUncached)
                            : hipMalloc(&ptr, (size_t)bytes);
  if (err != hipSuccess) return err;
  err = hipMemset(ptr, 0, (size_t)bytes);
  if (err != hipSuccess) {
    (void)hipFree(ptr);
    return err;
  }
  *out = reinterpret_cast<uintptr_t>(ptr);
  return hipDeviceSynchronize();
}

int allreduce_buffer_free(uintptr_t ptr) { return hipFree(reinterpret_cast<void*>(ptr)); }

int ipc_get_handle(uintptr_t ptr, std::string* handle) {
  hipIpcMemHandle_t h;
  const hipError_t err = hipIpcGetMemHandle(&h, reinterpret_cast<void*>(ptr));
  if (err != hipSuccess) return err;
  handle->assign(reinterpret_cast<const char*>(&h), sizeof(h));
  return 0;
}

int ipc_open_handle(const std::string& handle, uintptr_t* out) {
  if (handle.size() != sizeof(hipIpcMemHandle_t)) return hipErrorInvalidValue;
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle.data(), sizeof(h));
  void* ptr = nullptr;
  const hipError_t err = hipIpcOpenMemHandle(&ptr, h, hipIpcMemLazyEnablePeerAccess);
  if (err != hipSuccess) return err;
  *out = reinterpret_cast<uintptr_t>(ptr);
  return 0;
}

// host-driven read of a mapped peer buffer: a broken mapping fails here as an API error instead of
// as a memory fault inside the all-reduce kernel
int ipc_probe(uintptr_t ptr) {
  uint32_t tmp[4];
  const hipError_t err = hipMemcpy(tmp, reinterpret_cast<const void*>(ptr), sizeof(tmp), hipMemcpyDeviceToHost);
  return err;
}

int ipc_close_handle(uintptr_t ptr) { return hipIpcCloseMemHandle(reinterpret_cast<void*>(ptr)); }

// the error word copied to host memory behind the work already on `s` (no synchronisation: the
// engine reads it after the step's own sync point)
int allreduce_error_async(uintptr_t base, void* host_word, hipStream_t s) {
  ArSignal* sig = reinterpret_cast<ArSignal*>(base);
  return hipMemcpyAsync(host_word, &sig->error, sizeof(uint32_t), hipMemcpyDeviceToHost, s);
}

int allreduce_error(uintptr_t base, int clear) {
  uint32_t err = 0;
  ArSignal* sig = reinterpret_cast<ArSignal*>(base);
  if (hipMemcpy(&err, &sig->error, sizeof(err), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  if (clear && err) {
    const uint32_t z = 0;
    (void)hipMemcpy(&sig->error, &z, sizeof(z), hipMemcpyHostToDevice);
  }
  return (int)err;
}

}  // namespace dab

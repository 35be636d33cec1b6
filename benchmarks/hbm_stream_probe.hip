// HBM streaming-rate probe: how fast can one workgroup per CU read a once-used weight stream on
// gfx950, by the two transports the decode GEMMs could use?
//
//   vgpr: W waves per workgroup, each keeping D 1-KB fragments in flight in a register ring
//         (buffer_load_dwordx4, 16 B per lane; stream_gemm.hip's compute waves do this);
//   lds : L loader waves per workgroup filling a ring of 16-KB LDS slots with LDS-DMA
//         (global_load_lds, 16 B per lane), I slots in flight, counted vmcnt, no consumer.
//
// Each launch streams a fresh 256 MB window of a 2 GB buffer (the Infinity Cache holds 256 MB), so
// every byte comes from HBM.  Prints one JSON line per configuration: TB/s (median of 9 launches).
//
//   hipcc --offload-arch=gfx950 -O3 -o benchmarks/hbm_stream_probe benchmarks/hbm_stream_probe.hip
//   ./benchmarks/hbm_stream_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                        \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                     \
    }                                                                                   \
  } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N <= 63, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x70 | 0xF00);
}

// W waves x D-deep register ring; wave w reads 1-KB chunks w, w + W, w + 2W, ... of its
// workgroup's region (out-of-range loads of the buffer descriptor return zeros: no fault).
template <int W, int D, bool NT>
__global__ __launch_bounds__(64 * W) void vgpr_stream(const char* src, unsigned bytes_per_wg, unsigned* out) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(src + (size_t)blockIdx.x * bytes_per_wg), 0,
                                                    (int)bytes_per_wg, 0x00020000);
  const unsigned nchunks = bytes_per_wg / 1024;
  u32x4 ring[D];
  unsigned acc = 0;
#pragma unroll
  for (int d = 0; d < D; ++d)
    ring[d] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, ((w + d * W) * 64 + lane) * 16, 0,
                                                                              NT ? 2 : 0));
  for (unsigned c0 = w + D * W; c0 < nchunks + D * W; c0 += D * W) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      acc ^= ring[d][0] ^ ring[d][3];
      const unsigned c = c0 + d * W;  // past the end: a zero-returning load, never consumed
      ring[d] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (c * 64 + lane) * 16, 0,
                                                                                NT ? 2 : 0));
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if (acc == 0x9e3779b9u) out[blockIdx.x] = acc;  // keeps the loads alive
}

// The same ring, but every wave streams its own contiguous part of the workgroup's region (as
// stream_gemm's compute waves do: one 16-row block of the fragment layout each, 16 rows x K apart).
template <int W, int D, bool NT>
__global__ __launch_bounds__(64 * W) void vgpr_stream_private(const char* src, unsigned bytes_per_wg, unsigned* out) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const unsigned per_wave = bytes_per_wg / W / 1024 * 1024;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(src + (size_t)blockIdx.x * bytes_per_wg + (size_t)w * per_wave),
                                                    0, (int)per_wave, 0x00020000);
  const unsigned nchunks = per_wave / 1024;
  u32x4 ring[D];
  unsigned acc = 0;
#pragma unroll
  for (int d = 0; d < D; ++d)
    ring[d] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (d * 64 + lane) * 16, 0, NT ? 2 : 0));
  for (unsigned c0 = D; c0 < nchunks + D; c0 += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      acc ^= ring[d][0] ^ ring[d][3];
      ring[d] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, ((c0 + d) * 64 + lane) * 16, 0,
                                                                                NT ? 2 : 0));
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if (acc == 0x9e3779b9u) out[blockIdx.x] = acc;
}

// L loader waves fill 16-KB LDS slots (16 x 1 KB per slot, 16 / L instructions per wave), I slots in
// flight per wave's counted vmcnt; SLOTS-deep ring (nobody reads it: the transfer rate alone).
template <int L, int SLOTS, int I, bool NT>
__global__ __launch_bounds__(64 * L) void lds_stream(const char* src, unsigned bytes_per_wg, unsigned* out) {
  static_assert(16 % L == 0 && I < SLOTS, "shape");
  constexpr int PER = 16 / L;  // 1-KB instructions per wave per slot
  static_assert(I * PER <= 63, "vmcnt range");
  __shared__ __attribute__((aligned(16))) char ring[SLOTS * 16384];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const char* base = src + (size_t)blockIdx.x * bytes_per_wg;
  const unsigned nslots = bytes_per_wg / 16384;
  for (unsigned s = 0; s < nslots; ++s) {
    char* dst = ring + (s % SLOTS) * 16384;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int i = w * PER + j;
      __builtin_amdgcn_global_load_lds((const void*)(base + (size_t)s * 16384 + i * 1024 + lane * 16),
                                       (__attribute__((address_space(3))) void*)(dst + i * 1024), 16, 0, NT ? 2 : 0);
    }
    if (s >= (unsigned)I) wait_vm<I * PER>();  // slot s - I landed
  }
  wait_vm<0>();
  if (threadIdx.x == 0 && ring[lane] == 123 && ring[1] == 45) out[blockIdx.x] = 1;
}

template <class F>
static double time_tbps(F launch, size_t bytes) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  std::vector<float> ms;
  for (int r = 0; r < 10; ++r) {
    CHECK(hipEventRecord(a));
    launch(r);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float t = 0.f;
    CHECK(hipEventElapsedTime(&t, a, b));
    if (r) ms.push_back(t);  // the first launch warms up the code object
  }
  std::sort(ms.begin(), ms.end());
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
  return bytes / (ms[ms.size() / 2] * 1e-3) / 1e12;
}

int main() {
  const size_t total = size_t(2) << 30, window = size_t(256) << 20;
  char* buf = nullptr;
  unsigned* out = nullptr;
  CHECK(hipMalloc(&buf, total));
  CHECK(hipMalloc(&out, 4096 * sizeof(unsigned)));
  CHECK(hipMemset(buf, 1, total));
  CHECK(hipDeviceSynchronize());
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  for (int per_cu : {1, 2}) {
    const int nwg = cus * per_cu;
    const unsigned bpw = (unsigned)((window / nwg) / 16384 * 16384);
    const size_t bytes = (size_t)bpw * nwg;
    auto win = [&](int r) { return buf + (size_t)(r % 8) * window; };
#define VG(W, D, NT)                                                                                         \
  {                                                                                                          \
    double t = time_tbps([&](int r) { hipLaunchKernelGGL((vgpr_stream<W, D, NT>), dim3(nwg), dim3(64 * W), 0, 0, \
                                                         win(r), bpw, out); }, bytes);                        \
    std::printf("{\"transport\": \"vgpr\", \"wg_per_cu\": %d, \"waves\": %d, \"depth\": %d, \"nt\": %d, "   \
                "\"tbps\": %.2f}\n", per_cu, W, D, (int)NT, t);                                              \
  }
#define LD(L, S, I, NT)                                                                                      \
  {                                                                                                          \
    double t = time_tbps([&](int r) { hipLaunchKernelGGL((lds_stream<L, S, I, NT>), dim3(nwg), dim3(64 * L), 0, 0, \
                                                         win(r), bpw, out); }, bytes);                        \
    std::printf("{\"transport\": \"lds\", \"wg_per_cu\": %d, \"loaders\": %d, \"slots\": %d, "             \
                "\"in_flight\": %d, \"nt\": %d, \"tbps\": %.2f}\n", per_cu, L, S, I, (int)NT, t);            \
  }
#define VP(W, D, NT)                                                                                         \
  {                                                                                                          \
    double t = time_tbps([&](int r) { hipLaunchKernelGGL((vgpr_stream_private<W, D, NT>), dim3(nwg), dim3(64 * W), 0, \
                                                         0, win(r), bpw, out); }, bytes);                     \
    std::printf("{\"transport\": \"vgpr-private\", \"wg_per_cu\": %d, \"waves\": %d, \"depth\": %d, \"nt\": %d, " \
                "\"tbps\": %.2f}\n", per_cu, W, D, (int)NT, t);                                            \
  }
    if (per_cu == 1) {
      VG(4, 8, true) VG(7, 8, true) VG(7, 16, true) VG(8, 8, true)
      VP(4, 8, true) VP(4, 16, true) VP(4, 24, true) VP(7, 8, true) VP(7, 16, true) VP(8, 8, true) VP(8, 16, true)
      LD(4, 8, 3, true)
    } else {
      VG(4, 4, true) VG(4, 8, true) VP(4, 8, true) VP(4, 16, true) VP(7, 8, true)
    }
    std::fflush(stdout);
  }
  CHECK(hipFree(buf));
  CHECK(hipFree(out));
  return 0;
}

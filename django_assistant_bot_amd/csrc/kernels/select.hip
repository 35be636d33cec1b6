// Per-row selection kernels (one 1024-thread workgroup per row):
//   sample_tokens : HF-parity sampling  temperature -> top-k -> top-p -> multinomial  (N12;
//                   reference ai/providers/transformers.py:57-66 do_sample=True, top_k=50, top_p=0.95),
//                   greedy when temperature <= 0.  Counter-based RNG: graph replays draw fresh numbers.
//   topk_rows     : exact top-k (k <= 1024) of fp32 score rows, sorted descending, for the in-HBM
//                   cosine index (N13/N14; replaces pgvector ORDER BY distance LIMIT n).
//
// Both use an MSB-first 4 x 8-bit radix select of the k-th largest orderable key.  Histogram
// increments are wave-aggregated (one LDS atomic per distinct bin per wave) because score /
// logit keys cluster in a handful of top-byte bins and plain per-lane LDS atomics would serialise.
#include "common.h"
#include "launchers.h"

namespace dab {

// float_key(-inf): keys at or below it are -inf logits (masked) or the 0 padding of candidate lists
constexpr uint32_t kNegInfKey = 0x007FFFFFu;


constexpr int SEL_NT = 1024;
constexpr int SEL_MAXK = 1024;

struct SelShared {
  uint32_t hist[256];
  uint32_t bcast[4];
  uint32_t cnt_gt, cnt_eq;
  uint32_t cand_key[SEL_MAXK];
  int cand_idx[SEL_MAXK];
};

// Appends `pred` lanes with one atomic per wave; returns this lane's slot (or -1).
__device__ __forceinline__ int wave_append(uint32_t* counter, bool pred) {
  const unsigned long long m = __ballot(pred);
  if (!m) return -1;
  const int lane = threadIdx.x & 63;
  const int leader = __ffsll((long long)m) - 1;
  uint32_t base = 0;
  if (lane == leader) base = atomicAdd(counter, (uint32_t)__popcll(m));
  base = __shfl(base, leader, 64);
  const unsigned long long below = lane ? (m & ((1ull << lane) - 1ull)) : 0ull;
  return pred ? (int)(base + __popcll(below)) : -1;
}

template <class KeyAt>
__device__ uint32_t radix_kth(KeyAt key_at, int n, int k, SelShared& sh, uint32_t& ties_needed) {
  uint32_t prefix = 0, pmask = 0, kk = (uint32_t)k;
  const int tid = threadIdx.x, lane = tid & 63;
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int i = tid; i < 256; i += SEL_NT) sh.hist[i] = 0;
    __syncthreads();
    for (int i0 = 0; i0 < n; i0 += SEL_NT) {
      const int i = i0 + tid;
      int bin = -1;
      if (i < n) {
        const uint32_t key = key_at(i);
        if ((key & pmask) == prefix) bin = (int)((key >> shift) & 255u);
      }
      unsigned long long active = __ballot(bin >= 0);
      while (active) {
        const int leader = __ffsll((long long)active) - 1;
        const int lb = __shfl(bin, leader, 64);
        const unsigned long long eq = __ballot(bin == lb);
        if (lane == leader) atomicAdd(&sh.hist[lb], (uint32_t)__popcll(eq));
        active &= ~eq;
      }
    }
    __syncthreads();
    if (tid < 64) {
      uint32_t c[4], sum = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        c[j] = sh.hist[255 - 4 * tid - j];
        sum += c[j];
      }
      uint32_t incl = sum;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(incl, o, 64);
        if (tid >= o) incl += t;
      }
      const uint32_t excl = incl - sum;
      if (excl < kk && kk <= incl) {
        uint32_t acc = excl;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (acc + c[j] >= kk) {
            sh.bcast[0] = 255u - 4u * tid - j;
            sh.bcast[1] = kk - acc;
            break;
          }
          acc += c[j];
        }
      }
    }
    __syncthreads();
    const uint32_t digit = sh.bcast[0];
    kk = sh.bcast[1];
    prefix |= digit << shift;
    pmask |= 255u << shift;
    __syncthreads();
  }
  ties_needed = kk;
  return prefix;
}

// Gathers the k largest keys (ties at the k-th key taken in arbitrary order) into sh.cand_*[0..k)
// and sorts them descending by key (ascending index among equal keys).  TIES_ALL: every key equal
// to the k-th is kept too (HF TopKLogitsWarper keeps all logits >= the k-th value), up to SEL_MAXK
// candidates; returns the number kept (k without TIES_ALL).
template <bool TIES_ALL = false, class KeyAt>
__device__ int select_topk(KeyAt key_at, int n, int k, SelShared& sh) {
  const int tid = threadIdx.x;
  uint32_t ties;
  const uint32_t kth = radix_kth(key_at, n, k, sh, ties);
  const uint32_t n_gt0 = (uint32_t)k - ties;
  // capacity for the tied keys -- unless the k-th value is -inf (a masked row with fewer than k
  // allowed tokens): those ties carry probability 0, and extending over them would only sort and
  // walk up to SEL_MAXK dead candidates
  if (TIES_ALL && kth > kNegInfKey) ties = (uint32_t)SEL_MAXK - n_gt0;
  if (tid == 0) {
    sh.cnt_gt = 0;
    sh.cnt_eq = 0;
  }
  __syncthreads();
  const uint32_t n_gt = n_gt0;
  for (int i0 = 0; i0 < n; i0 += SEL_NT) {
    const int i = i0 + tid;
    uint32_t key = 0;
    if (i < n) key = key_at(i);
    const int pg = wave_append(&sh.cnt_gt, i < n && key > kth);
    if (pg >= 0) {
      sh.cand_key[pg] = key;
      sh.cand_idx[pg] = i;
    }
    const int pe = wave_append(&sh.cnt_eq, i < n && key == kth);
    if (pe >= 0 && (uint32_t)pe < ties) {
      sh.cand_key[n_gt + pe] = key;
      sh.cand_idx[n_gt + pe] = i;
    }
  }
  __syncthreads();
  if (TIES_ALL) k = (int)(n_gt + min(sh.cnt_eq, ties));
  int P = 1;
  while (P < k) P <<= 1;
  for (int i = k + tid; i < P; i += SEL_NT) {
    sh.cand_key[i] = 0u;
    sh.cand_idx[i] = 0x7fffffff;
  }
  __syncthreads();
  // bitonic sort, descending key, ascending index
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = tid; t < P; t += SEL_NT) {
        const int u = t ^ stride;
        if (u > t) {
          const bool desc = (t & size) == 0;
          const uint32_t ka = sh.cand_key[t], kb = sh.cand_key[u];
          const int ia = sh.cand_idx[t], ib = sh.cand_idx[u];
          const bool a_first = ka > kb || (ka == kb && ia < ib);
          if (a_first != desc) {
            sh.cand_key[t] = kb;
            sh.cand_key[u] = ka;
            sh.cand_idx[t] = ib;
            sh.cand_idx[u] = ia;
          }
        }
      }
      __syncthreads();
    }
  }
  return k;
}

__device__ __forceinline__ unsigned long long splitmix64(unsigned long long x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__global__ __launch_bounds__(SEL_NT) void sample_kernel(const void* __restrict__ logits, int logits_f32, long ld,
                                                        int vocab, const float* __restrict__ temperature,
                                                        const int* __restrict__ top_k,
                                                        const float* __restrict__ top_p, unsigned long long seed,
                                                        int64_t* __restrict__ counters, int* __restrict__ out_tokens,
                                                        float* __restrict__ out_logprobs) {
  __shared__ SelShared sh;
  __shared__ float probs[SEL_MAXK];
  const int row = blockIdx.x;
  const float T = temperature ? temperature[row] : 1.f;
  int k = (T <= 0.f) ? 1 : (top_k && top_k[row] > 0 ? top_k[row] : SEL_MAXK);
  if (k > SEL_MAXK) k = SEL_MAXK;
  if (k > vocab) k = vocab;
  const float P = top_p ? top_p[row] : 1.f;
  const bool f32 = logits_f32 != 0;
  const float* lf = reinterpret_cast<const float*>(logits) + (size_t)row * ld;
  const bf16* lb = reinterpret_cast<const bf16*>(logits) + (size_t)row * ld;
  auto key_at = [&](int i) -> uint32_t { return float_key(f32 ? lf[i] : bf2f(lb[i])); };
  // HF TopKLogitsWarper keeps every logit >= the k-th value (ties beyond k included); greedy takes
  // the lowest index among equal maxima (torch.argmax)
  k = select_topk<true>(key_at, vocab, k, sh);
  if (threadIdx.x != 0) return;
  if (T <= 0.f) {
    out_tokens[row] = sh.cand_idx[0];
    if (out_logprobs) out_logprobs[row] = 0.f;
    return;
  }
  // softmax over the top-k set (HF: top-k sets the rest to -inf before top-p's softmax)
  const float x0 = key_float(sh.cand_key[0]) / T;
  float total = 0.f;
  for (int i = 0; i < k; ++i) {
    const float e = __expf(key_float(sh.cand_key[i]) / T - x0);
    probs[i] = e;
    total += e;
  }
  // HF TopPLogitsWarper: ascending cumsum, drop tokens with cumsum <= 1 - top_p, keep >= 1.
  int keep = k;
  if (P < 1.f) {
    const float thr = (1.f - P) * total;
    float cum = 0.f;
    keep = k;
    for (int i = k - 1; i >= 1; --i) {  // ascending order = reverse of the sorted list
      cum += probs[i];
      if (cum <= thr) keep = i;
      else break;
    }
  }
  float kept = 0.f;
  for (int i = 0; i < keep; ++i) kept += probs[i];
  const long long c = counters ? counters[row] : 0;
  if (counters) counters[row] = c + 1;
  const unsigned long long r =
      splitmix64(seed ^ splitmix64((unsigned long long)c * 0x9E3779B97F4A7C15ull + (unsigned long long)row));
  const float u = (float)(r >> 40) * (1.f / 16777216.f);
  const float target = u * kept;
  float acc = 0.f;
  int pick = keep - 1;
  for (int i = 0; i < keep; ++i) {
    acc += probs[i];
    if (acc > target) {
      pick = i;
      break;
    }
  }
  out_tokens[row] = sh.cand_idx[pick];
  if (out_logprobs) out_logprobs[row] = __logf(probs[pick] / kept);
}

__global__ __launch_bounds__(SEL_NT) void topk_rows_kernel(const float* __restrict__ scores, long ld, int n, int k,
                                                           float* __restrict__ out_vals, int* __restrict__ out_idx,
                                                           int64_t index_base, int64_t* __restrict__ out_idx64) {
  __shared__ SelShared sh;
  const int row = blockIdx.x;
  const float* s = scores + (size_t)row * ld;
  auto key_at = [&](int i) -> uint32_t { return float_key(s[i]); };
  select_topk(key_at, n, k, sh);
  for (int i = threadIdx.x; i < k; i += SEL_NT) {
    out_vals[(size_t)row * k + i] = key_float(sh.cand_key[i]);
    if (out_idx) out_idx[(size_t)row * k + i] = sh.cand_idx[i];
    if (out_idx64) out_idx64[(size_t)row * k + i] = index_base + sh.cand_idx[i];
  }
}

// ---------------------------------------------------------------------------------------------
// Two-stage selection for long rows (vocabulary logits, index score rows): stage 1 spreads a row
// over many workgroups -- each holds a chunk of 256*PT keys in REGISTERS, radix-selects the chunk's
// top-k with register-resident passes (no global re-reads) and emits exactly k candidates; stage 2
// merges rows x chunks x kc candidates.  One workgroup per row (the single-stage kernels above)
// keeps only `rows` CUs busy and re-reads the row 5 times.

constexpr int CH_NT = 256;
constexpr int CH_FAST_MAXK = 64;   // threshold pre-filter for k <= this (sampling candidates)
constexpr int CH_FAST_CAP = 512;   // survivors ranked in LDS; more fall back to the radix select

struct ChunkFast {
  u32x4 tmax[CH_NT / 4];
  u32x4 kv[CH_FAST_CAP / 2];  // survivors as (key, index) pairs, two per 16 B
  uint32_t n, thr;
};

template <int PT>
__global__ __launch_bounds__(CH_NT) void chunk_topk_kernel(const void* __restrict__ src, int src_bf16, long ld, int n,
                                                           int k, int kc, uint32_t* __restrict__ cand_key,
                                                           int* __restrict__ cand_idx, int index_base = 0) {
  __shared__ uint32_t hist[256];
  __shared__ uint32_t bc[2];
  __shared__ uint32_t cnt[2];
  __shared__ ChunkFast fst;
  const int row = blockIdx.y, c = blockIdx.x, nchunks = gridDim.x;
  const int chunk = CH_NT * PT;
  const int start = c * chunk;
  const int len = min(chunk, n - start);
  const int tid = threadIdx.x, lane = tid & 63;
  const float* sf = reinterpret_cast<const float*>(src) + (size_t)row * ld + start;
  const bf16* sb = reinterpret_cast<const bf16*>(src) + (size_t)row * ld + start;
  // Each thread reads 16-B vectors (8 bf16 or 4 fp32 keys): key j of this thread is element
  // idx_of(j) of the chunk.  Strided 2-4 B loads (one 128-256 B request per wave instruction) held
  // the kernel to ~1 TB/s.
  static_assert(CH_NT == 256 && PT % 8 == 0, "idx_of assumes 256 threads and whole 16-B vectors");
  const int lg = src_bf16 ? 3 : 2;
  auto idx_of = [&](int j) { return ((j >> lg) << (8 + lg)) + (tid << lg) + (j & ((1 << lg) - 1)); };
  const bool vec_ok = ((reinterpret_cast<uintptr_t>(src_bf16 ? (const void*)sb : (const void*)sf)) & 15) == 0;
  uint32_t key[PT];
  if (src_bf16) {
#pragma unroll
    for (int v = 0; v < PT / 8; ++v) {
      const int i0 = v * (CH_NT * 8) + tid * 8;
      if (vec_ok && i0 + 8 <= len) {
        float f[8];
        unpack8(*reinterpret_cast<const u32x4*>(sb + i0), f);
#pragma unroll
        for (int e = 0; e < 8; ++e) key[8 * v + e] = float_key(f[e]);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) key[8 * v + e] = i0 + e < len ? float_key(bf2f(sb[i0 + e])) : 0u;
      }
    }
  } else {
#pragma unroll
    for (int v = 0; v < PT / 4; ++v) {
      const int i0 = v * (CH_NT * 4) + tid * 4;
      if (vec_ok && i0 + 4 <= len) {
        const f32x4 f = *reinterpret_cast<const f32x4*>(sf + i0);
#pragma unroll
        for (int e = 0; e < 4; ++e) key[4 * v + e] = float_key(f[e]);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) key[4 * v + e] = i0 + e < len ? float_key(sf[i0 + e]) : 0u;
      }
    }
  }
  const int kk = min(k, len);
  uint32_t* ok = cand_key + ((size_t)row * nchunks + c) * kc;
  int* oi = cand_idx + ((size_t)row * nchunks + c) * kc;
  if (kk <= CH_FAST_MAXK) {
    // Threshold pre-filter (sampling: k = 64 of 8192 logits).  t = the kk-th largest of the 256
    // per-thread maxima: at least kk keys are >= t (those maxima), so every top-kk key is >= t, and
    // typically only a few hundred keys pass.  The survivors are compacted into LDS and ranked
    // exactly (key desc, index asc): one pass over the registers instead of four histogram passes
    // whose LDS atomics serialise on the handful of top-byte bins logits fall into.  Too many
    // survivors (heavy ties) fall through to the radix select below.
    uint32_t m = 0;
#pragma unroll
    for (int j = 0; j < PT; ++j)
      if (idx_of(j) < len) m = max(m, key[j]);
    reinterpret_cast<uint32_t*>(fst.tmax)[tid] = m;
    if (tid == 0) fst.n = 0;
    __syncthreads();
    // rank of this thread's maximum (desc, thread index asc): 16-B broadcast reads, eight in flight
    // (one dependent LDS round trip per element would cost ~7 us per workgroup)
    int rank = 0;
#pragma unroll 4
    for (int j4 = 0; j4 < CH_NT / 4; ++j4) {
      const u32x4 o4 = fst.tmax[j4];
#pragma unroll
      for (int e = 0; e < 4; ++e) rank += (o4[e] > m) || (o4[e] == m && 4 * j4 + e < tid);
    }
    if (rank == kk - 1) fst.thr = m;
    __syncthreads();
    const uint32_t t = fst.thr;
#pragma unroll
    for (int j = 0; j < PT; ++j) {
      const int i = idx_of(j);
      const int slot = wave_append(&fst.n, i < len && key[j] >= t);
      if (slot >= 0 && slot < CH_FAST_CAP) {
        uint32_t* e2 = reinterpret_cast<uint32_t*>(fst.kv) + 2 * slot;
        e2[0] = key[j];
        e2[1] = (uint32_t)(index_base + start + i);
      }
    }
    __syncthreads();
    const int ns = (int)fst.n;
    if (ns <= CH_FAST_CAP) {
      // pad to a multiple of 8 pairs with (key 0, index max): never ranked above a survivor
      const int ns8 = min(CH_FAST_CAP, (ns + 7) & ~7);
      if (tid < ns8 - ns) {
        uint32_t* e2 = reinterpret_cast<uint32_t*>(fst.kv) + 2 * (ns + tid);
        e2[0] = 0u;
        e2[1] = 0xffffffffu;
      }
      __syncthreads();
      for (int a = tid; a < ns; a += CH_NT) {
        const uint32_t* ea = reinterpret_cast<const uint32_t*>(fst.kv) + 2 * a;
        const uint32_t ka = ea[0], ia = ea[1];
        int r = 0;
        for (int u2 = 0; u2 < ns8 / 2; u2 += 4) {
          u32x4 q[4];
#pragma unroll
          for (int z = 0; z < 4; ++z) q[z] = fst.kv[u2 + z];
#pragma unroll
          for (int z = 0; z < 4; ++z) {
            r += (q[z][0] > ka) || (q[z][0] == ka && q[z][1] < ia);
            r += (q[z][2] > ka) || (q[z][2] == ka && q[z][3] < ia);
          }
        }
        if (r < kk) {
          ok[r] = ka;
          oi[r] = (int)ia;
        }
      }
      for (int i = kk + tid; i < kc; i += CH_NT) {
        ok[i] = 0u;
        oi[i] = -1;
      }
      return;
    }
    __syncthreads();  // uniform: every thread read the same count
  }
  uint32_t prefix = 0, pmask = 0, need = (uint32_t)kk;
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int i = tid; i < 256; i += CH_NT) hist[i] = 0;
    __syncthreads();
    // LDS atomics straight into the 256-bin histogram: they serialise only on equal bins, so the
    // one badly clustered case -- a whole wave in one bin (cosine scores share the top byte) -- takes
    // one wave-aggregated add instead (a ballot/leader loop per distinct bin measured slower on
    // logits, whose keys spread over a dozen top-byte bins)
#pragma unroll
    for (int j = 0; j < PT; ++j) {
      const int i = idx_of(j);
      const int bin = (i < len && (key[j] & pmask) == prefix) ? (int)((key[j] >> shift) & 255u) : -1;
      const int b0 = __builtin_amdgcn_readfirstlane(bin);
      if (__all(bin == b0)) {
        if (lane == 0 && b0 >= 0) atomicAdd(&hist[b0], 64u);
      } else if (bin >= 0) {
        atomicAdd(&hist[bin], 1u);
      }
    }
    __syncthreads();
    if (tid < 64) {
      uint32_t cc[4], sum = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        cc[j] = hist[255 - 4 * tid - j];
        sum += cc[j];
      }
      uint32_t incl = sum;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(incl, o, 64);
        if (tid >= o) incl += t;
      }
      const uint32_t excl = incl - sum;
      if (excl < need && need <= incl) {
        uint32_t acc = excl;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (acc + cc[j] >= need) {
            bc[0] = 255u - 4u * tid - j;
            bc[1] = need - acc;
            break;
          }
          acc += cc[j];
        }
      }
    }
    __syncthreads();
    prefix |= bc[0] << shift;
    pmask |= 255u << shift;
    need = bc[1];
    __syncthreads();
  }
  if (tid == 0) {
    cnt[0] = 0;
    cnt[1] = 0;
  }
  __syncthreads();
  const uint32_t n_gt = (uint32_t)kk - need;
#pragma unroll
  for (int j = 0; j < PT; ++j) {
    const int i = idx_of(j);
    const bool valid = i < len;
    const int pg = wave_append(&cnt[0], valid && key[j] > prefix);
    if (pg >= 0) {
      ok[pg] = key[j];
      oi[pg] = index_base + start + i;
    }
    const int pe = wave_append(&cnt[1], valid && key[j] == prefix);
    if (pe >= 0 && (uint32_t)pe < need) {
      ok[n_gt + pe] = key[j];
      oi[n_gt + pe] = index_base + start + i;
    }
  }
  for (int i = kk + tid; i < kc; i += CH_NT) {
    ok[i] = 0u;
    oi[i] = -1;
  }
}

// Stage 2 of sampling: <= 1024 candidates per row -> sorted top-k -> HF top-p -> multinomial.
__global__ __launch_bounds__(SEL_NT) void sample_merge_kernel(const uint32_t* __restrict__ cand_key,
                                                              const int* __restrict__ cand_idx, int ncand,
                                                              const float* __restrict__ temperature,
                                                              const int* __restrict__ top_k,
                                                              const float* __restrict__ top_p, int vocab,
                                                              unsigned long long seed, int64_t* __restrict__ counters,
                                                              int* __restrict__ out_tokens) {
  __shared__ uint32_t skey[SEL_MAXK];
  __shared__ int sidx[SEL_MAXK];
  __shared__ float probs[SEL_MAXK];
  const int row = blockIdx.x, tid = threadIdx.x;
  const float T = temperature ? temperature[row] : 1.f;
  int k = (T <= 0.f) ? 1 : (top_k && top_k[row] > 0 ? top_k[row] : 64);
  k = min(k, min(64, vocab));
  const int nc = min(ncand, SEL_MAXK);
  for (int i = tid; i < SEL_MAXK; i += SEL_NT) {
    skey[i] = i < ncand ? cand_key[(size_t)row * ncand + i] : 0u;
    sidx[i] = i < ncand ? cand_idx[(size_t)row * ncand + i] : 0x7fffffff;
  }
  __syncthreads();
  for (int size = 2; size <= SEL_MAXK; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = tid; t < SEL_MAXK; t += SEL_NT) {
        const int u2 = t ^ stride;
        if (u2 > t) {
          const bool desc = (t & size) == 0;
          const uint32_t ka = skey[t], kb = skey[u2];
          const int ia = sidx[t], ib = sidx[u2];
          const bool a_first = ka > kb || (ka == kb && ia < ib);
          if (a_first != desc) {
            skey[t] = kb;
            skey[u2] = ka;
            sidx[t] = ib;
            sidx[u2] = ia;
          }
        }
      }
      __syncthreads();
    }
  }
  if (tid != 0) return;
  if (T <= 0.f) {
    out_tokens[row] = sidx[0];
    return;
  }
  // HF TopKLogitsWarper: the candidates tied with the k-th value stay in (exact while no 8192-token
  // chunk holds more than 64 logits >= the k-th value: the chunk stage keeps 64 per chunk)
  while (k < nc && skey[k] == skey[k - 1] && skey[k] > kNegInfKey) ++k;  // (never over -inf / padding)
  const float P = top_p ? top_p[row] : 1.f;
  const float x0 = key_float(skey[0]) / T;
  float total = 0.f;
  for (int i = 0; i < k; ++i) {
    const float e = __expf(key_float(skey[i]) / T - x0);
    probs[i] = e;
    total += e;
  }
  int keep = k;
  if (P < 1.f) {
    const float thr = (1.f - P) * total;
    float cum = 0.f;
    for (int i = k - 1; i >= 1; --i) {
      cum += probs[i];
      if (cum <= thr) keep = i;
      else break;
    }
  }
  float kept = 0.f;
  for (int i = 0; i < keep; ++i) kept += probs[i];
  const long long cval = counters ? counters[row] : 0;
  if (counters) counters[row] = cval + 1;
  const unsigned long long r =
      splitmix64(seed ^ splitmix64((unsigned long long)cval * 0x9E3779B97F4A7C15ull + (unsigned long long)row));
  const float uu = (float)(r >> 40) * (1.f / 16777216.f);
  const float target = uu * kept;
  float acc = 0.f;
  int pick = keep - 1;
  for (int i = 0; i < keep; ++i) {
    acc += probs[i];
    if (acc > target) {
      pick = i;
      break;
    }
  }
  out_tokens[row] = sidx[pick];
}

// Stage 2 of index top-k: radix select over the candidate keys (L2-resident) + sort + emit.
__global__ __launch_bounds__(SEL_NT) void topk_merge_kernel(const uint32_t* __restrict__ cand_key,
                                                            const int* __restrict__ cand_idx, int ncand, int k,
                                                            float* __restrict__ out_vals, int* __restrict__ out_idx,
                                                            int64_t index_base, int64_t* __restrict__ out_idx64) {
  __shared__ SelShared sh;
  const int row = blockIdx.x;
  const uint32_t* ck = cand_key + (size_t)row * ncand;
  const int* ci = cand_idx + (size_t)row * ncand;
  auto key_at = [&](int i) -> uint32_t { return ck[i]; };
  select_topk(key_at, ncand, k, sh);
  for (int i = threadIdx.x; i < k; i += SEL_NT) {
    const int pos = sh.cand_idx[i];
    const int idx = (pos >= 0 && pos < ncand) ? ci[pos] : -1;
    out_vals[(size_t)row * k + i] = key_float(sh.cand_key[i]);
    if (out_idx) out_idx[(size_t)row * k + i] = idx;
    if (out_idx64) out_idx64[(size_t)row * k + i] = idx >= 0 ? index_base + idx : -1;
  }
}

int sample_tokens_2stage(const void* logits, int logits_f32, long ld, int rows, int vocab, const float* temperature,
                         const int* top_k, const float* top_p, unsigned long long seed, int64_t* counters,
                         int* out_tokens, void* workspace, size_t workspace_bytes, hipStream_t s) {
  if (rows <= 0) return 0;
  constexpr int PT = 32, KC = 64;
  const int chunk = CH_NT * PT;
  const int nchunks = (vocab + chunk - 1) / chunk;
  const int ncand = nchunks * KC;
  const size_t need = (size_t)rows * ncand * 8;
  if (ncand > SEL_MAXK || workspace_bytes < need) return hipErrorInvalidValue;
  uint32_t* ck = reinterpret_cast<uint32_t*>(workspace);
  int* ci = reinterpret_cast<int*>(ck + (size_t)rows * ncand);
  hipLaunchKernelGGL(chunk_topk_kernel<PT>, dim3(nchunks, rows), dim3(CH_NT), 0, s, logits, logits_f32 ? 0 : 1, ld,
                     vocab, KC, KC, ck, ci);
  hipLaunchKernelGGL(sample_merge_kernel, dim3(rows), dim3(SEL_NT), 0, s, ck, ci, ncand, temperature, top_k, top_p,
                     vocab, seed, counters, out_tokens);
  return hipGetLastError();
}

// Vocab-parallel sampling under tensor parallelism: stage 1 on this rank's slice of the vocabulary
// (token ids offset by the slice start), candidates [rows][ncand] keys then [rows][ncand] ids; the TP
// ranks all-gather them and every rank runs stage 2 on the same union with the same counters, so all
// ranks draw the same token without a broadcast.  The union of per-chunk top-64s holds the global
// top-k (k <= 64), so the draw is the replicated head's draw on the same logits.
int sample_candidates(const void* logits, int logits_f32, long ld, int rows, int vocab, int index_base,
                      uint32_t* cand_key, int* cand_idx, int ncand, hipStream_t s) {
  if (rows <= 0) return 0;
  constexpr int PT = 32, KC = 64;
  const int nchunks = (vocab + CH_NT * PT - 1) / (CH_NT * PT);
  if (vocab <= 0 || ncand != nchunks * KC) return hipErrorInvalidValue;
  hipLaunchKernelGGL(chunk_topk_kernel<PT>, dim3(nchunks, rows), dim3(CH_NT), 0, s, logits, logits_f32 ? 0 : 1, ld,
                     vocab, KC, KC, cand_key, cand_idx, index_base);
  return hipGetLastError();
}

int sample_merge(const uint32_t* cand_key, const int* cand_idx, int ncand, int rows, int vocab,
                 const float* temperature, const int* top_k, const float* top_p, unsigned long long seed,
                 int64_t* counters, int* out_tokens, hipStream_t s) {
  if (rows <= 0) return 0;
  if (ncand <= 0 || ncand > SEL_MAXK) return hipErrorInvalidValue;
  hipLaunchKernelGGL(sample_merge_kernel, dim3(rows), dim3(SEL_NT), 0, s, cand_key, cand_idx, ncand, temperature, top_k,
                     top_p, vocab, seed, counters, out_tokens);
  return hipGetLastError();
}

int topk_rows_2stage(const float* scores, long ld, int rows, int n, int k, float* out_vals, int* out_idx,
                     int64_t index_base, int64_t* out_idx64, void* workspace, size_t workspace_bytes, hipStream_t s) {
  if (rows <= 0) return 0;
  if (k < 1 || k > SEL_MAXK || k > n) return hipErrorInvalidValue;
  constexpr int PT = 32;
  const int chunk = CH_NT * PT;
  const int kc = ((k + 63) / 64) * 64;
  const int nchunks = (n + chunk - 1) / chunk;
  const int ncand = nchunks * kc;
  if (workspace_bytes < (size_t)rows * ncand * 8) return hipErrorInvalidValue;
  uint32_t* ck = reinterpret_cast<uint32_t*>(workspace);
  int* ci = reinterpret_cast<int*>(ck + (size_t)rows * ncand);
  hipLaunchKernelGGL(chunk_topk_kernel<PT>, dim3(nchunks, rows), dim3(CH_NT), 0, s, scores, 0, ld, n, k, kc, ck, ci);
  hipLaunchKernelGGL(topk_merge_kernel, dim3(rows), dim3(SEL_NT), 0, s, ck, ci, ncand, k, out_vals, out_idx,
                     index_base, out_idx64);
  return hipGetLastError();
}

// One thread per 32 tokens (one mask word): the row flag and the word are read once, the logits
// of the disallowed tokens are overwritten with -inf.  Grid (ceil(words / 256), rows); rows
// without the flag return after one load.
__global__ __launch_bounds__(256) void mask_logits_kernel(void* __restrict__ logits, int logits_f32, long ld,
                                                          int vocab, const uint32_t* __restrict__ mask, int words,
                                                          long mask_ld, const int* __restrict__ row_flags) {
  const int row = blockIdx.y;
  if (row_flags[row] == 0) return;
  const int w = blockIdx.x * 256 + threadIdx.x;
  if (w >= words) return;
  const uint32_t bits = mask[(size_t)row * mask_ld + w];
  if (bits == 0xFFFFFFFFu) return;
  const int t0 = w * 32, n = min(32, vocab - t0);
  if (logits_f32) {
    float* l = reinterpret_cast<float*>(logits) + (size_t)row * ld + t0;
    for (int j = 0; j < n; ++j)
      if (!((bits >> j) & 1u)) l[j] = -INFINITY;
  } else {
    bf16* l = reinterpret_cast<bf16*>(logits) + (size_t)row * ld + t0;
    for (int j = 0; j < n; ++j)
      if (!((bits >> j) & 1u)) l[j] = f2bf(-INFINITY);
  }
}

int mask_logits(void* logits, int logits_f32, long ld, int rows, int vocab, const uint32_t* mask, int words,
                const int* row_flags, hipStream_t s, long mask_ld) {
  if (rows <= 0) return 0;
  if (mask_ld <= 0) mask_ld = words;
  if (vocab <= 0 || words * 32 < vocab || mask_ld < words) return hipErrorInvalidValue;
  hipLaunchKernelGGL(mask_logits_kernel, dim3((words + 255) / 256, rows), dim3(256), 0, s, logits, logits_f32, ld,
                     vocab, mask, words, mask_ld, row_flags);
  return hipGetLastError();
}

int sample_tokens(const void* logits, int logits_f32, long ld, int rows, int vocab, const float* temperature,
                  const int* top_k, const float* top_p, unsigned long long seed, int64_t* counters, int* out_tokens,
                  float* out_logprobs, hipStream_t s) {
  if (rows <= 0) return 0;
  if (vocab <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(sample_kernel, dim3(rows), dim3(SEL_NT), 0, s, logits, logits_f32, ld, vocab, temperature, top_k,
                     top_p, seed, counters, out_tokens, out_logprobs);
  return hipGetLastError();
}

int topk_rows(const float* scores, long ld, int rows, int n, int k, float* out_vals, int* out_idx, int64_t index_base,
              int64_t* out_idx64, hipStream_t s) {
  if (rows <= 0) return 0;
  if (k < 1 || k > SEL_MAXK || k > n) return hipErrorInvalidValue;
  hipLaunchKernelGGL(topk_rows_kernel, dim3(rows), dim3(SEL_NT), 0, s, scores, ld, n, k, out_vals, out_idx, index_base,
                     out_idx64);
  return hipGetLastError();
}

}  // namespace dab

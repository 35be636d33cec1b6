// Host-side launchers of the gfx950 kernel library.  Every launcher validates the shape
// constraints its kernel relies on, enqueues on the given stream (graph-capture safe: no
// allocation, no synchronisation) and returns a hipError_t value (0 = success).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <string>
#include <vector>

namespace dab {

inline int div_up_host(int a, int b) { return (a + b - 1) / b; }

// Optional Infinity-Cache warm-up riding on a latency-bound launch (common.h l3_warm): up to two byte
// ranges (16-B multiples) read by ``blocks`` workgroups appended to the kernel's grid.
struct L3Warm {
  const char* ptr[2];
  long bytes[2];
  int blocks;  // 0: off
};

// norm.hip
int rmsnorm(void* out, void* res_out, const void* x, const void* res_in, const void* w, int rows, int cols, float eps,
            hipStream_t s);
int rmsnorm_slabs(void* out, void* res_out, const void* slabs, int S, long slab_stride, const void* res_in,
                  const void* w, int rows, int cols, float eps, hipStream_t s, int slab_bf16 = 0);
int layernorm(void* out, const void* x, const void* res_in, const void* gamma, const void* beta, int rows, int cols,
              float eps, hipStream_t s);
int bert_embed(void* out, const int* ids, const int* pos_ids, const int* type_ids, const void* word, const void* pos,
               const void* type, const void* gamma, const void* beta, int rows, int cols, float eps, hipStream_t s);
int embed_gather(void* out, const int* ids, const void* table, int rows, int cols, hipStream_t s);
int mean_pool(float* out, void* out_bf16, const void* hidden, const int* cu_seqlens, int batch, int cols,
              int normalize, hipStream_t s);

// elementwise.hip
int gelu(void* out, const void* x, const void* bias, size_t rows, int cols, hipStream_t s);
int silu_mul(void* out, const void* x, size_t rows, int F, hipStream_t s, int interleaved = 0);
int rope_kv_write(const void* qkv, int ld, const int* positions, const void* cos_sin, void* q_out, void* k_cache,
                  void* v_cache, const int64_t* slots, int T, int Hq, int Hkv, int D, int block_size, hipStream_t s,
                  const void* slabs = nullptr, int S = 0, long slab_stride = 0, int slab_bf16 = 0);

// attention.hip
int flash_attention(const void* q, long q_stride_tok, long q_stride_head, const void* k, const void* v,
                    long kv_stride_tok, long kv_stride_head, const void* k_cache, const void* v_cache,
                    const int* block_tables, int max_blocks, int block_size, void* out, long o_stride_tok,
                    long o_stride_head, const int* cu_q, const int* cu_k, const int* ctx_k, int batch,
                    int max_seqlen_q, int Hq, int Hkv, int D, int causal, int paged, float scale, hipStream_t s,
                    const int* rope_pos = nullptr, const void* rope_cs = nullptr);
int paged_decode_attention(const void* q, const void* k_cache, const void* v_cache, const int* block_tables,
                           int max_blocks, int block_size, const int* ctx_lens, void* out, float* part_o,
                           float* part_m, float* part_l, int* counters, int batch, int Hq, int Hkv, int D,
                           int part_size, int max_parts, float scale, hipStream_t s,
                           const int* order = nullptr, const L3Warm* warm = nullptr);

// gemm.hip
// b_rows > 0: B is an ops.shuffle_weights copy of b_rows (>= N) rows; epilogue 4 = SwiGLU over 8-row
// [gate | up] groups
int gemm_bt(const void* A, long lda, const void* B, long ldb, void* C, long ldc, const void* bias, const void* residual,
            long ldr, int M, int N, int K, int epilogue, int out_f32, const int* row_group, const int* q_group,
            const uint32_t* allow, int allow_words, hipStream_t s, int b_rows = 0, int b_group = 1);

// gemm256.hip (large-M prefill / encoder GEMM, 256x256 phased schedule; epilogue 0 none, 1 GELU,
// 2 SwiGLU on [gate 16 | up 16]-interleaved weight rows; bias / residual optional)
int gemm256_ok(int M, int N, int K, long lda, long ldb);
int gemm256_candidates(const void* A, long lda, const void* B, long ldb, int M, int N, int K, const int* row_group,
                       const int* q_group, const float* thr, int* cnt, float* cand_val, int* cand_idx, int cap,
                       hipStream_t s, int b_rows = 0);
// b_shuf: B in the ops.shuffle_weights layout (the decode GEMM's copy); epilogue 4 = SwiGLU over
// 8-row [gate | up] groups
// diagnostic per-tile s_memtime stamps (benchmarks/gemm_stamps.py); returns the grid or -error
int gemm256_candidates_stamped(const void* A, long lda, const void* B, int M, int N, int K, int b_rows,
                               const float* thr, int* cnt, float* cand_val, int* cand_idx, int cap, void* stamps,
                               int stamp_tiles, hipStream_t s);
int gemm256_stamped(const void* A, long lda, const void* B, void* C, const void* bias, const void* residual, int M,
                    int N, int K, int epilogue, int b_shuf, void* stamps, int stamp_tiles, hipStream_t s, int store_aux);
int gemm256(const void* A, long lda, const void* B, long ldb, void* C, long ldc, const void* bias,
            const void* residual, long ldr, int M, int N, int K, int epilogue, hipStream_t s, int b_shuf = 0,
            int b_group = 1);

// gemm_mid.hip (M = 256..4096: mixed serving steps / single prompts; grouped stream-K over the N x K
// plane, 128 x 256 tiles, in-launch last-arriver combine; B in the shuffle_weights layout;
// epilogue 0 none (+ residual) or 4 SwiGLU over 8-row [gate | up] groups)
int gemm_mid_ok(int M, int N, int K, long lda);
long gemm_mid_slab_bytes();
int gemm_mid_counters(int M, int N);
int gemm_mid(const void* A, long lda, const void* B, void* C, long ldc, const void* residual, long ldr, int M, int N,
             int K, int epilogue, void* slabs, long slab_bytes, int* cnt, int n_cnt, hipStream_t s, int variant = 0,
             int b_group = 1);

// stream_gemm.hip (warp-specialised decode GEMM, M <= 256: bf16 / SwiGLU / fp32 split-K slabs; cfg selects
// the tile / ring configuration, stream_gemm_bn(cfg) = weight rows per workgroup)
int stream_gemm(const void* X, long ldx, const void* W, long ldw, void* out, long ldo, const void* residual, long ldr,
                int M, int N, int K, int S, int epilogue, hipStream_t s, int nt_weights, int cfg, float norm_eps = 0.f,
                int slab_bf16 = 0, int w_group = 1);
int stream_gemm_bn(int cfg);
// fp32 (or bf16: slab_bf16) split-K slabs [S][M][N] -> bf16 [M, N] (+ residual)
int slab_reduce(void* out, long ldo, const void* slabs, int S, int M, int N, const void* residual, long ldr,
                hipStream_t s, int slab_bf16 = 0);
// index_scan.hip: persistent scan for 1..64 queries at K <= 1024, 65..96 at K <= 768 (queries staged in
// LDS once), K % 256 == 0
int index_scan_candidates(const void* X, long ldx, const void* W, long ldw, int M, int N, int K, const int* row_group,
                          const int* q_group, const float* thr, int* cnt, float* cand_val, int* cand_idx, int cap,
                          hipStream_t s);
// ... the same scan over a copy of the rows in the shuffle_weights layout (>= round_up(N, 32) rows)
int index_scan_candidates_shuf(const void* X, long ldx, const void* W, int M, int N, int K, const int* row_group,
                               const int* q_group, const float* thr, int* cnt, float* cand_val, int* cand_idx,
                               int cap, hipStream_t s);
int stream_score_candidates(const void* X, long ldx, const void* W, long ldw, int M, int N, int K, const int* row_group,
                            const int* q_group, const float* thr, int* cnt, float* cand_val, int* cand_idx, int cap,
                            hipStream_t s);
int stream_score_candidates_shuf(const void* X, long ldx, const void* W, int M, int N, int K, const int* row_group,
                                 const int* q_group, const float* thr, int* cnt, float* cand_val, int* cand_idx,
                                 int cap, hipStream_t s);
int stream_gemm_max_m(int cfg);
void stream_gemm_set_slice_xcd(int on);
int stream_gemm_slice_xcd();
int stream_gemm_shuffled(int cfg);  // 1: cfg reads weights in the ops.shuffle_weights layout

// select.hip
// Disallowed tokens of the rows with row_flags[r] != 0 (mask bit clear) -> -inf logits, in place
// (JSON-constrained decoding); rows without the flag are untouched.
int mask_logits(void* logits, int logits_f32, long ld, int rows, int vocab, const uint32_t* mask, int words,
                const int* row_flags, hipStream_t s, long mask_ld = 0);
// vocab-parallel sampling (TP): stage 1 on a vocabulary slice, stage 2 on the all-gathered candidates
int sample_candidates(const void* logits, int logits_f32, long ld, int rows, int vocab, int index_base,
                      uint32_t* cand_key, int* cand_idx, int ncand, hipStream_t s);
int sample_merge(const uint32_t* cand_key, const int* cand_idx, int ncand, int rows, int vocab,
                 const float* temperature, const int* top_k, const float* top_p, unsigned long long seed,
                 int64_t* counters, int* out_tokens, hipStream_t s);
int sample_tokens(const void* logits, int logits_f32, long ld, int rows, int vocab, const float* temperature,
                  const int* top_k, const float* top_p, unsigned long long seed, int64_t* counters, int* out_tokens,
                  float* out_logprobs, hipStream_t s);
int topk_rows(const float* scores, long ld, int rows, int n, int k, float* out_vals, int* out_idx, int64_t index_base,
              int64_t* out_idx64, hipStream_t s);

// two-stage variants (chunked across workgroups); workspace = rows * candidates * 8 bytes
int sample_tokens_2stage(const void* logits, int logits_f32, long ld, int rows, int vocab, const float* temperature,
                         const int* top_k, const float* top_p, unsigned long long seed, int64_t* counters,
                         int* out_tokens, void* workspace, size_t workspace_bytes, hipStream_t s);
int topk_rows_2stage(const float* scores, long ld, int rows, int n, int k, float* out_vals, int* out_idx,
                     int64_t index_base, int64_t* out_idx64, void* workspace, size_t workspace_bytes, hipStream_t s);

// gemm.hip: scores >= thr[m] appended per query (exact threshold top-k of the vector index)
int gemm_score_candidates(const void* A, long lda, const void* B, long ldb, int M, int N, int K, const int* row_group,
                          const int* q_group, const float* thr, int* cnt, float* cand_val, int* cand_idx, int cap,
                          hipStream_t s, int b_rows = 0);

// allreduce.hip: one-shot all-reduce over IPC-mapped peer buffers (TP decode on one node)
size_t allreduce_signal_bytes();
// TP decode: this rank's split-K slabs (S > 0) or bf16 partial (S == 0) -> all-reduce -> + residual
// -> RMSNorm, one launch (bitwise slab_reduce + custom_allreduce + rmsnorm)
int custom_allreduce_rmsnorm(const std::vector<uintptr_t>& bases, int rank, const float* slabs, int S,
                             long slab_stride, const void* x, const void* res_in, void* res_out, void* out,
                             const void* w, int rows, int cols, float eps, long half_bytes, long spin_limit,
                             hipStream_t s);
int custom_allreduce(const std::vector<uintptr_t>& bases, int rank, void* data, long nbytes, long half_bytes,
                     long spin_limit, hipStream_t s);
int allreduce_buffer_alloc(long bytes, int uncached, uintptr_t* out);
int allreduce_buffer_free(uintptr_t ptr);
int ipc_get_handle(uintptr_t ptr, std::string* handle);
int ipc_open_handle(const std::string& handle, uintptr_t* out);
int ipc_close_handle(uintptr_t ptr);
int ipc_probe(uintptr_t ptr);
int allreduce_error(uintptr_t base, int clear);
int allreduce_error_async(uintptr_t base, void* host_word, hipStream_t s);

}  // namespace dab

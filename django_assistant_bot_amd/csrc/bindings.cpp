// pybind11 module `_native`: kernel launchers (raw device pointers + stream handles passed as
// integers from the python ops layer, which owns shape/dtype validation) and the native host
// runtime (tokenizer, paged-KV block manager, retrieval post-processing).
#include <hip/hip_runtime.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <stdexcept>
#include <string>

#include "kernels/launchers.h"
#include "runtime/json_grammar.h"
#include "runtime/kv_manager.h"
#include "runtime/rag.h"
#include "runtime/tokenizer.h"
#include "runtime/trace.h"

namespace py = pybind11;
using u = uintptr_t;

#define VP(x) reinterpret_cast<void*>(x)
#define CVP(x) reinterpret_cast<const void*>(x)
#define ST(x) reinterpret_cast<hipStream_t>(x)

static void check(int err, const char* name) {
  if (err) throw std::runtime_error(std::string("dab kernel '") + name + "' failed: " + hipGetErrorString((hipError_t)err));
}

PYBIND11_MODULE(_native, m) {
  m.doc() = "MI355X (gfx950) kernels and native runtime of django_assistant_bot_amd";
  m.def("roctx_available", &dab::trace::available);
  // one-shot all-reduce over IPC peer buffers (parallel/custom_allreduce.py)
  m.def("allreduce_signal_bytes", &dab::allreduce_signal_bytes);
  m.def("custom_allreduce", [](const std::vector<uintptr_t>& bases, int rank, u data, long nbytes, long half_bytes,
                               long spin_limit, u s) {
    check(dab::custom_allreduce(bases, rank, VP(data), nbytes, half_bytes, spin_limit, ST(s)), "custom_allreduce");
  });
  m.def("custom_allreduce_rmsnorm", [](const std::vector<uintptr_t>& bases, int rank, u slabs, int S, long slab_stride,
                                       u x, u res_in, u res_out, u out, u w, int rows, int cols, float eps,
                                       long half_bytes, long spin_limit, u s) {
    check(dab::custom_allreduce_rmsnorm(bases, rank, (const float*)slabs, S, slab_stride, CVP(x), CVP(res_in),
                                        VP(res_out), VP(out), CVP(w), rows, cols, eps, half_bytes, spin_limit, ST(s)),
          "custom_allreduce_rmsnorm");
  });
  m.def("allreduce_buffer_alloc", [](long bytes, bool uncached) {
    uintptr_t p = 0;
    check(dab::allreduce_buffer_alloc(bytes, uncached ? 1 : 0, &p), "allreduce_buffer_alloc");
    return p;
  }, py::arg("bytes"), py::arg("uncached") = true);
  m.def("allreduce_buffer_free", [](u ptr) { check(dab::allreduce_buffer_free(ptr), "allreduce_buffer_free"); });
  m.def("ipc_get_handle", [](u ptr) {
    std::string h;
    check(dab::ipc_get_handle(ptr, &h), "ipc_get_handle");
    return py::bytes(h);
  });
  m.def("ipc_open_handle", [](const std::string& h) {
    uintptr_t p = 0;
    check(dab::ipc_open_handle(h, &p), "ipc_open_handle");
    return p;
  });
  m.def("ipc_probe", [](u ptr) { check(dab::ipc_probe(ptr), "ipc_probe"); });
  m.def("ipc_close_handle", [](u ptr) { check(dab::ipc_close_handle(ptr), "ipc_close_handle"); });
  m.def("allreduce_error", &dab::allreduce_error, py::arg("base"), py::arg("clear") = 1);
  m.def("allreduce_error_async", [](u base, u host_word, u s) {
    check(dab::allreduce_error_async(base, VP(host_word), ST(s)), "allreduce_error_async");
  });
  m.def("roctx_push", [](const std::string& name) { return dab::trace::range_push(name.c_str()); });
  m.def("roctx_pop", &dab::trace::range_pop);
  m.def("roctx_mark", [](const std::string& name) { dab::trace::mark(name.c_str()); });

  // ---------------- kernels ----------------
  m.def("rmsnorm", [](u out, u res_out, u x, u res_in, u w, int rows, int cols, float eps, u s) {
    check(dab::rmsnorm(VP(out), VP(res_out), CVP(x), CVP(res_in), CVP(w), rows, cols, eps, ST(s)), "rmsnorm");
  });
  m.def("layernorm", [](u out, u x, u res_in, u gamma, u beta, int rows, int cols, float eps, u s) {
    check(dab::layernorm(VP(out), CVP(x), CVP(res_in), CVP(gamma), CVP(beta), rows, cols, eps, ST(s)), "layernorm");
  });
  m.def("bert_embed", [](u out, u ids, u pos_ids, u type_ids, u word, u pos, u type, u gamma, u beta, int rows, int cols,
                         float eps, u s) {
    check(dab::bert_embed(VP(out), (const int*)ids, (const int*)pos_ids, (const int*)type_ids, CVP(word), CVP(pos),
                          CVP(type), CVP(gamma), CVP(beta), rows, cols, eps, ST(s)),
          "bert_embed");
  });
  m.def("embed_gather", [](u out, u ids, u table, int rows, int cols, u s) {
    check(dab::embed_gather(VP(out), (const int*)ids, CVP(table), rows, cols, ST(s)), "embed_gather");
  });
  m.def("mean_pool", [](u out, u out_bf16, u hidden, u cu, int batch, int cols, int normalize, u s) {
    check(dab::mean_pool((float*)out, VP(out_bf16), CVP(hidden), (const int*)cu, batch, cols, normalize, ST(s)),
          "mean_pool");
  });
  m.def("gelu", [](u out, u x, u bias, size_t rows, int cols, u s) {
    check(dab::gelu(VP(out), CVP(x), CVP(bias), rows, cols, ST(s)), "gelu");
  });
  m.def("silu_mul", [](u out, u x, size_t rows, int F, u s, int interleaved) {
    check(dab::silu_mul(VP(out), CVP(x), rows, F, ST(s), interleaved), "silu_mul");
  }, py::arg("out"), py::arg("x"), py::arg("rows"), py::arg("F"), py::arg("s"), py::arg("interleaved") = 0);
  m.def("rope_kv_write", [](u qkv, int ld, u positions, u cos_sin, u q_out, u k_cache, u v_cache, u slots, int T,
                            int Hq, int Hkv, int D, int block_size, u s, u slabs, int S, long slab_stride,
                            int slab_bf16) {
    check(dab::rope_kv_write(CVP(qkv), ld, (const int*)positions, CVP(cos_sin), VP(q_out), VP(k_cache), VP(v_cache),
                             (const int64_t*)slots, T, Hq, Hkv, D, block_size, ST(s), CVP(slabs), S, slab_stride,
                             slab_bf16),
          "rope_kv_write");
  }, py::arg("qkv"), py::arg("ld"), py::arg("positions"), py::arg("cos_sin"), py::arg("q_out"), py::arg("k_cache"),
     py::arg("v_cache"), py::arg("slots"), py::arg("T"), py::arg("Hq"), py::arg("Hkv"), py::arg("D"),
     py::arg("block_size"), py::arg("s"), py::arg("slabs") = 0, py::arg("S") = 0, py::arg("slab_stride") = 0,
     py::arg("slab_bf16") = 0);
  m.def("rmsnorm_slabs", [](u out, u res_out, u slabs, int S, long slab_stride, u res_in, u w, int rows, int cols,
                            float eps, u s, int slab_bf16) {
    check(dab::rmsnorm_slabs(VP(out), VP(res_out), CVP(slabs), S, slab_stride, CVP(res_in), CVP(w), rows, cols, eps,
                             ST(s), slab_bf16),
          "rmsnorm_slabs");
  }, py::arg("out"), py::arg("res_out"), py::arg("slabs"), py::arg("S"), py::arg("slab_stride"), py::arg("res_in"),
     py::arg("w"), py::arg("rows"), py::arg("cols"), py::arg("eps"), py::arg("s"), py::arg("slab_bf16") = 0);
  m.def("flash_attention",
        [](u q, long qst, long qsh, u k, u v, long kvst, long kvsh, u kc, u vc, u bt, int max_blocks, int bs, u out,
           long ost, long osh, u cu_q, u cu_k, u ctx_k, int batch, int max_sq, int Hq, int Hkv, int D, int causal,
           int paged, float scale, u s) {
          check(dab::flash_attention(CVP(q), qst, qsh, CVP(k), CVP(v), kvst, kvsh, CVP(kc), CVP(vc), (const int*)bt,
                                     max_blocks, bs, VP(out), ost, osh, (const int*)cu_q, (const int*)cu_k,
                                     (const int*)ctx_k, batch, max_sq, Hq, Hkv, D, causal, paged, scale, ST(s)),
                "flash_attention");
        });
  // Llama prefill attention with RoPE applied to Q on load (positions int32 [Tq], cos/sin table)
  m.def("flash_attention_rope",
        [](u q, long qst, long qsh, u kc, u vc, u bt, int max_blocks, int bs, u out, long ost, long osh, u cu_q,
           u ctx_k, int batch, int max_sq, int Hq, int Hkv, int D, int causal, float scale, u rope_pos, u rope_cs,
           u s) {
          check(dab::flash_attention(CVP(q), qst, qsh, nullptr, nullptr, 0, 0, CVP(kc), CVP(vc), (const int*)bt,
                                     max_blocks, bs, VP(out), ost, osh, (const int*)cu_q, nullptr, (const int*)ctx_k,
                                     batch, max_sq, Hq, Hkv, D, causal, 1, scale, ST(s), (const int*)rope_pos,
                                     CVP(rope_cs)),
                "flash_attention_rope");
        });
  // HIP stream restricted to a set of CUs (bit i of the mask words = CU i): lets a compute-bound
  // workload run beside a bandwidth-bound one on disjoint CUs (benchmarks/overlap_probe.py).  The
  // handle is wrapped by torch.cuda.ExternalStream; destroy it with destroy_stream.
  m.def("create_cu_masked_stream", [](std::vector<uint32_t> mask) {
    hipStream_t st = nullptr;
    check(hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data()), "hipExtStreamCreateWithCUMask");
    return reinterpret_cast<uintptr_t>(st);
  });
  m.def("destroy_stream", [](u s) { check(hipStreamDestroy(ST(s)), "hipStreamDestroy"); });
  m.def("paged_decode_attention", [](u q, u kc, u vc, u bt, int max_blocks, int bs, u ctx, u out, u po, u pm, u pl,
                                     u cnt, int batch, int Hq, int Hkv, int D, int part_size, int max_parts,
                                     float scale, u s, u order, u w0, long w0_bytes, u w1, long w1_bytes,
                                     int w_blocks) {
    dab::L3Warm warm{{(const char*)w0, (const char*)w1}, {w0_bytes, w1_bytes}, w_blocks};
    check(dab::paged_decode_attention(CVP(q), CVP(kc), CVP(vc), (const int*)bt, max_blocks, bs, (const int*)ctx, VP(out),
                                      (float*)po, (float*)pm, (float*)pl, (int*)cnt, batch, Hq, Hkv, D, part_size,
                                      max_parts, scale, ST(s), (const int*)order, &warm),
          "paged_decode_attention");
  }, py::arg("q"), py::arg("kc"), py::arg("vc"), py::arg("bt"), py::arg("max_blocks"), py::arg("bs"), py::arg("ctx"),
     py::arg("out"), py::arg("po"), py::arg("pm"), py::arg("pl"), py::arg("cnt"), py::arg("batch"), py::arg("Hq"),
     py::arg("Hkv"), py::arg("D"), py::arg("part_size"), py::arg("max_parts"), py::arg("scale"), py::arg("s"),
     py::arg("order") = 0, py::arg("w0") = 0, py::arg("w0_bytes") = 0, py::arg("w1") = 0, py::arg("w1_bytes") = 0,
     py::arg("w_blocks") = 0);
  m.def("gemm_bt", [](u A, long lda, u B, long ldb, u C, long ldc, u bias, u residual, long ldr, int M, int N, int K,
                      int epilogue, int out_f32, u row_group, u q_group, u allow, int allow_words, u s, int b_rows,
                      int b_group) {
    check(dab::gemm_bt(CVP(A), lda, CVP(B), ldb, VP(C), ldc, CVP(bias), CVP(residual), ldr, M, N, K, epilogue, out_f32,
                       (const int*)row_group, (const int*)q_group, (const uint32_t*)allow, allow_words, ST(s), b_rows,
                       b_group),
          "gemm_bt");
  }, py::arg("A"), py::arg("lda"), py::arg("B"), py::arg("ldb"), py::arg("C"), py::arg("ldc"), py::arg("bias"),
     py::arg("residual"), py::arg("ldr"), py::arg("M"), py::arg("N"), py::arg("K"), py::arg("epilogue"),
     py::arg("out_f32"), py::arg("row_group"), py::arg("q_group"), py::arg("allow"), py::arg("allow_words"),
     py::arg("s"), py::arg("b_rows") = 0, py::arg("b_group") = 1);
  m.def("gemm_mid_ok", &dab::gemm_mid_ok);
  m.def("gemm_mid_slab_bytes", &dab::gemm_mid_slab_bytes);
  m.def("gemm_mid_counters", &dab::gemm_mid_counters);
  m.def("gemm_mid", [](u A, long lda, u B, u C, long ldc, u residual, long ldr, int M, int N, int K, int epilogue,
                       u slabs, long slab_bytes, u cnt, int n_cnt, u s, int variant, int b_group) {
    check(dab::gemm_mid(CVP(A), lda, CVP(B), VP(C), ldc, CVP(residual), ldr, M, N, K, epilogue, VP(slabs), slab_bytes,
                        (int*)cnt, n_cnt, ST(s), variant, b_group),
          "gemm_mid");
  }, py::arg("A"), py::arg("lda"), py::arg("B"), py::arg("C"), py::arg("ldc"), py::arg("residual"), py::arg("ldr"),
     py::arg("M"), py::arg("N"), py::arg("K"), py::arg("epilogue"), py::arg("slabs"), py::arg("slab_bytes"),
     py::arg("cnt"), py::arg("n_cnt"), py::arg("s"), py::arg("variant") = 0, py::arg("b_group") = 1);
  m.def("gemm256_ok", &dab::gemm256_ok);
  m.def("gemm256_stamped", [](u A, long lda, u B, u C, u bias, u residual, int M, int N, int K, int epilogue,
                              int b_shuf, u stamps, int stamp_tiles, u s, int store_aux) {
    const int r = dab::gemm256_stamped(CVP(A), lda, CVP(B), VP(C), CVP(bias), CVP(residual), M, N, K, epilogue, b_shuf,
                                       VP(stamps), stamp_tiles, ST(s), store_aux);
    if (r < 0) check(-r, "gemm256_stamped");
    return r;
  }, py::arg("A"), py::arg("lda"), py::arg("B"), py::arg("C"), py::arg("bias"), py::arg("residual"), py::arg("M"),
     py::arg("N"), py::arg("K"), py::arg("epilogue"), py::arg("b_shuf"), py::arg("stamps"), py::arg("stamp_tiles"),
     py::arg("s"), py::arg("store_aux") = 0);
  m.def("gemm256_candidates_stamped", [](u A, long lda, u B, int M, int N, int K, int b_rows, u thr, u cnt, u cand_val,
                                          u cand_idx, int cap, u stamps, int stamp_tiles, u s) {
    const int r = dab::gemm256_candidates_stamped(CVP(A), lda, CVP(B), M, N, K, b_rows, (const float*)thr, (int*)cnt,
                                                  (float*)cand_val, (int*)cand_idx, cap, VP(stamps), stamp_tiles, ST(s));
    if (r < 0) check(-r, "gemm256_candidates_stamped");
    return r;
  });
  m.def("gemm256", [](u A, long lda, u B, long ldb, u C, long ldc, u bias, u residual, long ldr, int M, int N, int K,
                      int epilogue, u s, int b_shuf, int b_group) {
    check(dab::gemm256(CVP(A), lda, CVP(B), ldb, VP(C), ldc, CVP(bias), CVP(residual), ldr, M, N, K, epilogue, ST(s),
                       b_shuf, b_group),
          "gemm256");
  }, py::arg("A"), py::arg("lda"), py::arg("B"), py::arg("ldb"), py::arg("C"), py::arg("ldc"), py::arg("bias"),
     py::arg("residual"), py::arg("ldr"), py::arg("M"), py::arg("N"), py::arg("K"), py::arg("epilogue"), py::arg("s"),
     py::arg("b_shuf") = 0, py::arg("b_group") = 1);
  m.def("gemm_score_candidates", [](u A, long lda, u B, long ldb, int M, int N, int K, u row_group, u q_group, u thr,
                                    u cnt, u cand_val, u cand_idx, int cap, u s) {
    check(dab::gemm_score_candidates(CVP(A), lda, CVP(B), ldb, M, N, K, reinterpret_cast<const int*>(row_group),
                                     reinterpret_cast<const int*>(q_group), reinterpret_cast<const float*>(thr),
                                     reinterpret_cast<int*>(cnt), reinterpret_cast<float*>(cand_val),
                                     reinterpret_cast<int*>(cand_idx), cap, ST(s)),
          "gemm_score_candidates");
  });
  // candidates over a shuffle_weights copy of the rows (b_rows of them): 1..16 queries on the
  // persistent scan, 17..128 on the weight-streaming kernel, more on the 8-phase GEMM
  m.def("score_candidates_shuf", [](u A, long lda, u Wshuf, int M, int N, int K, u row_group, u q_group, u thr,
                                    u cnt, u cand_val, u cand_idx, int cap, u s, int b_rows) {
    auto* rg = reinterpret_cast<const int*>(row_group);
    auto* qg = reinterpret_cast<const int*>(q_group);
    auto* th = reinterpret_cast<const float*>(thr);
    auto* ct = reinterpret_cast<int*>(cnt);
    auto* cv = reinterpret_cast<float*>(cand_val);
    auto* ci = reinterpret_cast<int*>(cand_idx);
    int rc = hipErrorInvalidValue;
    if (K % 256 == 0 && ((M <= 64 && K <= 1024) || (M <= 96 && K <= 768)))
      rc = dab::index_scan_candidates_shuf(CVP(A), lda, CVP(Wshuf), M, N, K, rg, qg, th, ct, cv, ci, cap, ST(s));
    else if (M <= 64 || K % 128)
      rc = dab::stream_score_candidates_shuf(CVP(A), lda, CVP(Wshuf), M, N, K, rg, qg, th, ct, cv, ci, cap, ST(s));
    else  // 65+ queries past the scan's limits: the persistent 256x256 kernel (gemm256 G_CAND); at
          // 97-127 queries of 768 the streaming kernel took 5.6-6.0 ms on 10M rows, gemm256 ~3.9
      rc = dab::gemm_score_candidates(CVP(A), lda, CVP(Wshuf), K, M, N, K, rg, qg, th, ct, cv, ci, cap, ST(s), b_rows);
    check(rc, "score_candidates_shuf");
  }, py::arg("A"), py::arg("lda"), py::arg("Wshuf"), py::arg("M"), py::arg("N"), py::arg("K"), py::arg("row_group"),
     py::arg("q_group"), py::arg("thr"), py::arg("cnt"), py::arg("cand_val"), py::arg("cand_idx"), py::arg("cap"),
     py::arg("s"), py::arg("b_rows") = 0);
  m.def("stream_gemm", [](u X, long ldx, u W, long ldw, u out, long ldo, u residual, long ldr, int M, int N, int K,
                          int S, int epilogue, u s, int nt, int cfg, float norm_eps, int slab_bf16, int w_group) {
    check(dab::stream_gemm(CVP(X), ldx, CVP(W), ldw, VP(out), ldo, CVP(residual), ldr, M, N, K, S, epilogue, ST(s), nt,
                           cfg, norm_eps, slab_bf16, w_group),
          "stream_gemm");
  }, py::arg("X"), py::arg("ldx"), py::arg("W"), py::arg("ldw"), py::arg("out"), py::arg("ldo"), py::arg("residual"),
     py::arg("ldr"), py::arg("M"), py::arg("N"), py::arg("K"), py::arg("S"), py::arg("epilogue"), py::arg("s"),
     py::arg("nt"), py::arg("cfg"), py::arg("norm_eps") = 0.f, py::arg("slab_bf16") = 0, py::arg("w_group") = 1);
  m.def("stream_gemm_bn", &dab::stream_gemm_bn);
  m.def("stream_gemm_max_m", &dab::stream_gemm_max_m);
  m.def("stream_gemm_set_slice_xcd", &dab::stream_gemm_set_slice_xcd);
  m.def("stream_gemm_slice_xcd", &dab::stream_gemm_slice_xcd);
  m.def("stream_gemm_shuffled", &dab::stream_gemm_shuffled);
  m.def("slab_reduce", [](u out, long ldo, u slabs, int S, int M, int N, u residual, long ldr, u s, int slab_bf16) {
    check(dab::slab_reduce(VP(out), ldo, CVP(slabs), S, M, N, CVP(residual), ldr, ST(s), slab_bf16), "slab_reduce");
  }, py::arg("out"), py::arg("ldo"), py::arg("slabs"), py::arg("S"), py::arg("M"), py::arg("N"), py::arg("residual"),
     py::arg("ldr"), py::arg("s"), py::arg("slab_bf16") = 0);
  m.def("sample_tokens", [](u logits, int f32, long ld, int rows, int vocab, u temp, u top_k, u top_p,
                            unsigned long long seed, u counters, u out_tokens, u out_logprobs, u s) {
    check(dab::sample_tokens(CVP(logits), f32, ld, rows, vocab, (const float*)temp, (const int*)top_k,
                             (const float*)top_p, seed, (int64_t*)counters, (int*)out_tokens, (float*)out_logprobs,
                             ST(s)),
          "sample_tokens");
  });
  m.def("topk_rows", [](u scores, long ld, int rows, int n, int k, u out_vals, u out_idx, long long base, u out_idx64,
                        u s) {
    check(dab::topk_rows((const float*)scores, ld, rows, n, k, (float*)out_vals, (int*)out_idx, base,
                         (int64_t*)out_idx64, ST(s)),
          "topk_rows");
  });

  m.def("sample_tokens_2stage", [](u logits, int f32, long ld, int rows, int vocab, u temp, u top_k, u top_p,
                                   unsigned long long seed, u counters, u out_tokens, u ws, size_t ws_bytes, u s) {
    check(dab::sample_tokens_2stage(CVP(logits), f32, ld, rows, vocab, (const float*)temp, (const int*)top_k,
                                    (const float*)top_p, seed, (int64_t*)counters, (int*)out_tokens, VP(ws), ws_bytes,
                                    ST(s)),
          "sample_tokens_2stage");
  });
  m.def("mask_logits", [](u logits, int f32, long ld, int rows, int vocab, u mask, int words, u row_flags, u s,
                          long mask_ld) {
    check(dab::mask_logits(VP(logits), f32, ld, rows, vocab, (const uint32_t*)mask, words, (const int*)row_flags,
                           ST(s), mask_ld),
          "mask_logits");
  });
  m.def("sample_candidates", [](u logits, int f32, long ld, int rows, int vocab, int base, u keys, u idx, int ncand,
                                u s) {
    check(dab::sample_candidates(CVP(logits), f32, ld, rows, vocab, base, (uint32_t*)keys, (int*)idx, ncand, ST(s)),
          "sample_candidates");
  });
  m.def("sample_merge", [](u keys, u idx, int ncand, int rows, int vocab, u temp, u top_k, u top_p,
                           unsigned long long seed, u counters, u out_tokens, u s) {
    check(dab::sample_merge((const uint32_t*)keys, (const int*)idx, ncand, rows, vocab, (const float*)temp,
                            (const int*)top_k, (const float*)top_p, seed, (int64_t*)counters, (int*)out_tokens, ST(s)),
          "sample_merge");
  });
  m.def("topk_rows_2stage", [](u scores, long ld, int rows, int n, int k, u out_vals, u out_idx, long long base,
                               u out_idx64, u ws, size_t ws_bytes, u s) {
    check(dab::topk_rows_2stage((const float*)scores, ld, rows, n, k, (float*)out_vals, (int*)out_idx, base,
                                (int64_t*)out_idx64, VP(ws), ws_bytes, ST(s)),
          "topk_rows_2stage");
  });

  // ---------------- tokenizer ----------------
  py::class_<dab::TokenizerConfig>(m, "TokenizerConfig")
      .def(py::init<>())
      .def_readwrite("vocab_size", &dab::TokenizerConfig::vocab_size)
      .def_readwrite("first_id", &dab::TokenizerConfig::first_id)
      .def_readwrite("last_id", &dab::TokenizerConfig::last_id)
      .def_readwrite("pad_id", &dab::TokenizerConfig::pad_id)
      .def_readwrite("unk_id", &dab::TokenizerConfig::unk_id)
      .def_readwrite("cls_id", &dab::TokenizerConfig::cls_id)
      .def_readwrite("sep_id", &dab::TokenizerConfig::sep_id)
      .def_readwrite("max_word_chars", &dab::TokenizerConfig::max_word_chars);
  py::class_<dab::HashTokenizer>(m, "HashTokenizer")
      .def(py::init<const dab::TokenizerConfig&>())
      .def("encode", &dab::HashTokenizer::encode, py::arg("text"), py::arg("add_special") = true,
           py::arg("max_len") = 0)
      .def(
          "encode_batch",
          [](const dab::HashTokenizer& t, const std::vector<std::string>& texts, bool add_special, int max_len,
             int threads) {
            std::vector<int32_t> ids;
            std::vector<int64_t> offs;
            {
              py::gil_scoped_release rel;
              t.encode_batch(texts, add_special, max_len, threads, ids, offs);
            }
            py::array_t<int32_t> a(ids.size());
            std::copy(ids.begin(), ids.end(), a.mutable_data());
            py::array_t<int64_t> o(offs.size());
            std::copy(offs.begin(), offs.end(), o.mutable_data());
            return py::make_tuple(a, o);
          },
          py::arg("texts"), py::arg("add_special") = true, py::arg("max_len") = 0, py::arg("threads") = 8)
      .def("decode", &dab::HashTokenizer::decode, py::arg("ids"), py::arg("skip_special") = true)
      .def("token_texts",
           [](const dab::HashTokenizer& t) {
             py::list out;
             for (const auto& w : t.token_texts()) out.append(py::bytes(w));
             return out;
           })
      .def_static("count_words", &dab::HashTokenizer::count_words);

  // ---------------- JSON-constrained decoding ----------------
  py::class_<dab::JsonVocab, std::shared_ptr<dab::JsonVocab>>(m, "JsonVocab")
      .def(py::init([](const std::vector<py::bytes>& toks, const std::vector<int32_t>& eos) {
             std::vector<std::string> t;
             t.reserve(toks.size());
             for (const auto& b : toks) t.emplace_back(b);
             return std::make_shared<dab::JsonVocab>(t, eos);
           }),
           py::arg("tokens"), py::arg("eos_ids"))
      .def("vocab_size", &dab::JsonVocab::vocab_size)
      .def("words", &dab::JsonVocab::words)
      .def("trie_nodes", &dab::JsonVocab::trie_nodes)
      .def("cache_entries", &dab::JsonVocab::cache_entries);
  py::class_<dab::JsonMatcher>(m, "JsonMatcher")
      .def(py::init<std::shared_ptr<dab::JsonVocab>, int, int>(), py::arg("vocab"), py::arg("max_depth") = 24,
           py::arg("max_ws") = 8)
      .def("fill_mask",
           [](dab::JsonMatcher& j, int remaining, u out) {
             py::gil_scoped_release rel;
             return j.fill_mask(remaining, (uint32_t*)out);
           })
      .def("advance", &dab::JsonMatcher::advance)
      .def("done", &dab::JsonMatcher::done)
      .def("broken", &dab::JsonMatcher::broken)
      .def("completion", [](const dab::JsonMatcher& j) { return py::bytes(j.completion()); })
      .def("completion_len", &dab::JsonMatcher::completion_len)
      .def("text", [](const dab::JsonMatcher& j) { return py::bytes(j.text()); });
  py::class_<dab::SchemaAutomaton, std::shared_ptr<dab::SchemaAutomaton>>(m, "SchemaAutomaton")
      .def(py::init<std::shared_ptr<dab::JsonVocab>, int, int, const std::vector<int32_t>&,
                    const std::vector<std::vector<int32_t>>&, const std::vector<std::vector<int32_t>>&>(),
           py::arg("vocab"), py::arg("n_states"), py::arg("start"), py::arg("accept"), py::arg("edges"),
           py::arg("eps"))
      .def("dfa_states", &dab::SchemaAutomaton::dfa_states)
      .def("accepts", [](dab::SchemaAutomaton& a, const py::bytes& b) {
        int d = a.start();
        for (unsigned char c : std::string(b)) {
          d = a.step(d, c);
          if (d < 0) return false;
        }
        return a.accepting(d);
      });
  py::class_<dab::SchemaMatcher>(m, "SchemaMatcher")
      .def(py::init<std::shared_ptr<dab::SchemaAutomaton>>(), py::arg("automaton"))
      .def("fill_mask",
           [](dab::SchemaMatcher& j, int remaining, u out) {
             py::gil_scoped_release rel;
             return j.fill_mask(remaining, (uint32_t*)out);
           })
      .def("advance", &dab::SchemaMatcher::advance)
      .def("done", &dab::SchemaMatcher::done)
      .def("broken", &dab::SchemaMatcher::broken)
      .def("completion_len", &dab::SchemaMatcher::completion_len)
      .def("text", [](const dab::SchemaMatcher& j) { return py::bytes(j.text()); });
  m.def("json_accepts", [](const py::bytes& b, bool complete, int max_depth, int max_ws) {
    return dab::json_accepts(std::string(b), complete, max_depth, max_ws);
  }, py::arg("bytes"), py::arg("complete") = true, py::arg("max_depth") = 64, py::arg("max_ws") = 255);

  // ---------------- KV block manager ----------------
  py::class_<dab::KVBlockManager>(m, "KVBlockManager")
      .def(py::init<int, int, bool>(), py::arg("num_blocks"), py::arg("block_size"), py::arg("prefix_cache") = true)
      .def("add_sequence", &dab::KVBlockManager::add_sequence)
      .def("extend", &dab::KVBlockManager::extend)
      .def("append_tokens", &dab::KVBlockManager::append_tokens)
      .def("commit_prefix", &dab::KVBlockManager::commit_prefix)
      .def("free_sequence", &dab::KVBlockManager::free_sequence)
      .def("has", &dab::KVBlockManager::has)
      .def("num_tokens", &dab::KVBlockManager::num_tokens)
      .def("capacity_tokens", &dab::KVBlockManager::capacity_tokens)
      .def("num_free_blocks", &dab::KVBlockManager::num_free_blocks)
      .def("num_blocks", &dab::KVBlockManager::num_blocks)
      .def("block_size", &dab::KVBlockManager::block_size)
      .def("prefix_hits", &dab::KVBlockManager::prefix_hits)
      .def("blocks", &dab::KVBlockManager::blocks)
      .def("slot_mapping_into",
           [](const dab::KVBlockManager& k, int64_t seq, int start, int n, u out) {
             k.slot_mapping(seq, start, n, (int64_t*)out);
           })
      .def("prepare_decode_into",
           [](dab::KVBlockManager& k, const std::vector<int64_t>& seqs, const std::vector<int32_t>& toks,
              int max_blocks, u ids, u pos, u slots, u ctx, u bt) {
             return k.prepare_decode(seqs, toks, max_blocks, (int32_t*)ids, (int32_t*)pos, (int64_t*)slots,
                                     (int32_t*)ctx, (int32_t*)bt);
           })
      .def("block_table_into", [](const dab::KVBlockManager& k, const std::vector<int64_t>& seqs, int max_blocks,
                                  u out) { k.block_table(seqs, max_blocks, (int32_t*)out); });

  // ---------------- retrieval post-processing ----------------
  m.def(
      "aggregate_documents",
      [](py::array_t<float, py::array::c_style | py::array::forcecast> dist,
         py::array_t<int64_t, py::array::c_style | py::array::forcecast> doc_ids, int max_scores_n, int top_n) {
        if (dist.size() != doc_ids.size()) throw std::invalid_argument("distances / doc_ids length mismatch");
        auto r = dab::aggregate_documents(dist.data(), doc_ids.data(), (int)dist.size(), max_scores_n, top_n);
        py::list out;
        for (auto& d : r) out.append(py::make_tuple(d.doc_id, d.score));
        return out;
      },
      py::arg("distances"), py::arg("doc_ids"), py::arg("max_scores_n"), py::arg("top_n"));
  m.def(
      "merge_topk",
      [](py::array_t<float, py::array::c_style | py::array::forcecast> vals,
         py::array_t<int64_t, py::array::c_style | py::array::forcecast> ids, int k_out) {
        if (vals.ndim() != 2 || ids.ndim() != 2 || vals.shape(0) != ids.shape(0) || vals.shape(1) != ids.shape(1))
          throw std::invalid_argument("vals / ids must be [S, k] arrays of the same shape");
        const int S = (int)vals.shape(0), k = (int)vals.shape(1);
        py::array_t<float> ov(k_out);
        py::array_t<int64_t> oi(k_out);
        dab::merge_topk(vals.data(), ids.data(), S, k, k_out, ov.mutable_data(), oi.mutable_data());
        return py::make_tuple(ov, oi);
      },
      py::arg("vals"), py::arg("ids"), py::arg("k_out"));
}

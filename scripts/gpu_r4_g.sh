#!/bin/bash
# Round 4, call G: candidate-list kernels (tests), index search with the 1/16 and 1/64 samples, and
# the epilogue store cache-policy A/B on the real GEMM launcher.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r4g_tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
    -k "score_candidates or index_ or gemm256" &&
$S r4g_idx16 300 python -u benchmarks/index_bench.py --iters 10 --warmup 3 --batch 1 16 64 96 128 512 --sample-stride 16 &&
$S r4g_idx64 300 python -u benchmarks/index_bench.py --iters 10 --warmup 3 --batch 1 16 64 96 128 512 --sample-stride 64 &&
$S r4g_gemm 500 python -u benchmarks/gemm_bench.py --shapes llama,bge --store-aux 2 18 --rounds 3 --iters 10 &&
$S r4g_stagger 400 python -u benchmarks/gemm_stamps.py --shapes bge-qkv,bge-up,cand-shape,llama-qkv --aux 18 --stagger 0 0.5

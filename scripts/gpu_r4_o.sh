#!/bin/bash
# Round 4, call O: gemm256 K-loop in 4 merged phases (two quadrants per MFMA block, half the barriers).
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r4o_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
    -k "gemm256 or score_candidates or index_ or swiglu or gelu" &&
$S r4o_gemm 400 python -u benchmarks/gemm_bench.py --shapes llama,bge --rounds 3 --iters 10 &&
$S r4o_stamps 300 python -u benchmarks/gemm_stamps.py --shapes bge-qkv,bge-o,llama-qkv,llama-o --cand 0.0016 &&
$S r4o_index 300 python -u benchmarks/index_bench.py --iters 10 --warmup 3 --batch 128 512

#!/bin/bash
# Round 4, call N: the group stagger re-made per tile (the two groups' epilogues side by side).
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r4n_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
    -k "gemm256 or score_candidates or index_ or gemm_bt or swiglu or gelu" &&
$S r4n_stamps 300 python -u benchmarks/gemm_stamps.py --shapes bge-qkv,bge-o,bge-up,bge-down,llama-o --cand 0.0016 &&
$S r4n_gemm 400 python -u benchmarks/gemm_bench.py --shapes llama,bge --rounds 3 --iters 10 &&
$S r4n_embed 300 python -u benchmarks/embed_bench.py --chunks 1000000 &&
$S r4n_index 300 python -u benchmarks/index_bench.py --iters 10 --warmup 3 --batch 128 256 512

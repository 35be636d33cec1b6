#!/bin/bash
# Round 4, call L: compact candidate epilogue (branch-free hit masks + one append loop).
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r4l_tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
    -k "score_candidates or index_ or gemm256" &&
$S r4l_stamps 300 python -u benchmarks/gemm_stamps.py --shapes "" --cand 0.0016 0.0004 &&
$S r4l_index 300 python -u benchmarks/index_bench.py --iters 10 --warmup 3 --batch 64 128 256 512

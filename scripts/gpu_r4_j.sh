#!/bin/bash
# Round 4, call J: index-scan ring depth A/B (8 vs 12 chunks in flight per wave) + its kernel tests.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r4j_tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
    -k "score_candidates or index_" &&
$S r4j_ring 300 python -u benchmarks/index_bench.py --iters 10 --warmup 3 --batch 1 16 32 64 96 --scan-ring 8 12 8 12

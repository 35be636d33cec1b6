#!/bin/bash
# Round 6, call B: gemm_mid with the 6-stage 32-deep ring (default) vs the 3-stage 64-deep ring, and
# with the split-tile combine skipped (timing only), on the mid shapes.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r6b_mid_tests 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm_mid" &&
$S r6b_mid_bench 600 python -u benchmarks/gemm_bench.py --shapes mid --rounds 3 --iters 10 --mid-variants

#!/bin/bash
# Round 6, call A: numerics of the new mid-M stream-K GEMM (gemm_mid.hip), then its timing against
# the current native dispatch, gemm256 and hipBLASLt on the mid shapes.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r6a_mid_tests 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm_mid" &&
$S r6a_mid_bench 600 python -u benchmarks/gemm_bench.py --shapes mid --rounds 3 --iters 10

#!/bin/bash
# Round 6, call AJ: the reverted gemm_mid combine (A/B against call AI) --
# GEMM tests, then the mid-M table against hipBLASLt.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r6aj_tests 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread \
  -k "gemm_mid or grouped or fragment_layout" &&
$S r6aj_mid 600 python -u benchmarks/gemm_bench.py --shapes mid --rounds 3 --iters 10

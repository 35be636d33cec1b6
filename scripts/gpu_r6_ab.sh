#!/bin/bash
# Round 6, call AB: short prefill steps on the streaming kernels -- model tests, the GEMM microbench,
# the headline bench.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r6ab_tests 600 python -u -m pytest tests/test_models_gpu.py tests/test_hf_dirs.py tests/test_bench_gpu.py -x -q \
  --timeout 300 --timeout-method thread &&
$S r6ab_small 300 python -u benchmarks/small_prefill_gemm.py &&
$S r6ab_bench 600 python -u bench.py --steps 10 --warmup 3

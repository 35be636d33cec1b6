#!/bin/bash
# Round 6, call AC: gemm_mid from M = 1 on the fragment-layout weights -- GEMM and model tests, the
# small-prefill microbench, the headline bench.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r6ac_tests 700 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_hf_dirs.py -x -q \
  --timeout 300 --timeout-method thread -k "gemm or model or prefill or decode or hf" &&
$S r6ac_small 300 python -u benchmarks/small_prefill_gemm.py &&
$S r6ac_bench 600 python -u bench.py --steps 10 --warmup 3

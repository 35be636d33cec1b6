#!/bin/bash
# Round 6, call Z: prefill tail absorption -- engine / model GPU tests, then the headline bench.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r6z_tests 600 python -u -m pytest tests/test_models_gpu.py tests/test_bench_gpu.py tests/test_app_gpu.py -x -q \
  --timeout 300 --timeout-method thread &&
$S r6z_bench 600 python -u bench.py --steps 10 --warmup 3

#!/bin/bash
# Round 4, call A: new TP D=128 + self-launch tests, then the 1-GPU headline bench.
cd "$(dirname "$0")/.." || exit 1
S=scripts/gpu_step.sh
$S r4a_tests 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
    tests/test_tp_gpu.py tests/test_bench_gpu.py -k "d128 or self_launch or config5" &&
$S r4a_bench 420 python -u bench.py --steps 10 --warmup 3

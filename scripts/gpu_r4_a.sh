#!/bin/bash
# Round 4, call A: config-5 rehearsal (8 TP ranks on the card), then the 1-GPU headline bench.
cd "$(dirname "$0")/.." || exit 1
S=scripts/gpu_step.sh
$S r4a_tests 600 python -u -m pytest -x -v --timeout 450 --timeout-method thread \
    tests/test_bench_gpu.py -k "config5" &&
$S r4a_bench 420 python -u bench.py --steps 10 --warmup 3

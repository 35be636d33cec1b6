#!/bin/bash
# Round 6, call P: deeper weight rings for gate_up on the grouped copy (stream_gemm cfgs 41 / 42).
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r6p_tests 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread \
  -k "grouped or swiglu8" &&
$S r6p_group 300 python -u benchmarks/stream_group_bench.py &&
$S r6p_ab 900 python -u benchmarks/decode_ab.py --arms base,gu22,gu41,gu42 --rounds 3 --steps 40

#!/bin/bash
# Round 6, call X: prefill attention with G = 2 + heaviest-first walk -- numerics, shape A/B, bench.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r6x_tests 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 200 \
  --timeout-method thread -k "attention or flash or prefill or hf or decode_stream" &&
$S r6x_attn 400 python -u benchmarks/attn_prefill_shape.py &&
$S r6x_bench 600 python -u bench.py --steps 10 --warmup 3

#!/bin/bash
# Round 6, call T: heaviest-first, 2-pair walk of the causal prefill attention -- numerics, the
# prefill-shape A/B, and the headline bench.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r6t_tests 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 200 \
  --timeout-method thread -k "attention or flash or prefill or hf or decode_stream" &&
$S r6t_attn 300 python -u benchmarks/attn_prefill_shape.py &&
$S r6t_bench 600 python -u bench.py --steps 10 --warmup 3

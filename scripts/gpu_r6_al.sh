#!/bin/bash
# Round 6, call AL: single-prompt attention on one block per workgroup -- attention / model tests,
# the single-prompt shapes, time to first token.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r6al_tests 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 200 \
  --timeout-method thread -k "attention or flash or prefill or hf or model" &&
ATTN_SINGLE=1 $S r6al_attn 300 python -u benchmarks/attn_prefill_shape.py &&
$S r6al_ttft 400 python -u benchmarks/ttft_bench.py

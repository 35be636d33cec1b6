#!/bin/bash
# Round 6, call N: grouped layouts for every decoder projection (LlamaModel.PROJ_GROUPS) -- the
# model-level bit-equality, then the batch-128 decode A/B per projection.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r6n_tests 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 200 \
  --timeout-method thread -k "grouped or small or consumer" &&
$S r6n_ab 900 python -u benchmarks/decode_ab.py --arms base,all_g8,down_g8,qkvo_g8 --rounds 3 --steps 40

#!/bin/bash
# Round 6, call M: the grouped gate_up layout (shuffle_weights(w, 8)) -- bit-equality on every GEMM that
# reads it, the model-level equality, the per-projection microbench, then the batch-128 decode A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r6m_tests 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 200 \
  --timeout-method thread -k "grouped or gemm_mid or gemm256 or fragment_layout or bf16_decode_slabs or swiglu8" &&
$S r6m_group 300 python -u benchmarks/stream_group_bench.py &&
$S r6m_ab 700 python -u benchmarks/decode_ab.py --arms base,gu_g1 --rounds 3 --steps 40

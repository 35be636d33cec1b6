#!/bin/bash
# Round 6, call AM: decode batches 129..256 with gate_up on gemm_mid -- model / TP tests, decode A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r6am_tests 600 python -u -m pytest tests/test_models_gpu.py tests/test_tp_gpu.py tests/test_bench_gpu.py -x -q \
  --timeout 300 --timeout-method thread &&
$S r6am_b256 600 python -u benchmarks/decode_ab.py --batch 256 --arms base,gu27 --rounds 3 --steps 30 &&
$S r6am_b192 600 python -u benchmarks/decode_ab.py --batch 192 --arms base,gu27 --rounds 3 --steps 30

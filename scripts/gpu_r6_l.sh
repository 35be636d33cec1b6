#!/bin/bash
# Round 6, call L: bf16 split-K decode slabs -- numerics, then the batch-128 decode A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r6l_tests 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 200 \
  --timeout-method thread -k "bf16_split_k or bf16_decode_slabs or rmsnorm_slabs or rope_kv or stream_gemm or slab" &&
$S r6l_ab 700 python -u benchmarks/decode_ab.py --arms slab32,slab16 --rounds 3 --steps 40

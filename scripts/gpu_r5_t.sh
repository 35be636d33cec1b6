#!/bin/bash
# Round 5, call T: two workgroups per CU for the batch-128 streaming GEMMs (cfg 36 / 37, BN 64, 2-stage
# X ring): numerics, then the batch-128 decode A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r5t_tests 300 python -u -m pytest tests/test_kernels_gpu.py -k "test_stream_gemm and (36- or 37-)" -x -q --timeout 120 --timeout-method thread &&
$S r5t_ab 700 python -u benchmarks/decode_ab.py --batch 128 --arms base,occ2,o36_8,down36_8,qkv36_4,qkv36_8,o37_8,down37_8 --rounds 3 --steps 40

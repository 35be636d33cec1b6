#!/bin/bash
# Round 5, call Q: narrow-tile streaming GEMM configs for batch 65-128 decode (cfg 34 BN 32, cfg 35
# BN 48, 2 K-slices: a quarter of the fp32 slab bytes): numerics, then the batch-128 decode A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r5q_tests 300 python -u -m pytest tests/test_kernels_gpu.py -k "test_stream_gemm and (-34- or -35- or 34- or 35-)" -x -q --timeout 120 --timeout-method thread &&
$S r5q_ab 600 python -u benchmarks/decode_ab.py --batch 128 --arms base,narrow,o34_2,down34_2,qkv35_2 --rounds 3 --steps 40

#!/bin/bash
# Round 5, call X: gemm256 next-tile A1 piece staged ahead of the epilogue stores -- numerics (vs
# the phase-1 stage, DAB_G256_PRE=0), the GEMM A/B and the embed bench both ways.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r5x_tests 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "gemm256 or gemm_bt or exact_layout" &&
$S r5x_gemm 500 python -u benchmarks/gemm_bench.py --shapes bge,llama --native-only --ab-pre --rounds 7 &&
$S r5x_embed_pre 300 python -u benchmarks/embed_bench.py --chunks 1000000 &&
DAB_G256_PRE=0 $S r5x_embed_nopre 300 python -u benchmarks/embed_bench.py --chunks 1000000 &&
$S r5x_embed_pre2 300 python -u benchmarks/embed_bench.py --chunks 1000000 &&
DAB_G256_PRE=0 $S r5x_embed_nopre2 300 python -u benchmarks/embed_bench.py --chunks 1000000

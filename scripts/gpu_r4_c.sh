#!/bin/bash
# Round 4, call C: gemm256 on the 32x32x16 MFMA against the 16x16x32 default and hipBLASLt.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r4c_gemm 400 python -u benchmarks/gemm_bench.py --shapes llama,bge --m32 --rounds 3 --iters 10

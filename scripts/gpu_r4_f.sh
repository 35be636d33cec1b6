#!/bin/bash
# Round 4, call F: epilogue store cache policy A/B on the per-tile stamps (short- and long-K shapes).
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r4f_stamps 400 python -u benchmarks/gemm_stamps.py --shapes bge-qkv,bge-o,bge-up,cand-shape,llama-o --aux 0 2 16 18

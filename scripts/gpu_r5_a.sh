#!/bin/bash
# Round 5, call A: mid-M GEMM status, gemm256 after the read-barrier change
# (ADVICE r4), serve-mode reference point.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r5a_gemm_mid 300 python -u benchmarks/gemm_bench.py --shapes mid,llama --rounds 3 --iters 10 &&
$S r5a_serve 600 python -u bench.py --mode serve --steps 3 --warmup 1

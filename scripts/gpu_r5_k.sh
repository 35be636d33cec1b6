#!/bin/bash
# Round 5, call K: prefill-attention scan (fixed tokens, T 256..4096, causal / full) to separate the
# per-workgroup fixed cost from the per-tile cost; the embed bench with the 5-wave encoder attention.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r5k_scan 300 python -u benchmarks/kernel_bench.py attnscan &&
$S r5k_embed 400 python -u benchmarks/embed_bench.py --chunks 1000000

#!/bin/bash
# Round 6, call AO: the secondary BASELINE configs on the final round-6 tree -- config 2 (bge-base batch
# embedding of 1M chunks) and config 3 (in-HBM cosine top-250 over 10M x 768 rows, one shard).
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r6ao_embed 600 python -u benchmarks/embed_bench.py --chunks 1000000 &&
$S r6ao_index 400 python -u benchmarks/index_bench.py

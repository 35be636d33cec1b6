#!/bin/bash
# Round 4, call D: launch-size A/Bs -- encoder batch tokens (config 2) and prefill chunk tokens (headline).
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r4d_emb64k 240 python -u benchmarks/embed_bench.py --chunks 1000000 --max-batch-tokens 65536 &&
$S r4d_emb128k 240 python -u benchmarks/embed_bench.py --chunks 1000000 --max-batch-tokens 131072 &&
$S r4d_emb256k 240 python -u benchmarks/embed_bench.py --chunks 1000000 --max-batch-tokens 262144 &&
$S r4d_pf64k 420 python -u bench.py --steps 5 --warmup 2 --prefill-tokens 65536 &&
$S r4d_pf140k 420 python -u bench.py --steps 5 --warmup 2 --prefill-tokens 140000

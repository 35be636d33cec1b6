#!/bin/bash
# Round 4, call AE: 8-rank DP rehearsal of the driver's scaling command on one card (gloo): bge-base
# retriever, tiny generator, the 1M-row index sharded 8 ways, batch 128 per rank, so every rank's
# search scores 1024 all-gathered queries on the candidate GEMM (M = kCandMaxM).
cd "$GRAFT_REPO_ROOT" || exit 1
export DAB_DIST_BACKEND=gloo
scripts/gpu_step.sh r4ae_dp8 500 python -u bench.py --gpus 8 --llm-model tiny-llama --index-rows 1000000 \
    --batch 128 --max-new-tokens 8 --steps 2 --warmup 1 --no-fast-steps

#!/bin/bash
# Round 4, call V: throughput at the headline's latency -- overlap mode (two engines, one weight
# copy) at smaller per-engine batches.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r4v_ov64 400 python -u bench.py --mode overlap --batch 64 --steps 12 --warmup 2 --no-fast-steps &&
$S r4v_ov96 400 python -u bench.py --mode overlap --batch 96 --steps 10 --warmup 2 --no-fast-steps

#!/bin/bash
# Round 6, call AH: serve mode with mixed prefill + decode steps, re-measured on the final tree.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r6ah_mixed512 600 python -u bench.py --mode serve --mixed-tokens 512 --steps 6 --warmup 2 &&
$S r6ah_mixed1024 600 python -u bench.py --mode serve --mixed-tokens 1024 --steps 6 --warmup 2

#!/bin/bash
# Round 5, call U: prompt tokens per prefill step (the bench's 128 x ~1.09k-token prompts = ~131k
# tokens per batch; 32768 leaves a ~200-token fifth step) -- headline A/B, no fast JSON steps.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
for pt in 32768 33792 45056 66560 135168 32768b; do
  $S r5u_pt$pt 300 python -u bench.py --steps 5 --warmup 2 --no-fast-steps --prefill-tokens ${pt%b} || exit $?
done

#!/bin/bash
# Round 6, call Q: prefill attention at the headline's prefill shape; grouped gate_up A/B in reverse order.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r6q_attn 300 python -u benchmarks/attn_prefill_shape.py &&
$S r6q_ab 700 python -u benchmarks/decode_ab.py --arms gu_g1,base --rounds 3 --steps 40

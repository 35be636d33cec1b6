#!/bin/bash
# Round 6, call AF: grouped layouts at small decode batches (1 / 16).
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r6af_b1 500 python -u benchmarks/decode_ab.py --batch 1 --arms base,all_g8,gu_g1 --rounds 3 --steps 60 &&
$S r6af_b16 500 python -u benchmarks/decode_ab.py --batch 16 --arms base,all_g8,gu_g1 --rounds 3 --steps 60

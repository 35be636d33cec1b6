#!/bin/bash
# Round 6, call AG: down in the grouped layout too? batch 1 / 16 / 128 A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r6ag_b1 500 python -u benchmarks/decode_ab.py --batch 1 --arms base,down_g8 --rounds 3 --steps 60 &&
$S r6ag_b16 500 python -u benchmarks/decode_ab.py --batch 16 --arms base,down_g8 --rounds 3 --steps 60 &&
$S r6ag_b128 700 python -u benchmarks/decode_ab.py --batch 128 --arms base,down_g8 --rounds 4 --steps 40

#!/bin/bash
# Round 5, call H: Infinity-Cache warm-up of the next o / gate_up weights by workgroups appended to
# the small-batch decode attention (VERDICT r4 item 5 structural attempt): parity, then A/B at B=1/8.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r5h_tests 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -k "l3_warm or paged_decode or small_batch" -x -v --timeout 120 --timeout-method thread &&
$S r5h_ab_b1 500 python -u benchmarks/decode_ab.py --batch 1 --arms base,warm32,warm64,warm96,warm160,warm96b128 --rounds 3 --steps 100 &&
$S r5h_ab_b8 500 python -u benchmarks/decode_ab.py --batch 8 --arms base,warm32,warm64,warm96,warm160,warm96b128 --rounds 3 --steps 100

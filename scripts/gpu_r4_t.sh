#!/bin/bash
# Round 4, call T: single-tile encoder attention (<= 64-token chunks at 8 workgroups per CU).
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r4t_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
    tests/test_models_gpu.py -k "flash_packed or bert or embed" &&
$S r4t_embed 300 python -u benchmarks/embed_bench.py --chunks 1000000 &&
bash scripts/prof_embed.sh

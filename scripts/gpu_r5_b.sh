#!/bin/bash
# Round 5, call B: the world-1 RCCL group tests.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r5b_w1 400 python -u -m pytest tests/test_rccl_world1_gpu.py -x -v --timeout 300 --timeout-method thread

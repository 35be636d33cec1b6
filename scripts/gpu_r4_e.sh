#!/bin/bash
# Round 4, call E: the whole GPU suite + smoke, the index search at 1..512 queries (1/64 sample), then
# the launch-size A/Bs of call D.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r4e_suite 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread &&
$S r4e_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" &&
$S r4e_index 300 python -u benchmarks/index_bench.py --iters 10 --warmup 3 --batch 1 16 64 96 128 512 &&
$S r4e_stamps 300 python -u benchmarks/gemm_stamps.py &&
bash scripts/gpu_r4_d.sh

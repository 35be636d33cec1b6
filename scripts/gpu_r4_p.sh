#!/bin/bash
# Round 4, call P (after the 4-phase K-loop): the whole GPU suite + smoke, the headline bench, the
# config 2 / config 3 benches and a rocprofv3 kernel profile of the headline step.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r4p_suite 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread &&
$S r4p_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" &&
$S r4p_bench 600 python -u bench.py --steps 10 --warmup 3 &&
$S r4p_embed 300 python -u benchmarks/embed_bench.py --chunks 1000000 &&
$S r4p_index 300 python -u benchmarks/index_bench.py --iters 10 --warmup 3 --batch 1 16 64 96 128 256 512 &&
bash scripts/prof_bench.sh

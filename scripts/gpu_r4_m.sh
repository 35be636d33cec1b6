#!/bin/bash
# Round 4, call M (after the candidate-epilogue rebuild): the whole GPU suite + smoke, the headline
# bench and the config 3 bench at every batch size.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r4m_suite 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread &&
$S r4m_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" &&
$S r4m_bench 600 python -u bench.py --steps 10 --warmup 3 &&
$S r4m_index 300 python -u benchmarks/index_bench.py --iters 10 --warmup 3 --batch 1 16 64 96 128 256 512

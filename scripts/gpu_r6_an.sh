#!/bin/bash
# Round 6, call AN: validation of the final tree: the whole GPU suite, smoke(), the default bench.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r6an_gpu_tests 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread &&
$S r6an_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" &&
$S r6an_bench 600 python -u bench.py --steps 10 --warmup 3

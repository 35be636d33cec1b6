#!/bin/bash
# Round 4, call AH (final tree): the whole GPU suite + smoke + the headline bench.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r4ah_suite 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread &&
$S r4ah_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" &&
$S r4ah_bench 600 python -u bench.py --steps 10 --warmup 3

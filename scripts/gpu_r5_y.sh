#!/bin/bash
# Round 5, call Y: last validation of the committed tree (in-tree .so rebuilt after the gemm256
# A/B was reverted): the whole GPU suite, smoke(), and the default bench.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r5y_gpu_tests 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread &&
$S r5y_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" &&
$S r5y_bench 600 python -u bench.py --steps 10 --warmup 3

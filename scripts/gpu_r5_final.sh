#!/bin/bash
# Round 5, final checks: the whole GPU test suite as the driver runs it, smoke(), the default bench
# twice, and a rocprofv3 kernel profile of a short bench run (-> gpurun_out/prof_bench_*.md).
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r5z_gpu_tests 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread &&
$S r5z_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" &&
$S r5z_bench 600 python -u bench.py --steps 10 --warmup 3 &&
$S r5z_bench2 600 python -u bench.py --steps 10 --warmup 3 &&
GAP_LAST_MS=4000 $S r5z_prof 600 bash scripts/prof_bench.sh

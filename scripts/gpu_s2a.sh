#!/bin/bash
# session-2 re-entry check: GPU suite, smoke, default bench
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s2a_tests.log 2>&1
rc=$?; tail -3 gpurun_out/s2a_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s2a_smoke.log 2>&1
rc=$?; tail -2 gpurun_out/s2a_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/s2a_bench.log 2>&1
rc=$?; tail -1 gpurun_out/s2a_bench.log; exit $rc

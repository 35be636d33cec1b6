#!/bin/bash
# round-end rehearsal: full gpu suite, smoke(), default bench (as the driver runs them)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s3m_tests.log 2>&1
rc=$?; tail -2 gpurun_out/s3m_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/s3m_smoke.log 2>&1
rc=$?; tail -2 gpurun_out/s3m_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/s3m_bench.log 2>&1
rc=$?; tail -1 gpurun_out/s3m_bench.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc

#!/bin/bash
# selection kernels: numerics + bench (before/after the histogram change via git stash is not possible on the box: run twice)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "topk or sampling or index" > gpurun_out/s2h_tests.log 2>&1
rc=$?; tail -2 gpurun_out/s2h_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python benchmarks/kernel_bench.py select > gpurun_out/s2h_select.log 2>&1
rc=$?; grep op gpurun_out/s2h_select.log; exit $rc

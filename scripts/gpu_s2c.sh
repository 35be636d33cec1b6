#!/bin/bash
# stream_gemm: numerics, then the decode-projection sweep (graph-timed, cold weights)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "stream or skinny" > gpurun_out/s2c_tests.log 2>&1
rc=$?; tail -3 gpurun_out/s2c_tests.log; [ $rc -eq 0 ] || exit $rc
STREAM_NT=1 STREAM_CFGS=10,13,14,15,16 timeout -k 10 600 python benchmarks/kernel_bench.py stream all 128,64 > gpurun_out/s2c_sweep.log 2>&1
rc=$?; cat gpurun_out/s2c_sweep.log; exit $rc

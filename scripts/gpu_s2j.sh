#!/bin/bash
# paged decode: numerics + kernel bench
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread -k "decode or mixed or engine" > gpurun_out/s2j_tests.log 2>&1
rc=$?; tail -1 gpurun_out/s2j_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python benchmarks/kernel_bench.py attn > gpurun_out/s2j_attn.log 2>&1
rc=$?; grep paged gpurun_out/s2j_attn.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python benchmarks/kernel_bench.py decode > gpurun_out/s2j_sweep.log 2>&1
rc=$?; grep sweep gpurun_out/s2j_sweep.log; exit $rc

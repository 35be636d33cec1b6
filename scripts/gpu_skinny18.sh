#!/bin/bash
# M <= 128 weight-streaming GEMM: numerics, then split sweep vs hipBLASLt (cold weights)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -k skinny tests/test_models_gpu.py -x -q > gpurun_out/t18.log 2>&1
rc=$?; tail -3 gpurun_out/t18.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python benchmarks/kernel_bench.py skinny > gpurun_out/sk18.log 2>&1
rc=$?; cat gpurun_out/sk18.log; exit $rc

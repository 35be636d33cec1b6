#!/bin/bash
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q -k "index or scores or topk" > gpurun_out/t28.log 2>&1
rc=$?; tail -3 gpurun_out/t28.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python benchmarks/index_bench.py --rows 10000000 --batch 1 64 512 > gpurun_out/idx28.log 2>&1
rc=$?; tail -1 gpurun_out/idx28.log; exit $rc

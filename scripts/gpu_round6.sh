#!/bin/bash
# skinny decode GEMM: correctness, per-shape timings, end-to-end bench (batch 64)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -q -x -p no:cacheprovider > gpurun_out/gputests6.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/gputests6.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python benchmarks/kernel_bench.py gemm llama8b > gpurun_out/kbench_gemm6.log 2>&1
rc=$?; echo "kbench rc=$rc"; cat gpurun_out/kbench_gemm6.log | grep op
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench6.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench6.log
exit $rc

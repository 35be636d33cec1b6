#!/bin/bash
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -x -p no:cacheprovider > gpurun_out/gputests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/gputests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python benchmarks/kernel_bench.py select > gpurun_out/kbench_sel.log 2>&1
rc=$?; echo "kbench rc=$rc"; grep op gpurun_out/kbench_sel.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py --steps 3 --warmup 1 > gpurun_out/bench4.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench4.log
exit $rc

#!/bin/bash
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
ok_rc() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -x -p no:cacheprovider > gpurun_out/gputests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/gputests.log
ok_rc $rc || exit $rc
timeout -k 10 300 python benchmarks/kernel_bench.py attn > gpurun_out/kbench_attn.log 2>&1
rc=$?; echo "kbench rc=$rc"; cat gpurun_out/kbench_attn.log | grep op
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py --steps 2 --warmup 1 > gpurun_out/bench2.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/bench2.log
exit $rc

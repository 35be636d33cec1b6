#!/bin/bash
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -q -x -p no:cacheprovider -k "skinny or rmsnorm or rope or silu or decode" > gpurun_out/gputests7.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gputests7.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python benchmarks/kernel_bench.py gemm llama8b > gpurun_out/kbench_gemm7.log 2>&1
rc=$?; echo "kbench rc=$rc"; grep skinny gpurun_out/kbench_gemm7.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['op'], d['M'], 'S', d['skinny_splits'], 'warm', d['skinny_us'], d['hipblaslt_us'], 'cold', d['cold_skinny_us'], d['cold_skinny_nt_us'], d['cold_hipblaslt_us'])"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench7.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench7.log
[ $rc -eq 0 ] || exit $rc
DAB_SKINNY_NT=1 timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench7nt.log 2>&1
rc=$?; echo "bench nt rc=$rc"; tail -1 gpurun_out/bench7nt.log
exit $rc

#!/bin/bash
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -x -p no:cacheprovider -k "gemm" > gpurun_out/gputests14.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gputests14.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python benchmarks/kernel_bench.py gemm bge > gpurun_out/kbench_gemm14.log 2>&1
rc=$?; echo "kbench rc=$rc"; python3 -c "
import json
for l in open('gpurun_out/kbench_gemm14.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['op'], d['M'], d['N'], d['K'], 'native', d['native_us'], d['native_tflops'], 'lib', d['hipblaslt_us'], d['hipblaslt_tflops'])"
timeout -k 10 300 python benchmarks/kernel_bench.py gemm index > gpurun_out/kbench_idx14.log 2>&1
grep op gpurun_out/kbench_idx14.log
timeout -k 10 600 python benchmarks/embed_bench.py --chunks 1000000 > gpurun_out/embed14.log 2>&1
rc=$?; echo "embed rc=$rc"; tail -1 gpurun_out/embed14.log
exit $rc

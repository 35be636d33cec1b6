#!/bin/bash
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/prof_attn gpurun_out/prof_bench
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_attn -o attn --output-format csv -- python benchmarks/kernel_bench.py attn > gpurun_out/prof_attn.log 2>&1
rc=$?; echo "prof attn rc=$rc"; tail -8 gpurun_out/prof_attn.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o bench --output-format csv -- python bench.py --steps 1 --warmup 1 --batch 64 --max-new-tokens 64 > gpurun_out/prof_bench.log 2>&1
rc=$?; echo "prof bench rc=$rc"; tail -3 gpurun_out/prof_bench.log
find gpurun_out/prof_attn gpurun_out/prof_bench -name "*stats*"
exit $rc

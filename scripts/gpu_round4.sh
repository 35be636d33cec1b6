#!/bin/bash
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/prof_bench2
export PYTHONUNBUFFERED=1
timeout -k 10 900 python bench.py --steps 3 --warmup 1 > gpurun_out/bench3.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench3.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench2 -o bench --output-format csv -- python bench.py --steps 1 --warmup 1 > gpurun_out/prof_bench2.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -1 gpurun_out/prof_bench2.log
exit $rc

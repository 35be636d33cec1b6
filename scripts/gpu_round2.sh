#!/bin/bash
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python benchmarks/kernel_bench.py all > gpurun_out/kbench.log 2>&1
rc=$?; echo "kbench rc=$rc"; tail -60 gpurun_out/kbench.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py --steps 2 --warmup 1 --batch 64 --max-new-tokens 128 > gpurun_out/bench1.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -8 gpurun_out/bench1.log
exit $rc

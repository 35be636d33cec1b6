#!/bin/bash
# GPU validation: kernel numerics, smoke, first bench. Stops at the first crash-type exit code.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
ok_rc() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 900 python -m pytest tests/test_kernels_gpu.py -q -x -p no:cacheprovider > gpurun_out/gputests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/gputests.log
ok_rc $rc || exit $rc
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py --steps 2 --warmup 1 --batch 32 --max-new-tokens 64 > gpurun_out/bench1.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench1.log
exit $rc

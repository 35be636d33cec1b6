#!/bin/bash
# new GPU tests, reference re-run (HF, sequential), default bench, roctx-attributed kernel trace
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -m pytest tests/test_trace.py tests/test_models_gpu.py -m gpu -x -q > gpurun_out/t20.log 2>&1
rc=$?; tail -3 gpurun_out/t20.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python benchmarks/reference_rerun.py --queries 4 --warmup 1 > gpurun_out/rerun20.log 2>&1
rc=$?; echo "rerun rc=$rc"; tail -2 gpurun_out/rerun20.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/b20.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/b20.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=gpurun_out/prof20_roctx
rm -rf $OUT; mkdir -p $OUT
DAB_ROCTX=1 timeout -k 10 600 rocprofv3 --marker-trace --kernel-trace --stats -d $OUT -o bench --output-format csv -- python bench.py --steps 1 --warmup 1 --batch 32 --max-new-tokens 32 --index-rows 200000 > $OUT/run.log 2>&1
rc=$?; echo "prof rc=$rc"; ls -la $OUT $OUT/* | head -30; exit $rc

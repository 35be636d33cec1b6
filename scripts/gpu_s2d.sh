#!/bin/bash
# stream-kernel decode: full GPU suite, smoke, headline bench, per-step kernel breakdown
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s2d_tests.log 2>&1
rc=$?; tail -3 gpurun_out/s2d_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s2d_smoke.log 2>&1
rc=$?; tail -1 gpurun_out/s2d_smoke.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/s2d_bench.log 2>&1
rc=$?; tail -1 gpurun_out/s2d_bench.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
OUT=gpurun_out/prof_s2d; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT -o bench --output-format csv -- python bench.py --steps 1 --warmup 1 > $OUT/run.log 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc
python scripts/step_breakdown.py $OUT bench --out $OUT/steps.md > /dev/null
python scripts/prof_summary.py $OUT bench $OUT/summary.md --drop-trace > /dev/null
rm -f $OUT/*.csv
sed -n '/last decode step/,$p' $OUT/steps.md

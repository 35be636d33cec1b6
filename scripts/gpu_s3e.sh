#!/bin/bash
# rocprofv3 kernel trace of the current headline bench: whole-run stats + per-step breakdown
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/prof_s3e
rm -rf $OUT; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT -o bench --output-format csv -- python bench.py --steps 1 --warmup 1 > $OUT/run.log 2>&1
rc=$?; echo "prof rc=$rc"; grep metric $OUT/run.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
python scripts/step_breakdown.py $OUT bench --out $OUT/steps.md || true
python scripts/prof_summary.py $OUT bench $OUT/summary.md --drop-trace > /dev/null || true
ls $OUT
rm -f $OUT/*.csv

#!/bin/bash
# kernel trace of the default headline bench -> per-step breakdown (prefill / decode)
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out/prof_s2b
rm -rf $OUT; mkdir -p $OUT
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT -o bench --output-format csv -- python bench.py --steps 1 --warmup 1 > $OUT/run.log 2>&1
rc=$?; echo "prof rc=$rc"; grep metric $OUT/run.log
[ $rc -eq 0 ] || exit $rc
python scripts/step_breakdown.py $OUT bench --out $OUT/steps.md > /dev/null
python scripts/prof_summary.py $OUT bench $OUT/summary.md --drop-trace > /dev/null
rm -f $OUT/*.csv
cat $OUT/steps.md

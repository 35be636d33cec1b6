#!/bin/bash
# rocprofv3 kernel-trace + stats of the headline bench; leaves only a markdown summary.
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out/prof_bench_${1:-cur}
rm -rf $OUT; mkdir -p $OUT
export PYTHONUNBUFFERED=1
shift
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT -o bench --output-format csv -- python bench.py --steps 1 --warmup 1 "$@" > $OUT/run.log 2>&1
rc=$?; echo "prof rc=$rc"; grep metric $OUT/run.log
[ $rc -eq 0 ] || exit $rc
python scripts/prof_summary.py $OUT bench $OUT/summary.md --drop-trace | head -45
rm -f $OUT/*.csv

#!/bin/bash
# decode-window profile: library path vs skinny o/down; bench numbers for both
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for V in none o,down all; do
  OUT=gpurun_out/prof9_${V//,/_}
  rm -rf $OUT; mkdir -p $OUT
  DAB_SKINNY=$V timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT -o bench --output-format csv -- python bench.py --steps 1 --warmup 1 > $OUT/run.log 2>&1
  rc=$?; echo "prof $V rc=$rc"; grep -o '"value": [0-9.]*' $OUT/run.log
  [ $rc -eq 0 ] || exit $rc
  python scripts/prof_summary.py $OUT bench $OUT/summary.md --drop-trace | sed -n 3,8p
  rm -f $OUT/*.csv
done

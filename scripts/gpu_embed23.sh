#!/bin/bash
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python benchmarks/embed_bench.py --chunks 1000000 > gpurun_out/embed23.log 2>&1
rc=$?; echo "embed rc=$rc"; tail -1 gpurun_out/embed23.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=gpurun_out/prof23_embed
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT -o embed --output-format csv -- python benchmarks/embed_bench.py --chunks 200000 > $OUT/run.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python scripts/prof_summary.py $OUT embed $OUT/summary.md --drop-trace | sed -n 1,30p
rm -f $OUT/*.csv

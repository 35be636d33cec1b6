#!/bin/bash
# per-kernel times of the selection microbench (chunk top-k vs merge)
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/prof_s3i
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o sel --output-format csv -- python benchmarks/kernel_bench.py select > $OUT/run.log 2>&1
rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || exit $rc
find $OUT -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-200 | head -12
find $OUT -name "*.csv" ! -name "*kernel_stats.csv" -delete

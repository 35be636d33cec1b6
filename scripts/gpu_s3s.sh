#!/bin/bash
# TEMP A/B: paged decode grid cap (persistent 512 / 768 workgroups vs one per item)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for i in 1 2; do
for g in 2048 512 768; do
DAB_DECODE_GRID=$g timeout -k 10 120 python benchmarks/kernel_bench.py decode > gpurun_out/s3s_g${g}_$i.log 2>&1
rc=$?; echo "grid=$g $(grep -o '"B": 128.*p2048_tbps": [0-9.]*' gpurun_out/s3s_g${g}_$i.log | grep -o 'p2048_us": [0-9.]*')"; [ $rc -eq 0 ] || exit $rc
done
done

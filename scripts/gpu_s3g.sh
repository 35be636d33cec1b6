#!/bin/bash
# A/B of early block-table lookups in paged decode (kernel sweep, 2x each, interleaved)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for i in 1 2; do
for e in 1 0; do
DAB_EARLY_BT=$e timeout -k 10 300 python benchmarks/kernel_bench.py decode > gpurun_out/s3g_sweep_e${e}_$i.log 2>&1
rc=$?; echo "early=$e"; cat gpurun_out/s3g_sweep_e${e}_$i.log | grep -o '"B": [0-9]*.*p2048_tbps": [0-9.]*' ; [ $rc -eq 0 ] || exit $rc
done
done

#!/bin/bash
# TEMP A/B: decode RoPE/KV-write block size (graph-timed)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for i in 1 2; do for nt in 256 128 64; do
DAB_ROPE_NT=$nt timeout -k 10 120 python benchmarks/rope_bench.py > gpurun_out/s3v_${nt}_$i.log 2>&1
rc=$?; grep op gpurun_out/s3v_${nt}_$i.log; [ $rc -eq 0 ] || exit $rc
done; done

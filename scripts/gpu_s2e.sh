#!/bin/bash
# stream_gemm ablations (no X / no MFMA / weight stream only) at M=128
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
STREAM_NT=1 STREAM_CFGS=${CFGS:-10,17,18,19} timeout -k 10 600 python benchmarks/kernel_bench.py stream all ${MS:-128} > gpurun_out/s2e_sweep.log 2>&1
rc=$?; cat gpurun_out/s2e_sweep.log; exit $rc

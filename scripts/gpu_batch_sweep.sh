#!/bin/bash
# QPS / p50 vs per-GPU batch for the flagship RAG bench.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for B in 128 256; do
  timeout -k 10 600 python bench.py --steps 2 --warmup 1 --batch $B > gpurun_out/bench_b$B.log 2>&1
  rc=$?; echo "batch $B rc=$rc"; tail -1 gpurun_out/bench_b$B.log
  [ $rc -eq 0 ] || exit $rc
done

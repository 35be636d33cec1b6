#!/bin/bash
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for F in 0 1; do
  DAB_BERT_FUSED_UP=$F timeout -k 10 600 python benchmarks/embed_bench.py --chunks 1000000 > gpurun_out/embed25_$F.log 2>&1
  rc=$?; echo "fused=$F rc=$rc"; tail -1 gpurun_out/embed25_$F.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 600 python -m pytest tests -m gpu -q -k "bert or embed or encoder" > gpurun_out/t25.log 2>&1
rc=$?; tail -2 gpurun_out/t25.log; exit $rc

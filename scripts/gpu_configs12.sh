#!/bin/bash
# BASELINE configs 2 and 5 on one MI355X: DP=1 batch embedding of 1M chunks; Llama-3-70B RAG (TP=1 fits in 288 GB)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python benchmarks/embed_bench.py --chunks 1000000 > gpurun_out/embed12.log 2>&1
rc=$?; echo "embed rc=$rc"; tail -1 gpurun_out/embed12.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py --llm-model llama-3-70b --embed-model bge-large-en --batch 64 --steps 1 --warmup 1 > gpurun_out/bench12_70b.log 2>&1
rc=$?; echo "70b rc=$rc"; tail -1 gpurun_out/bench12_70b.log
exit $rc

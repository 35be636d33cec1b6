#!/bin/bash
# refresh the secondary BASELINE configs at the current commit: 2 (bge-base 1M-chunk embedding),
# 3 (in-HBM index search, 10M rows), 5 (Llama-3-70B + bge-large RAG on one GPU, batch 64)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python benchmarks/embed_bench.py --chunks 1000000 > gpurun_out/s3q_embed.log 2>&1
rc=$?; echo "embed rc=$rc"; tail -1 gpurun_out/s3q_embed.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python benchmarks/index_bench.py --rows 10000000 --batch 1 64 512 > gpurun_out/s3q_idx.log 2>&1
rc=$?; echo "index rc=$rc"; tail -3 gpurun_out/s3q_idx.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py --llm-model llama-3-70b --embed-model bge-large-en --batch 64 --steps 1 --warmup 1 > gpurun_out/s3q_70b.log 2>&1
rc=$?; echo "70b rc=$rc"; tail -1 gpurun_out/s3q_70b.log | cut -c1-600; exit $rc

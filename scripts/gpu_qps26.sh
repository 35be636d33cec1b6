#!/bin/bash
# fixed-QPS (open-loop) latency curves: 8B + bge-base, then 70B + bge-large on one GPU
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
summ() { tail -1 "$1" | python3 -c "
import sys, json; d=json.loads(sys.stdin.read()); c=d['config']
print(c['model'], '|', c['mode'], '| achieved', d['value'], 'q/s | p50', d['p50_latency_ms'], '| p90', d.get('p90_latency_ms'))"; }
for q in 8 16 24 30; do
  L=gpurun_out/q26_8b_$q.log
  timeout -k 10 600 python bench.py --mode serve --qps $q --batch 128 --steps 2 --warmup 1 > $L 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "8b qps $q rc=$rc"; tail -5 $L; exit $rc; }
  summ $L
done
for q in 1.5 3; do
  L=gpurun_out/q26_70b_$q.log
  timeout -k 10 900 python bench.py --mode serve --qps $q --batch 64 --steps 2 --warmup 1 --llm-model llama-3-70b --embed-model bge-large-en > $L 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "70b qps $q rc=$rc"; tail -5 $L; exit $rc; }
  summ $L
done

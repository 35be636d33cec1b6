#!/bin/bash
# full GPU suite + batch-1 latency + smoke
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/t21.log 2>&1
rc=$?; tail -3 gpurun_out/t21.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build(); g.smoke(); print('smoke ok')" > gpurun_out/smoke21.log 2>&1
rc=$?; tail -2 gpurun_out/smoke21.log; [ $rc -eq 0 ] || exit $rc
for b in 1 8; do
  timeout -k 10 600 python bench.py --batch $b --steps 3 --warmup 1 > gpurun_out/b21_$b.log 2>&1
  rc=$?; echo "batch $b rc=$rc"; [ $rc -eq 0 ] || exit $rc
  tail -1 gpurun_out/b21_$b.log | python3 -c "
import sys, json; d=json.loads(sys.stdin.read()); c=d['config']; e=c['engine_rank0']
print(d['value'], d['p50_latency_ms'], c['phases_rank0_s'], round(e.get('gpu_decode_ms',0)/max(1,e['decode_steps']),3), 'ms/decode')"
done

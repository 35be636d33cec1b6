#!/bin/bash
# mixed prefill+decode serving mode vs batch mode (bench.py), plus the mixed-step GPU tests
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
summ() { tail -1 "$1" | python3 -c "
import sys, json; d=json.loads(sys.stdin.read()); c=d['config']; e=c['engine_rank0']
print(c['mode'], '| qps', d['value'], '| p50', d['p50_latency_ms'], '| p90', d.get('p90_latency_ms'), '| seq', c['seq_len'], '|', e)"; }
timeout -k 10 600 python -m pytest tests/test_models_gpu.py -x -q > gpurun_out/t16.log 2>&1
rc=$?; tail -3 gpurun_out/t16.log; [ $rc -eq 0 ] || exit $rc
for cfg in "serve:2048:128" "serve:4096:128" "serve:2048:192" "batch:0:128"; do
  IFS=: read mode mt b <<< "$cfg"
  timeout -k 10 600 python bench.py --mode $mode --mixed-tokens $mt --batch $b --steps 4 --warmup 2 > gpurun_out/b16_${mode}_${mt}_${b}.log 2>&1
  rc=$?; echo "$cfg rc=$rc"; [ $rc -eq 0 ] || exit $rc
  summ gpurun_out/b16_${mode}_${mt}_${b}.log
done

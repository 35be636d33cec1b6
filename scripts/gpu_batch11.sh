#!/bin/bash
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for B in 64 128 256; do
  timeout -k 10 600 python bench.py --steps 2 --warmup 1 --batch $B > gpurun_out/bench11_b$B.log 2>&1
  rc=$?; echo "batch $B rc=$rc"; tail -1 gpurun_out/bench11_b$B.log | python3 -c "
import sys, json; d=json.loads(sys.stdin.read()); c=d['config']; e=c['engine_rank0']
print(d['value'], d['p50_latency_ms'], c['seq_len'], c['docs_per_prompt'], c['tuned_gemm_shapes'], round(e['decode_gpu_wait_s']/max(1,e['decode_steps'])*1000,2), 'ms/decode')"
  [ $rc -eq 0 ] || exit $rc
done
DAB_GEMM_TUNING=0 timeout -k 10 600 python bench.py --steps 2 --warmup 1 --batch 128 > gpurun_out/bench11_b128_notune.log 2>&1
rc=$?; echo "notune rc=$rc"; tail -1 gpurun_out/bench11_b128_notune.log | cut -c1-200
exit $rc

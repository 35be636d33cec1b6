#!/bin/bash
# end-to-end effect of the weight-streaming GEMM on o/down(/qkv) at decode batch 128
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for V in o,down none o,down,qkv; do
  L=gpurun_out/b19_${V//,/_}.log
  DAB_SKINNY=$V timeout -k 10 600 python bench.py --mode batch --steps 3 --warmup 1 > $L 2>&1
  rc=$?; echo "$V rc=$rc"; [ $rc -eq 0 ] || exit $rc
  tail -1 $L | python3 -c "
import sys, json; d=json.loads(sys.stdin.read()); e=d['config']['engine_rank0']
print(d['value'], d['p50_latency_ms'], round(e['decode_gpu_wait_s']/e['decode_steps']*1000, 3), 'ms/decode-step')"
done

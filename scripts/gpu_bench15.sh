#!/bin/bash
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python bench.py --steps 3 --warmup 1 > gpurun_out/bench15.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench15.log | python3 -c "
import sys, json; d=json.loads(sys.stdin.read()); c=d['config']; e=c['engine_rank0']
print(d['value'], d['p50_latency_ms'], c['seq_len'], c['phases_rank0_s'], round(e['decode_gpu_wait_s']/max(1,e['decode_steps'])*1000,2), 'ms/decode')"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python benchmarks/embed_bench.py --chunks 1000000 > gpurun_out/embed15.log 2>&1
rc=$?; echo "embed rc=$rc"; tail -1 gpurun_out/embed15.log | cut -c1-200
exit $rc

#!/bin/bash
# prefill step size sweep on the headline bench (tokens per prefill forward)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
pp() { python -c "
import sys,json; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); e=d['config']['engine_rank0']
print(sys.argv[1], d['value'], d['p50_latency_ms'], 'prefill ms/batch', round(e['gpu_prefill_ms']/3,1), 'steps', e['prefill_steps'], 'decode ms/step', round(e['gpu_decode_ms']/e['decode_steps'],3))" $1; }
for pt in 32768 65536 131072 32768 65536 131072; do
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --prefill-tokens $pt > gpurun_out/s3r_$pt.log 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc; pp gpurun_out/s3r_$pt.log
done

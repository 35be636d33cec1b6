#!/bin/bash
# two-stream prefill: numerics, then the headline bench with 1 and 2 prefill streams (and 64K steps)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s3a_tests.log 2>&1
rc=$?; tail -1 gpurun_out/s3a_tests.log; [ $rc -eq 0 ] || exit $rc
pp() { python -c "
import sys,json; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); e=d['config']['engine_rank0']
print(sys.argv[1], d['value'], d['p50_latency_ms'], 'prefill ms/batch', round(e['gpu_prefill_ms']/3,1), 'decode ms/step', round(e['gpu_decode_ms']/e['decode_steps'],3))" $1; }
DAB_PREFILL_STREAMS=1 timeout -k 10 400 python bench.py --steps 3 --warmup 1 > gpurun_out/s3a_b1.log 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc; pp gpurun_out/s3a_b1.log
DAB_PREFILL_STREAMS=2 timeout -k 10 400 python bench.py --steps 3 --warmup 1 > gpurun_out/s3a_b2.log 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc; pp gpurun_out/s3a_b2.log
DAB_PREFILL_STREAMS=2 timeout -k 10 400 python bench.py --steps 3 --warmup 1 --prefill-tokens 65536 > gpurun_out/s3a_b3.log 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc; pp gpurun_out/s3a_b3.log

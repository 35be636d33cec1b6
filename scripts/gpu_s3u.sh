#!/bin/bash
# 512-thread slab RMSNorm for 4096-wide rows: numerics, graph-timed microbench, headline bench
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s3u_tests.log 2>&1
rc=$?; tail -1 gpurun_out/s3u_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python benchmarks/slab_norm_bench.py > gpurun_out/s3u_slab.log 2>&1
rc=$?; grep op gpurun_out/s3u_slab.log; [ $rc -eq 0 ] || exit $rc
pp() { python -c "
import sys,json; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); e=d['config']['engine_rank0']
print(sys.argv[1], d['value'], d['p50_latency_ms'], 'prefill ms/batch', round(e['gpu_prefill_ms']/3,1), 'decode ms/step', round(e['gpu_decode_ms']/e['decode_steps'],3))" $1; }
for i in 1 2; do
timeout -k 10 400 python bench.py --steps 3 --warmup 1 > gpurun_out/s3u_b$i.log 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc; pp gpurun_out/s3u_b$i.log
done

#!/bin/bash
# flash prefill attention: numerics + kernel bench + headline bench
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread -k "flash or mixed or decode or engine" > gpurun_out/s2g_tests.log 2>&1
rc=$?; tail -2 gpurun_out/s2g_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python benchmarks/kernel_bench.py attn > gpurun_out/s2g_attn.log 2>&1
rc=$?; cat gpurun_out/s2g_attn.log | grep op; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/s2g_bench.log 2>&1
rc=$?; tail -1 gpurun_out/s2g_bench.log | cut -c1-300; tail -1 gpurun_out/s2g_bench.log | python3 -c "
import sys,json; d=json.loads(sys.stdin.read()); e=d['config']['engine_rank0']; print('prefill ms/batch', e['gpu_prefill_ms']/3, 'decode ms/step', e['gpu_decode_ms']/e['decode_steps'])"
exit $rc

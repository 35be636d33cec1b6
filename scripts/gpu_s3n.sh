#!/bin/bash
# flash forward variants: default (8 waves x 16 queries), qt2 (4 waves x 2x16, 2 waves/SIMD), q8 (8 waves x 2x16)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for v in qt2 q8; do
DAB_FLASH_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "flash or prefill or encoder or embed or forward" > gpurun_out/s3n_tests_$v.log 2>&1
rc=$?; echo "$v: $(tail -1 gpurun_out/s3n_tests_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for i in 1 2; do
for v in w8 qt2 q8; do
DAB_FLASH_VARIANT=$v timeout -k 10 120 python benchmarks/kernel_bench.py attn > gpurun_out/s3n_attn_${v}_$i.log 2>&1
rc=$?; echo "$v: $(grep flash gpurun_out/s3n_attn_${v}_$i.log | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
done
done

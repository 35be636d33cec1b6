#!/bin/bash
# flash forward variants: numerics (default) + A/B timing of w4 / w8 / qt2
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for v in w4 w8 qt2; do
  DAB_FLASH_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "flash" > gpurun_out/s2i_tests_$v.log 2>&1
  rc=$?; echo "$v tests: $(tail -1 gpurun_out/s2i_tests_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for v in w4 w8 qt2 w4 w8 qt2; do
  DAB_FLASH_VARIANT=$v timeout -k 10 300 python benchmarks/kernel_bench.py attn > gpurun_out/s2i_attn_$v.log 2>&1
  rc=$?; echo "$v: $(grep flash gpurun_out/s2i_attn_$v.log | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
done

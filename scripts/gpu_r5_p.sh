#!/bin/bash
# Round 5, call P: 64 queries per wave, one wave per SIMD (DAB_FLASH_Q64=1): parity, flash / prefill
# tests with it on (incl. RoPE on load), the attention A/B and the scan.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r5p_variant_tests 300 python -u -m pytest tests/test_kernels_gpu.py -k "variants_match" -x -v --timeout 120 --timeout-method thread &&
DAB_FLASH_Q64=1 $S r5p_flash_tests 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -k "flash or prefill" -x -q --timeout 120 --timeout-method thread &&
$S r5p_attn 300 python -u benchmarks/kernel_bench.py attn &&
$S r5p_scan 300 python -u benchmarks/kernel_bench.py attnscan

#!/bin/bash
# Round 5, call L: paired causal query blocks (DAB_FLASH_PAIR=1): parity tests, flash / prefill tests
# with it on (incl. the model's RoPE-on-load prefill), then the attention A/B and the scan.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r5l_variant_tests 300 python -u -m pytest tests/test_kernels_gpu.py -k "variants_match" -x -v --timeout 120 --timeout-method thread &&
DAB_FLASH_PAIR=1 $S r5l_flash_tests 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -k "flash or prefill" -x -q --timeout 120 --timeout-method thread &&
$S r5l_attn 300 python -u benchmarks/kernel_bench.py attn &&
$S r5l_scan 300 python -u benchmarks/kernel_bench.py attnscan

#!/bin/bash
# Round 5, call O: one barrier per tile in the paired causal kernel (DAB_FLASH_1BAR=1): parity, A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r5o_variant_tests 300 python -u -m pytest tests/test_kernels_gpu.py -k "variants_match" -x -v --timeout 120 --timeout-method thread &&
DAB_FLASH_1BAR=1 $S r5o_flash_tests 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -k "flash or prefill" -x -q --timeout 120 --timeout-method thread &&
$S r5o_attn 300 python -u benchmarks/kernel_bench.py attn

#!/bin/bash
# Round 5, call J: 8-wave / 3-deep-ring prefill attention (DAB_FLASH_W8=1) and the 5-waves-per-SIMD
# encoder attention (DAB_ENC_W5=1): parity tests, flash tests with W8 on, then the interleaved
# kernel A/B (causal and full prefill; the embed bench's packed encoder batch).
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r5j_variant_tests 300 python -u -m pytest tests/test_kernels_gpu.py -k "variants_match" -x -v --timeout 120 --timeout-method thread &&
DAB_FLASH_W8=1 $S r5j_flash_tests 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -k "flash or prefill" -x -q --timeout 120 --timeout-method thread &&
$S r5j_attn 300 python -u benchmarks/kernel_bench.py attn

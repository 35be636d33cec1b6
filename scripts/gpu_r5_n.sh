#!/bin/bash
# Round 5, call N: G causal block pairs per workgroup (DAB_FLASH_G): parity + flash / prefill tests,
# attention A/B (G from the launch size vs 1 vs 4) and the scan.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r5n_variant_tests 300 python -u -m pytest tests/test_kernels_gpu.py -k "variants_match" -x -v --timeout 120 --timeout-method thread &&
DAB_FLASH_G=3 $S r5n_flash_tests 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -k "flash or prefill" -x -q --timeout 120 --timeout-method thread &&
$S r5n_attn 300 python -u benchmarks/kernel_bench.py attn &&
$S r5n_scan 300 python -u benchmarks/kernel_bench.py attnscan

#!/bin/bash
# Round 5, call V: softmax split across the PV k-steps (DAB_FLASH_SMS=1): flash / prefill tests with
# it on (the variants test compares against the unsplit kernel bit for bit, so it runs without the
# switch), the attention A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
DAB_FLASH_SMS=1 $S r5v_flash_tests 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -k "(flash or prefill) and not variants" -x -q --timeout 120 --timeout-method thread &&
$S r5v_attn 300 python -u benchmarks/kernel_bench.py attn

#!/bin/bash
# Round 5, call F: software-pipelined V reads in the prefill attention:
# numerics with the variant on (DAB_FLASH_VPIPE=1: flash tests incl. forced rescales), then the
# interleaved A/B in kernel_bench attn.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
DAB_FLASH_VPIPE=1 $S r5f_flash_tests 400 python -u -m pytest tests/test_kernels_gpu.py -k "flash" -x -q --timeout 300 --timeout-method thread &&
$S r5f_attn 300 python -u benchmarks/kernel_bench.py attn

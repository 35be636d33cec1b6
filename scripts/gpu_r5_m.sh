#!/bin/bash
# Round 5, call M: paired causal blocks on by default + block-table loads hoisted: kernel and model
# GPU tests (flash / prefill / variants), the attention A/B and scan, the default bench.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r5m_tests 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 300 --timeout-method thread &&
$S r5m_attn 300 python -u benchmarks/kernel_bench.py attn &&
$S r5m_scan 300 python -u benchmarks/kernel_bench.py attnscan &&
$S r5m_bench 600 python -u bench.py --steps 10 --warmup 3

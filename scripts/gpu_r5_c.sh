#!/bin/bash
# Round 5, call C: vocab-parallel sampling + TP tests, world-1 RCCL, the CU-split probe, then the
# full-size 70B TP-8 rehearsal on the one card.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r5c_tests 900 python -u -m pytest tests/test_tp_gpu.py tests/test_rccl_world1_gpu.py "tests/test_kernels_gpu.py::test_vocab_parallel_sampling_draws_the_replicated_token" -x -v --timeout 300 --timeout-method thread &&
$S r5c_tp70b_small 300 python -u benchmarks/tp70b_rehearsal.py --model tiny-llama-70b-d128 --world 8 --out gpurun_out/tp70b_small.json &&
$S r5c_cusplit 600 python -u benchmarks/cu_split_probe.py &&
$S r5c_tp70b 1000 python -u benchmarks/tp70b_rehearsal.py --out gpurun_out/tp70b_rehearsal.json

#!/bin/bash
# Round 6, call D: the gemm_mid dispatch in gemm_bt -- kernel + model tests, the mid-M table on the
# production dispatch, then serve mode with mixed steps (512 / 1024 prompt tokens per step) against
# batch mode on the same box.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r6d_tests 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 200 --timeout-method thread -k "gemm or decode or prefill or mixed or fold or default_path or llama or sampl" &&
$S r6d_tp 900 python -u -m pytest tests/test_sampling_parity_gpu.py tests/test_tp_fault_gpu.py tests/test_custom_allreduce_gpu.py tests/test_tp_gpu.py -x -q --timeout 300 --timeout-method thread &&
$S r6d_mid 400 python -u benchmarks/gemm_bench.py --shapes mid --rounds 3 --iters 10 &&
$S r6d_batch 400 python -u bench.py --steps 4 --warmup 2 &&
$S r6d_mixed512 400 python -u bench.py --mode serve --mixed-tokens 512 --steps 4 --warmup 2 &&
$S r6d_mixed1024 400 python -u bench.py --mode serve --mixed-tokens 1024 --steps 4 --warmup 2

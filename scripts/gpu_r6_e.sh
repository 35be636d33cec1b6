#!/bin/bash
# Round 6, call E: the rest of call D (killed by the silence watchdog during the 8-rank all-reduce
# test; GPU tests now print a heartbeat): TP / sampling / fault tests, the mid-M table on the
# production dispatch, batch vs mixed serve.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r6e_tp 900 python -u -m pytest tests/test_tp_fault_gpu.py tests/test_custom_allreduce_gpu.py tests/test_tp_gpu.py -x -v --timeout 400 --timeout-method thread &&
$S r6e_mid 400 python -u benchmarks/gemm_bench.py --shapes mid --rounds 3 --iters 10 &&
$S r6e_batch 400 python -u bench.py --steps 4 --warmup 2 &&
$S r6e_mixed512 400 python -u bench.py --mode serve --mixed-tokens 512 --steps 4 --warmup 2 &&
$S r6e_mixed1024 400 python -u bench.py --mode serve --mixed-tokens 1024 --steps 4 --warmup 2

#!/bin/bash
# Round 6 call G: slice-per-XCD block mapping of the batch-128 split-K decode GEMMs (A/B)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "slice_per_xcd or test_stream_gemm" > gpurun_out/r6g_test.log 2>&1 || exit $?
STREAM_CFGS=10 timeout -k 10 200 python -u benchmarks/kernel_bench.py stream all 128 > gpurun_out/r6g_k0.log 2>&1 || exit $?
DAB_STREAM_SLICE_XCD=1 STREAM_CFGS=10 timeout -k 10 200 python -u benchmarks/kernel_bench.py stream all 128 > gpurun_out/r6g_k1.log 2>&1 || exit $?
timeout -k 10 600 python -u benchmarks/decode_ab.py --arms base,slicexcd --rounds 3 --steps 40 > gpurun_out/r6g_ab.log 2>&1 || exit $?

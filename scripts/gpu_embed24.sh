#!/bin/bash
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python benchmarks/embed_bench.py --chunks 1000000 > gpurun_out/embed24.log 2>&1
rc=$?; echo "embed rc=$rc"; tail -1 gpurun_out/embed24.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python benchmarks/kernel_bench.py gemm bge > gpurun_out/kb24.log 2>&1
rc=$?; echo "kb rc=$rc"; cat gpurun_out/kb24.log | grep -v amdgpu.ids; exit $rc

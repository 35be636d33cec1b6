#!/bin/bash
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python benchmarks/kernel_bench.py decode > gpurun_out/s2k_sweep.log 2>&1
rc=$?; grep sweep gpurun_out/s2k_sweep.log; exit $rc

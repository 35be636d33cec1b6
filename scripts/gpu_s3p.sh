#!/bin/bash
# probe: prefill GEMMs on a low-priority stream beside decode-shaped work
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python benchmarks/overlap_probe.py > gpurun_out/s3p_probe.log 2>&1
rc=$?; grep overlap gpurun_out/s3p_probe.log || tail -5 gpurun_out/s3p_probe.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python benchmarks/overlap_probe.py > gpurun_out/s3p_probe2.log 2>&1
rc=$?; grep overlap gpurun_out/s3p_probe2.log || tail -5 gpurun_out/s3p_probe2.log; [ $rc -eq 0 ] || exit $rc

#!/bin/bash
# prefill study: kernel breakdown of a full 32K-token prefill step + native vs library GEMM at prefill M
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
OUT=gpurun_out/prof_s2f; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT -o bench --output-format csv -- python bench.py --steps 1 --warmup 1 > $OUT/run.log 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc
python scripts/step_breakdown.py $OUT bench --out $OUT/steps.md > /dev/null
rm -f $OUT/*.csv
sed -n '1,/last decode step/p' $OUT/steps.md
timeout -k 10 600 python benchmarks/kernel_bench.py gemm llama8b > gpurun_out/s2f_gemm.log 2>&1
rc=$?; grep -E '"M": (4096|16384)' gpurun_out/s2f_gemm.log; exit $rc

#!/bin/bash
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cp django_assistant_bot_amd/tuning/tunableop_llama-3-8b_tp1_gfx950.csv gpurun_out/tune_before13.csv
timeout -k 10 1100 python benchmarks/tune_gemms.py --no-decode --prefill-m 32768,16384 --out gpurun_out/tune_prefill13.csv > gpurun_out/tune13.log 2>&1
rc=$?; echo "tune rc=$rc"; grep '"M"' gpurun_out/tune13.log
exit $rc

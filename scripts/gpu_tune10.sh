#!/bin/bash
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python benchmarks/tune_gemms.py --max-m 256 > gpurun_out/tune10.log 2>&1
rc=$?; echo "tune rc=$rc"; grep -v tuned gpurun_out/tune10.log | tail -80
cp django_assistant_bot_amd/tuning/*.csv gpurun_out/ 2>/dev/null
exit $rc

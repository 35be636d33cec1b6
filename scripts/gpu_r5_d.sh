#!/bin/bash
# Round 5, call D: full-size Llama-3-70B TP-8 rehearsal on the one card; serve mode with mixed
# prefill + decode steps at 512 / 1024 prompt tokens per step, and a kernel
# trace of the 512 case for the per-step breakdown.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r5d_tp70b 1000 python -u benchmarks/tp70b_rehearsal.py --out gpurun_out/tp70b_rehearsal.json &&
$S r5d_mixed512 400 python -u bench.py --mode serve --mixed-tokens 512 --admit-group 8 --steps 2 --warmup 1 &&
$S r5d_mixed1024 400 python -u bench.py --mode serve --mixed-tokens 1024 --admit-group 8 --steps 2 --warmup 1 &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mixed -o run \
  -- python bench.py --mode serve --mixed-tokens 512 --admit-group 8 --steps 1 --warmup 1 > gpurun_out/prof_mixed.log 2>&1 &&
d=$(dirname "$(find gpurun_out/prof_mixed -name 'run_kernel_stats.csv' | head -1)") &&
python scripts/step_breakdown.py "$d" run --out gpurun_out/prof_mixed_steps.md > /dev/null &&
python scripts/prof_summary.py "$d" run gpurun_out/prof_mixed_stats.md --drop-trace

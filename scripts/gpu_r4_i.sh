#!/bin/bash
# Round 4, call I: kernel breakdown of the 512-query search after the candidate-list changes.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_idx512b -o run \
  -- python benchmarks/index_bench.py --iters 5 --warmup 2 --batch 512 > gpurun_out/prof_idx512b.log 2>&1 || exit $?
d=$(dirname "$(find gpurun_out/prof_idx512b -name 'run_kernel_stats.csv' | head -1)")
python scripts/prof_summary.py "$d" run gpurun_out/prof_idx512b_stats.md --drop-trace

#!/bin/bash
# Round 4, call B: kernel breakdown of the 10M-row index search at 64 and 512 queries.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for b in 64 512; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_idx$b -o run \
    -- python benchmarks/index_bench.py --iters 5 --warmup 2 --batch $b > gpurun_out/prof_idx$b.log 2>&1 || exit $?
  d=$(dirname "$(find gpurun_out/prof_idx$b -name 'run_kernel_stats.csv' | head -1)")
  python scripts/prof_summary.py "$d" run gpurun_out/prof_idx${b}_stats.md --drop-trace || exit $?
  tail -2 gpurun_out/prof_idx$b.log
done

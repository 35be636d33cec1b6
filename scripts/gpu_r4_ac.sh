#!/bin/bash
# Round 4, call AC: kernel breakdown of the 128- and 512-query searches at the end of the round.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for B in 128 512; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_idx_end_$B -o run \
    -- python benchmarks/index_bench.py --iters 5 --warmup 2 --batch $B > gpurun_out/prof_idx_end_$B.log 2>&1 || exit $?
  d=$(dirname "$(find gpurun_out/prof_idx_end_$B -name 'run_kernel_stats.csv' | head -1)")
  python scripts/prof_summary.py "$d" run gpurun_out/prof_idx_end_${B}_stats.md --drop-trace || exit $?
done

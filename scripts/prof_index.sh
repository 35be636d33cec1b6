#!/bin/bash
# rocprofv3 kernel trace + stats of the index search bench (10M rows) -> gpurun_out/prof_index/
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_index -o run \
  -- python benchmarks/index_bench.py --iters 5 --warmup 2 "$@" > gpurun_out/prof_index.log 2>&1 || exit $?
d=$(dirname "$(find gpurun_out/prof_index -name 'run_kernel_stats.csv' | head -1)")
python scripts/prof_summary.py "$d" run gpurun_out/prof_index_stats.md --drop-trace

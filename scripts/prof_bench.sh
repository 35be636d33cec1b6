#!/bin/bash
# rocprofv3 kernel trace + stats of one short headline-bench run -> gpurun_out/prof_bench/
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o run \
  -- python bench.py --steps 1 --warmup 1 "$@" > gpurun_out/prof_bench.log 2>&1 || exit $?
d=$(dirname "$(find gpurun_out/prof_bench -name 'run_kernel_stats.csv' | head -1)")
python scripts/step_breakdown.py "$d" run --out gpurun_out/prof_bench_steps.md && \
python scripts/gap_report.py "$d" run --min-us 50 --top 40 ${GAP_LAST_MS:+--last-ms $GAP_LAST_MS} --out gpurun_out/prof_bench_gaps.md > /dev/null && \
python scripts/prof_summary.py "$d" run gpurun_out/prof_bench_stats.md --drop-trace

#!/bin/bash
# rocprofv3 kernel stats of the bge-base batch-embedding bench (BASELINE config 2) -> gpurun_out/prof_embed_stats.md
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_embed -o run \
  -- python benchmarks/embed_bench.py --chunks 200000 "$@" > gpurun_out/prof_embed.log 2>&1 || exit $?
d=$(dirname "$(find gpurun_out/prof_embed -name 'run_kernel_stats.csv' | head -1)")
python scripts/gap_report.py "$d" run --min-us 20 --top 40 --last-ms 1800 --out gpurun_out/prof_embed_gaps.md
python scripts/prof_summary.py "$d" run gpurun_out/prof_embed_stats.md --drop-trace

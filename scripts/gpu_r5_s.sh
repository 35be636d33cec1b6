#!/bin/bash
# Round 5, call S: embed-bench kernel profiles with the default and the persistent encoder attention.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pe_def -o run \
  -- python benchmarks/embed_bench.py --chunks 200000 > gpurun_out/r5s_def.log 2>&1 &&
DAB_ENC_PERSIST=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pe_per -o run \
  -- python benchmarks/embed_bench.py --chunks 200000 > gpurun_out/r5s_per.log 2>&1 &&
for d in pe_def pe_per; do
  s=$(dirname "$(find gpurun_out/$d -name 'run_kernel_stats.csv' | head -1)")
  python scripts/prof_summary.py "$s" run gpurun_out/${d}_stats.md --drop-trace || exit 1
done

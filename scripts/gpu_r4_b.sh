#!/bin/bash
# Round 4, call B: index kernels (1-64 queries on the persistent LDS-query scan), the 10M-row
# search at 1..512 queries, and a kernel breakdown of the 64- and 512-query searches.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r4b_tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
    -k "score_candidates or index_threshold or index_recall or index_fragment" &&
$S r4b_bench 300 python -u benchmarks/index_bench.py --iters 10 --warmup 3 --batch 1 16 32 48 64 96 100 128 512 || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for b in 64 512; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_idx$b -o run \
    -- python benchmarks/index_bench.py --iters 5 --warmup 2 --batch $b > gpurun_out/prof_idx$b.log 2>&1 || exit $?
  d=$(dirname "$(find gpurun_out/prof_idx$b -name 'run_kernel_stats.csv' | head -1)")
  python scripts/prof_summary.py "$d" run gpurun_out/prof_idx${b}_stats.md --drop-trace || exit $?
  tail -2 gpurun_out/prof_idx$b.log
done
cd "$GRAFT_REPO_ROOT" && S=scripts/gpu_step.sh &&
$S r4b_stride64 300 python -u benchmarks/index_bench.py --iters 10 --warmup 3 --batch 128 512 --sample-stride 64

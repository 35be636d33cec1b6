#!/bin/bash
# rocprofv3 kernel trace of a short headline-bench run -> per-slot decode layer table
# usage: scripts/prof_decode.sh NAME [bench args...]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
name=$1; shift
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_$name -o run \
  -- python bench.py --steps 1 --warmup 0 --no-fast-steps "$@" > gpurun_out/prof_$name.log 2>&1 || exit $?
d=$(dirname "$(find gpurun_out/prof_$name -name 'run_kernel_trace.csv' | head -1)")
python scripts/decode_layer_profile.py "$d" run --out gpurun_out/decode_layer_$name.md && \
python scripts/step_breakdown.py "$d" run --out gpurun_out/steps_$name.md && rm -rf gpurun_out/prof_$name

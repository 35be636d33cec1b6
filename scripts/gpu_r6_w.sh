#!/bin/bash
# Round 6, call W: kernel trace of a short headline run, every prefill-attention launch listed.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/attn_trace -o run \
  -- python bench.py --steps 1 --warmup 1 > gpurun_out/attn_trace.log 2>&1 || exit $?
d=$(dirname "$(find gpurun_out/attn_trace -name 'run_kernel_trace.csv' | head -1)")
head -1 "$d/run_kernel_trace.csv" > gpurun_out/attn_trace_header.txt
python scripts/attn_trace.py "$d" run gpurun_out/attn_trace.md && rm -rf gpurun_out/attn_trace

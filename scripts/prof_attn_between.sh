#!/bin/bash
# Decode attention kernel duration with different kernels between launches (rocprofv3 kernel
# stats of benchmarks/decode_attn_bench.py): none / streaming GEMM / device copy / spin.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for kind in none gemm copy spin; do
  if [ $kind = none ]; then extra=""; else extra="--between 1 --between-kind $kind"; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pab_$kind -o run \
    -- python benchmarks/decode_attn_bench.py --parts 2048 --dists mixed $extra > gpurun_out/pab_$kind.log 2>&1 || exit $?
  f=$(find gpurun_out/pab_$kind -name 'run_kernel_stats.csv' | head -1)
  python - "$f" "$kind" <<'PY' >> gpurun_out/pab_summary.md
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if "paged_decode" in n or "stream_gemm" in n or "copy" in n.lower() or "sleep" in n.lower() or "spin" in n.lower():
        print(f"| {sys.argv[2]} | `{n[:70]}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} |")
PY
  rm -rf gpurun_out/pab_$kind
done

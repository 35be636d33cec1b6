#!/bin/bash
# chunk top-k pre-filter with vectorised LDS ranks: numerics + per-kernel times of the selection microbench
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "topk or sampl" > gpurun_out/s3j_tests.log 2>&1
rc=$?; tail -1 gpurun_out/s3j_tests.log; [ $rc -eq 0 ] || exit $rc
OUT=gpurun_out/prof_s3j
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o sel --output-format csv -- python benchmarks/kernel_bench.py select > $OUT/run.log 2>&1
rc=$?; echo "rc=$rc"; grep '"op"' $OUT/run.log; [ $rc -eq 0 ] || exit $rc
python - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/prof_s3j/**/*kernel_trace.csv", recursive=True) + glob.glob("gpurun_out/prof_s3j/*kernel_trace.csv")
rows = list(csv.DictReader(open(f[0])))
from collections import defaultdict
d = defaultdict(list)
for r in rows:
    n = r["Kernel_Name"]
    if "chunk_topk" in n or "merge" in n:
        d[(n.split("(")[0][-40:], r["Grid_Size_X"] if "Grid_Size_X" in r else r.get("Grid_Size", ""), r.get("Grid_Size_Y", ""))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in d.items():
    v.sort(); print(k, len(v), "median us", round(v[len(v) // 2], 1))
PY
find $OUT -name "*.csv" -delete

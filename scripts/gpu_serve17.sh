#!/bin/bash
# thin mixed steps (prefill spread over every decode step) + batch-128 decode-window profile
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
summ() { tail -1 "$1" | python3 -c "
import sys, json; d=json.loads(sys.stdin.read()); c=d['config']; e=c['engine_rank0']
print(c['mode'], '| qps', d['value'], '| p50', d['p50_latency_ms'], '| p90', d.get('p90_latency_ms'), '| seq', c['seq_len'], '|', e)"; }
for cfg in "8:640:128" "4:320:128" "8:1024:128" "4:512:192"; do
  IFS=: read g mt b <<< "$cfg"
  L=gpurun_out/b17_${g}_${mt}_${b}.log
  timeout -k 10 600 python bench.py --admit-group $g --mixed-tokens $mt --batch $b --steps 4 --warmup 2 > $L 2>&1
  rc=$?; echo "$cfg rc=$rc"; [ $rc -eq 0 ] || exit $rc
  summ $L
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=gpurun_out/prof17_batch128
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT -o bench --output-format csv -- python bench.py --mode batch --steps 1 --warmup 1 > $OUT/run.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python scripts/prof_summary.py $OUT bench $OUT/summary.md --drop-trace | sed -n 3,8p
rm -f $OUT/*.csv
OUT=gpurun_out/prof17_serve
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT -o bench --output-format csv -- python bench.py --admit-group 8 --mixed-tokens 640 --steps 1 --warmup 1 > $OUT/run.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python scripts/prof_summary.py $OUT bench $OUT/summary.md --drop-trace | sed -n 3,8p
rm -f $OUT/*.csv

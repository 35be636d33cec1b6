#!/bin/bash
# One GPU step of a gpurun call: gpu_step.sh NAME SECONDS CMD...
#   runs CMD under `timeout -k 10 SECONDS`, output to gpurun_out/NAME.log, prints its tail and
#   exits with CMD's status (chain steps with && so a failed / timed-out step ends the call).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
name=$1; secs=$2; shift 2
export PYTHONUNBUFFERED=1
timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
rc=$?
tail -n 25 "gpurun_out/$name.log"
echo "[$name] rc=$rc"
exit $rc

#!/bin/bash
# 2-rank rehearsal of the multi-GPU bench path on a 1-GPU box: two DP ranks share the card over
# gloo (the driver's 8-GPU run uses RCCL), each with a 40 GB KV pool.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export DAB_DIST_BACKEND=gloo PYTHONUNBUFFERED=1
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 --kv-gb 40 "$@" > gpurun_out/dp2.log 2>&1
rc=$?
tail -n 5 gpurun_out/dp2.log
exit $rc

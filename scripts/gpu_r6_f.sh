#!/bin/bash
# Round 6, call F: BASELINE config 5 end-to-end at FULL size on ONE card: 8 gloo
# ranks share the GPU -- bge-large retriever, replicated index, Llama-3-70B TP 8 (80 layers, hidden
# 8192, vocab 128256; the IPC one-shot all-reduce, fused with the RMSNorm in the decode graphs; the
# vocab-parallel LM head), open-loop arrivals.  A rehearsal of the code path, NOT a performance
# number (8 ranks time-share one GPU and sync over gloo).
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
export DAB_DIST_BACKEND=gloo
$S r6f_cfg5 1100 python -u bench.py --config 5 --gpus 8 --batch 4 --steps 1 --warmup 1 --max-new-tokens 32 \
  --kv-gb 6 --index-rows 100000 --qps 2 --json-out gpurun_out/r6f_cfg5.json

#!/bin/bash
# Round 5, call G: kernel + model GPU tests with the new defaults (pipelined V reads on, consumer-side
# norm opt-in), the attention A/B again, a PMC pass over the batch-1 decode (VERDICT r4 item 5's
# fallback table), and the encoder kernel profile (item 7).
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r5g_tests 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 300 --timeout-method thread &&
$S r5g_attn 300 python -u benchmarks/kernel_bench.py attn &&
PDEC_PREFIX=pdec_b1 $S r5g_pmc_b1 800 bash scripts/prof_decode_pmc.sh --batch 1 --steps 40 &&
$S r5g_embed_prof 500 bash scripts/prof_embed.sh

#!/bin/bash
# Round 5, call I: encoder pipeline (faster batch tokenizer, small first block) -- embed bench x2,
# then the kernel profile with a GPU gap report; PMC passes of the prefill attention (item 6).
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r5i_embed 400 python -u benchmarks/embed_bench.py --chunks 1000000 &&
$S r5i_embed2 400 python -u benchmarks/embed_bench.py --chunks 1000000 &&
$S r5i_embed_prof 500 bash scripts/prof_embed.sh &&
PDEC_PREFIX=pattn PDEC_DRIVER="benchmarks/kernel_bench.py attn" $S r5i_pmc_attn 800 bash scripts/prof_decode_pmc.sh

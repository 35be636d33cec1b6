#!/bin/bash
# Round 5, call W: PMC passes of the prefill attention kernels at the new defaults (paired causal
# blocks) -> gpurun_out/pattn2_table.md.
cd "$GRAFT_REPO_ROOT" || exit 1
PDEC_PREFIX=pattn2 PDEC_DRIVER="benchmarks/kernel_bench.py attn" timeout -k 10 900 bash scripts/prof_decode_pmc.sh

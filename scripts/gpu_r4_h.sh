#!/bin/bash
# Round 4, call H (end-of-round evidence): the whole GPU suite + smoke, the headline bench, config 2
# and config 3 benches, and a rocprofv3 kernel profile of one headline step.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r4h_suite 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread &&
$S r4h_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" &&
$S r4h_gemm 400 python -u benchmarks/gemm_bench.py --shapes llama,bge --rounds 3 --iters 10 &&
$S r4h_stamps 300 python -u benchmarks/gemm_stamps.py --shapes bge-qkv,bge-o,bge-up,cand-shape,llama-o &&
$S r4h_bench 600 python -u bench.py --steps 10 --warmup 3 &&
$S r4h_embed 300 python -u benchmarks/embed_bench.py --chunks 1000000 &&
$S r4h_index 300 python -u benchmarks/index_bench.py --iters 10 --warmup 3 --batch 1 16 64 96 128 512 &&
bash scripts/prof_bench.sh

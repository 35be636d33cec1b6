#!/bin/bash
# Round 5, call R: persistent encoder attention (DAB_ENC_PERSIST=1): parity, the packed flash and
# encoder-model tests with it on, the kernel A/B on the embed bench's batch, and the embed bench
# end to end with and without it.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r5r_variant_tests 300 python -u -m pytest tests/test_kernels_gpu.py -k "variants_match" -x -v --timeout 120 --timeout-method thread &&
DAB_ENC_PERSIST=1 $S r5r_enc_tests 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -k "flash_packed or bert or encoder or embed" -x -q --timeout 120 --timeout-method thread &&
$S r5r_attn 300 python -u benchmarks/kernel_bench.py attn &&
$S r5r_embed 400 python -u benchmarks/embed_bench.py --chunks 1000000 &&
DAB_ENC_PERSIST=1 $S r5r_embed_p 400 python -u benchmarks/embed_bench.py --chunks 1000000 &&
$S r5r_embed2 400 python -u benchmarks/embed_bench.py --chunks 1000000 &&
DAB_ENC_PERSIST=1 $S r5r_embed_p2 400 python -u benchmarks/embed_bench.py --chunks 1000000

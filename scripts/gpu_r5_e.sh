#!/bin/bash
# Round 5, call E: the consumer-side RMSNorm for small decode batches: numerics
# (kernel + model, folded gains), then un-profiled interleaved A/B at batch 1 / 8 / 128; then the
# software-pipelined V reads of the prefill attention (item 6): flash tests with it on, kernel A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
S=scripts/gpu_step.sh
$S r5e_tests 600 python -u -m pytest tests/test_kernels_gpu.py -k "consumer_rmsnorm or (test_stream_gemm and (-32- or -33-))" tests/test_models_gpu.py -x -v --timeout 300 --timeout-method thread &&
$S r5e_ab_b1 400 python -u benchmarks/decode_ab.py --batch 1 --arms base,normkernels,res32 --rounds 3 --steps 100 &&
$S r5e_ab_b8 400 python -u benchmarks/decode_ab.py --batch 8 --arms base,normkernels,res32 --rounds 3 --steps 100 &&
$S r5e_ab_b128 400 python -u benchmarks/decode_ab.py --batch 128 --arms base --rounds 2 --steps 40 &&
DAB_FLASH_VPIPE=1 $S r5f_flash_tests 400 python -u -m pytest tests/test_kernels_gpu.py -k "flash" -x -q --timeout 300 --timeout-method thread &&
$S r5f_attn 300 python -u benchmarks/kernel_bench.py attn

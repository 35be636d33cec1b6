cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for c in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAIT_ANY" "TCC_HIT_sum TCC_MISS_sum"; do
  n=$(echo $c | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/prof_$n -- python benchmarks/gemm_bench.py --shapes llama,bge --only llama8b-o,llama8b-down,bge-qkv --rounds 1 --iters 2 --native-only > gpurun_out/prof_$n.log 2>&1 || exit $?
done

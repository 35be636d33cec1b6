#!/bin/bash
# rocprofv3 PMC passes over the attention microbench (flash prefill / encoder / paged decode) ->
# gpurun_out/pattn_*/ ; one pass per counter group (the SQ block holds 8 counters per pass)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for c in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAIT_ANY" \
         "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVES"; do
  n=$(echo $c | cut -d' ' -f2)
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pattn_$n -o run \
    -- python benchmarks/kernel_bench.py attn > gpurun_out/pattn_$n.log 2>&1 || exit $?
done
python scripts/pmc_table.py gpurun_out/pattn_SQ_WAVE_CYCLES gpurun_out/pattn_SQ_ACTIVE_INST_ANY > gpurun_out/pattn_table.md

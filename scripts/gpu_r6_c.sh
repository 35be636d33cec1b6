#!/bin/bash
# Round 6, call C: PMC passes over gemm_mid (BK 32 / 64, combine on / off) and gemm256 on two mid shapes.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for shp in 768,4096,4096 2048,4096,4096; do
  for c in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAIT_ANY" "TCC_HIT_sum TCC_MISS_sum" "SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM"; do
    n=$(echo $c | cut -d' ' -f1)_${shp//,/x}
    timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/r6c_$n -- python benchmarks/gmid_probe.py --shape $shp --g256 > gpurun_out/r6c_$n.log 2>&1 || exit $?
  done
  python scripts/pmc_table.py gpurun_out/r6c_GRBM_GUI_ACTIVE_${shp//,/x} gpurun_out/r6c_TCC_HIT_sum_${shp//,/x} gpurun_out/r6c_SQ_LDS_IDX_ACTIVE_${shp//,/x} > gpurun_out/r6c_table_${shp//,/x}.md || exit 1
done
cat gpurun_out/r6c_table_*.md

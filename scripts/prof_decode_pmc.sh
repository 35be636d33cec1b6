#!/bin/bash
# rocprofv3 PMC passes over an eager Llama-3-8B prefill + decode (benchmarks/decode_pmc_driver.py)
# -> gpurun_out/pdec_*/ and gpurun_out/pdec_table.md.  One pass per counter group, each with
# --kernel-trace only (durations for bytes / time); the TCC block holds 4 counters per pass
# (FETCH_SIZE takes 3, WRITE_SIZE 2), the SQ block 8.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
p=${PDEC_PREFIX:-pdec}  # output prefix; extra arguments go to the driver (e.g. --batch 1 --steps 40)
# PDEC_DRIVER: another python program (+ its arguments) to profile, e.g. "benchmarks/kernel_bench.py attn"
i=0
for c in "FETCH_SIZE GRBM_GUI_ACTIVE" \
         "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" \
         "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_WAVES"; do
  i=$((i + 1))
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/${p}_$i -o run \
    -- python ${PDEC_DRIVER:-benchmarks/decode_pmc_driver.py --steps 6} "$@" > gpurun_out/${p}_$i.log 2>&1 || exit $?
done
python scripts/pmc_table.py gpurun_out/${p}_1 gpurun_out/${p}_2 gpurun_out/${p}_3 > gpurun_out/${p}_table.md

#!/bin/bash
# PMC passes (one rocprofv3 run each, counters within the per-block slot limits) over a command.
# Usage: tools/pmc_passes.sh <outdir> -- <program args...>   (program: python3 / a binary, run directly)
set -e
out=$1; shift; shift
export TMPDIR=/tmp
mkdir -p "$out"
i=0
for pmc in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS" \
           "FETCH_SIZE GRBM_GUI_ACTIVE" \
           "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VALU_TRANS_F32 SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d "$out/p$i" -o run -- "$@" > "$out/p$i.log" 2>&1
done

#!/bin/bash
# PMC passes restricted to kernels matching a regex (small output), one rocprofv3 run per pass.
# Usage: tools/pmc_kernel.sh <outdir> <kernel-regex> -- <program args...>
set -e
out=$1; rx=$2; shift; shift; shift
export TMPDIR=/tmp
mkdir -p "$out"
i=0
for pmc in "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VALU_TRANS_F32 SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $pmc --kernel-include-regex "$rx" --output-format csv -d "$out/p$i" -o run -- "$@" > "$out/p$i.log" 2>&1
done

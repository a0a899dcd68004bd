mkdir -p gpurun_out && export TMPDIR=/tmp
H=$(cat gpurun_out/.head 2>/dev/null || echo cur)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_gputest.log 2>&1; rc=$?; tail -3 gpurun_out/r3_gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/r3_bench.log 2>&1 || exit 1; tail -1 gpurun_out/r3_bench.log | cut -c1-400
bash tools/prof_bench.sh gpurun_out/r3prof || exit 1
python tools/rocprof_summary.py gpurun_out/r3prof/run_results.db --last 5 --top 45 > gpurun_out/r3_stats.md || exit 1
head -20 gpurun_out/r3_stats.md
out=gpurun_out/pmcwb; mkdir -p $out; i=0
for pmc in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VALU_TRANS_F32 SQ_WAVES" "FETCH_SIZE GRBM_GUI_ACTIVE"; do
  i=$((i+1)); WATTN_STAGE=0 timeout -s KILL 90 rocprofv3 --pmc $pmc --output-format csv -d "$out/p$i" -o run -- python3 tools/wattn_bench.py > "$out/p$i.log" 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
python tools/pmc_summary.py $out wattn_bwd > gpurun_out/r3_pmc_wattn_bwd_stage1_counters.txt; cat gpurun_out/r3_pmc_wattn_bwd_stage1_counters.txt

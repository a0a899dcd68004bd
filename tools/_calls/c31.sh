set -o pipefail
export PYTHONUNBUFFERED=1
B="python3 bench.py --steps 1 --warmup 1 --roofline-steps 1 --no-cpu-baseline --agent-steps 0"
bash tools/pmc_kernel.sh /tmp/pq wattn_qkv_fwd -- $B && \
python3 tools/pmc_traffic.py /tmp/pq wattn_qkv_fwd gpurun_out/r5_pmc_wattn_qkv_fwd.json "bench.py --steps 1 --warmup 1 --roofline-steps 1, kernel-filtered rocprofv3 --pmc passes (tools/pmc_kernel.sh), round-5 tree" > /dev/null && \
python3 tools/pmc_summary.py /tmp/pq wattn_qkv_fwd > gpurun_out/r5_pmc_wattn_qkv_fwd_counters.txt && \
bash tools/pmc_kernel.sh /tmp/pg "false, true>" -- $B && \
python3 tools/pmc_traffic.py /tmp/pg "false, true>" gpurun_out/r5_pmc_gemm_grouped_dw.json "grouped weight-gradient launches (stages 1-4) of one step, kernel-filtered rocprofv3 --pmc passes" > /dev/null && \
python3 tools/pmc_summary.py /tmp/pg "false, true>" > gpurun_out/r5_pmc_gemm_grouped_dw_counters.txt
rc=$?; cat gpurun_out/r5_pmc_wattn_qkv_fwd.json gpurun_out/r5_pmc_gemm_grouped_dw.json; rm -rf /tmp/pq /tmp/pg; exit $rc

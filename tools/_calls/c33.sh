set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u tools/dw_batch_bench.py --iters 3 > gpurun_out/r5_c33_dwbench.txt 2>&1 && \
tools/ab_env.sh r5ss 2 - "LRCE_DW_SHORT_SPLIT=2" > gpurun_out/r5_c33_ab.txt 2>&1
rc=$?; grep -v amdgpu gpurun_out/r5_c33_dwbench.txt | tail -4; cat gpurun_out/r5_c33_ab.txt; exit $rc

set -o pipefail
export PYTHONUNBUFFERED=1
LRCE_DW_LOCKSTEP=1 timeout -k 10 240 python -u -m pytest tests/test_ops_gpu.py -k "dw_grouped or dw_batched" -q --timeout 120 --timeout-method thread > gpurun_out/r5_c34_ops.log 2>&1 && \
LRCE_DW_LOCKSTEP=1 timeout -k 10 400 python -u tools/dw_batch_bench.py --iters 3 > gpurun_out/r5_c34_dw_lock.txt 2>&1 && \
timeout -k 10 400 python -u tools/dw_batch_bench.py --iters 3 > gpurun_out/r5_c34_dw_base.txt 2>&1 && \
tools/ab_env.sh r5ls 2 - "LRCE_DW_LOCKSTEP=1" > gpurun_out/r5_c34_ab.txt 2>&1
rc=$?; tail -1 gpurun_out/r5_c34_ops.log; grep -h "blocks x" gpurun_out/r5_c34_dw_lock.txt gpurun_out/r5_c34_dw_base.txt; cat gpurun_out/r5_c34_ab.txt; exit $rc

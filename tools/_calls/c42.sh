set -o pipefail
export PYTHONUNBUFFERED=1
LRCE_RED_NT=1 timeout -k 10 240 python -u -m pytest tests/test_ops_gpu.py -k "dw or linear" -q --timeout 120 --timeout-method thread > gpurun_out/r5_c42_ops.log 2>&1 && \
timeout -k 10 400 python -u tools/dw_batch_bench.py --iters 3 > gpurun_out/r5_c42_dw_base.txt 2>&1 && \
LRCE_RED_NT=1 timeout -k 10 400 python -u tools/dw_batch_bench.py --iters 3 > gpurun_out/r5_c42_dw_nt.txt 2>&1 && \
tools/ab_env.sh r5rn 2 - "LRCE_RED_NT=1" > gpurun_out/r5_c42_ab.txt 2>&1
rc=$?; tail -1 gpurun_out/r5_c42_ops.log; grep -h "launches\|split" gpurun_out/r5_c42_dw_base.txt gpurun_out/r5_c42_dw_nt.txt | cut -c1-120; cat gpurun_out/r5_c42_ab.txt; exit $rc

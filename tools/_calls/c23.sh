set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 240 python -u -m pytest tests/test_ops_gpu.py -k "dw_grouped or dw_batched" -v --timeout 120 --timeout-method thread > gpurun_out/r5_c23_ops.log 2>&1 && \
timeout -k 10 400 python -u tools/dw_batch_bench.py --iters 3 > gpurun_out/r5_c23_dwbench.txt 2>&1 && \
timeout -k 10 700 python -u -m pytest tests/test_model_gpu.py tests/test_train_parity_gpu.py tests/test_swin_gpu.py -q --maxfail=3 --timeout 300 --timeout-method thread > gpurun_out/r5_c23_tests.log 2>&1 && \
tools/ab_env.sh r5sd 2 - "LRCE_SPLIT_DW=0" > gpurun_out/r5_c23_ab.txt 2>&1
rc=$?; tail -7 gpurun_out/r5_c23_ops.log; cat gpurun_out/r5_c23_dwbench.txt; tail -3 gpurun_out/r5_c23_tests.log; cat gpurun_out/r5_c23_ab.txt; exit $rc

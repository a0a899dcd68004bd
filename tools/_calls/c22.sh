set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 240 python -u -m pytest tests/test_ops_gpu.py -k "dw_grouped or dw_batched" -v --timeout 120 --timeout-method thread > gpurun_out/r5_c22_ops.log 2>&1 && \
timeout -k 10 700 python -u -m pytest tests/test_model_gpu.py tests/test_train_parity_gpu.py tests/test_agent_gpu.py -q --maxfail=3 --timeout 300 --timeout-method thread > gpurun_out/r5_c22_tests.log 2>&1 && \
tools/ab_env.sh r5bg 2 - "LRCE_BERT_WGRAD_GROUPED=0" > gpurun_out/r5_c22_ab.txt 2>&1
rc=$?; tail -5 gpurun_out/r5_c22_ops.log; tail -3 gpurun_out/r5_c22_tests.log; cat gpurun_out/r5_c22_ab.txt; exit $rc

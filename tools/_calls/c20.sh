set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 240 python -u -m pytest tests/test_ops_gpu.py -k "linear_resid_ln or dw_batched or adamw_keeps" -v --timeout 120 --timeout-method thread > gpurun_out/r5_c20_ops.log 2>&1 && \
timeout -k 10 700 python -u -m pytest tests/test_model_gpu.py tests/test_ops_gpu.py tests/test_agent_gpu.py tests/test_train_parity_gpu.py -q --maxfail=5 --timeout 300 --timeout-method thread > gpurun_out/r5_c20_tests.log 2>&1 ; rt=$?; \
{ [ $rt -eq 0 ] || [ $rt -eq 1 ]; } && tools/ab_env.sh r5rl 2 - "LRCE_BERT_REDUCE_LN=0" "LRCE_STORE_FRESH_GRADS=0" > gpurun_out/r5_c20_ab.txt 2>&1
rc=$?; tail -5 gpurun_out/r5_c20_ops.log; tail -4 gpurun_out/r5_c20_tests.log; cat gpurun_out/r5_c20_ab.txt; exit $rc

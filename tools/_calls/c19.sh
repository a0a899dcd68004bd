set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest tests/test_model_gpu.py tests/test_ops_gpu.py tests/test_agent_gpu.py tests/test_train_parity_gpu.py -q --maxfail=5 --timeout 300 --timeout-method thread > gpurun_out/r5_c19_tests.log 2>&1 ; rt=$?; \
{ [ $rt -eq 0 ] || [ $rt -eq 1 ]; } && tools/ab_env.sh r5sf 2 - "LRCE_STORE_FRESH_GRADS=0" > gpurun_out/r5_c19_ab.txt 2>&1
rc=$?; tail -4 gpurun_out/r5_c19_tests.log; cat gpurun_out/r5_c19_ab.txt; exit $rc

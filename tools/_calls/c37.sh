set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_agent_gpu.py tests/test_train_parity_gpu.py -k "adamw or agent or train or early" -q --maxfail=3 --timeout 300 --timeout-method thread > gpurun_out/r5_c37_tests.log 2>&1 && \
tools/ab_env.sh r5aw 2 - "LRCE_ADAMW_VARIANT=0" > gpurun_out/r5_c37_ab.txt 2>&1
rc=$?; tail -2 gpurun_out/r5_c37_tests.log; cat gpurun_out/r5_c37_ab.txt; exit $rc

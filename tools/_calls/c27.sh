set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_agent_gpu.py tests/test_train_parity_gpu.py -q --maxfail=3 --timeout 300 --timeout-method thread > gpurun_out/r5_c27_tests.log 2>&1 && \
tools/ab_env.sh r5cl 2 - "LRCE_CLEAR_AT_DECODER=0" > gpurun_out/r5_c27_ab.txt 2>&1
rc=$?; tail -3 gpurun_out/r5_c27_tests.log; cat gpurun_out/r5_c27_ab.txt; exit $rc

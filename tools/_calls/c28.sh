set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests/test_distributed_gpu.py tests/test_model_gpu.py tests/test_agent_gpu.py tests/test_train_parity_gpu.py -k "dp_ or deferred or agent or train or early" -q --maxfail=3 --timeout 400 --timeout-method thread > gpurun_out/r5_c28_tests.log 2>&1 && \
tools/ab_env.sh r5cl 2 - "LRCE_CLEAR_AT_DECODER=0" > gpurun_out/r5_c28_ab.txt 2>&1 && \
timeout -k 10 300 python -u tools/cumask_probe.py > gpurun_out/r5_cumask_probe.txt 2>&1
rc=$?; tail -3 gpurun_out/r5_c28_tests.log; cat gpurun_out/r5_c28_ab.txt; cat gpurun_out/r5_cumask_probe.txt; exit $rc

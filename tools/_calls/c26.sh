set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests/test_distributed_gpu.py tests/test_model_gpu.py -k "dp_ or deferred" -v --timeout 400 --timeout-method thread > gpurun_out/r5_c26_tests.log 2>&1
rc=$?; [ $rc -eq 0 ] && { timeout -k 10 300 python -u tools/cumask_probe.py > gpurun_out/r5_cumask_probe.txt 2>&1; cat gpurun_out/r5_cumask_probe.txt; }
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r5_c26_tests.log | tail -12; exit $rc

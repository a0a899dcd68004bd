set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 180 python tools/dw_batch_bench.py > gpurun_out/r5_c15_dwbatch.txt 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py tests/test_ops_gpu.py tests/test_agent_gpu.py -k "deferred or bit_identical or dw_batched or early_updates or e2e_train" -q --timeout 200 --timeout-method thread > gpurun_out/r5_c15_tests.log 2>&1 ; rt=$?; \
{ [ $rt -eq 0 ] || [ $rt -eq 1 ]; } && tools/ab_env.sh r5dw 2 - "LRCE_SWIN_DEFER_WGRAD=0" > gpurun_out/r5_c15_ab.txt 2>&1
rc=$?; grep -v amdgpu gpurun_out/r5_c15_dwbatch.txt; tail -4 gpurun_out/r5_c15_tests.log; cat gpurun_out/r5_c15_ab.txt; exit $rc

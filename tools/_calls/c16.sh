set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py tests/test_ops_gpu.py tests/test_agent_gpu.py -k "deferred or bit_identical or dw_batched or early_updates or e2e_train or fused_decoder" -q --timeout 200 --timeout-method thread > gpurun_out/r5_c16_tests.log 2>&1 ; rt=$?; \
{ [ $rt -eq 0 ] || [ $rt -eq 1 ]; } && tools/ab_env.sh r5dw2 2 - "LRCE_SWIN_DEFER_WGRAD=0" "LRCE_DEC_KV_WGRAD_BATCHED=0" > gpurun_out/r5_c16_ab.txt 2>&1 && \
bash tools/prof_step.sh r5p4
rc=$?; tail -4 gpurun_out/r5_c16_tests.log; cat gpurun_out/r5_c16_ab.txt; head -3 gpurun_out/r5p4_timeline.txt; exit $rc

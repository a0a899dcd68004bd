set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 200 python tools/determinism_probe.py > gpurun_out/r5_c13_determinism.txt 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py tests/test_swin_gpu.py tests/test_ops_gpu.py -k "deferred or swin or layernorm or window or e2e_train or stage or bert" -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_c13_tests.log 2>&1 ; rt=$?; \
{ [ $rt -eq 0 ] || [ $rt -eq 1 ]; } && tools/ab_env.sh r5dr 3 - "LRCE_SWIN_DEFER_RED=0 LRCE_BERT_LN_DEFER=0" "LRCE_DEC_WGRAD_EARLY=0" > gpurun_out/r5_c13_ab.txt 2>&1
rc=$?; cat gpurun_out/r5_c13_determinism.txt | grep -v amdgpu; tail -3 gpurun_out/r5_c13_tests.log; cat gpurun_out/r5_c13_ab.txt; exit $rc

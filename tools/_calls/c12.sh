set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -k "fused_decoder or bit_identical or fusion_backward or e2e_train" -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_c12_tests.log 2>&1 && \
tools/ab_env.sh r5wg 3 - "LRCE_DEC_WGRAD_EARLY=0" > gpurun_out/r5_c12_ab.txt 2>&1
rc=$?; tail -3 gpurun_out/r5_c12_tests.log; cat gpurun_out/r5_c12_ab.txt; exit $rc

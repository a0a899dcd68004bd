set -o pipefail
export PYTHONUNBUFFERED=1
LRCE_DEC_KV_WGRAD_BATCHED=1 timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -k "decoder or fused or kv" -q --timeout 200 --timeout-method thread > gpurun_out/r5_c41_tests.log 2>&1 && \
tools/ab_env.sh r5kv 2 - "LRCE_DEC_KV_WGRAD_BATCHED=1" > gpurun_out/r5_c41_ab.txt 2>&1
rc=$?; tail -1 gpurun_out/r5_c41_tests.log; cat gpurun_out/r5_c41_ab.txt; exit $rc

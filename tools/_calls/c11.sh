set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_model_gpu.py tests/test_ops_gpu.py tests/test_swin_gpu.py -k "fusion or decoder or fused_decoder or e2e or layernorm or swin or block" -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_c11_tests.log 2>&1 && \
timeout -k 10 120 python tools/decoder_trace.py > gpurun_out/r5_c11_dectrace.txt 2>&1 && \
timeout -k 10 120 python tools/ln_bench.py > gpurun_out/r5_c11_ln_base.txt 2>&1 && \
LRCE_LN_PF2=1 timeout -k 10 120 python tools/ln_bench.py > gpurun_out/r5_c11_ln_pf2.txt 2>&1 && \
tools/ab_env.sh r5kv 2 - "LRCE_DEC_KV_ASYNC=0" "LRCE_SWIN_WGRAD_ASYNC=0" "LRCE_DEC_KV_ASYNC=0 LRCE_SWIN_WGRAD_ASYNC=0" > gpurun_out/r5_c11_ab.txt 2>&1
rc=$?; tail -3 gpurun_out/r5_c11_tests.log; cat gpurun_out/r5_c11_ab.txt; exit $rc

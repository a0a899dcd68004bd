set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/ln_bench.py > gpurun_out/r5_c38_ln_base.txt 2>&1 && \
LRCE_LN_NT=1 timeout -k 10 300 python -u tools/ln_bench.py > gpurun_out/r5_c38_ln_nt.txt 2>&1 && \
LRCE_LN_NT=1 timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py tests/test_swin_gpu.py -k "layernorm or ln_ or stage or handoff" -q --timeout 120 --timeout-method thread > gpurun_out/r5_c38_tests.log 2>&1 && \
tools/ab_env.sh r5ln 2 - "LRCE_LN_NT=1" > gpurun_out/r5_c38_ab.txt 2>&1
rc=$?; paste gpurun_out/r5_c38_ln_base.txt gpurun_out/r5_c38_ln_nt.txt | head -30; tail -1 gpurun_out/r5_c38_tests.log; cat gpurun_out/r5_c38_ab.txt; exit $rc

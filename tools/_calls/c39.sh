set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_agent_gpu.py tests/test_train_parity_gpu.py -k "adamw or agent or train or early" -q --maxfail=3 --timeout 300 --timeout-method thread > gpurun_out/r5_c39_tests.log 2>&1 && \
timeout -k 10 300 python -u tools/ln_bench.py > gpurun_out/r5_c39_ln_base.txt 2>&1 && \
LRCE_LN_NT=1 timeout -k 10 300 python -u tools/ln_bench.py > gpurun_out/r5_c39_ln_nt.txt 2>&1 && \
LRCE_LN_NT=1 timeout -k 10 300 python -u -m pytest tests/test_swin_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/r5_c39_swin_nt.log 2>&1 && \
tools/ab_env.sh r5an 2 - "LRCE_ADAMW_VARIANT=0" "LRCE_LN_NT=1" > gpurun_out/r5_c39_ab.txt 2>&1
rc=$?; tail -1 gpurun_out/r5_c39_tests.log; paste -d'|' gpurun_out/r5_c39_ln_base.txt gpurun_out/r5_c39_ln_nt.txt | head -24; tail -1 gpurun_out/r5_c39_swin_nt.log; cat gpurun_out/r5_c39_ab.txt; exit $rc

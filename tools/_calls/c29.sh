set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_agent_gpu.py tests/test_train_parity_gpu.py -q --maxfail=3 --timeout 300 --timeout-method thread > gpurun_out/r5_c29_tests.log 2>&1 && \
tools/ab_env.sh r5sf 2 - "LRCE_BERT_SPLIT_FLUSH=0" > gpurun_out/r5_c29_ab.txt 2>&1
rc=$?; tail -3 gpurun_out/r5_c29_tests.log; cat gpurun_out/r5_c29_ab.txt; exit $rc

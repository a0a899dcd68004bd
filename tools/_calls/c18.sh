set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -k "e2e_train or bit_identical or fused_decoder" -q --timeout 200 --timeout-method thread > gpurun_out/r5_c18_tests.log 2>&1 ; rt=$?; \
{ [ $rt -eq 0 ] || [ $rt -eq 1 ]; } && tools/ab_env.sh r5il 2 - "LRCE_TEXT_INTERLEAVE=1" "LRCE_DEC_KV_AHEAD=0" > gpurun_out/r5_c18_ab.txt 2>&1
rc=$?; tail -3 gpurun_out/r5_c18_tests.log; cat gpurun_out/r5_c18_ab.txt; exit $rc

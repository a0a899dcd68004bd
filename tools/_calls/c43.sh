set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r5_c43_tests.log 2>&1 ; rt=$?; \
{ [ $rt -eq 0 ] || [ $rt -eq 1 ]; } && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5_c43_smoke.log 2>&1
rc=$?; tail -1 gpurun_out/r5_c43_tests.log; tail -1 gpurun_out/r5_c43_smoke.log; exit $rc

set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r5_c40_tests.log 2>&1 ; rt=$?; \
{ [ $rt -eq 0 ] || [ $rt -eq 1 ]; } && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5_c40_smoke.log 2>&1 && \
timeout -k 10 600 python -u bench.py > gpurun_out/r5_c40_bench.log 2>&1 && \
bash tools/prof_step.sh r5_c40p
rc=$?; tail -3 gpurun_out/r5_c40_tests.log; tail -3 gpurun_out/r5_c40_smoke.log; tail -2 gpurun_out/r5_c40_bench.log; head -30 gpurun_out/r5_c40p_stats.md; exit $rc

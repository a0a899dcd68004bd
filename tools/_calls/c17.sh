set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 120 python tools/graph_overlap_probe.py > gpurun_out/r5_c17_overlap.txt 2>&1 && \
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail=8 --timeout 300 --timeout-method thread > gpurun_out/r5_c17_tests.log 2>&1
rc=$?; grep -v amdgpu gpurun_out/r5_c17_overlap.txt; tail -12 gpurun_out/r5_c17_tests.log; exit $rc

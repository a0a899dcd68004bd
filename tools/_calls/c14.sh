set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 200 python tools/determinism_probe.py > gpurun_out/r5_c14_determinism.txt 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5_c14_tests.log 2>&1
rc=$?; grep -v amdgpu gpurun_out/r5_c14_determinism.txt; tail -5 gpurun_out/r5_c14_tests.log; exit $rc

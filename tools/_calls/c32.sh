set -o pipefail
export PYTHONUNBUFFERED=1
tools/ab_env.sh r5nc 2 - "LRCE_DEV_NO_CLEAR=1" > gpurun_out/r5_c32_ab.txt 2>&1
rc=$?; cat gpurun_out/r5_c32_ab.txt; exit $rc

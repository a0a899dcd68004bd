set -o pipefail
export PYTHONUNBUFFERED=1
tools/ab_env.sh r5cs 2 - "LRCE_CLEAR_AT=swin3" > gpurun_out/r5_c30_ab.txt 2>&1
rc=$?; cat gpurun_out/r5_c30_ab.txt; exit $rc

set -o pipefail
export PYTHONUNBUFFERED=1
for v in 0 1 2 3 0; do LRCE_ADAMW_VARIANT=$v timeout -k 10 120 python -u tools/adamw_bench.py >> gpurun_out/r5_c36_adamw.txt 2>&1 || exit $?; done
cat gpurun_out/r5_c36_adamw.txt | grep variant

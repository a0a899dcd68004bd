set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
B="--no-cpu-baseline --agent-steps 0 --roofline-steps 0 --steps 20"
for i in 1 2; do
  for v in 2 1 4; do
    LRCE_SPLITK_PER_CU=$v timeout -k 10 300 python bench.py $B > gpurun_out/split_${v}_$i.log 2>&1
  done
done

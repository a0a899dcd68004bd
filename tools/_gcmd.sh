set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_swin_gpu.py tests/test_model_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_sel.log 2>&1
B="--no-cpu-baseline --agent-steps 0 --roofline-steps 0 --steps 20"
for i in 1 2; do
  (cd dev/ab_base && timeout -k 10 300 python bench.py $B) > gpurun_out/ab_base_$i.log 2>&1
  timeout -k 10 300 python bench.py $B > gpurun_out/ab_new_$i.log 2>&1
done
bash tools/prof_bench.sh gpurun_out/sprof8

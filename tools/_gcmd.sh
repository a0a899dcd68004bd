set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_agent_gpu.py tests/test_model_gpu.py tests/test_distributed_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_early.log 2>&1
for i in 1 2; do
LRCE_AB_NO_SWIN_EARLY=1 timeout -k 10 300 python bench.py --no-cpu-baseline --agent-steps 0 --roofline-steps 0 --steps 20 > gpurun_out/b_off$i.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --agent-steps 0 --roofline-steps 0 --steps 20 > gpurun_out/b_on$i.log 2>&1
done

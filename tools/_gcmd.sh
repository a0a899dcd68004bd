set -e
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_agent_gpu.py -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/t_agent.log 2>&1
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1

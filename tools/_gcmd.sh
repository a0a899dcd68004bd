set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_agent_gpu.py -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/t_agent2.log 2>&1

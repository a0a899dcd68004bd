set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py tests/test_model_gpu.py tests/test_agent_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/t_fd.log 2>&1
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --roofline-steps 0 > gpurun_out/bench_fd.log 2>&1

set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py tests/test_agent_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/t_e2e.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke3.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/bench_e2e.log 2>&1

set -e
timeout -k 10 120 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q --timeout 60 --timeout-method thread -k "gemm or layernorm" > gpurun_out/t_ops.log 2>&1
timeout -k 10 240 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1
bash tools/prof_bench.sh gpurun_out/prof

set -e
timeout -k 10 120 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q --timeout 60 --timeout-method thread -k "gemm or layernorm" > gpurun_out/t_ops.log 2>&1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_new.log 2>&1
timeout -k 10 120 python tools/ln_bench.py > gpurun_out/ln_bench.txt 2>&1
timeout -k 10 200 python tools/gemm_bench.py --first 15 > gpurun_out/gb_new.txt 2>&1
timeout -k 10 240 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1

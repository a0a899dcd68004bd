set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm" > gpurun_out/t_g160.log 2>&1
timeout -k 10 300 python tools/gemm_bench.py --iters 30 > gpurun_out/gemm_bench160.log 2>&1
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --roofline-steps 0 > gpurun_out/bench_160.log 2>&1
LRCE_NATIVE_LIB=$PWD/vqa-lrce-kbs-2023_amd/lrce/_native/liblrce_hip_prev.so timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --roofline-steps 0 > gpurun_out/bench_prev.log 2>&1

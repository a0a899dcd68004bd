set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_ops.log 2>&1
timeout -k 10 300 python tools/gemm_bench.py --first 21 --iters 20 > gpurun_out/gemm_nt.log 2>&1
bash tools/pmc_passes.sh gpurun_out/pmc_g1c -- python3 tools/gemm_bench.py --only 1 --iters 5

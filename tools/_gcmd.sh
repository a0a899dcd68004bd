set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py tests/test_swin_gpu.py tests/test_ops_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_sel.log 2>&1
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1
bash tools/prof_bench.sh gpurun_out/sprof6

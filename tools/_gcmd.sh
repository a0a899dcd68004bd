set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_swin_gpu.py tests/test_ops_gpu.py tests/test_model_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_pad.log 2>&1

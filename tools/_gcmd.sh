set -e
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_video_gpu.py -m gpu -x -v --timeout 100 --timeout-method thread > gpurun_out/t_video.log 2>&1

mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "window_attention_fwd_bwd" > gpurun_out/t6.log 2>&1; rc=$?; grep -E "^E  |passed|failed|Error" gpurun_out/t6.log | head -20; [ $rc -eq 0 ] || exit $rc

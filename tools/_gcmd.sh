mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "fused_decoder" > gpurun_out/t3.log 2>&1; rc=$?; grep -E "^E  |passed|failed|Error" gpurun_out/t3.log | head -30; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_agent_gpu.py tests/test_ops_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "early or window_attention_fwd_bwd" > gpurun_out/t2.log 2>&1; rc=$?; grep -E "^E  |passed|failed" gpurun_out/t2.log | head -30
timeout -k 10 300 python bench.py --no-cpu-baseline --agent-steps 0 --steps 20 > gpurun_out/b3.log 2>&1; tail -1 gpurun_out/b3.log | cut -c1-400

mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "fused_decoder" > gpurun_out/t3.log 2>&1; rc=$?; grep -E "^E  |passed|failed|Error" gpurun_out/t3.log | head -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/decoder_trace.py > gpurun_out/trace.log 2>&1; grep -v "last done\|amdgpu.ids" gpurun_out/trace.log
for f in 1 0 1; do LRCE_DEC_FUSED=$f timeout -k 10 200 python bench.py --no-cpu-baseline --agent-steps 0 --steps 20 > gpurun_out/ab_$f.log 2>&1 || exit 1; echo "fused=$f $(tail -1 gpurun_out/ab_$f.log | cut -c100-175)"; done

mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_swin_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_sw.log 2>&1; rc=$?; tail -2 gpurun_out/t_sw.log; [ $rc -eq 0 ] || exit $rc
for v in 0 512 1024 dbias 0 512; do LRCE_SWIN_WGRAD_STREAM=$v timeout -k 10 200 python bench.py --no-cpu-baseline --agent-steps 0 --steps 20 > gpurun_out/ab_w$v.log 2>&1 || exit 1; echo "w=$v $(tail -1 gpurun_out/ab_w$v.log | cut -c100-140)"; done

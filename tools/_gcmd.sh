mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "window_attention" > gpurun_out/t6.log 2>&1; rc=$?; grep -E "^E  |passed|failed|Error" gpurun_out/t6.log | head -20; [ $rc -eq 0 ] || exit $rc
for v in old new old new; do unset LRCE_NATIVE_LIB; if [ $v = old ]; then export LRCE_NATIVE_LIB=$PWD/tools/_ab_old.so; fi; echo "== $v"; timeout -k 10 120 python tools/wattn_bench.py 2>&1 | grep "all stages" || exit 1; done

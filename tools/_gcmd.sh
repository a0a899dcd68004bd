mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_gputest.log 2>&1; rc=$?; tail -3 gpurun_out/r3_gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/r3_bench.log 2>&1 || exit 1; tail -1 gpurun_out/r3_bench.log | cut -c1-300
bash tools/prof_bench.sh gpurun_out/r3prof || exit 1
python tools/rocprof_summary.py $(python -c "import glob;print(glob.glob('gpurun_out/r3prof/**/*results.db',recursive=True)[0])") --last 5 > gpurun_out/r3_stats.md 2>&1; head -40 gpurun_out/r3_stats.md

set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/t_all.log 2>&1
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1
bash tools/prof_bench.sh gpurun_out/prof4
python tools/rocprof_summary.py gpurun_out/prof4/run_results.db > gpurun_out/prof4_stats.md

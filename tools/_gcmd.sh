set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread -k "mha or fusion or e2e" > gpurun_out/t_mha.log 2>&1
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --roofline-steps 0 > gpurun_out/bench_mha.log 2>&1
bash tools/prof_bench.sh gpurun_out/prof7
python tools/rocprof_summary.py gpurun_out/prof7/run_results.db > gpurun_out/prof7_stats.md

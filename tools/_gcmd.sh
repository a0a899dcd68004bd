set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_final
B="python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 --roofline-steps 1 --mode eager"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_final/p1 -o run -- $B > gpurun_out/pmc_final/p1.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_final/p2 -o run -- $B > gpurun_out/pmc_final/p2.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmc_final/p3 -o run -- $B > gpurun_out/pmc_final/p3.log 2>&1
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_final.log 2>&1

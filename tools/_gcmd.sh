set -e
mkdir -p gpurun_out
for mk in 512 2048 100000; do LRCE_SKINNY_MINK=$mk timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --roofline-steps 0 > gpurun_out/bench_mk$mk.log 2>&1; done

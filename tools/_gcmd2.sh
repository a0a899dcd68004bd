mkdir -p gpurun_out && export TMPDIR=/tmp
out=gpurun_out/pmc3
mkdir -p $out
i=0
for pmc in "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $pmc --output-format csv -d "$out/p$i" -o run -- python3 bench.py --steps 1 --warmup 1 --roofline-steps 1 --no-cpu-baseline --agent-steps 0 > "$out/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$out/p$i.log"; exit 1; }
done
python tools/pmc_traffic.py $out wattn_qkv_fwd gpurun_out/r3_pmc_wattn_qkv_fwd.json "bench.py --steps 1 --warmup 1 --roofline-steps 1 (eager + graph steps), FETCH_SIZE and WRITE_SIZE passes, round-3 kernel (head pairs, 3-stage BK=32 ring, fp16 bias tiles)"

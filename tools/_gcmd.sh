mkdir -p gpurun_out && export TMPDIR=/tmp
for v in aux defer main aux defer main; do LRCE_DEC_WGRAD_STREAM=$v timeout -k 10 300 python bench.py --no-cpu-baseline --agent-steps 0 --steps 20 > gpurun_out/b7_$v.log 2>&1 || exit 1; echo "wgrad stream $v: $(tail -1 gpurun_out/b7_$v.log | cut -c100-190)"; done

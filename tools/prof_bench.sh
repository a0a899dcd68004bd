#!/bin/bash
# rocprofv3 kernel trace of a short bench run (GPU box).  Usage: tools/prof_bench.sh <outdir> [bench args]
set -e
out=${1:-gpurun_out/prof}
shift || true
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out" -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --roofline-steps 0 --agent-steps 0 "$@" > "$out.log" 2>&1

#!/bin/bash
# Same-box A/B of bench.py (GPU box): alternate runs of the baseline worktree (.ab/r5base) and this
# tree.  Usage: tools/ab_bench.sh <tag> <rounds> [bench args]
tag=$1; rounds=$2; shift 2
for r in $(seq 1 "$rounds"); do
  (cd .ab/r5base && timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --agent-steps 0 --roofline-steps 0 "$@") \
    > gpurun_out/${tag}_base_$r.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --agent-steps 0 --roofline-steps 0 "$@" \
    > gpurun_out/${tag}_new_$r.log 2>&1 || exit $?
done
grep -h -o '"ms_per_step": [0-9.]*' gpurun_out/${tag}_*_*.log /dev/null | head -0
for f in gpurun_out/${tag}_*_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | head -1)"; done

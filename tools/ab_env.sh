#!/bin/bash
# Same-box A/B over environment variants of this tree plus the baseline worktree (.ab/r5base).
# Usage: tools/ab_env.sh <tag> <rounds> "<ENV=..>" ["<ENV=..>" ...]   ("-" = no extra env; "base" = baseline tree)
tag=$1; rounds=$2; shift 2
for r in $(seq 1 "$rounds"); do
  i=0
  for v in "$@"; do
    i=$((i + 1))
    if [ "$v" = "base" ]; then
      (cd .ab/r5base && timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --agent-steps 0 --roofline-steps 0) \
        > gpurun_out/${tag}_v${i}_$r.log 2>&1 || exit $?
    else
      e=""; [ "$v" != "-" ] && e="$v"
      env $e timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --agent-steps 0 --roofline-steps 0 \
        > gpurun_out/${tag}_v${i}_$r.log 2>&1 || exit $?
    fi
  done
done
i=0
for v in "$@"; do
  i=$((i + 1))
  echo "v$i [$v]: $(grep -h -o '"value": [0-9.]*' gpurun_out/${tag}_v${i}_*.log | tr '\n' ' ')"
done

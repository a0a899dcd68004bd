#!/bin/bash
# rocprofv3 kernel trace of a short bench run, summarised ON the GPU box (only text comes back; the
# trace database is deleted).  Usage: tools/prof_step.sh <tag> [bench args]   (run from a tree root)
set -e
tag=$1; shift || true
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d /tmp/$tag -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --roofline-steps 0 --agent-steps 0 "$@" > $out.log 2>&1
db=$(ls /tmp/$tag/*/run_results.db /tmp/$tag/run_results.db 2>/dev/null | head -1)
python $GRAFT_REPO_ROOT/tools/rocprof_summary.py $db --last 4 --top 60 > ${out}_stats.md
(cd $GRAFT_REPO_ROOT/tools && python step_phases.py $db > ${out}_phases.txt && python text_branch.py $db --list > ${out}_text.txt)
python $GRAFT_REPO_ROOT/tools/timeline_gaps.py $db > ${out}_gaps.txt 2>&1 || true
(cd $GRAFT_REPO_ROOT/tools && python step_timeline.py $db > ${out}_timeline.txt 2>&1) || true
rm -rf /tmp/$tag

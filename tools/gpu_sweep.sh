#!/bin/bash
# In-process A/B sweep (tools/sweep.py) with the given arguments, e.g.
#   gpurun -- 'bash tools/gpu_sweep.sh --workload c4 --us 1 --variants base,decearly'
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 500 python3 -u tools/sweep.py "$@" > $O/sweep.jsonl 2> $O/sweep.err || { tail -30 $O/sweep.err; exit 1; }
cat $O/sweep.jsonl

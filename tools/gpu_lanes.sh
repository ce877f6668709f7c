#!/bin/bash
# tile width A/B (lanes per U = 1 tile) on C2, C4, C5 — one process per workload, interleaved variants
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
V="base,base@SEC_FULL_LANES=128,base@SEC_FULL_LANES=192,base@SEC_FULL_LANES=448,base@SEC_FULL_LANES=512"
for w in c2 c4 c5; do
  timeout -k 10 300 python -u tools/sweep.py --variants $V --us 1 --workload $w >> $O/lanes.jsonl 2>$O/lanes.err || { tail -20 $O/lanes.err; exit 1; }
done
cat $O/lanes.jsonl

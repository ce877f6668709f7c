#!/bin/bash
# Per-chunk upload timeline (tools/upload_timeline.py): page-locked (default) vs staged host path
# (SEC_REGISTER_MIN above the chunk), at two hash-pool sizes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
: > $O/upload_ab.jsonl
for RM in "" 67108864; do for W in 15 8; do
  SEC_REGISTER_MIN=$RM STORB_HASH_WORKERS=$W timeout -k 10 200 python3 -u tools/upload_timeline.py --mib 512 >> $O/upload_ab.jsonl 2> $O/upload_ab.err || { tail -20 $O/upload_ab.err; exit 1; }
done; done
cat $O/upload_ab.jsonl

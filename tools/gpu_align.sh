#!/bin/bash
# C4 alignment study: parity stride padded to 16 / 128 B, and an aligned-B shape of the same size
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
for pa in 1 16 128; do
  timeout -k 10 240 python -u tools/sweep.py --variants base --us 1 --workload c4 --palign $pa >> $O/align.jsonl 2>$O/align.err || { tail -20 $O/align.err; exit 1; }
done
timeout -k 10 240 python -u tools/sweep.py --variants base --us 1 --workload 8192,65600,10,14 >> $O/align.jsonl 2>$O/align.err || { tail -20 $O/align.err; exit 1; }
cat $O/align.jsonl

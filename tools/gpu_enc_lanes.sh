#!/bin/bash
# Encode tile width A/B (SEC_ENC_LANES: 256 default vs 64 / 128) on C2, C4 and C5, one process each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
: > $O/enc_lanes.jsonl
for W in ${WORKLOADS:-c2 c4 c5 1024,1048576,8,11 1024,1048576,16,24}; do
  timeout -k 10 300 python3 -u tools/sweep.py --workload $W --us 1 --rounds 7 --variants ${VARIANTS:-base,base@SEC_ENC_LANES=64,base@SEC_ENC_LANES=128} >> $O/enc_lanes.jsonl 2> $O/enc_lanes.err || { tail -20 $O/enc_lanes.err; exit 1; }
done
cat $O/enc_lanes.jsonl

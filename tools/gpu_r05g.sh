#!/bin/bash
# Round 5: the per-call profile (memo reset between loops) and the 1 GiB object's upload /
# download loops with sec_encode_pieces (tools/stream_rate.py --gpu-ids: GPU vs host ids).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
echo "== small calls" && timeout -k 10 300 python3 -u tools/small_call_profile.py --reps 100 > $O/small_calls.json 2> $O/small_calls.err || { tail -20 $O/small_calls.err; exit 1; }
cat $O/small_calls.json
echo "== stream rate" && timeout -k 10 600 python3 -u tools/stream_rate.py --mib 1024 --reps 3 --gpu-ids > $O/stream_rate.json 2> $O/stream_rate.err || { tail -20 $O/stream_rate.err; exit 1; }
cat $O/stream_rate.json

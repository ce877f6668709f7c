#!/bin/bash
# Round 5: native join of reassembled chunks (sec_host_copy): the GPU suite, then the 1 GiB
# object's upload / download loops (tools/stream_rate.py --gpu-ids).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
bash tools/gpu_tests.sh || exit 1
echo "== stream rate" && timeout -k 10 600 python3 -u tools/stream_rate.py --mib 1024 --reps 3 --gpu-ids > $O/stream_rate.json 2> $O/stream_rate.err || { tail -20 $O/stream_rate.err; exit 1; }
cat $O/stream_rate.json

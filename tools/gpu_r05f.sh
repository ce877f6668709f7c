#!/bin/bash
# Round 5: sec_encode_pieces (the per-call floor at storb's granularity) -- the GPU suite, then
# the per-call profile and the C1 loopback with the library path on and off (piece.HOST_PIECES).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
bash tools/gpu_tests.sh || exit 1
echo "== small calls" && timeout -k 10 300 python3 -u tools/small_call_profile.py --reps 100 > $O/small_calls.json 2> $O/small_calls.err || { tail -20 $O/small_calls.err; exit 1; }
cat $O/small_calls.json
echo "== c1" && timeout -k 10 300 python3 -u tools/c1_loopback.py --reps 20 > $O/c1.json 2> $O/c1.err || { tail -20 $O/c1.err; exit 1; }
cat $O/c1.json

#!/bin/bash
# Host path: SEC_F_STAGED test and the piece tests, then the per-chunk upload timeline, the stream
# rates and the C1 loopback with the staged piece copies and the half-CPU hash pool.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
echo "== tests" && timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_piece_gpu.py tests/test_stream_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pt_host.log 2>&1 || { tail -40 $O/pt_host.log; exit 1; }
tail -1 $O/pt_host.log
echo "== upload timeline" && timeout -k 10 200 python3 -u tools/upload_timeline.py --mib 512 > $O/upload_timeline.json 2> $O/upload_timeline.err || { tail -20 $O/upload_timeline.err; exit 1; }
cat $O/upload_timeline.json
echo "== stream rate" && timeout -k 10 300 python3 -u tools/stream_rate.py --mib 1024 > $O/stream_rate.json 2> $O/stream_rate.err || { tail -10 $O/stream_rate.err; exit 1; }
cat $O/stream_rate.json
echo "== c1 loopback" && timeout -k 10 300 python3 -u tools/c1_loopback.py > $O/c1_loopback.json 2> $O/c1_loopback.err || { tail -10 $O/c1_loopback.err; exit 1; }
cat $O/c1_loopback.json

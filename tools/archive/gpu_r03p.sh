#!/bin/bash
# Piece API host path: piece / stream tests, then the per-chunk upload timeline and stream rates.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
echo "== tests" && timeout -k 10 400 python3 -u -m pytest tests/test_piece_gpu.py tests/test_stream_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pt_host.log 2>&1 || { tail -40 $O/pt_host.log; exit 1; }
tail -1 $O/pt_host.log
echo "== upload timeline" && for i in 1; do timeout -k 10 200 python3 -u tools/upload_timeline.py --mib 512 >> $O/upload_timeline2.json 2> $O/upload_timeline.err || { tail -20 $O/upload_timeline.err; exit 1; }; done
cat $O/upload_timeline2.json



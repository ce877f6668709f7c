#!/bin/bash
# Round 6: GPU parity ids (SEC_F_GPU_PARITY_IDS): the piece tests, then the 1 GiB upload stream
# with host ids against GPU parity ids per window (tools/stream_rate.py --parity-ids).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_pieces.py tests/test_gpu_sha1.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_e.log 2>&1 || { tail -40 $O/pytest_e.log; exit 1; }
tail -1 $O/pytest_e.log
timeout -k 10 600 python3 -u tools/stream_rate.py --parity-ids --mib 1024 --reps 2 > $O/r06_parity_ids.json 2> $O/r06_parity_ids.err || { tail -20 $O/r06_parity_ids.err; exit 1; }
cat $O/r06_parity_ids.json

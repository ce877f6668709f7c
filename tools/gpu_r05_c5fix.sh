#!/bin/bash
# Round 5: the C5 line after routing all-pinned joining decodes back to the direct path.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
echo "== tests" && timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pieces.py tests/test_gpu_decode_ex.py tests/test_gpu_bench_c5.py tests/test_piece_gpu.py tests/test_stream_gpu.py > $O/c5fix_tests.log 2>&1 || { tail -30 $O/c5fix_tests.log; exit 1; }
tail -2 $O/c5fix_tests.log
echo "== bench c5" && timeout -k 10 300 python3 -u bench.py --workload c5 > $O/c5fix_bench.log 2>&1 || { tail -30 $O/c5fix_bench.log; exit 1; }
tail -1 $O/c5fix_bench.log
echo "== stream rate" && timeout -k 10 600 python3 -u tools/stream_rate.py --mib 1024 --reps 3 > $O/c5fix_stream.json 2> $O/c5fix_stream.err || { tail -20 $O/c5fix_stream.err; exit 1; }
cat $O/c5fix_stream.json

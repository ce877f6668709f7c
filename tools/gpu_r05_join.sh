#!/bin/bash
# Round 5: host reassembly by buffer kind (pinned / locked -> concurrent direct form; staged ->
# join_staged): GPU tests of the host paths, the bench's e2e and C5 lines, the 1 GiB stream.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
echo "== tests" && timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pieces.py tests/test_gpu_decode_ex.py tests/test_gpu_parity.py tests/test_gpu_bench_c5.py tests/test_piece_gpu.py tests/test_stream_gpu.py > $O/join_tests.log 2>&1 || { tail -30 $O/join_tests.log; exit 1; }
tail -2 $O/join_tests.log
echo "== bench" && timeout -k 10 300 python3 -u bench.py --no-c4 > $O/join_bench.log 2>&1 || { tail -30 $O/join_bench.log; exit 1; }
tail -1 $O/join_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('e2e'), d.get('c5',{}).get('value'), d.get('c5',{}).get('staged'))"
echo "== stream rate" && timeout -k 10 600 python3 -u tools/stream_rate.py --mib 1024 --reps 3 > $O/join_stream.json 2> $O/join_stream.err || { tail -20 $O/join_stream.err; exit 1; }
cat $O/join_stream.json

#!/bin/bash
# XOR3 accumulation (current sources, "base") against the previous build ("prev"): parity tests, then shapes
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out; mkdir -p $O
echo "== parity tests" && timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_piece_gpu.py > $O/xor3_tests.log 2>&1 || { tail -30 $O/xor3_tests.log; exit 1; }
tail -1 $O/xor3_tests.log
: > $O/xor3_sweep.jsonl
for w in ${WL:-c2 c4 c5 512,2097152,16,24 256,4194304,32,48}; do
  echo "== $w" && timeout -k 10 300 python -u tools/sweep.py --workload $w --variants base,prev --us 1 --rounds 5 >> $O/xor3_sweep.jsonl 2>&1 || { tail -20 $O/xor3_sweep.jsonl; exit 1; }
done
grep '^{' $O/xor3_sweep.jsonl

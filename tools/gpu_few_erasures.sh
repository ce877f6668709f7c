#!/bin/bash
# Wide policy shapes at their chunk sizes, decoding with 1, 2 and 4 data blocks lost (the
# usual download) and recover-only; one process per (shape, erasure set).
set -o pipefail
O=gpurun_out; mkdir -p $O; : > $O/few_erasures.jsonl
for W in 64,16777216,32,48 256,4194304,16,24 16,16777216,64,96; do
  for E in 0 0,5 0,5,9,13; do
    timeout -k 10 300 python3 -u tools/sweep.py --workload $W --erased $E --recover --us 1 --rounds 5 --variants base >> $O/few_erasures.jsonl 2> $O/few.err || { tail -20 $O/few.err; exit 1; }
  done
done
cat $O/few_erasures.jsonl

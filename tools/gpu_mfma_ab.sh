#!/bin/bash
# MFMA (bit-sliced) against v_perm encode on the wide policy shapes, in-process A/B per shape.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
: > $O/mfma_ab.jsonl
for W in 32,33554432,32,48 1024,1048576,32,48 4,268435456,64,96 32,33554432,32,40; do
  timeout -k 10 300 python3 -u tools/sweep.py --workload $W --us 1 --rounds 5 --variants ${VARIANTS:-base@SEC_MFMA=0,base@SEC_MFMA=1} >> $O/mfma_ab.jsonl 2> $O/mfma_ab.err || { tail -20 $O/mfma_ab.err; exit 1; }
done
cat $O/mfma_ab.jsonl

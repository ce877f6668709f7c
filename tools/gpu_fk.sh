#!/bin/bash
# A/B: compile-time k (SEC_FIXED_K) against the runtime-k kernels on C2, C4, C5
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out; mkdir -p $O
echo "== c2" && timeout -k 10 300 python -u tools/sweep.py --variants base,fk4 --us 1 --rounds 5 > $O/fk_c2.jsonl 2>&1 || { tail -20 $O/fk_c2.jsonl; exit 1; }
cat $O/fk_c2.jsonl
echo "== c4" && timeout -k 10 300 python -u tools/sweep.py --workload c4 --variants base,fk10 --us 1 --rounds 5 > $O/fk_c4.jsonl 2>&1 || { tail -20 $O/fk_c4.jsonl; exit 1; }
cat $O/fk_c4.jsonl
echo "== c5" && timeout -k 10 300 python -u tools/sweep.py --workload c5 --variants base,fk8 --us 1 --rounds 5 > $O/fk_c5.jsonl 2>&1 || { tail -20 $O/fk_c5.jsonl; exit 1; }
cat $O/fk_c5.jsonl

#!/bin/bash
# Round-3 encode LDS-ring A/B ((64,96): the ring for both groups, the same capped at 256
# registers, none; (32,48): ring / none), then the round batch (tools/gpu_round.sh).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
echo "== enc A/B (64,96)" && timeout -k 10 300 python3 -u tools/sweep.py --variants base,encl2,bsw2,noencl --us 1 --rounds 5 --workload 256,1048576,64,96 > $O/enc_lds_6496.jsonl 2>&1 || { tail -20 $O/enc_lds_6496.jsonl; exit 1; }
cat $O/enc_lds_6496.jsonl
echo "== enc A/B (32,48)" && timeout -k 10 300 python3 -u tools/sweep.py --variants base,noencl --us 1 --rounds 7 --workload 512,524288,32,48 > $O/enc_lds_3248.jsonl 2>&1 || { tail -20 $O/enc_lds_3248.jsonl; exit 1; }
cat $O/enc_lds_3248.jsonl
bash tools/gpu_round.sh

#!/bin/bash
# Round 5: C5-shaped access-pattern ceiling (tools/rw_ceiling.hip), the in-process bench form
# (one device; two contexts on the one GPU), and the N = 2 rehearsal with the nested in-process
# measurement (both ranks and both in-process workers on cuda:0, gloo).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
echo "== rw_ceiling" && timeout -k 10 120 tools/rw_ceiling > $O/rw_ceiling.json 2>&1 || { tail -20 $O/rw_ceiling.json; exit 1; }
cat $O/rw_ceiling.json
echo "== in-process x1" && timeout -k 10 240 python3 -u bench.py --gpus 1 --in-process --steps 20 --warmup 3 --c5-steps 5 > $O/inproc1.log 2>&1 || { tail -30 $O/inproc1.log; exit 1; }
grep '^{' $O/inproc1.log
echo "== in-process 0,0" && timeout -k 10 240 python3 -u bench.py --gpus 2 --in-process --inproc-devices 0,0 --steps 20 --warmup 3 --c5-steps 5 > $O/inproc00.log 2>&1 || { tail -30 $O/inproc00.log; exit 1; }
grep '^{' $O/inproc00.log
echo "== rehearse n2 + nested in-process" && STORB_BENCH_DEVICE=0 STORB_DIST_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu --no-e2e --c4-chunks 16384 --c5-bytes 268435456 --inproc-devices 0,0 > $O/rehearse_n2_inproc.log 2>&1 || { tail -30 $O/rehearse_n2_inproc.log; exit 1; }
grep '^{' $O/rehearse_n2_inproc.log

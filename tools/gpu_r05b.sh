#!/bin/bash
# Round 5: in-process multi-device tests (two contexts on the one GPU) and the headline-step
# store-policy A/B (tools/step_ab.py, wall clock per step as bench.py times it).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
echo "== group tests" && timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_group.py > $O/group_tests.log 2>&1 || { tail -40 $O/group_tests.log; exit 1; }
tail -12 $O/group_tests.log
echo "== step A/B" && timeout -k 10 400 python3 -u tools/step_ab.py --variants ${VARS:-base,est2,est3,est0,est2dst2,dst2,dst3} --rounds 7 --steps 20 > $O/step_ab.jsonl 2> $O/step_ab.err || { tail -20 $O/step_ab.err; exit 1; }
cat $O/step_ab.jsonl

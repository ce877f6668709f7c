#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
echo "== pytest gpu" && timeout -k 10 600 python -m pytest tests -x -q -m gpu > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
echo "== ceiling" && timeout -k 10 120 ./tools/stream_ceiling > $O/ceiling.json 2>&1 || { cat $O/ceiling.json; exit 1; }
cat $O/ceiling.json
echo "== sweep c2" && timeout -k 10 400 python tools/sweep.py > $O/sweep_c2.jsonl 2>&1 || { tail -20 $O/sweep_c2.jsonl; exit 1; }
cat $O/sweep_c2.jsonl
echo "== sweep c4" && timeout -k 10 400 python tools/sweep.py --workload c4 --us 1,2 > $O/sweep_c4.jsonl 2>&1 || { tail -20 $O/sweep_c4.jsonl; exit 1; }
cat $O/sweep_c4.jsonl

#!/bin/bash
# GPU parity tests, then interleaved A/B sweeps given as SWEEP1 / SWEEP2 / SWEEP3 (tools/sweep.py args)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
echo "== pytest gpu" && timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for i in 1 2 3; do
  v=SWEEP$i; [ -z "${!v}" ] && continue
  echo "== sweep $i: ${!v}" && timeout -k 10 400 python -u tools/sweep.py ${!v} > $O/ab$i.jsonl 2>&1 || { tail -20 $O/ab$i.jsonl; exit 1; }
  grep variant $O/ab$i.jsonl
done

#!/bin/bash
# tests -> smoke -> bench (-> optional sweep) ; stops at the first failure
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
echo "== pytest gpu" && timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log; grep -h "took the" $O/pytest_gpu.log || true
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
echo "== bench" && timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log
if [ -n "$SWEEP" ]; then
  echo "== sweep" && timeout -k 10 400 python -u tools/sweep.py $SWEEP > $O/sweep.jsonl 2>&1 || { tail -20 $O/sweep.jsonl; exit 1; }
  cat $O/sweep.jsonl
fi

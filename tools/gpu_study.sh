#!/bin/bash
# GPU parity tests -> HBM store/load study -> PCIe e2e study -> bench.  Stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
if [ -z "$SKIP_TESTS" ]; then
  echo "== pytest gpu" && timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
fi
echo "== hbm study" && timeout -k 10 180 ./tools/hbm_study > $O/hbm_study.jsonl 2>&1 || { cat $O/hbm_study.jsonl; exit 1; }
cat $O/hbm_study.jsonl
echo "== e2e study" && timeout -k 10 300 python -u tools/e2e_study.py > $O/e2e_study.json 2>&1 || { tail -20 $O/e2e_study.json; exit 1; }
tail -1 $O/e2e_study.json
echo "== bench" && timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log

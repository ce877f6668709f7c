#!/bin/bash
# One GPU session: smoke -> gpu tests -> bench -> rocprofv3 kernel stats.  Stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -30 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
echo "== pytest gpu" && timeout -k 10 600 python -m pytest tests -x -q -m gpu > $O/pytest_gpu.log 2>&1 || { echo gpu tests failed; tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
echo "== bench" && timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > $O/bench.log 2>&1 || { echo bench failed; tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log
if [ -n "$PROFILE" ]; then
  echo "== rocprofv3"
  export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu --no-e2e > $O/prof.log 2>&1 || { echo prof failed; tail -30 $O/prof.log; exit 1; }
  find $O/prof -name "*stats*" | head
fi
echo done

#!/bin/bash
# GPU test run: the given pytest targets (default: the whole -m gpu suite), one process,
# per-test timeout, output under gpurun_out/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
T=${*:-tests}
timeout -k 10 900 python3 -u -m pytest $T -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
tail -40 $O/pytest_gpu.log
exit $rc

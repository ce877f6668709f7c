#!/bin/bash
# kernel-attached timing events: GPU tests, bench with / without events, rocprof kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out; mkdir -p $O
echo "== pytest gpu" && timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for i in 1 2; do
  timeout -k 10 120 python bench.py --no-cpu --no-e2e --steps 200 > $O/ev_on.log 2>&1 && timeout -k 10 120 python bench.py --no-cpu --no-e2e --steps 200 --no-events > $O/ev_off.log 2>&1 || { tail -20 $O/ev_on.log $O/ev_off.log; exit 1; }
  python -c "
import json
for f in ('$O/ev_on.log','$O/ev_off.log'):
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['decode_kernel']['avg_launch_ms'])"
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu --no-e2e > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
tail -1 $O/prof.log | cut -c1-200
grep sec_ $O/prof/run_kernel_stats.csv | cut -d, -f1,2,4 | cut -c1-40,150-

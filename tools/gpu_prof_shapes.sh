#!/bin/bash
# rocprofv3 kernel stats per shape (full vs edge kernels), one process per shape
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
for w in ${SHAPES:-c4 8192,65600,10,14}; do
  tag=$(echo $w | tr ',' '_')
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ps_$tag -o run -- python3 $R/tools/sweep.py --variants base --us 1 --rounds 2 --reps 5 --workload $w > $O/ps_$tag.log 2>&1 || { tail -20 $O/ps_$tag.log; exit 1; }
  echo "== $w"; grep variant $O/ps_$tag.log
  python3 - $O/ps_$tag/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "sec_" in r["Name"]:
        print(f'{r["Name"][:90]:90s} calls={r["Calls"]:>4} avg_us={float(r["AverageNs"])/1e3:8.2f}')
PY
done

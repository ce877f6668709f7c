#!/bin/bash
# rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE passes of one shape (default C4)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R; export TMPDIR=/tmp
W=${W:-c4}
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$W -o run -- python3 tools/prof_shape.py --workload $W > $O/prof_$W.log 2>&1 || { tail -20 $O/prof_$W.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmcf_$W -o run -- python3 tools/prof_shape.py --workload $W --reps 5 > $O/pmcf_$W.log 2>&1 || { tail -20 $O/pmcf_$W.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmcw_$W -o run -- python3 tools/prof_shape.py --workload $W --reps 5 > $O/pmcw_$W.log 2>&1 || { tail -20 $O/pmcw_$W.log; exit 1; }
find $O/prof_$W -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-60,200- | head -20
for f in $(find $O/pmcf_$W $O/pmcw_$W -name "*counter_collection.csv"); do
  python3 - "$f" <<'PY'
import csv, sys, collections
v = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    v[(r["Kernel_Name"][:40], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), xs in v.items():
    print(c, k, "per-dispatch KiB avg", round(sum(xs) / max(1, len(set(range(len(xs))))), 1), "n", len(xs))
PY
done

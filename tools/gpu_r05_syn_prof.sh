#!/bin/bash
# Round 5: per-kernel times of the two-kernel wide decode (zfec(64,96), 32 / 24 lost), reassembly.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
for C in "32 lost" "24 lost (random"; do
  T=$(echo "$C" | cut -c1-2)
  echo "== $C" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/synprof_$T -o run -- python3 tools/syn_ab.py --rounds 1 --reps 5 --variants auto --modes reassemble --cases "$C" > $O/synprof_$T.log 2>&1 || { tail -20 $O/synprof_$T.log; exit 1; }
  python3 -c "
import csv,sys
for r in csv.DictReader(open('$O/synprof_$T/run_kernel_stats.csv')):
    if 'sec_' in r['Name']: print(r['Name'][:90], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
"
done

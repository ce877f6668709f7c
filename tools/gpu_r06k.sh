#!/bin/bash
# Round 6: the wide decode's two phases with no field arithmetic (build/variants/libstorbec_nogf.so,
# SEC_PROBE_NOGF: every load, copy and store kept) against the product, per phase (kernel trace),
# 32 and 24 lost: the access patterns' own time.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
for C in "32 lost" "24 lost (random"; do
  for V in "auto" "nogf/nogf"; do
    T=$O/p6_cal_${V%%/*}_${C%% *}
    rm -rf $T
    timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $T -o run -- python3 tools/syn_ab.py --cases "$C" --variants "$V" --no-check nogf --rounds 1 --reps 4 --modes reassemble > $T.log 2>&1 || { tail -20 $T.log; exit 1; }
    python3 -c "
import csv
for r in csv.DictReader(open('$T/run_kernel_stats.csv')):
    if 'syndrome' in r['Name'] or 'solve' in r['Name']: print('$C', '$V', r['Name'][:60], r['Calls'], r['AverageNs'])"
  done
done

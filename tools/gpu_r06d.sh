#!/bin/bash
# Round 6 iteration: the wide-decode GPU tests, the syn A/B (this build against VARS) and the
# per-phase kernel times of this build (trace) on 32 / 24 lost.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
VARS=${VARS:-"auto,r05/r05"}
TAG=${TAG:-d}
timeout -k 10 300 python -u -m pytest tests/test_gpu_syndrome.py tests/test_gpu_bs.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_$TAG.log 2>&1 || { tail -40 $O/pytest_$TAG.log; exit 1; }
tail -1 $O/pytest_$TAG.log
timeout -k 10 500 python3 -u tools/syn_ab.py --rounds 3 --variants "$VARS" --cases "32 lost;24 lost (random;16 lost (random;30 %" > $O/r06_syn_ab_$TAG.jsonl 2> $O/r06_syn_ab_$TAG.err || { tail -20 $O/r06_syn_ab_$TAG.err; exit 1; }
python3 -c "
import json,sys
for l in open('$O/r06_syn_ab_$TAG.jsonl'):
    d=json.loads(l); print(d['case'][:60], {k:(v['reassemble'],v['recover_only']) for k,v in d.items() if isinstance(v,dict)})"
for C in "32 lost" "24 lost (random"; do
  T=$O/p6_${TAG}_${C%% *}
  rm -rf $T
  timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $T -o run -- python3 tools/syn_ab.py --cases "$C" --variants "auto" --rounds 1 --reps 4 --modes reassemble > $T.log 2>&1 || { tail -20 $T.log; exit 1; }
  python3 -c "
import csv
for r in csv.DictReader(open('$T/run_kernel_stats.csv')):
    if 'sec_' in r['Name']: print('  $C', r['Name'][:70], r['Calls'], r['AverageNs'])"
done

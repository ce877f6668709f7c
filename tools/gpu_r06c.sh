#!/bin/bash
# Round 6: counters of both wide-decode phases at 32 and 24 lost (this build), the round-5 kernels'
# per-phase times on the same cases (trace only), and the wide encodes (pair / interleaved).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
TAG=syn32 CASES="32 lost" bash tools/gpu_r06_pmc.sh > $O/r06c_1.log 2>&1 || { tail -20 $O/r06c_1.log; exit 1; }
TAG=syn24 CASES="24 lost (random" bash tools/gpu_r06_pmc.sh > $O/r06c_2.log 2>&1 || { tail -20 $O/r06c_2.log; exit 1; }
for C in "32 lost" "24 lost (random"; do
  T=$O/p6_r05_${C%% *}
  rm -rf $T
  timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $T -o run -- python3 tools/syn_ab.py --cases "$C" --variants "r05/r05" --rounds 1 --reps 4 --modes reassemble > $T.log 2>&1 || { tail -20 $T.log; exit 1; }
  T=$O/p6_cur_${C%% *}
  rm -rf $T
  timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $T -o run -- python3 tools/syn_ab.py --cases "$C" --variants "auto" --rounds 1 --reps 4 --modes reassemble > $T.log 2>&1 || { tail -20 $T.log; exit 1; }
done
TAG=enc TOOL=enc CASES="1MiB x1024" VARS="pair,bs2@SEC_BS_PAIR=0" bash tools/gpu_r06_pmc.sh > $O/r06c_3.log 2>&1 || { tail -20 $O/r06c_3.log; exit 1; }
ls $O

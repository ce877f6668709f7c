#!/bin/bash
# PMC traffic of a bench line's kernels: FETCH_SIZE and WRITE_SIZE in separate passes (TCC slots),
# --kernel-trace only beside --pmc (no sys/runtime trace), then summarised into JSON.
#   bash tools/gpu_pmc.sh [c2|c4|c5]   -> gpurun_out/pmc_<wl>.json (copy to profiles/pmc_<wl>.json)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
WL=${1:-c2}
case $WL in
  c4) ARGS="--workload c4 --steps 10 --warmup 2 --no-cpu";;
  c5) ARGS="--workload c5 --c5-device-only --steps 5 --warmup 1 --no-cpu --no-e2e";;
  *) ARGS="--steps 10 --warmup 2 --no-cpu --no-e2e --no-recover --no-c4 --no-c5";;
esac
rm -rf $O/pmc_fetch $O/pmc_write $O/prof_$WL
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py $ARGS > $O/pmc_fetch.log 2>&1 || { tail -20 $O/pmc_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py $ARGS > $O/pmc_write.log 2>&1 || { tail -20 $O/pmc_write.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$WL -o run -- python3 $R/bench.py $ARGS > $O/prof_$WL.log 2>&1 || { tail -20 $O/prof_$WL.log; exit 1; }
python3 tools/pmc_summary.py $O $WL > $O/pmc_$WL.json && cat $O/pmc_$WL.json

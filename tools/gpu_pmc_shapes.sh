#!/bin/bash
# PMC passes over tools/prof_shape.py for one or more workloads (default: c4 c2):
#   FETCH_SIZE, WRITE_SIZE (separate TCC passes), an SQ issue/wait pass with GRBM_GUI_ACTIVE,
#   and a --kernel-trace --stats pass.  Each pass is its own rocprofv3 run under its own
#   timeout; the first failure ends the script.  Summarised by tools/pmc_shapes.py.
#   PMC_TAG: suffix of the output directory (for runs under different SEC_* settings).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/pmc_shapes${PMC_TAG:-}; mkdir -p $O; cd $R
export TMPDIR=/tmp
WL=${*:-c4 c2}
SQ="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
for w in $WL; do
  for pass in fetch write sq stats; do
    case $pass in
      fetch) P="--pmc FETCH_SIZE --kernel-trace";;
      write) P="--pmc WRITE_SIZE --kernel-trace";;
      sq)    P="--pmc $SQ --kernel-trace";;
      stats) P="--kernel-trace --stats";;
    esac
    echo "== $w $pass"
    timeout -k 10 180 rocprofv3 $P --output-format csv -d $O/$w/$pass -o run -- python3 $R/tools/prof_shape.py --workload $w --reps 10 > $O/$w.$pass.log 2>&1 || { tail -20 $O/$w.$pass.log; exit 1; }
  done
done
python3 tools/pmc_shapes.py $O $WL > $O/summary.json && cat $O/summary.json

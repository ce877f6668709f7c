#!/bin/bash
# PMC of the syndrome decode (the fused kernel on zfec(64,96) 1 MiB x 1024, 16 lost, parity rows
# of one group) and of the direct decode on the same chunks: FETCH_SIZE, WRITE_SIZE and the SQ
# wave-state counters in separate passes, summarised by tools/pmc_syn_summary.py.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
CASE="zfec(64,96) 1MiB x1024, 16 lost"
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES"
for VAR in "fused@SEC_SYN=1" "direct@SEC_SYN=0"; do
  N=${VAR%%@*}
  for P in FETCH_SIZE WRITE_SIZE SQ; do
    if [ $P = SQ ]; then C=$SQ; D=$O/pmc_sq_$N; else C=$P; D=$O/pmc_syn_${N}_$P; fi
    rm -rf $D
    timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $D -o run -- python3 tools/syn_ab.py --cases "$CASE" --variants "$VAR" --rounds 1 --reps 2 > $D.log 2>&1 || { tail -20 $D.log; exit 1; }
  done
done
python3 tools/pmc_syn_summary.py $O > $O/pmc_syn.json && cat $O/pmc_syn.json

#!/bin/bash
# Wide decodes: the A/B of tools/syn_ab.py over its cases (direct / two kernels / fused / default),
# then rocprofv3 kernel stats of the default choice on the e > 16 and random-parity cases (time per
# kernel: syndromes vs solve), then SQ wave-state counters of the two-kernel path on 32 lost.
#   CASES="...;..." bash tools/gpu_syn_prof.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
VARS=${VARS:-direct@SEC_SYN=0,two@SEC_SYN=1+SEC_SYN_FUSED=0,auto}
echo "== syn_ab" && timeout -k 10 600 python3 -u tools/syn_ab.py --rounds ${ROUNDS:-3} --variants "$VARS" ${CASES:+--cases "$CASES"} > $O/syn_ab.jsonl 2> $O/syn_ab.err || { tail -20 $O/syn_ab.err; exit 1; }
cat $O/syn_ab.jsonl
[ -n "$SKIP_PROF" ] && exit 0
PC="zfec(64,96) 1MiB x1024, 32 lost;zfec(64,96) 1MiB x1024, 24 lost;zfec(64,96) 1MiB x1024, 16 lost (random, parity random)"
rm -rf $O/prof_syn
echo "== stats" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_syn -o run -- python3 tools/syn_ab.py --cases "$PC" --variants auto --rounds 1 --reps 3 > $O/prof_syn.log 2>&1 || { tail -20 $O/prof_syn.log; exit 1; }
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES"
rm -rf $O/pmc_sq_two
echo "== sq" && timeout -s KILL 120 rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d $O/pmc_sq_two -o run -- python3 tools/syn_ab.py --cases "zfec(64,96) 1MiB x1024, 32 lost" --variants auto --rounds 1 --reps 2 > $O/pmc_sq_two.log 2>&1 || { tail -20 $O/pmc_sq_two.log; exit 1; }
echo done

#!/bin/bash
# Round 6: counters of the zfec(64,96) kernels furthest below roofline:
# the two-kernel wide reassembly at 32 / 24 lost (sec_syndrome_bs_pair_kernel, sec_solve_bs_lds_kernel)
# and the wide encode that makes its parity (sec_encode_bs2_kernel).  FETCH_SIZE, WRITE_SIZE, two SQ
# passes (wave states; instruction mix + instruction cache) and a trace, each its own run, summarised
# by tools/syn_pmc.py -> gpurun_out/r06_pmc.json.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
CASES=${CASES:-"32 lost;24 lost (random"}
VARS=${VARS:-auto}
A=(tools/syn_ab.py --cases "$CASES" --variants "$VARS" --rounds 1 --reps 2 --modes reassemble)
SQA="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
SQB="SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQC_ICACHE_REQ SQC_ICACHE_MISSES SQ_IFETCH"
rm -rf $O/p6_f $O/p6_w $O/p6_a $O/p6_b $O/p6_t
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/p6_f -o run -- python3 "${A[@]}" > $O/p6_f.log 2>&1 || { tail -20 $O/p6_f.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/p6_w -o run -- python3 "${A[@]}" > $O/p6_w.log 2>&1 || { tail -20 $O/p6_w.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc $SQA --kernel-trace --output-format csv -d $O/p6_a -o run -- python3 "${A[@]}" > $O/p6_a.log 2>&1 || { tail -20 $O/p6_a.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc $SQB --kernel-trace --output-format csv -d $O/p6_b -o run -- python3 "${A[@]}" > $O/p6_b.log 2>&1 || { tail -20 $O/p6_b.log; exit 1; }
timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d $O/p6_t -o run -- python3 "${A[@]}" > $O/p6_t.log 2>&1 || { tail -20 $O/p6_t.log; exit 1; }
python3 tools/syn_pmc.py $O/p6_f $O/p6_w $O/p6_a $O/p6_t $O/p6_b > $O/r06_pmc.json && cat $O/r06_pmc.json

#!/bin/bash
# Round 6: counters of the zfec(64,96) kernels furthest below roofline:
# FETCH_SIZE, WRITE_SIZE, two SQ passes (wave states; instruction mix + instruction cache) and a
# trace, each its own rocprofv3 run, summarised per kernel by tools/syn_pmc.py into
# gpurun_out/r06_pmc_<TAG>.json.  TOOL = syn (tools/syn_ab.py reassembly, CASES / VARS) or enc
# (tools/enc_ab.py, CASES / VARS).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
TAG=${TAG:-syn}
TOOL=${TOOL:-syn}
CASES=${CASES:-"32 lost;24 lost (random"}
VARS=${VARS:-auto}
if [ "$TOOL" = enc ]; then
  A=(tools/enc_ab.py --cases "$CASES" --variants "$VARS" --rounds 1 --reps 2)
else
  A=(tools/syn_ab.py --cases "$CASES" --variants "$VARS" --rounds 1 --reps 2 --modes reassemble)
fi
SQA="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
SQB="SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQC_ICACHE_REQ SQC_ICACHE_MISSES SQ_IFETCH"
P=$O/p6_$TAG
rm -rf ${P}_f ${P}_w ${P}_a ${P}_b ${P}_t
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d ${P}_f -o run -- python3 "${A[@]}" > ${P}_f.log 2>&1 || { tail -20 ${P}_f.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d ${P}_w -o run -- python3 "${A[@]}" > ${P}_w.log 2>&1 || { tail -20 ${P}_w.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc $SQA --kernel-trace --output-format csv -d ${P}_a -o run -- python3 "${A[@]}" > ${P}_a.log 2>&1 || { tail -20 ${P}_a.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc $SQB --kernel-trace --output-format csv -d ${P}_b -o run -- python3 "${A[@]}" > ${P}_b.log 2>&1 || { tail -20 ${P}_b.log; exit 1; }
timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d ${P}_t -o run -- python3 "${A[@]}" > ${P}_t.log 2>&1 || { tail -20 ${P}_t.log; exit 1; }
python3 tools/syn_pmc.py ${P}_f ${P}_w ${P}_a ${P}_t ${P}_b > $O/r06_pmc_$TAG.json && cat $O/r06_pmc_$TAG.json

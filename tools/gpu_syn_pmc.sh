#!/bin/bash
# Wide-decode counters: HBM bytes and SQ wave states per decode kernel on
# zfec(64,96) reassembly -- 16 lost in one parity group (the one-wave kernel), 16 random (the wave
# pair), 32 lost (two kernels) -- FETCH_SIZE, WRITE_SIZE and SQ in separate passes, summarised by
# tools/syn_pmc.py -> gpurun_out/syn_pmc.json.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
CASES=${CASES:-"zfec(64,96) 1MiB x1024, 16 lost;zfec(64,96) 1MiB x1024, 32 lost"}
VARS=${VARS:-auto}
A=(tools/syn_ab.py --cases "$CASES" --variants "$VARS" --rounds 1 --reps 2 --modes reassemble)
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU"
rm -rf $O/spmc_f $O/spmc_w $O/spmc_s $O/spmc_t
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/spmc_f -o run -- python3 "${A[@]}" > $O/spmc_f.log 2>&1 || { tail -20 $O/spmc_f.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/spmc_w -o run -- python3 "${A[@]}" > $O/spmc_w.log 2>&1 || { tail -20 $O/spmc_w.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d $O/spmc_s -o run -- python3 "${A[@]}" > $O/spmc_s.log 2>&1 || { tail -20 $O/spmc_s.log; exit 1; }
timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d $O/spmc_t -o run -- python3 "${A[@]}" > $O/spmc_t.log 2>&1 || { tail -20 $O/spmc_t.log; exit 1; }
python3 tools/syn_pmc.py $O/spmc_f $O/spmc_w $O/spmc_s $O/spmc_t > $O/syn_pmc.json && cat $O/syn_pmc.json

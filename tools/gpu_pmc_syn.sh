#!/bin/bash
# PMC traffic of the syndrome decode (fused kernel, zfec(64,96) 1 MiB x 1024, 16 lost, parity rows of
# one group) and of the direct decode on the same chunks, FETCH_SIZE and WRITE_SIZE in separate
# passes; then the upload timeline.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
CASE="zfec(64,96) 1MiB x1024, 16 lost"
for V in "fused@SEC_SYN=1:sec_decode_bs_kernel" "direct@SEC_SYN=0:sec_decode_kernel"; do
  VAR=${V%%:*}; K=${V##*:}; N=${VAR%%@*}
  for C in FETCH_SIZE WRITE_SIZE; do
    rm -rf $O/pmc_syn_${N}_$C
    timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/pmc_syn_${N}_$C -o run -- python3 tools/syn_ab.py --cases "$CASE" --variants "$VAR" --rounds 1 --reps 2 > $O/pmc_syn_${N}_$C.log 2>&1 || { tail -20 $O/pmc_syn_${N}_$C.log; exit 1; }
  done
  python3 tools/pmc_syn_summary.py $O/pmc_syn_${N}_FETCH_SIZE $O/pmc_syn_${N}_WRITE_SIZE $K 64 16384 1024 16 1048576 > $O/pmc_syn_$N.json && cat $O/pmc_syn_$N.json
done
echo "== upload timeline" && timeout -k 10 200 python3 -u tools/upload_timeline.py --mib 512 > $O/upload_timeline.json 2> $O/upload_timeline.err || { tail -20 $O/upload_timeline.err; exit 1; }
cat $O/upload_timeline.json

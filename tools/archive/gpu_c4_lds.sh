#!/bin/bash
# Round 4 A/Bs: C4's LDS-staged encode (SEC_BS_LDS) and reassembly (SEC_DEC_LDS), zfec(64,96)'s shared-transpose wave pairs
# (SEC_BS_PAIR), each against the previous plan in one process (tools/sweep.py), after the
# bit-sliced parity tests; then the C4 bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
echo "== tests" && timeout -k 10 600 python3 -u -m pytest tests/test_gpu_bs.py tests/test_gpu_bench_c4.py tests/test_gpu_parity.py tests/test_gpu_decode_ex.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pt_lds.log 2>&1 || { tail -30 $O/pt_lds.log; exit 1; }
tail -1 $O/pt_lds.log
echo "== sweep c4" && timeout -k 10 300 python3 -u tools/sweep.py --workload c4 --us 1 --rounds 7 --palign 128 --variants base,base@SEC_BS_LDS=0+SEC_DEC_LDS=0,base@SEC_BS_LDS=0,base@SEC_DEC_LDS=0 > $O/c4_lds_ab.jsonl 2> $O/c4_lds_ab.err || { tail -20 $O/c4_lds_ab.err; exit 1; }
cat $O/c4_lds_ab.jsonl
for W in 512,1048576,64,96 4,268435456,64,96; do
  echo "== sweep $W" && timeout -k 10 300 python3 -u tools/sweep.py --workload $W --us 1 --rounds 5 --variants base,base@SEC_BS_PAIR=0 >> $O/pair_ab.jsonl 2> $O/pair_ab.err || { tail -20 $O/pair_ab.err; exit 1; }
done
cat $O/pair_ab.jsonl
echo "== bench c4" && timeout -k 10 300 python3 -u bench.py --workload c4 --no-cpu > $O/bench_c4.log 2>&1 || { tail -20 $O/bench_c4.log; exit 1; }
tail -1 $O/bench_c4.log

#!/bin/bash
# Round 4: phase 2 with each span's syndromes staged in LDS (SEC_SOLVE_LDS) -- its parity tests,
# then the A/B against the (span, row group) tiles on the two-kernel cases.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
echo "== tests" && timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_syndrome.py tests/test_gpu_choose.py > $O/pt_solve.log 2>&1 || { tail -30 $O/pt_solve.log; exit 1; }
tail -2 $O/pt_solve.log
echo "== syn A/B" && timeout -k 10 600 python3 -u tools/syn_ab.py --rounds 3 --variants "auto,tiles@SEC_SOLVE_LDS=0,direct@SEC_SYN=0" --cases "32 lost;24 lost (random;30 %;16 lost (random;32,48) 1MiB x1024, 16 lost (every" > $O/syn_ab_solve.jsonl 2> $O/syn_ab_solve.err || { tail -20 $O/syn_ab_solve.err; exit 1; }
cat $O/syn_ab_solve.jsonl

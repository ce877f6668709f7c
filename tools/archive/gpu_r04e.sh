#!/bin/bash
# Round 4: phase 1 of both-group chunks in two-wave workgroups (SEC_SYN_WG2) -- parity tests, then
# the A/B against the per-group tiles.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
echo "== tests" && timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_syndrome.py tests/test_gpu_choose.py > $O/pt_wg2.log 2>&1 || { tail -30 $O/pt_wg2.log; exit 1; }
tail -2 $O/pt_wg2.log
echo "== syn A/B" && timeout -k 10 600 python3 -u tools/syn_ab.py --rounds 3 --variants "auto,nowg2@SEC_SYN_WG2=0,two@SEC_SYN=1+SEC_SYN_FUSED=0,two_nowg2@SEC_SYN=1+SEC_SYN_FUSED=0+SEC_SYN_WG2=0" --cases "32 lost;24 lost (random;30 %;16 lost (random" > $O/syn_ab_wg2.jsonl 2> $O/syn_ab_wg2.err || { tail -20 $O/syn_ab_wg2.err; exit 1; }
cat $O/syn_ab_wg2.jsonl

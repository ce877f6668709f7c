#!/bin/bash
# Round 4 evidence: tools/gpu_round.sh (GPU tests, smoke, PMC c2/c4/c5 on this build, bench lines,
# kernel stats, --gpus 2 rehearsal, every BASELINE config), then the wide-decode A/B of the final
# defaults (tools/syn_ab.py).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
bash tools/gpu_round.sh || exit 1
echo "== syn A/B" && timeout -k 10 600 python3 -u tools/syn_ab.py --rounds 3 --variants "auto,nowg2@SEC_SYN_WG2=0,tiles@SEC_SOLVE_LDS=0,two@SEC_SYN=1+SEC_SYN_FUSED=0,direct@SEC_SYN=0" --cases "32 lost;24 lost (random;30 %;16 lost (random;20 %;rows 64..73" > $O/syn_ab_final.jsonl 2> $O/syn_ab_final.err || { tail -20 $O/syn_ab_final.err; exit 1; }
cat $O/syn_ab_final.jsonl

#!/bin/bash
# Round-3 final evidence: the round batch with every BASELINE config (gpu tests, smoke, bench,
# rocprof, c4, c5, --gpus 2 rehearsal, tools/bench_configs.py), the syndrome A/B, its PMC.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
bash tools/gpu_round.sh || exit 1
echo "== syn A/B" && timeout -k 10 700 python3 -u tools/syn_ab.py --rounds 2 --variants "direct@SEC_SYN=0,two@SEC_SYN=1+SEC_SYN_FUSED=0,fused@SEC_SYN=1,auto" > $O/syn_ab.jsonl 2> $O/syn_ab.err || { tail -20 $O/syn_ab.err; exit 1; }
cat $O/syn_ab.jsonl
bash tools/gpu_pmc_syn.sh

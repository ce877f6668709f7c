#!/bin/bash
# Round 5: phase-1 occupancy of the both-group wide decode -- the pair kernel capped at 3 waves per
# SIMD (SEC_SYN_WAVES=3, 168 VGPRs, spills) with the 8-slot and a 6-slot LDS ring, against the
# shipped build; tools/syn_ab.py, reassembly, interleaved rounds.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
echo "== syn occ" && timeout -k 10 500 python3 -u tools/syn_ab.py --rounds 3 --reps 5 --modes reassemble --variants "${SYN_VARIANTS:-auto,w3/w3,w3r6/w3r6}" --cases "32 lost;24 lost (random;16 lost (random, parity;30 % of blocks lost, first" > $O/syn_occ${SYN_TAG}.jsonl 2> $O/syn_occ${SYN_TAG}.err || { tail -20 $O/syn_occ${SYN_TAG}.err; exit 1; }
python3 -c "
import json
for l in open('$O/syn_occ${SYN_TAG}.jsonl'):
    d=json.loads(l); print(d['case'][:60], {k: v['reassemble'] for k, v in d.items() if isinstance(v, dict) and 'reassemble' in v})
"

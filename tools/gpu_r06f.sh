#!/bin/bash
# Round 6, after the knob prune: the GPU suite + smoke, then this build against the round-5
# library on the wide encodes and decodes (device-resident, one process, rounds interleaved).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
bash tools/gpu_tests.sh || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_pieces.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_pieces2.log 2>&1 || { tail -30 $O/pytest_pieces2.log; exit 1; }
tail -1 $O/pytest_pieces2.log
echo "== enc A/B" && timeout -k 10 400 python3 -u tools/enc_ab.py --rounds 3 --reps 5 --variants "cur,r05/r05" > $O/r06_enc_ab_final.jsonl 2> $O/r06_enc_ab_final.err || { tail -20 $O/r06_enc_ab_final.err; exit 1; }
cat $O/r06_enc_ab_final.jsonl
echo "== syn A/B" && timeout -k 10 500 python3 -u tools/syn_ab.py --rounds 3 --variants "auto,r05/r05" --cases "32 lost;24 lost (random;16 lost (random;x1024, 16 lost;30 %;14 data" > $O/r06_syn_ab_final.jsonl 2> $O/r06_syn_ab_final.err || { tail -20 $O/r06_syn_ab_final.err; exit 1; }
python3 -c "
import json
for l in open('$O/r06_syn_ab_final.jsonl'):
    d=json.loads(l); print(d['case'][:70], {k:(v['reassemble'],v['recover_only']) for k,v in d.items() if isinstance(v,dict)})"

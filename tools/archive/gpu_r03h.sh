#!/bin/bash
# Round evidence after the syndrome-path rework: the round batch (gpu tests, smoke, bench, rocprof,
# c4, c5, --gpus 2 rehearsal), then the syndrome A/B with the default choice and the per-chunk
# upload timeline.  First failure ends it.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
SKIP_CONFIGS=1 bash tools/gpu_round.sh || exit 1
echo "== syn A/B" && timeout -k 10 700 python3 -u tools/syn_ab.py --rounds 2 --variants "direct@SEC_SYN=0,two@SEC_SYN=1+SEC_SYN_FUSED=0,fused@SEC_SYN=1,auto" > $O/syn_ab.jsonl 2> $O/syn_ab.err || { tail -20 $O/syn_ab.err; exit 1; }
cat $O/syn_ab.jsonl
echo "== upload timeline" && timeout -k 10 300 python3 -u tools/upload_timeline.py > $O/upload_timeline.json 2> $O/upload_timeline.err || { tail -20 $O/upload_timeline.err; exit 1; }
cat $O/upload_timeline.json

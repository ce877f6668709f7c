#!/bin/bash
# Round 5: access-pattern ceilings with the product's own tiles (the no-GF calibration build,
# tools/c5_classes.py --libs base,nogf --extra; the headline step with it), and the per-call
# floor at storb's granularity (tools/small_call_profile.py, tools/c1_loopback.py).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
echo "== classes base/nogf" && timeout -k 10 300 python3 -u tools/c5_classes.py run --reps 10 --libs base,nogf --extra > $O/classes_nogf.json 2> $O/classes_nogf.err || { tail -20 $O/classes_nogf.err; exit 1; }
python3 - $O/classes_nogf.json <<'PY'
import json,sys
d=json.load(open(sys.argv[1]))
for k,v in d.items():
    if isinstance(v,dict): print(k, v["encode_TBs"], v["decode_TBs"])
PY
echo "== step base/nogf" && timeout -k 10 300 python3 -u tools/step_ab.py --variants base,nogf --rounds 5 --steps 20 > $O/step_nogf.jsonl 2> $O/step_nogf.err || { tail -20 $O/step_nogf.err; exit 1; }
cat $O/step_nogf.jsonl
echo "== small calls" && timeout -k 10 300 python3 -u tools/small_call_profile.py --reps 200 > $O/small_calls.json 2> $O/small_calls.err || { tail -20 $O/small_calls.err; exit 1; }
cat $O/small_calls.json
echo "== c1" && timeout -k 10 300 python3 -u tools/c1_loopback.py --reps 20 > $O/c1.json 2> $O/c1.err || { tail -20 $O/c1.err; exit 1; }
cat $O/c1.json

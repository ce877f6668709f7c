#!/bin/bash
# Round 5: tile order across the XCDs (SEC_XCD_ORDER 1: contiguous eighths; 2: runs of 8 consecutive
# tiles per XCD) against the plain order: C5 by size class, C3 and one GPU's C4 share
# in opposite library orders.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
echo "== run 1" && timeout -k 10 300 python3 -u tools/c5_classes.py run --reps 10 --extra --libs base,xcd1,xcd2 > $O/xcd_1.json 2> $O/xcd_1.err || { tail -20 $O/xcd_1.err; exit 1; }
echo "== run 2" && timeout -k 10 300 python3 -u tools/c5_classes.py run --reps 10 --extra --libs xcd2,xcd1,base > $O/xcd_2.json 2> $O/xcd_2.err || { tail -20 $O/xcd_2.err; exit 1; }
python3 - <<'PY'
import json
for f in ("gpurun_out/xcd_1.json", "gpurun_out/xcd_2.json"):
    d = json.load(open(f))
    for k, v in d.items():
        if isinstance(v, dict) and "decode_TBs" in v:
            print(f[-11:], k, "dec", v["decode_TBs"], "enc", v["encode_TBs"])
PY

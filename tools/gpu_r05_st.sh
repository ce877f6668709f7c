#!/bin/bash
# Round 5: plain (write-back) decode stores (SEC_DEC_ST=0) alone and with runs of 8 tiles per XCD
# (SEC_XCD_ORDER=2) against the shipped streaming stores: C5 by size class, C3 and a C4 share
# in opposite library orders.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
echo "== run 1" && timeout -k 10 300 python3 -u tools/c5_classes.py run --reps 10 --extra --libs base,st0,st0x2 > $O/st_1.json 2> $O/st_1.err || { tail -20 $O/st_1.err; exit 1; }
echo "== run 2" && timeout -k 10 300 python3 -u tools/c5_classes.py run --reps 10 --extra --libs st0x2,st0,base > $O/st_2.json 2> $O/st_2.err || { tail -20 $O/st_2.err; exit 1; }
python3 - <<'PY'
import json
for f in ("gpurun_out/st_1.json", "gpurun_out/st_2.json"):
    d = json.load(open(f))
    for k, v in d.items():
        if isinstance(v, dict) and "decode_TBs" in v:
            print(f[-11:], k, "dec", v["decode_TBs"], "enc", v["encode_TBs"])
PY

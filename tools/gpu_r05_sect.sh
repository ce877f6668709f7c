#!/bin/bash
# Round 5: sector-staged decode stores (SEC_DEC_SECTOR=1: rows staged in LDS, stored from each
# row's first 64-byte sector boundary) against the shipped stores: C5 classes, C3, C4 share
# in opposite library orders.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
echo "== run 1" && timeout -k 10 300 python3 -u tools/c5_classes.py run --reps 10 --extra --libs base,sect > $O/sect_1.json 2> $O/sect_1.err || { tail -20 $O/sect_1.err; exit 1; }
echo "== run 2" && timeout -k 10 300 python3 -u tools/c5_classes.py run --reps 10 --extra --libs sect,base > $O/sect_2.json 2> $O/sect_2.err || { tail -20 $O/sect_2.err; exit 1; }
python3 - <<'PY'
import json
for f in ("gpurun_out/sect_1.json", "gpurun_out/sect_2.json"):
    d = json.load(open(f))
    for k, v in d.items():
        if isinstance(v, dict) and "decode_TBs" in v:
            print(f[-11:], k, "dec", v["decode_TBs"], "enc", v["encode_TBs"])
PY

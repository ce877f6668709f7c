#!/bin/bash
# Round 5: decode tiles per workgroup (SEC_DEC_TPW 2 / 4 variant libraries) against the shipped
# one-tile workgroups: C5 by size class, C3 and one GPU's C4 share (tools/c5_classes.py), twice
# in opposite library orders.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
echo "== run 1" && timeout -k 10 300 python3 -u tools/c5_classes.py run --reps 10 --extra --libs base,dtpw2,dtpw4 > $O/dtpw_1.json 2> $O/dtpw_1.err || { tail -20 $O/dtpw_1.err; exit 1; }
echo "== run 2" && timeout -k 10 300 python3 -u tools/c5_classes.py run --reps 10 --extra --libs dtpw4,dtpw2,base > $O/dtpw_2.json 2> $O/dtpw_2.err || { tail -20 $O/dtpw_2.err; exit 1; }
python3 - <<'PY'
import json
for f in ("gpurun_out/dtpw_1.json", "gpurun_out/dtpw_2.json"):
    d = json.load(open(f))
    for k, v in d.items():
        if isinstance(v, dict) and "decode_TBs" in v:
            print(f[-11:], k, "dec", v["decode_TBs"], "enc", v["encode_TBs"])
PY

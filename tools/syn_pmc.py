#!/usr/bin/env python3
"""Per-kernel PMC summary of tools/syn_ab.py runs under rocprofv3 (tools/gpu_syn_pmc.sh): for each
sec_* decode kernel, dispatches, mean duration, HBM bytes per dispatch (read = 2 x FETCH_SIZE x
1024 on gfx950, write = WRITE_SIZE x 1024; MI355X_MICROARCH.md) and the SQ wave-state fractions
(SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_VALU over SQ_WAVE_CYCLES).  Not product code.

    python tools/syn_pmc.py gpurun_out/<fetch dir> <write dir> <sq dir> <trace dir> [<more sq dirs>...]

Every counter of the SQ passes is also reported as its mean per dispatch (`per_dispatch`), so a
pass of instruction counts (SQ_INSTS_*, SQC_ICACHE_*, SQ_IFETCH) reads off directly.
"""

import csv
import glob
import json
import os
import sys
from collections import defaultdict


def rows(d, pat):
    for p in glob.glob(os.path.join(d, "**", pat), recursive=True):
        with open(p) as f:
            yield from csv.DictReader(f)


def short(name):
    i = name.find("sec_")
    return name[i:name.find("(", i)] if i >= 0 else None


def per_dispatch(d):
    v = defaultdict(lambda: defaultdict(float))
    for r in rows(d, "*counter_collection*.csv"):
        k = short(r.get("Kernel_Name", ""))
        if k:
            v[(k, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    out = defaultdict(lambda: defaultdict(list))
    for (k, _), cs in v.items():
        for c, x in cs.items():
            out[k][c].append(x)
    return out


def main():
    fetch, write, sq, trace = sys.argv[1:5]
    f, w, s = per_dispatch(fetch), per_dispatch(write), per_dispatch(sq)
    for extra in sys.argv[5:]:
        for k, cs in per_dispatch(extra).items():
            for c, x in cs.items():
                s[k][c] = x
    dur = defaultdict(list)
    for r in rows(trace, "*kernel_trace*.csv"):
        k = short(r.get("Kernel_Name", ""))
        if k:
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    res = {}
    for k in sorted(set(f) | set(w) | set(s)):
        e = {}
        if f[k].get("FETCH_SIZE"):
            x = f[k]["FETCH_SIZE"]
            e["read_bytes_per_dispatch"] = 2 * 1024 * sum(x) / len(x)
        if w[k].get("WRITE_SIZE"):
            x = w[k]["WRITE_SIZE"]
            e["write_bytes_per_dispatch"] = 1024 * sum(x) / len(x)
        cyc = sum(s[k].get("SQ_WAVE_CYCLES", [])) or None
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_ANY"):
            if cyc and s[k].get(c):
                e[c.lower() + "_frac"] = round(sum(s[k][c]) / cyc, 3)
        if s[k]:
            e["per_dispatch"] = {c: round(sum(x) / len(x)) for c, x in sorted(s[k].items())}
        if dur.get(k):
            e["dispatches"] = len(dur[k])
            e["mean_ms"] = round(sum(dur[k]) / len(dur[k]), 4)
        res[k] = e
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""HBM traffic of the syndrome decode kernels from rocprofv3 --pmc passes over tools/syn_ab.py
(one case, one variant, --rounds 1 --reps R): the first 1 + R dispatches of the decode kernel are
the reassembling calls, the next 1 + R the recover-only ones (syn_ab's order).  gfx950
correction as tools/pmc_summary.py: read bytes = 2 x FETCH_SIZE KiB, written = WRITE_SIZE KiB.

    python tools/pmc_syn_summary.py <fetch dir> <write dir> <kernel substring> <k> <B> <chunks> <e> <n>
"""

from __future__ import annotations

import csv
import glob
import json
import sys


def per_dispatch(d, counter, kernel):
    rows = []
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
                rows.append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    agg = {}
    for i, v in rows:
        agg[i] = agg.get(i, 0.0) + v
    return [agg[i] for i in sorted(agg)]


def main():
    fd, wd, kern = sys.argv[1:4]
    k, B, nch, e, n = (int(x) for x in sys.argv[4:9])
    fetch = per_dispatch(fd, "FETCH_SIZE", kern)
    write = per_dispatch(wd, "WRITE_SIZE", kern)
    half = len(fetch) // 2
    out = {"kernel": kern, "correction": "read = 2 x FETCH_SIZE x 1024 B (gfx950), write = WRITE_SIZE x 1024 B",
           "dispatches": len(fetch)}
    for mode, sl, alg in (("reassemble", slice(0, half), nch * (k * B + n)),
                          ("recover_only", slice(half, 2 * half), nch * (k * B + e * B))):
        f = fetch[sl]
        w = write[sl][:len(f)]
        if not f:
            continue
        rd = 2 * 1024 * sum(f) / len(f)
        wr = 1024 * sum(w) / max(len(w), 1)
        out[mode] = {"read_bytes": round(rd), "write_bytes": round(wr), "algorithmic_bytes": alg,
                     "traffic_over_algorithmic": round((rd + wr) / alg, 4)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py into per-launch HBM bytes.

    python tools/pmc_summary.py gpurun_out > profiles/pmc_encode_c2.json

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half the bytes of a wide
coalesced streaming read, so read bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE is exact for
16 B/lane streaming stores (x 1024).  Both counters are in KiB per dispatch.
"""

from __future__ import annotations

import csv
import glob
import json
import os
import sys
from collections import defaultdict

ENC_ALG = 1024 * ((1 << 20) + 2 * (1 << 18))  # bytes per encode launch (bench workload c2)
DEC_ALG = 1024 * (4 * (1 << 18) + (1 << 20))  # bytes per decode launch (reassemble)


def counters(d: str, name: str) -> dict:
    vals = defaultdict(list)
    for path in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != name:
                    continue
                k = row.get("Kernel_Name", "")
                kind = "encode" if "sec_encode_kernel" in k else "decode" if "sec_decode_kernel" in k else None
                if kind:
                    vals[(kind, row.get("Dispatch_Id"))].append(float(row["Counter_Value"]))
    per = defaultdict(list)
    for (kind, _), v in vals.items():
        per[kind].append(sum(v))
    return {k: sum(v) / len(v) for k, v in per.items() if v}


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
    fetch = counters(os.path.join(d, "pmc_fetch"), "FETCH_SIZE")
    write = counters(os.path.join(d, "pmc_write"), "WRITE_SIZE")
    out = {"workload": "c2", "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) on "
                                      "python3 bench.py --steps 10 --warmup 2",
           "correction": "read = 2 x FETCH_SIZE KiB (gfx950 half-count), write = WRITE_SIZE KiB"}
    for kind, alg in (("encode", ENC_ALG), ("decode", DEC_ALG)):
        if kind in fetch and kind in write:
            rd = 2 * fetch[kind] * 1024
            wr = write[kind] * 1024
            out[kind] = {"fetch_size_kib": fetch[kind], "write_size_kib": write[kind], "read_bytes": rd,
                         "write_bytes": wr, "hbm_bytes_per_launch": rd + wr, "algorithmic_bytes": alg,
                         "traffic_over_algorithmic": round((rd + wr) / alg, 4)}
    if "encode" in out:
        out["hbm_bytes_per_launch"] = out["encode"]["hbm_bytes_per_launch"]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

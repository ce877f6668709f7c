#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py into per-launch HBM bytes.

    python tools/pmc_summary.py gpurun_out c2|c4|c5 > profiles/pmc_<workload>.json

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half the bytes of a wide
coalesced streaming read, so read bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE is exact for
16 B/lane streaming stores (x 1024).  Both counters are in KiB per dispatch.

The summary records `lib_digest`, the source digest of the libstorbec.so it was taken on
(storb_amd/_build.py); bench.py load_traffic uses a summary only when that digest equals the
current build's.

Workloads (the bench line each summary belongs to; bench.py load_traffic reads it):
  c2  python3 bench.py: encode (sec_encode_kernel) and decode (sec_decode_kernel) launches over
      1024 x 1 MiB RS(4,2) chunks (the timed region only: no recover-only, c4 or c5 launches)
  c4  python3 bench.py --workload c4: the encode launches (sec_encode_bs*_kernel) over the
      whole 65536 x 64 KiB RS(10,4) job at N = 1, and the decode launches after the timed region
  c5  python3 bench.py --workload c5 --c5-device-only: the device-resident encode / decode
      launches over the ~1 GiB mixed RS(8,3) job at N = 1
"""

from __future__ import annotations

import csv
import glob
import json
import os
import sys
from collections import defaultdict

def _c5_alg():
    import numpy as np

    sys.path.insert(0, ROOT)
    import bench

    sizes = np.array(bench.c5_sizes(), dtype=np.int64)
    B = (sizes + 7) // 8
    return int(sizes.sum() + 3 * B.sum()), int(8 * B.sum() + sizes.sum())


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKLOADS = {
    "c2": {"encode": ("sec_encode_kernel", 1024 * ((1 << 20) + 2 * (1 << 18))),
           "decode": ("sec_decode_kernel", 1024 * (4 * (1 << 18) + (1 << 20))),
           "cmd": "python3 bench.py --steps 10 --warmup 2 --no-cpu --no-e2e --no-recover --no-c4 --no-c5"},
    "c4": {"encode": ("sec_encode_bs", 65536 * (65536 + 4 * 6554)),
           "decode": ("sec_decode_kernel", 65536 * (10 * 6554 + 65536)),
           "cmd": "python3 bench.py --workload c4 --steps 10 --warmup 2 --no-cpu"},
    "c5": {"encode": ("sec_encode_kernel", None), "decode": ("sec_decode_kernel", None),
           "cmd": "python3 bench.py --workload c5 --c5-device-only --steps 5 --warmup 1 --no-cpu --no-e2e"},
}


def counters(d: str, name: str, kinds: dict) -> dict:
    vals = defaultdict(list)
    for path in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != name:
                    continue
                k = row.get("Kernel_Name", "")
                kind = next((kd for kd, (pat, _) in kinds.items() if pat in k), None)
                if kind:
                    vals[(kind, row.get("Dispatch_Id"))].append(float(row["Counter_Value"]))
    per = defaultdict(list)
    for (kind, _), v in vals.items():
        per[kind].append(sum(v))
    return {k: sum(v) / len(v) for k, v in per.items() if v}


def _digest() -> str:
    sys.path.insert(0, ROOT)
    from storb_amd import _build

    return _build._digest()


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
    wl = sys.argv[2] if len(sys.argv) > 2 else "c2"
    spec = dict(WORKLOADS[wl])
    if wl == "c5":
        ea, da = _c5_alg()
        spec["encode"], spec["decode"] = (spec["encode"][0], ea), (spec["decode"][0], da)
    kinds = {k: v for k, v in spec.items() if k in ("encode", "decode")}
    fetch = counters(os.path.join(d, "pmc_fetch"), "FETCH_SIZE", kinds)
    write = counters(os.path.join(d, "pmc_write"), "WRITE_SIZE", kinds)
    out = {"workload": wl, "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) on {spec['cmd']}",
           "correction": "read = 2 x FETCH_SIZE KiB (gfx950 half-count), write = WRITE_SIZE KiB",
           "lib_digest": _digest()}
    for kind, (pat, alg) in kinds.items():
        if kind in fetch and kind in write:
            rd = 2 * fetch[kind] * 1024
            wr = write[kind] * 1024
            out[kind] = {"kernel": pat, "fetch_size_kib": fetch[kind], "write_size_kib": write[kind], "read_bytes": rd,
                         "write_bytes": wr, "hbm_bytes_per_launch": rd + wr, "algorithmic_bytes": alg,
                         "traffic_over_algorithmic": round((rd + wr) / alg, 4)}
    if "encode" in out:
        out["hbm_bytes_per_launch"] = out["encode"]["hbm_bytes_per_launch"]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

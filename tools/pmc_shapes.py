#!/usr/bin/env python3
"""Summarise tools/gpu_pmc_shapes.sh's rocprofv3 passes into per-launch numbers per kernel.

    python tools/pmc_shapes.py gpurun_out/pmc_shapes c4 c2 > profiles/r02_pmc_shapes.json

Per workload and EC kernel (encode / decode main kernels, one name each):
  * HBM traffic: read = 2 x FETCH_SIZE KiB (gfx950 half-count on wide streaming reads,
    MI355X_MICROARCH.md §HBM), write = WRITE_SIZE KiB; against the algorithmic bytes;
  * issue: SQ_INSTS_VALU per wave; the shares of SQ_WAVE_CYCLES spent waiting (SQ_WAIT_ANY),
    issue-stalled (SQ_WAIT_INST_ANY) and issuing (SQ_ACTIVE_INST_ANY / _VALU); raw counters kept;
  * effective clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel duration (MI355X_MICROARCH.md DVFS note);
  * kernel duration from the --stats pass, and the VALU issue floor: SQ_INSTS_VALU x 4 cycles
    over 1024 SIMDs at that clock.
Shapes follow tools/prof_shape.py.
"""

from __future__ import annotations

import csv
import glob
import json
import os
import sys
from collections import defaultdict

SHAPES = {"c2": (1024, 1 << 20, 4, 6), "c4": (8192, 65536, 10, 14)}


def shape(w: str):
    if w in SHAPES:
        return SHAPES[w]
    return tuple(map(int, w.split(",")))


def kind_of(name: str):
    if "sec_encode_kernel" in name or "sec_encode_bs" in name or "sec_encode_xb" in name:
        return "encode"
    if "sec_decode_kernel" in name:
        return "decode"
    return None


def counters(d: str) -> dict:
    """{(kind, counter): [per-dispatch values]} summed over the dispatch's instances."""
    vals = defaultdict(float)
    names = {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                kind = kind_of(row.get("Kernel_Name", ""))
                if not kind:
                    continue
                names[kind] = row["Kernel_Name"].replace("void (anonymous namespace)::", "").split("(")[0]
                vals[(kind, row["Counter_Name"], row["Dispatch_Id"])] += float(row["Counter_Value"])
    per = defaultdict(list)
    for (kind, cn, _), v in vals.items():
        per[(kind, cn)].append(v)
    return {k: sum(v) / len(v) for k, v in per.items()}, names


def stats(d: str) -> dict:
    out = {}
    for path in glob.glob(os.path.join(d, "**", "*kernel_stats*.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                kind = kind_of(row["Name"])
                if kind:
                    out[kind] = {"avg_ns": float(row["AverageNs"]), "calls": int(row["Calls"]),
                                 "min_ns": float(row["MinNs"]), "max_ns": float(row["MaxNs"])}
    return out


def main():
    root = sys.argv[1]
    res = {"source": "tools/gpu_pmc_shapes.sh: rocprofv3 passes over tools/prof_shape.py --reps 10 "
                     "(FETCH_SIZE, WRITE_SIZE, SQ + GRBM, --stats; each its own run)",
           "correction": "read = 2 x FETCH_SIZE KiB, write = WRITE_SIZE KiB (MI355X_MICROARCH.md HBM section)"}
    for w in sys.argv[2:]:
        nch, n, k, m = shape(w)
        B = -(-n // k)
        alg = {"encode": nch * (n + (m - k) * B), "decode": nch * (k * B + n)}
        fetch, names = counters(os.path.join(root, w, "fetch"))
        write, _ = counters(os.path.join(root, w, "write"))
        sq, _ = counters(os.path.join(root, w, "sq"))
        st = stats(os.path.join(root, w, "stats"))
        wres = {}
        for kind in ("encode", "decode"):
            r = {"kernel": names.get(kind), "algorithmic_bytes": alg[kind]}
            if kind in st:
                r["avg_ms"] = st[kind]["avg_ns"] / 1e6
                r["achieved_GBs"] = round(alg[kind] / st[kind]["avg_ns"], 1)
            f, wr = fetch.get((kind, "FETCH_SIZE")), write.get((kind, "WRITE_SIZE"))
            if f is not None and wr is not None:
                r["read_bytes"] = 2 * f * 1024
                r["write_bytes"] = wr * 1024
                r["traffic_over_algorithmic"] = round((r["read_bytes"] + r["write_bytes"]) / alg[kind], 4)
            c = {cn: sq.get((kind, cn)) for cn in ("SQ_WAVES", "SQ_INSTS_VALU", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES",
                                                  "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                                                  "SQ_ACTIVE_INST_VALU", "GRBM_GUI_ACTIVE")}
            r["counters"] = c
            if c["SQ_WAVES"] and c["SQ_INSTS_VALU"]:
                r["valu_insts_per_wave"] = round(c["SQ_INSTS_VALU"] / c["SQ_WAVES"], 1)
            if c["SQ_WAVE_CYCLES"]:
                wc = c["SQ_WAVE_CYCLES"]
                r["share_of_wave_cycles"] = {
                    "waiting (s_waitcnt / barrier)": round((c["SQ_WAIT_ANY"] or 0) / wc, 3),
                    "issue stalled": round((c["SQ_WAIT_INST_ANY"] or 0) / wc, 3),
                    "issuing": round((c["SQ_ACTIVE_INST_ANY"] or 0) / wc, 3),
                    "issuing VALU": round((c["SQ_ACTIVE_INST_VALU"] or 0) / wc, 3)}
            if c["GRBM_GUI_ACTIVE"] and kind in st:
                clk = c["GRBM_GUI_ACTIVE"] / 8 / st[kind]["avg_ns"]  # GHz
                r["effective_clock_GHz"] = round(clk, 3)
                if c["SQ_INSTS_VALU"]:
                    # wave64 VALU issue: one instruction per SIMD every 4 cycles (SQ_ACTIVE_INST_VALU
                    # counts it as one quad-cycle); 256 CUs x 4 SIMDs
                    floor_ns = c["SQ_INSTS_VALU"] * 4 / 1024 / clk
                    r["valu_issue_floor_ms"] = round(floor_ns / 1e6, 4)
                    r["valu_issue_floor_over_duration"] = round(floor_ns / st[kind]["avg_ns"], 3)
            wres[kind] = r
        res[w] = wres
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""C5's dominant decode (sec_decode_kernel<3,1,false,0>) runs 0.65-0.67 of
HBM peak against C3's 0.75-0.77.  Split the C5 job (bench.c5_sizes: log-uniform 4 KiB-4 MiB,
RS(8,3), {1,3,5} erased, block 7 read in place) into size classes, run each class as its own
device-resident batch, and time the encode / decode kernels per class (HIP events).

    python tools/c5_classes.py run [--reps 10]            -> JSON (per class: ms, TB/s, bytes)
    python tools/c5_classes.py summarize DIR_SQ DIR_TRACE  -> per (class, kernel) SQ counters

Under rocprofv3 the launches of one class are contiguous in dispatch order (each class syncs
before the next starts), and `run` prints the plan (class order, launches per class) so
`summarize` can assign each sec_* dispatch to its class.
"""

from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import sys
from collections import defaultdict

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CLASSES = (("4K-64K", 0, 64 << 10), ("64K-1M", 64 << 10, 1 << 20), ("1M-4M", 1 << 20, 1 << 30), ("all", 0, 1 << 30))
K, M, ERASED = 8, 11, (1, 3, 5)


def run(reps: int, libs: str = "base", extra: bool = False):
    import torch

    import bench
    from storb_amd import _build
    from storb_amd.engine import Engine

    tags = libs.split(",")
    engs = {t: Engine(0, lib_path=_build.LIB if t == "base" else _build.variant_lib(t))
            for t in tags}
    sizes_all = np.array(bench.c5_sizes(), dtype=np.int64)
    res = {"config": f"C5 sizes (bench.c5_sizes) by class, RS(8,3), decode {ERASED} erased reassemble, "
                     f"{reps} launches each, per-launch HIP events", "lib_digest": bench.lib_digest(), "plan": []}
    cases = [(name, [int(s) for s in sizes_all if lo <= s < hi], K, M, ERASED) for name, lo, hi in CLASSES]
    if extra:  # the other BASELINE shapes through the same harness (C3: 1024 x 1 MiB RS(4,2); C4: one GPU's share)
        cases += [("C3_1024x1MiB_rs42", [1 << 20] * 1024, 4, 6, (1, 3)),
                  ("C4_8192x64KiB_rs104", [65536] * 8192, 10, 14, (0, 2, 5, 7))]
    for name, sizes, K_, M_, ER in cases:
        total = int(np.sum(sizes))
        ed, B = bench.enc_descs_var(sizes, K_, M_)
        src = torch.randint(0, 256, (total,), dtype=torch.uint8, device="cuda:0")
        par = torch.empty(int(np.sum(B)) * (M_ - K_), dtype=torch.uint8, device="cuda:0")
        out = torch.empty_like(src)
        dd, sn, offs, av = bench.dec_descs_var(sizes, K_, M_, B, src.data_ptr(), par.data_ptr(), ER)
        ea = total + int(np.sum(B)) * (M_ - K_)
        da = int(np.sum(B)) * K_ + total
        for tag, eng in engs.items():
            eng.encode_batch(ed, src, par)
            eng.decode_batch(dd, sn, offs, 0, out, block_avail=av)
            torch.cuda.synchronize()
            if not tag.startswith("nogf"):  # (a calibration variant's "parity" is not Reed-Solomon parity)
                assert torch.equal(out, src), (name, tag)
            eng.set_timing(True)
            for _ in range(reps):
                eng.encode_batch(ed, src, par, asynchronous=True)
            for _ in range(reps):
                eng.decode_batch(dd, sn, offs, 0, out, block_avail=av, asynchronous=True)
            eng.sync()
            eng.set_timing(False)
            ems, en = eng.collect_timing("encode")
            dms, dn = eng.collect_timing("decode")
            te, td = ems / en, dms / dn
            key = name if tag == "base" else f"{name}@{tag}"
            res[key] = {"chunks": len(sizes), "bytes": total, "encode_ms": round(te, 4),
                        "encode_TBs": round(ea / te / 1e9, 3), "decode_ms": round(td, 4),
                        "decode_TBs": round(da / td / 1e9, 3), "encode_alg_bytes": ea, "decode_alg_bytes": da,
                        "mean_chunk": round(total / max(len(sizes), 1))}
        res["plan"].append({"class": name, "launches": (1 + reps) * len(engs), "encode_alg": ea, "decode_alg": da})
        del src, par, out
        torch.cuda.empty_cache()
    print(json.dumps(res, indent=1), flush=True)
    for eng in engs.values():
        eng.close()


def _rows(d):
    rows = []
    for path in glob.glob(os.path.join(d, "**", "*.csv"), recursive=True):
        with open(path) as f:
            rows.extend(csv.DictReader(f))
    return rows


def summarize(sq_dir: str, plan_path: str):
    with open(plan_path) as f:
        plan = json.load(f)["plan"]
    vals = defaultdict(lambda: defaultdict(float))  # dispatch -> counter -> value
    names = {}
    for r in _rows(sq_dir):
        if "Counter_Name" not in r:
            continue
        k = r.get("Kernel_Name", "")
        if "sec_" not in k:
            continue
        did = int(r["Dispatch_Id"])
        vals[did][r["Counter_Name"]] += float(r["Counter_Value"])
        names[did] = k
    # each class: (1 + reps) encodes then (1 + reps) decodes; dispatches in order
    enc = sorted(d for d in names if "encode" in names[d])
    dec = sorted(d for d in names if "decode" in names[d])
    out = {}
    ei = di = 0
    for p in plan:
        n = p["launches"]
        for kind, lst, idx in (("encode", enc, ei), ("decode", dec, di)):
            ds = lst[idx + 1:idx + n]  # the first launch is the untimed check
            agg = defaultdict(float)
            for d in ds:
                for c, v in vals[d].items():
                    agg[c] += v / max(len(ds), 1)
            wc = agg.get("SQ_WAVE_CYCLES", 0.0)
            o = {"kernel": sorted({names[d] for d in ds}), "dispatches": len(ds), **{c: round(v) for c, v in agg.items()}}
            if wc:
                for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
                    if c in agg:
                        o[c + "_frac"] = round(agg[c] / wc, 4)
            if "SQ_WAVES" in agg and "SQ_BUSY_CYCLES" in agg and agg["SQ_BUSY_CYCLES"]:
                o["avg_waves_per_busy_cycle"] = round(wc / agg["SQ_BUSY_CYCLES"], 2)
            out[f"{p['class']}/{kind}"] = o
        ei += n
        di += n
    print(json.dumps(out, indent=1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=("run", "summarize"))
    ap.add_argument("dirs", nargs="*")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--libs", default="base", help="comma list: base and/or tools/sweep.py variant tags (built)")
    ap.add_argument("--extra", action="store_true", help="also C3 (1024 x 1 MiB RS(4,2)) and one GPU's C4 share")
    a = ap.parse_args()
    if a.mode == "run":
        run(a.reps, a.libs, a.extra)
    else:
        summarize(a.dirs[0], a.dirs[1])


if __name__ == "__main__":
    main()

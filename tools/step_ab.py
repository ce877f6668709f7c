#!/usr/bin/env python3
"""A/B of build variants on the headline STEP (bench.c2c3_run: encode then decode of 1024 x
1 MiB RS(4,2), {1,3} erased), timed as the bench times it: wall clock of `--steps` steps
between device syncs, median over interleaved rounds, one process, one set of buffers
(cdna_hip_programming.md §5.4 rule 24).  Kernel times (HIP events) are taken in separate
blocks so the events do not sit in the wall-clock blocks.

tools/decode_gap.py showed that the decode right after the encode runs 4 % slower than a
decode after a decode or after idle time; a store policy that writes the encode's parity
through may move that cost into the encode or remove it.  Only the step total counts.

    python tools/step_ab.py --variants base,est2,est3 [--rounds 7] [--steps 20]
Variants are tools/sweep.py's VARIANTS (built here with --build).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="base")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--build", action="store_true")
    a = ap.parse_args()
    import sweep

    tags = a.variants.split(",")
    if a.build:
        sweep.build(tags)
        return
    import torch

    import bench
    from storb_amd import _build
    from storb_amd.engine import Engine

    libs = {t: (_build.LIB if t == "base" else _build.variant_lib(t)) for t in tags}
    torch.cuda.set_device(0)
    nch, n, k, m = 1024, bench.CHUNK, bench.K, bench.M
    g = torch.Generator(device="cuda:0")
    g.manual_seed(1000)
    src = torch.randint(0, 256, (nch * n,), dtype=torch.uint8, device="cuda:0", generator=g)
    ed, B = bench.enc_descs(nch, n, k, m)
    par = torch.empty(nch * (m - k) * B, dtype=torch.uint8, device="cuda:0")
    out = torch.empty_like(src)
    dd, sn, offs, av = bench.dec_descs(nch, n, k, m, B, src.data_ptr(), par.data_ptr(), bench.ERASED)
    engs = {t: Engine(0, lib_path=libs[t]) for t in tags}
    for t, e in engs.items():
        out.zero_()
        e.encode_batch(ed, src, par)
        e.decode_batch(dd, sn, offs, 0, out, block_avail=av)
        if t != "nogf":  # (the calibration variant writes no Reed-Solomon bytes)
            assert torch.equal(out, src), t
    wall = {t: [] for t in tags}
    kern = {t: {"encode": [], "decode": []} for t in tags}
    for _ in range(a.rounds):
        for t, e in engs.items():
            def step():
                e.encode_batch(ed, src, par, asynchronous=True)
                e.decode_batch(dd, sn, offs, 0, out, block_avail=av, asynchronous=True)

            for _ in range(3):
                step()
            e.sync()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                step()
            e.sync()
            wall[t].append((time.perf_counter() - t0) / a.steps * 1e3)
            e.set_timing(True)
            for _ in range(a.steps):
                step()
            e.sync()
            e.set_timing(False)
            for kind in ("encode", "decode"):
                ms, nl = e.collect_timing(kind)
                kern[t][kind].append(ms / nl)
    for t in tags:
        w = float(np.median(wall[t]))
        print(json.dumps({"variant": t, "defines": sweep.VARIANTS.get(t, {}), "ms_per_step": round(w, 4),
                          "ms_per_step_all": [round(x, 4) for x in wall[t]],
                          "gibs": round(2 * nch * n / (w / 1e3) / (1 << 30), 1),
                          "encode_ms": round(float(np.median(kern[t]["encode"])), 4),
                          "decode_ms": round(float(np.median(kern[t]["decode"])), 4),
                          "steps": a.steps, "rounds": a.rounds}), flush=True)
    for e in engs.values():
        e.close()


if __name__ == "__main__":
    main()

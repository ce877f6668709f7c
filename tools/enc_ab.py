#!/usr/bin/env python3
"""A/B of the wide bit-sliced encodes (one process, fresh engine per variant, rounds interleaved),
device-resident.  Rates are TB/s of algorithmic bytes (n read + (m - k) B written per chunk) per
HIP-event kernel time of the encode call.  Every variant's parity is compared with the first
variant's (the GPU suite checks the kernels against the oracle).  Not product code.

    python tools/enc_ab.py [--rounds 3] [--reps 5] [--variants "cur,r05/r05"]

(Round 6 compared the pair kernel with the interleaved launch through the context option
SEC_BS_PAIR, since archived with that kernel; a variant is now a prebuilt library.)
"""

from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# (name, k, m, chunk bytes, chunks)
CASES = [
    ("zfec(64,96) 1MiB x1024", 64, 96, 1 << 20, 1024),
    ("zfec(64,96) 256MiB x4", 64, 96, 256 << 20, 4),
    ("zfec(64,96) 64MiB x16 (ragged)", 64, 96, (64 << 20) - 12345, 16),
    ("zfec(32,48) 1MiB x1024", 32, 48, 1 << 20, 1024),
    ("zfec(16,24) 8MiB x128", 16, 24, 8 << 20, 128),
    # the block stride (B) question of DESIGN §8 item 3: power-of-two B at several spans, and
    # non-power-of-two B at the 256 MiB span
    ("stride: zfec(64,96) 16MiB x64 (B 256 KiB)", 64, 96, 16 << 20, 64),
    ("stride: zfec(64,96) 64MiB x16 (B 1 MiB)", 64, 96, 64 << 20, 16),
    ("stride: zfec(64,96) 128MiB x8 (B 2 MiB)", 64, 96, 128 << 20, 8),
    ("stride: zfec(64,96) 256MiB x4 (B 4 MiB)", 64, 96, 256 << 20, 4),
    ("stride: zfec(64,96) 252MiB x4 (B 4032 KiB)", 64, 96, 252 << 20, 4),
    ("stride: zfec(64,96) 260MiB x4 (B 4160 KiB)", 64, 96, 260 << 20, 4),
    ("stride: zfec(64,96) 256MiB-4KiB x4 (B 4 MiB - 64)", 64, 96, (256 << 20) - 4096, 4),
]


def main():
    import torch

    import bench
    from storb_amd import _build
    from storb_amd.engine import Engine

    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--variants", default="cur,r05/r05",
                    help="name@OPT=V+OPT2=V2[/tag]: context options per variant, optionally a prebuilt variant "
                         "library build/variants/libstorbec_<tag>.so")
    ap.add_argument("--cases", default="")
    a = ap.parse_args()
    variants = []
    for v in a.variants.split(","):
        v, _, tag = v.partition("/")
        name, _, env = v.partition("@")
        opts = {kv.split("=")[0]: int(kv.split("=")[1]) for kv in env.split("+")} if env else {}
        variants.append((name, opts, _build.variant_lib(tag) if tag else None))
    sel = [c for c in CASES if not a.cases or any(t in c[0] for t in a.cases.split(";"))]
    for name, k, m, n, nch in sel:
        g = torch.Generator(device="cuda")
        g.manual_seed(7)
        src = torch.randint(0, 256, (nch * n,), dtype=torch.uint8, device="cuda", generator=g)
        ed, B = bench.enc_descs(nch, n, k, m)
        ref = None
        par = torch.empty(nch * (m - k) * B, dtype=torch.uint8, device="cuda")
        res = {v[0]: [] for v in variants}
        for _ in range(a.rounds):
            for vname, opts, lib in variants:
                eng = Engine(0, lib_path=lib, options=opts)
                par.zero_()
                eng.encode_batch(ed, src, par)
                if ref is None:
                    ref = par.clone()
                else:
                    assert torch.equal(par, ref), (name, vname)
                eng.set_timing(True)
                for _ in range(a.reps):
                    eng.encode_batch(ed, src, par, asynchronous=True)
                eng.sync()
                eng.set_timing(False)
                ms, _ = eng.collect_timing("encode")
                res[vname].append(nch * (n + (m - k) * B) / (ms / 1e3 / a.reps) / 1e12)
                eng.close()
        row = {"case": name, "k": k, "m": m, "chunk": n, "chunks": nch}
        for vname, r in res.items():
            row[vname] = {"TB/s median": round(float(np.median(r)), 3), "all": [round(x, 3) for x in r]}
        print(json.dumps(row), flush=True)
        del src, par, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

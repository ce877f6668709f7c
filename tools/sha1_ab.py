#!/usr/bin/env python3
"""Interleaved in-process A/B of the SHA-1 kernel's next-block prefetch: the
libstorbec_sha1pf.so and libstorbec_sha1nopf.so builds (SEC_SHA1_PF=1 / 0) each get an Engine
in ONE process; every round times each build on each message shape (HIP events around the
kernel, 5 launches), rounds interleaved; prints per (shape, build) the median and the min/max
over rounds.  Not product code.

    python tools/sweep.py --build --variants sha1pf,sha1nopf && python tools/sha1_ab.py
"""

from __future__ import annotations

import json
import os
import statistics
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# (messages, bytes each): C2's pieces, C4's per-GPU pieces, and shapes between them
SHAPES = [(6144, 262144), (114688, 6554), (16384, 65536), (65536, 16384), (32768, 6554), (4096, 1 << 20)]


def main():
    import torch

    from storb_amd._lib import MSG_DTYPE
    from storb_amd.engine import Engine

    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    libdir = os.path.join(ROOT, "storb_amd", "lib")
    engs = {t: Engine(0, lib_path=os.path.join(libdir, f"libstorbec_{t}.so")) for t in ("sha1pf", "sha1nopf")}
    bufs = {}
    for nm, ln in SHAPES:
        buf = torch.randint(0, 256, (nm * ln,), dtype=torch.uint8, device="cuda")
        msgs = np.zeros(nm, dtype=MSG_DTYPE)
        msgs["addr"] = buf.data_ptr() + np.arange(nm, dtype=np.uint64) * ln
        msgs["len"] = msgs["avail"] = ln
        dig = {t: torch.empty(nm * 20, dtype=torch.uint8, device="cuda") for t in engs}
        bufs[(nm, ln)] = (buf, msgs, dig)
    samples = {(s, t): [] for s in SHAPES for t in engs}
    for _ in range(rounds):
        for s in SHAPES:
            buf, msgs, dig = bufs[s]
            for t, e in engs.items():
                e.sha1_batch(msgs, dig[t])  # warm
                e.set_timing(True)
                for _ in range(5):
                    e.sha1_batch(msgs, dig[t], asynchronous=True)
                e.sync()
                e.set_timing(False)
                ms, n = e.collect_timing("sha1")
                samples[(s, t)].append(ms / n)
    for s in SHAPES:
        _, _, dig = bufs[s]
        assert torch.equal(dig["sha1pf"], dig["sha1nopf"]), s
        nm, ln = s
        row = {"messages": nm, "bytes": ln, "blocks_per_message": -(-(ln + 9) // 64),
               "waves_per_simd": round(nm / 64 / 1024, 2)}
        for t in engs:
            v = samples[(s, t)]
            row[t] = {"median_ms": round(statistics.median(v), 4), "min_ms": round(min(v), 4),
                      "max_ms": round(max(v), 4), "GBs": round(nm * ln / statistics.median(v) / 1e6, 1)}
        row["pf_over_nopf"] = round(row["sha1nopf"]["median_ms"] / row["sha1pf"]["median_ms"], 3)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()

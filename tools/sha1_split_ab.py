#!/usr/bin/env python3
"""Interleaved in-process A/B of the two-wave SHA-1 kernel (sec_sha1_split_kernel: message
schedule on a second wave) against the one-lane-per-message kernel, on device-resident
message shapes from latency-bound (few long pieces) to issue-bound (many short ones).  One
Engine per mode (SEC_SHA1_SPLIT read when each engine builds its plan), rounds interleaved,
HIP-event kernel time of 5 launches per round; prints per shape the median per mode and the
speedup.  Digests of both modes checked equal.  Not product code.

    python tools/sha1_split_ab.py [rounds]
"""

from __future__ import annotations

import json
import os
import statistics
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# (messages, bytes each): C2's pieces, the upload window's 512 KiB pieces, 1 MiB pieces, and
# shorter ones down to C4's
SHAPES = [(6144, 262144), (768, 524288), (3072, 524288), (4096, 1 << 20), (16384, 65536), (65536, 16384),
          (114688, 6554)]


def main():
    import torch

    from storb_amd._lib import MSG_DTYPE
    from storb_amd.engine import Engine

    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    bufs = {}
    for nm, ln in SHAPES:
        buf = torch.randint(0, 256, (nm * ln,), dtype=torch.uint8, device="cuda")
        msgs = np.zeros(nm, dtype=MSG_DTYPE)
        msgs["addr"] = buf.data_ptr() + np.arange(nm, dtype=np.uint64) * ln
        msgs["len"] = msgs["avail"] = ln
        bufs[(nm, ln)] = (buf, msgs, {})
    engs = {}
    for mode in ("1", "0"):
        e = engs[mode] = Engine(0, options={"SEC_SHA1_SPLIT": int(mode)})
        for s in SHAPES:  # one engine per mode; each shape's plan is built here with that mode
            _, msgs, dig = bufs[s]
            dig[mode] = torch.empty(s[0] * 20, dtype=torch.uint8, device="cuda")
    samples = {(s, m): [] for s in SHAPES for m in engs}
    for _ in range(rounds):
        for s in SHAPES:
            _, msgs, dig = bufs[s]
            for m, e in engs.items():
                e.sha1_batch(msgs, dig[m])
                e.set_timing(True)
                for _ in range(5):
                    e.sha1_batch(msgs, dig[m], asynchronous=True)
                e.sync()
                e.set_timing(False)
                ms, n = e.collect_timing("sha1")
                samples[(s, m)].append(ms / n)
    for s in SHAPES:
        _, _, dig = bufs[s]
        assert torch.equal(dig["1"], dig["0"]), s
        nm, ln = s
        row = {"messages": nm, "bytes": ln, "waves_one_lane_kernel": -(-nm // 64)}
        for m in engs:
            v = samples[(s, m)]
            row["split" if m == "1" else "one_lane"] = {"median_ms": round(statistics.median(v), 4),
                                                        "GBs": round(nm * ln / statistics.median(v) / 1e6, 1)}
        row["split_speedup"] = round(row["one_lane"]["median_ms"] / row["split"]["median_ms"], 3)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()

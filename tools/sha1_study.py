#!/usr/bin/env python3
"""F1 SHA-1 piece ids on the device: C2's 6144 pieces of 256 KiB (one chain per lane, too
few lanes to fill the chip: latency-bound) and C4's per-GPU 114688 pieces of 6554 B (enough
lanes: issue-bound).  Not product code; prints one JSON line."""

from __future__ import annotations

import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import hashlib

    import torch

    from storb_amd._lib import MSG_DTYPE
    from storb_amd.engine import Engine
    from tools.bench_configs import sha1_case, timed

    lib = sys.argv[1] if len(sys.argv) > 1 else None  # an A/B build, e.g. storb_amd/lib/libstorbec_base.so
    eng = Engine(0, lib_path=lib)
    res = {"lib": os.path.basename(lib or "libstorbec.so"), "c2": sha1_case(eng)}
    nch, n, k, m = 8192, 65536, 10, 14
    B = -(-n // k)
    buf = torch.randint(0, 256, (nch * m * B,), dtype=torch.uint8, device="cuda")
    dig = torch.empty(nch * m * 20, dtype=torch.uint8, device="cuda")
    msgs = np.zeros(nch * m, dtype=MSG_DTYPE)
    msgs["addr"] = buf.data_ptr() + np.arange(nch * m, dtype=np.uint64) * B
    msgs["len"] = B
    msgs["avail"] = B
    t = timed(lambda: eng.sha1_batch(msgs, dig), 5)
    h = dig.cpu().numpy().reshape(-1, 20)
    hb = buf.cpu().numpy()
    for i in (0, 1, nch * m - 1):
        assert h[i].tobytes() == hashlib.sha1(hb[i * B:(i + 1) * B].tobytes()).digest(), i
    res["c4_pieces"] = {"pieces": nch * m, "piece_bytes": B, "sha1_ms": round(t * 1e3, 3),
                        "sha1_GBs": round(nch * m * B / t / 1e9, 1)}
    print(json.dumps(res), flush=True)
    eng.close()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""One 8 MiB chunk through encode_host_raw (the per-chunk upload's GPU call), timed per variant:
fresh pageable bytes per call vs one reused object, page-locking (SEC_REGISTER_MIN default) vs
staged copies (SEC_REGISTER_MIN=0), and the kernel time (HIP events).  Not product code.

    python tools/host_encode_probe.py > gpurun_out/host_encode_probe.json
"""

from __future__ import annotations

import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from storb_amd import piece
    from storb_amd.engine import Engine

    cs = 8 << 20
    k, m, B, _ = piece.chunk_shape(cs)
    rng = np.random.default_rng(1)
    base = rng.integers(0, 256, 64 * cs, dtype=np.uint8).tobytes()
    res = {"chunk_bytes": cs, "k": k, "m": m, "unit": "ms per call, median of 40"}
    for label, env in (("lock", {}), ("staged", {"SEC_REGISTER_MIN": 0})):
        eng = Engine(0, options=env)
        for mode in ("fresh", "reused"):
            ts, ks = [], []
            same = base[:cs]
            for i in range(48):
                c = base[(i % 64) * cs:(i % 64 + 1) * cs] if mode == "fresh" else same
                eng.set_timing(True)
                t0 = time.perf_counter()
                eng.encode_host_raw([c], [(k, m)])
                t1 = time.perf_counter()
                eng.set_timing(False)
                ms, nl = eng.collect_timing("encode")
                if i >= 8:
                    ts.append(t1 - t0)
                    ks.append(ms / max(nl, 1))
            res[f"{label}_{mode}"] = round(statistics.median(ts) * 1e3, 3)
            res[f"{label}_{mode}_kernel"] = round(statistics.median(ks), 3)
        eng.close()
    t0 = time.perf_counter()
    for i in range(8):
        bytes(base[i * cs:(i + 1) * cs])
    res["bytes_copy_8MiB"] = round((time.perf_counter() - t0) / 8 * 1e3, 3)
    print(json.dumps(res))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Where one per-chunk upload (encode_chunk + piece_hash of every piece, validator.py:1380,1081)
spends its time: a timeline of each call, medians over the chunks of a 1 GiB object.

    python tools/upload_timeline.py [--mib 1024] [--chunk-mib 8] > gpurun_out/upload_timeline.json

Marks (ms from the call's start): gpu_call start / end (engine.encode_host_raw, wrapped), every
piece filled (_pieces_parallel's return), the pydantic models built (_build), encode_chunk's
return, and the last piece_hash's return.  Not product code.
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=1024)
    ap.add_argument("--chunk-mib", type=int, default=8)
    a = ap.parse_args()
    from storb_amd import piece
    from storb_amd.engine import Engine

    rng = np.random.default_rng(7)
    data = rng.integers(0, 256, a.mib << 20, dtype=np.uint8).tobytes()
    cs = a.chunk_mib << 20
    eng = piece.get_engine()
    marks = {}
    orig = type(eng).encode_host_raw

    def wrapped(self, *args, **kw):
        marks["gpu_start"] = time.perf_counter()
        r = orig(self, *args, **kw)
        marks["gpu_end"] = time.perf_counter()
        return r

    type(eng).encode_host_raw = wrapped
    orig_pp, orig_build = piece._pieces_parallel, piece._build

    def pp(*args, **kw):
        r = orig_pp(*args, **kw)
        marks["pieces_ready"] = time.perf_counter()
        return r

    def build(*args, **kw):
        r = orig_build(*args, **kw)
        marks["models_built"] = time.perf_counter()
        return r

    piece._pieces_parallel, piece._build = pp, build
    rows = []
    for rep in range(2):
        for off in range(0, len(data), cs):
            chunk = data[off:off + cs]
            marks.clear()
            t0 = time.perf_counter()
            ec = piece.encode_chunk(chunk, off // cs)
            t1 = time.perf_counter()
            ids = [piece.piece_hash(p.data) for p in ec.pieces]
            t2 = time.perf_counter()
            if rep:
                rows.append({"gpu_start": marks.get("gpu_start", t0) - t0, "gpu_end": marks.get("gpu_end", t0) - t0,
                             "pieces_ready": marks.get("pieces_ready", t0) - t0,
                             "models_built": marks.get("models_built", t0) - t0,
                             "encode_return": t1 - t0, "hash_done": t2 - t0})
    type(eng).encode_host_raw = orig
    piece._pieces_parallel, piece._build = orig_pp, orig_build
    med = {k: round(statistics.median(r[k] for r in rows) * 1e3, 3) for k in rows[0]}
    k, m, B, _ = piece.chunk_shape(cs)
    print(json.dumps({"MALLOC_TRIM_THRESHOLD_": os.environ.get("MALLOC_TRIM_THRESHOLD_", ""), "unit": "ms from the call's start, median", "chunk_bytes": cs, "k": k, "m": m, "B": B,
                      "chunks": len(rows), **med,
                      "GiB_per_s": round(cs / (med["hash_done"] / 1e3) / 2**30, 3),
                      "cpus": piece._usable_cpus(), "hash_workers": piece.HASH_WORKERS,
                      "pool_threads": piece._pool("hash")._max_workers}))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""A/B of encode_chunk's piece-id prefetch (piece.PREFETCH_PIECE_IDS; thread-pool sizes) at the validator's call pattern (encode_chunk, then
piece_hash of each piece, chunk after chunk).  Not product code."""
import hashlib
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from concurrent.futures import ThreadPoolExecutor

    from storb_amd import piece

    rng = np.random.default_rng(0)
    res = {}
    for n in (256 << 10, 512 << 10, 1 << 20, 4 << 20):
        chunks = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for _ in range(16)]
        want = None
        for mode, pool in (("off", 0), ("per_piece", 8), ("per_piece", 16), ("per_piece", 4), ("off", 0)):
            piece.PREFETCH_PIECE_IDS = mode != "off"
            piece.PREFETCH_MIN_CHUNK = 0
            if pool:
                piece._pools["hash"] = ThreadPoolExecutor(pool)
            ts = []
            for rep in range(8):
                t0 = time.perf_counter()
                ids = []
                for i, c in enumerate(chunks):
                    info = piece.encode_chunk(c, i)
                    ids.append([piece.piece_hash(p.data) for p in info.pieces])
                ts.append(time.perf_counter() - t0)
                if want is None:
                    want = [[hashlib.sha1(b).hexdigest() for b in piece.Encoder(info.k, info.m).encode(c)]
                            for c in chunks]
                assert ids == want
            res[f"{n >> 10}KiB {mode} pool{pool}"] = round(statistics.median(ts) / len(chunks) * 1e6, 1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""F2 at the API storb calls: the upload and download loops over one large object, per-chunk
(the reference's call pattern) against the pipelined entry points.  Not product code.

    python tools/stream_rate.py [--mib 1024] > gpurun_out/stream_rate.json

Object: --mib MiB of random bytes; the policy gives its chunk size (1 GiB -> 8 MiB chunks,
zfec(16,24)).  Rates are object bytes / wall time (GiB/s), best of --reps:
  upload_per_chunk       encode_chunk per chunk + piece_hash per piece (validator.py:1380,1081)
  upload_stream          encode_chunks_stream(piece_ids=True), defaults (GPU piece ids for
                         large pieces, STREAM_WINDOW_IDS_BYTES windows)
  --gpu-ids: also per-window encode_chunks_with_ids, and the stream with GPU / host ids at
             64..512 MiB windows
  download_per_chunk     decode_chunk per chunk (the reference's reconstruct_data_stream body)
  download_stream        reconstruct_data_stream, consumed chunk by chunk
each download both with every data piece present (joined, no GPU work) and with data piece 0
of every chunk lost (recovered on the GPU).
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
GIB = float(1 << 30)


def best(fn, reps):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return min(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--gpu-ids", action="store_true", help="also: piece ids from the GPU SHA-1, per window")
    ap.add_argument("--parity-ids", action="store_true",
                    help="only the upload stream: host ids vs GPU parity ids (GPU_PARITY_IDS) at 64..1024 MiB windows, "
                         "rounds interleaved, ids checked against hashlib")
    ap.add_argument("--ab", action="store_true",
                    help="A/B in one process, rounds interleaved: STREAM_WORKERS 1 vs the default (a single stream "
                         "should not care), and encode_chunk's id hashing on fill vs after all pieces")
    a = ap.parse_args()
    if a.ab:
        return ab(a)
    if a.parity_ids:
        return parity_ids(a)
    from storb_amd import piece

    data = np.random.default_rng(3).integers(0, 256, a.mib << 20, dtype=np.uint8).tobytes()
    cs = piece.piece_length(len(data))
    parts = [data[o:o + cs] for o in range(0, len(data), cs)]
    res = {"object_bytes": len(data), "chunk_bytes": cs, "chunks": len(parts),
           "shape": list(piece.chunk_shape(cs)[:2]), "unit": "GiB/s of object bytes, best of %d" % a.reps}

    def up_per_chunk():
        out = []
        for i, c in enumerate(parts):
            ec = piece.encode_chunk(c, i)
            out.append((ec, [piece.piece_hash(p.data) for p in ec.pieces]))
        return out

    def up_stream():
        return list(piece.encode_chunks_stream(iter(parts), piece_ids=True))

    def up_gpu_ids(window_mib):  # piece ids hashed on the GPU (fused after encode), one call per window
        def run():
            out, i = [], 0
            per = max(1, (window_mib << 20) // cs)
            for w in range(0, len(parts), per):
                ecs, ids = piece.encode_chunks_with_ids(parts[w:w + per], w)
                out.extend(zip(ecs, ids))
            return out
        return run

    enc = up_stream()
    res["upload_per_chunk"] = round(len(data) / best(up_per_chunk, a.reps) / GIB, 3)
    res["upload_stream"] = round(len(data) / best(up_stream, a.reps) / GIB, 3)
    if a.gpu_ids:
        ref = [ids for _, ids in enc]
        for wm in (64, 256, 1024):
            got = up_gpu_ids(wm)()
            assert [ids for _, ids in got] == ref
            res[f"upload_gpu_ids_window_{wm}MiB"] = round(len(data) / best(up_gpu_ids(wm), a.reps) / GIB, 3)
        for wm in (64, 128, 256, 512):
            for mode in (True, False):  # ids from the GPU SHA-1 / from hashlib on the pool
                def up(wm=wm, mode=mode):
                    old = piece.GPU_PIECE_IDS
                    piece.GPU_PIECE_IDS = mode
                    try:
                        return list(piece.encode_chunks_stream(iter(parts), piece_ids=True, window_bytes=wm << 20))
                    finally:
                        piece.GPU_PIECE_IDS = old
                got = up()
                assert [ids for _, ids in got] == ref
                assert [[p.data for p in ec.pieces] for ec, _ in got] == [[p.data for p in ec.pieces] for ec, _ in enc]
                res[f"upload_stream_{'gpu' if mode else 'host'}_ids_window_{wm}MiB"] = round(
                    len(data) / best(up, a.reps) / GIB, 3)
    chunks = [ec.model_copy(update={"pieces": None}) for ec, _ in enc]
    for label, drop in (("all_data_present", ()), ("data_piece_0_lost", (0,))):
        pieces = [p for ec, _ in enc for p in ec.pieces if p.piece_idx not in drop]

        def down_per_chunk():
            for ch in chunks:
                ch.pieces = sorted([p for p in pieces if p.chunk_idx == ch.chunk_idx], key=lambda p: p.piece_idx)
                piece.decode_chunk(ch)

        def down_stream():
            n = 0
            for b in piece.reconstruct_data_stream(pieces, chunks):
                n += len(b)
            assert n == len(data)

        from storb_amd.engine import Engine

        for lj in (True, False):  # A/B: the library's one-call reassembly vs round 4's recover + join
            Engine.LIBRARY_JOIN = lj
            sfx = "" if lj else "_round4_join"
            assert b"".join(piece.reconstruct_data_stream(pieces, chunks)) == data
            res[f"download_per_chunk_{label}{sfx}"] = round(len(data) / best(down_per_chunk, a.reps) / GIB, 3)
            res[f"download_stream_{label}{sfx}"] = round(len(data) / best(down_stream, a.reps) / GIB, 3)
        Engine.LIBRARY_JOIN = True
    print(json.dumps(res, indent=1))


def parity_ids(a):
    """Upload stream (encode_chunks_stream(piece_ids=True)) with every id on the host threads
    against the parity ids from the GPU, per window size; median over 3 rounds of best-of-reps."""
    import hashlib

    from storb_amd import piece

    data = np.random.default_rng(3).integers(0, 256, a.mib << 20, dtype=np.uint8).tobytes()
    cs = piece.piece_length(len(data))
    parts = [data[o:o + cs] for o in range(0, len(data), cs)]
    res = {}
    for rnd in range(3):
        for wm in (64, 256, 512, 1024):
            for gp in (False, True):
                def up(wm=wm, gp=gp):
                    old = piece.GPU_PARITY_IDS
                    piece.GPU_PARITY_IDS = gp
                    try:
                        return list(piece.encode_chunks_stream(iter(parts), piece_ids=True, window_bytes=wm << 20))
                    finally:
                        piece.GPU_PARITY_IDS = old
                if rnd == 0:
                    got = up()
                    for ec, ids in got:
                        assert ids == [hashlib.sha1(p.data).hexdigest() for p in ec.pieces]
                    del got
                res.setdefault(f"window_{wm}MiB_{'gpu_parity' if gp else 'host'}_ids", []).append(
                    len(data) / best(up, a.reps) / GIB)
    print(json.dumps({"object_bytes": len(data), "chunk_bytes": cs, "shape": list(piece.chunk_shape(cs)[:2]),
                      "unit": "GiB/s, median of 3 rounds of best-of-%d" % a.reps,
                      **{k: round(float(np.median(v)), 3) for k, v in res.items()}}, indent=1))


def ab(a):
    """Interleaved A/B of the stream pool size and of HASH_ON_FILL (best of --reps per round,
    median over 3 rounds)."""
    from storb_amd import piece

    data = np.random.default_rng(3).integers(0, 256, a.mib << 20, dtype=np.uint8).tobytes()
    cs = piece.piece_length(len(data))
    parts = [data[o:o + cs] for o in range(0, len(data), cs)]
    enc = list(piece.encode_chunks_stream(iter(parts), piece_ids=True))
    chunks = [ec.model_copy(update={"pieces": None}) for ec, _ in enc]
    all_p = [p for ec, _ in enc for p in ec.pieces]
    lost_p = [p for ec, _ in enc for p in ec.pieces if p.piece_idx != 0]
    workers0 = piece.STREAM_WORKERS

    def set_workers(n):
        piece.STREAM_WORKERS = n

    def up_chunk():
        for i, c in enumerate(parts):
            ec = piece.encode_chunk(c, i)
            [piece.piece_hash(p.data) for p in ec.pieces]

    def up_stream():
        list(piece.encode_chunks_stream(iter(parts), piece_ids=True))

    def down(pieces):
        def run():
            n = 0
            for b in piece.reconstruct_data_stream(pieces, chunks):
                n += len(b)
            assert n == len(data)
        return run

    res = {}
    for _ in range(3):
        for w in (1, workers0):
            set_workers(w)
            for name, fn in (("upload_stream", up_stream), ("download_stream_all_present", down(all_p)),
                             ("download_stream_piece0_lost", down(lost_p))):
                fn()  # warm the pool's engines
                res.setdefault(f"{name}_workers{w}", []).append(len(data) / best(fn, a.reps) / GIB)
        for hof in (True, False):
            piece.HASH_ON_FILL = hof
            up_chunk()
            res.setdefault(f"upload_per_chunk_hash_on_fill_{hof}", []).append(len(data) / best(up_chunk, a.reps) / GIB)
        piece.HASH_ON_FILL = True
    set_workers(workers0)
    print(json.dumps({"object_bytes": len(data), "chunk_bytes": cs, "unit": "GiB/s, median of 3 rounds of best-of-%d" % a.reps,
                      **{k: round(float(np.median(v)), 3) for k, v in res.items()}}, indent=1))


if __name__ == "__main__":
    main()

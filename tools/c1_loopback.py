#!/usr/bin/env python3
"""BASELINE configs[0] (C1): one object through storb's upload -> store -> retrieve -> download
path in a loopback harness (an in-memory dict keyed by piece id stands in for the miners; the
real validator/miner need a chain, fibers and kademlia).  Not product code.

    python tools/c1_loopback.py [--reps 20] > gpurun_out/c1.json

Objects: 4 MiB (the policy gives 8 x 512 KiB chunks, zfec(4,6)) and 1 MiB (4 x 256 KiB,
zfec(2,3): BASELINE's "RS(k=2,m=1)", exactly piece_test.py:15).  Paths, each timed on the
same bytes, median of --reps runs, one thread of caller code:

  reference_cpu   the reference's path restated: storb/util/piece.py's encode_chunk /
                  decode_chunk / reconstruct_data logic (policy, easyfec split + pad, pydantic
                  Piece / EncodedChunk models, one decode per chunk, join) with zfec's arithmetic
                  from oracle/fec_oracle.c (the C restatement of zfec's fec.c), piece ids by
                  hashlib (validator.py:1081) — the reference's own CPU path
  dropin          storb_amd.piece with the caller unchanged: encode_chunk per chunk,
                  piece_hash per piece, reconstruct_data
  dropin_no_prefetch  the same with PREFETCH_PIECE_IDS = False (piece ids hashed serially by
                  the caller, exactly as the reference)
  dropin_round4_host_path  the same with HOST_PIECES = False (round 4's host side: Python piece
                  fills and a hashlib thread pool instead of sec_encode_pieces)
  streamed        the pipelined entry points: encode_chunks_stream(piece_ids=True) and
                  reconstruct_data_stream
"""

from __future__ import annotations

import argparse
import hashlib
import json
import math
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

MIB = float(1 << 20)


def _ref_path():
    """The reference's piece.py logic with the oracle standing in for zfec (pydantic models from
    storb_amd.piece, which mirror piece.py:21-51 field for field)."""
    from oracle import cfec, zfec_ref
    from storb_amd.piece import EncodedChunk, Piece, PieceType

    def encode_chunk(chunk, chunk_idx):  # piece.py:103-166
        n = len(chunk)
        k, m, B, padlen = zfec_ref.chunk_shape(n)
        blocks = cfec.easy_encode(bytes(chunk), k, m)
        pieces = [Piece(piece_type=PieceType.Data if i < k else PieceType.Parity, data=b, chunk_idx=chunk_idx,
                        piece_idx=i) for i, b in enumerate(blocks)]
        return EncodedChunk(pieces=pieces, chunk_idx=chunk_idx, k=k, m=m, chunk_size=B, padlen=padlen,
                            original_chunk_size=n)

    def decode_chunk(ec):  # piece.py:169-198 (positional sharenums: exact when 0..k-1 present)
        use = ec.pieces[:ec.k]
        return cfec.easy_decode([p.data for p in use], list(range(len(use))), ec.padlen, ec.k, ec.m)

    def reconstruct_data(pieces, chunks):  # piece.py:201-236
        out = []
        for chunk in chunks:
            relevant = sorted([p for p in pieces if p.chunk_idx == chunk.chunk_idx], key=lambda p: p.piece_idx)
            if len(relevant) < chunk.k:
                raise ValueError("Not enough pieces")
            chunk.pieces = relevant
            out.append(decode_chunk(chunk))
        return b"".join(out)

    return encode_chunk, (lambda d: hashlib.sha1(d).hexdigest()), reconstruct_data, zfec_ref.piece_length


def loopback(data, encode_chunk, piece_hash, reconstruct_data, piece_length):
    chunk_size = piece_length(len(data))
    store, chunks = {}, []
    for ci in range(math.ceil(len(data) / chunk_size)):
        info = encode_chunk(data[ci * chunk_size:(ci + 1) * chunk_size], ci)
        for p in info.pieces:
            store[piece_hash(p.data)] = p  # validator.py:1081 -> miners
        chunks.append(info.model_copy(update={"pieces": None}))
    pieces = list(store.values())  # retrieval
    return reconstruct_data(pieces, chunks)


def streamed(data):
    from storb_amd import piece

    chunk_size = piece.piece_length(len(data))
    store, chunks = {}, []
    parts = (data[o:o + chunk_size] for o in range(0, len(data), chunk_size))
    for info, ids in piece.encode_chunks_stream(parts, piece_ids=True):
        for p, h in zip(info.pieces, ids):
            store[h] = p
        chunks.append(info.model_copy(update={"pieces": None}))
    return b"".join(piece.reconstruct_data_stream(list(store.values()), chunks))


def timed(fn, data, reps):
    assert fn(data) == data
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn(data)
        ts.append(time.perf_counter() - t0)
    return len(data) / statistics.median(ts) / MIB


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    from storb_amd import piece

    ref = _ref_path()
    drop = (piece.encode_chunk, piece.piece_hash, piece.reconstruct_data, piece.piece_length)
    rng = np.random.default_rng(1)
    res = {"unit": "MiB/s of object bytes (upload + download), median",
           "harness": "tools/c1_loopback.py: encode -> piece ids -> dict 'miners' -> retrieve -> reconstruct"}
    for label, size in (("4MiB_object_8x512KiB_zfec(4,6)", 4 << 20), ("1MiB_object_4x256KiB_zfec(2,3)", 1 << 20)):
        data = rng.integers(0, 256, size, dtype=np.uint8).tobytes()
        r = {"reference_cpu": timed(lambda d: loopback(d, *ref), data, a.reps),
             "dropin": timed(lambda d: loopback(d, *drop), data, a.reps)}
        piece.PREFETCH_PIECE_IDS = False
        try:
            r["dropin_no_prefetch"] = timed(lambda d: loopback(d, *drop), data, a.reps)
        finally:
            piece.PREFETCH_PIECE_IDS = True
        piece.HOST_PIECES = False  # A/B: round 4's Python piece fills and hashlib pool
        try:
            r["dropin_round4_host_path"] = timed(lambda d: loopback(d, *drop), data, a.reps)
        finally:
            piece.HOST_PIECES = True
        r["streamed"] = timed(streamed, data, a.reps)
        res[label] = {k: round(v, 1) for k, v in r.items()}
        res[label]["dropin_over_reference"] = round(r["dropin"] / r["reference_cpu"], 2)
        res[label]["dropin_no_prefetch_over_reference"] = round(r["dropin_no_prefetch"] / r["reference_cpu"], 2)
        res[label]["dropin_round4_over_reference"] = round(r["dropin_round4_host_path"] / r["reference_cpu"], 2)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()

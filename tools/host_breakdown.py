#!/usr/bin/env python3
"""Host-side time breakdown of one drop-in call: where does encode_chunk / decode_chunk spend
its time at storb's real call granularity (one chunk per call, validator.py:1380 / piece.py
:169-198)?  Not product code: it replays the stages of storb_amd.piece / easyfec / engine with
a timer around each, on one MI355X, and prints one JSON object.

    python tools/host_breakdown.py > gpurun_out/host_breakdown.json

Stages (median over `--reps` calls, microseconds):
  encode_chunk:  policy (piece_length + chunk_shape) | split (k data slices as bytes, easyfec's
                 copy) | descs (numpy descriptor + addresses) | c_call (sec_encode_batch: the
                 host path's staging copies, PCIe, kernel, sync) of which kernel (HIP events) |
                 parity_bytes (parity out of the pinned result buffer) | models (pydantic Piece x m
                 + EncodedChunk) | total (the real encode_chunk, timed separately)
  decode_chunk:  sharenums | descs | c_call (sec_decode_batch) of which kernel | out_bytes |
                 total (the real decode_chunk)
  piece_hash:    hashlib SHA-1 of every piece of the chunk (the validator's next step)
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


def med(xs):
    return round(statistics.median(xs) * 1e6, 1)


def encode_stages(eng, piece, chunk, reps):
    from storb_amd._lib import ENC_DTYPE

    st = {k: [] for k in ("policy", "split", "descs", "c_call", "kernel", "parity_bytes", "models", "total")}
    n = len(chunk)
    for _ in range(reps):
        t0 = time.perf_counter()
        piece.piece_length(n)
        k, m, B, padlen = piece.chunk_shape(n)
        t1 = time.perf_counter()
        prim = piece._split(chunk, k, B)
        t2 = time.perf_counter()
        mv = memoryview(chunk).cast("B")
        descs = np.zeros(1, dtype=ENC_DTYPE)
        arr = np.frombuffer(mv, dtype=np.uint8)
        descs[0] = (arr.ctypes.data, n, 0, B, k, m)
        out = eng._out_buffer((m - k) * B)
        t3 = time.perf_counter()
        eng.set_timing(True)
        eng.encode_batch(descs, 0, out, host=True)
        t4 = time.perf_counter()
        eng.set_timing(False)
        kms, kn = eng.collect_timing("encode")
        omv = memoryview(out)
        par = [bytes(omv[r * B:(r + 1) * B]) for r in range(m - k)]
        t5 = time.perf_counter()
        piece._build(0, k, m, B, padlen, n, prim + par)
        t6 = time.perf_counter()
        for key, v in zip(("policy", "split", "descs", "c_call", "parity_bytes", "models"),
                          (t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4, t6 - t5)):
            st[key].append(v)
        st["kernel"].append(kms / 1e3 / max(kn, 1))
    for _ in range(reps):
        t0 = time.perf_counter()
        piece.encode_chunk(chunk, 0)
        st["total"].append(time.perf_counter() - t0)
    return {k: med(v) for k, v in st.items()}


def decode_stages(eng, piece, enc, reps, erase):
    from storb_amd._lib import DEC_DTYPE

    st = {k: [] for k in ("sharenums", "descs", "c_call", "kernel", "out_bytes", "total")}
    ch = enc.model_copy()
    ch.pieces = [p for p in enc.pieces if p.piece_idx not in erase]
    for _ in range(reps):
        t0 = time.perf_counter()
        blocks, sn = piece._sharenums(ch, False)
        t1 = time.perf_counter()
        k, B = ch.k, len(blocks[0])
        descs = np.zeros(1, dtype=DEC_DTYPE)
        descs[0] = (0, B, ch.padlen, 0, k, ch.m)
        bo = np.array([np.frombuffer(b, np.uint8).ctypes.data for b in blocks], np.uint64)
        total = k * B - ch.padlen
        out = eng._out_buffer(total)
        t2 = time.perf_counter()
        eng.set_timing(True)
        eng.decode_batch(descs, np.array(sn, np.int32), bo, 0, out, host=True)
        t3 = time.perf_counter()
        eng.set_timing(False)
        kms, kn = eng.collect_timing("decode")
        bytes(memoryview(out)[:total])
        t4 = time.perf_counter()
        for key, v in zip(("sharenums", "descs", "c_call", "out_bytes"), (t1 - t0, t2 - t1, t3 - t2, t4 - t3)):
            st[key].append(v)
        st["kernel"].append(kms / 1e3 / max(kn, 1))
    for _ in range(reps):
        t0 = time.perf_counter()
        piece.decode_chunk(ch)
        st["total"].append(time.perf_counter() - t0)
    return {k: med(v) for k, v in st.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    import hashlib

    from storb_amd import piece
    from storb_amd.engine import get_engine

    eng = get_engine(0)
    rng = np.random.default_rng(2)
    res = {"unit": "microseconds, median", "reps": a.reps}
    for label, n in (("256KiB_zfec(2,3)", 256 << 10), ("512KiB_zfec(4,6)", 512 << 10), ("1MiB_zfec(4,6)", 1 << 20),
                     ("4MiB_zfec(8,12)", 4 << 20)):
        chunk = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        enc = piece.encode_chunk(chunk, 0)
        k = enc.k
        r = {"encode_chunk": encode_stages(eng, piece, chunk, a.reps),
             "decode_chunk_all_data_present": decode_stages(eng, piece, enc, a.reps, erase=()),
             "decode_chunk_one_data_lost": decode_stages(eng, piece, enc, a.reps, erase=(0,))}
        hs = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            for p in enc.pieces:
                hashlib.sha1(p.data).hexdigest()
            hs.append(time.perf_counter() - t0)
        r["piece_hash_all_pieces"] = med(hs)
        r["shape"] = {"k": k, "m": enc.m, "B": enc.chunk_size}
        res[label] = r
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""where a per-chunk call at storb's own granularity spends its time (C1's
1 MiB object = 4 x 256 KiB chunks, zfec(2,3), 128 KiB pieces; the 4 MiB object = 8 x 512 KiB,
zfec(4,6)).  Medians over --reps calls of each step, in microseconds, on one thread:

  encode_chunk        the drop-in call (storb_amd.piece.encode_chunk); *_round4: with
                      piece.HOST_PIECES = False (round 4's Python fills and hashlib pool)
  piece_ids           hashlib SHA-1 of the chunk's m pieces (validator.py:1081), serial
  ref_encode          the reference's arithmetic restated (oracle/fec_oracle.c easy_encode)
  split               easyfec's k slices (+ pad) as bytes
  encode_host         Engine.encode_host on the chunk (the GPU call + parity as bytes)
  lib_call            sec_encode_batch alone (SEC_F_HOST, pinned result buffer): staging, launch,
                      sync
  lib_call_pinned_in  the same with the chunk already in pinned memory (zero-copy)
  models              the pydantic Piece / EncodedChunk objects (_build)
  decode_chunk_lost0  decode_chunk with piece 0 lost (one GPU recover)
  ref_decode_lost0    the oracle's decode of the same blocks

    python tools/small_call_profile.py [--reps 200] > gpurun_out/small_calls.json
"""

from __future__ import annotations

import argparse
import hashlib
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def med_us(fn, reps):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(statistics.median(ts) * 1e6, 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    a = ap.parse_args()
    from oracle import cfec
    from storb_amd import piece
    from storb_amd._lib import ENC_DTYPE
    from storb_amd.engine import get_engine

    eng = get_engine()
    res = {"unit": "us per call, median", "reps": a.reps}
    for label, n in (("256KiB_chunk_zfec(2,3)", 256 << 10), ("512KiB_chunk_zfec(4,6)", 512 << 10),
                     ("1MiB_chunk_zfec(4,6)", 1 << 20), ("8MiB_chunk_zfec(16,24)", 8 << 20)):
        chunk = np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8).tobytes()
        k, m, B, padlen = piece.chunk_shape(n)
        r = {"k": k, "m": m, "B": B}
        for hp in (True, False):  # sec_encode_pieces (HOST_PIECES) against round 4's host side
            piece.HOST_PIECES = hp
            sfx = "" if hp else "_round4"
            r["encode_chunk" + sfx] = med_us(lambda: piece.encode_chunk(chunk, 0), a.reps)
            # a fresh piece-id memo: the loop above took no ids, so the memo would have paused
            # prefetching (its idle rule) and most of the next loop would hash serially
            piece._memo = piece._PieceIdMemo()
            r["encode_chunk_plus_ids" + sfx] = med_us(
                lambda: [piece.piece_hash(p.data) for p in piece.encode_chunk(chunk, 0).pieces], a.reps)
        piece.HOST_PIECES = True
        ec = piece.encode_chunk(chunk, 0)
        datas = [p.data for p in ec.pieces]
        r["piece_ids"] = med_us(lambda: [hashlib.sha1(d).hexdigest() for d in datas], a.reps)
        r["ref_encode"] = med_us(lambda: cfec.easy_encode(chunk, k, m), a.reps)
        r["split"] = med_us(lambda: piece._split(chunk, k, B), a.reps)
        r["encode_host"] = med_us(lambda: eng.encode_host([chunk], [(k, m)]), a.reps)
        d = np.zeros(1, dtype=ENC_DTYPE)
        src = np.frombuffer(chunk, np.uint8)
        out = eng.host_empty((m - k) * B)
        d[0] = (src.ctypes.data, n, 0, B, k, m)
        r["lib_call"] = med_us(lambda: eng.encode_batch(d, 0, out, host=True), a.reps)
        pin = eng.host_empty(n)
        pin[:] = src
        dp = d.copy()
        dp["in_off"] = pin.ctypes.data
        r["lib_call_pinned_in"] = med_us(lambda: eng.encode_batch(dp, 0, out, host=True), a.reps)
        r["models"] = med_us(lambda: piece._build(0, k, m, B, padlen, n, datas), a.reps)
        lost = [p for p in ec.pieces if p.piece_idx != 0]
        dec = ec.model_copy(update={"pieces": lost})
        assert piece.decode_chunk(dec) == chunk
        r["decode_chunk_lost0"] = med_us(lambda: piece.decode_chunk(dec), a.reps)
        blocks = [p.data for p in lost][:k]
        sn = [p.piece_idx for p in lost][:k]
        r["ref_decode_lost0"] = med_us(lambda: cfec.easy_decode(blocks, sn, padlen, k, m), a.reps)
        r["host_paths"] = list(eng.host_paths())
        res[label] = r
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()

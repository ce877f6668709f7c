#!/usr/bin/env python3
"""Measures every BASELINE.json config on one MI355X (C4 at its per-GPU share) and prints one
JSON object.  Complements bench.py (which is the C2+C3 headline line).

    python tools/bench_configs.py > gpurun_out/configs.json

C1  see tools/c1_loopback.py.
C2/C3  1024 x 1 MiB RS(4,2) encode / decode ({1,3} erased), device-resident; C3 also over
    the erasure sets of SURVEY 8(d) (c3_patterns), reassemble and recover-only.
Policy shapes for 1 GiB / 16 GiB / 1 TiB files: zfec(16,24), (32,48), (64,96) on 8 / 32 / 256
    MiB chunks, 1 GiB per case.
C4  8192 x 64 KiB RS(10,4) (one GPU's share of 65536), device-resident encode / decode with
    data blocks {0,2,5,7} erased (block 9, zfec's padded one, read in place: avail = B - padlen).
C5  mixed chunk sizes log-uniform in [4 KiB, 4 MiB] (seed 5) up to ~1 GiB, RS(8,3):
    device-resident encode / decode (blocks {1,3,5} erased, block 7 read in place) and end-to-end from host memory
    (pageable buffers, staged; and pinned buffers, zero-copy).
"""

from __future__ import annotations

import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

GIB = float(1 << 30)
MIB = float(1 << 20)


def timed(fn, reps):
    fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t0) / reps


# ---------------------------------------------------------------- device-resident
def enc_descs_var(sizes, k, m):
    from storb_amd._lib import ENC_DTYPE

    sizes = np.asarray(sizes, dtype=np.uint64)
    B = (sizes + k - 1) // k
    d = np.zeros(len(sizes), dtype=ENC_DTYPE)
    d["in_off"] = np.concatenate([[0], np.cumsum(sizes)[:-1]])
    d["n"] = sizes
    d["parity_off"] = np.concatenate([[0], np.cumsum(B * (m - k))[:-1]])
    d["parity_stride"] = B
    d["k"], d["m"] = k, m
    return d, B


def dec_descs_var(sizes, k, m, B, data_base, par_base, erased):
    """Decode descriptors + per-slot avail (an in-place block k-1 has B - padlen bytes)."""
    from storb_amd._lib import DEC_DTYPE

    keep = [s for s in range(m) if s not in erased][:k]
    n = len(sizes)
    sizes = np.asarray(sizes, dtype=np.uint64)
    in_off = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
    par_off = np.concatenate([[0], np.cumsum(B * (m - k))[:-1]]).astype(np.uint64)
    d = np.zeros(n, dtype=DEC_DTYPE)
    d["out_off"] = in_off
    d["B"] = B
    d["padlen"] = B * k - sizes
    d["slot0"] = np.arange(n, dtype=np.uint64) * k
    d["k"], d["m"] = k, m
    sn = np.tile(np.array(keep, np.int32), n)
    offs = np.zeros(n * k, np.uint64)
    avail = np.zeros(n * k, np.uint64)
    for j, s in enumerate(keep):
        offs[j::k] = (data_base + in_off + s * B) if s < k else (par_base + par_off + (s - k) * B)
        avail[j::k] = (sizes - (k - 1) * B) if s == k - 1 else B
    return d, sn, offs, avail


def c5_sizes() -> list[int]:
    """BASELINE configs[4] chunk sizes: log-uniform integers in [4 KiB, 4 MiB], seed 5, ~1 GiB."""
    r5 = np.random.default_rng(5)
    sizes, tot = [], 0
    while tot < (1 << 30):
        s = int(np.exp(r5.uniform(np.log(4096), np.log(4 << 20))))
        sizes.append(s)
        tot += s
    return sizes


def device_case(eng, sizes, k, m, erased, reps=20):
    import torch

    total = int(np.sum(sizes))
    ed, B = enc_descs_var(sizes, k, m)
    src = torch.randint(0, 256, (total,), dtype=torch.uint8, device="cuda")
    par = torch.empty(int(np.sum(B)) * (m - k), dtype=torch.uint8, device="cuda")
    out = torch.empty_like(src)
    dd, sn, offs, av = dec_descs_var(sizes, k, m, B, src.data_ptr(), par.data_ptr(), erased)
    eng.encode_batch(ed, src, par)
    eng.decode_batch(dd, sn, offs, 0, out, block_avail=av)
    assert torch.equal(out, src)
    eng.set_timing(True)
    for _ in range(reps):
        eng.encode_batch(ed, src, par, asynchronous=True)
    for _ in range(reps):
        eng.decode_batch(dd, sn, offs, 0, out, block_avail=av, asynchronous=True)
    eng.sync()
    eng.set_timing(False)
    ems, en = eng.collect_timing("encode")
    dms, dn = eng.collect_timing("decode")
    te, td = ems / en / 1e3, dms / dn / 1e3
    enc_bytes = total + int(np.sum(B)) * (m - k)
    dec_bytes = int(np.sum(B)) * k + total
    return {"chunks": len(sizes), "input_bytes": total, "encode_ms": round(te * 1e3, 4),
            "encode_gibs": round(total / te / GIB, 2), "encode_hbm_GBs": round(enc_bytes / te / 1e9, 1),
            "decode_ms": round(td * 1e3, 4), "decode_gibs": round(total / td / GIB, 2),
            "decode_hbm_GBs": round(dec_bytes / td / 1e9, 1)}


C3_PATTERNS = ((1, 3), (0, 1), (2, 3), (1, 4), (0, 5), (4, 5))


def c3_patterns(eng, nch=1024, n=1 << 20, k=4, m=6, reps=10, rounds=5):
    """C3 decode over several erasure sets: two data blocks ({1,3}, {0,1}, {2,3}),
    a data block and a parity block ({1,4}, {0,5}: one row recovered) and both parity blocks
    ({4,5}: a pure reassembly).  Reassemble (kB read + n written) and recover-only (kB read +
    eB written) kernel rates, outputs checked against the source bytes.  The patterns are
    timed round-robin, `rounds` times `reps` launches each, median per pattern (timed one after
    the other, the first pattern of a process measured up to 5 % low)."""
    import torch

    sizes = [n] * nch
    ed, B = enc_descs_var(sizes, k, m)
    B = int(B[0])
    src = torch.randint(0, 256, (nch * n,), dtype=torch.uint8, device="cuda")
    par = torch.empty(nch * (m - k) * B, dtype=torch.uint8, device="cuda")
    out = torch.empty_like(src)
    eng.encode_batch(ed, src, par)
    cases = []  # (name, mode, bytes per launch, launch function)
    for erased in C3_PATTERNS:
        name = "{" + ",".join(map(str, erased)) + "}"
        dd, sn, offs, av = dec_descs_var(sizes, k, m, np.full(nch, B, np.uint64), src.data_ptr(), par.data_ptr(), erased)
        out.zero_()
        eng.decode_batch(dd, sn, offs, 0, out, block_avail=av)
        assert torch.equal(out, src), erased
        cases.append((name, "reassemble", nch * (k * B + n),
                      lambda dd=dd, sn=sn, offs=offs, av=av: eng.decode_batch(dd, sn, offs, 0, out, block_avail=av,
                                                                                 asynchronous=True)))
        lost = sorted(s for s in erased if s < k)
        if lost:
            e = len(lost)
            rd = dd.copy()
            rd["out_off"] = np.arange(nch, dtype=np.uint64) * (e * B)
            rec = torch.empty(nch * e * B, dtype=torch.uint8, device="cuda")
            eng.decode_batch(rd, sn, offs, 0, rec, block_avail=av, recover_only=True)
            r3, s3 = rec.view(nch, e, B), src.view(nch, k, B)
            for j, blk in enumerate(lost):
                assert torch.equal(r3[:, j], s3[:, blk]), (erased, blk)
            cases.append((name, "recover_only", nch * (k + e) * B,
                          lambda rd=rd, sn=sn, offs=offs, av=av, rec=rec: eng.decode_batch(
                              rd, sn, offs, 0, rec, block_avail=av, recover_only=True, asynchronous=True)))
    samples = {(c[0], c[1]): [] for c in cases}
    for _ in range(rounds):
        for name, mode, _, fn in cases:
            eng.set_timing(True)
            for _ in range(reps):
                fn()
            eng.sync()
            eng.set_timing(False)
            ms, nl = eng.collect_timing("decode")
            samples[(name, mode)].append(ms / nl / 1e3)
    res = {}
    for name, mode, nbytes, _ in cases:
        t = float(np.median(samples[(name, mode)]))
        res.setdefault(name, {}).update({f"{mode}_ms": round(t * 1e3, 4), f"{mode}_hbm_GBs": round(nbytes / t / 1e9, 1)})
    return res


def sha1_case(eng, nch=1024, n=1 << 20, k=4, m=6, reps=5):
    """F1: SHA-1 of all m pieces of every C2 chunk on the device, alone and fused after encode."""
    import torch

    from storb_amd._lib import MSG_DTYPE

    ed, B = enc_descs_var([n] * nch, k, m)
    B = int(B[0])
    src = torch.randint(0, 256, (nch * n,), dtype=torch.uint8, device="cuda")
    par = torch.empty(nch * (m - k) * B, dtype=torch.uint8, device="cuda")
    dig = torch.empty(nch * m * 20, dtype=torch.uint8, device="cuda")
    msgs = np.zeros(nch * m, dtype=MSG_DTYPE)
    ci = np.arange(nch, dtype=np.uint64)
    for j in range(m):
        msgs["addr"][j::m] = (src.data_ptr() + ci * n + j * B) if j < k else (par.data_ptr() + ci * (m - k) * B + (j - k) * B)
    msgs["len"] = B
    msgs["avail"] = B
    eng.encode_batch(ed, src, par)
    t_sha = timed(lambda: eng.sha1_batch(msgs, dig), reps)
    t_enc = timed(lambda: eng.encode_batch(ed, src, par), reps)
    t_both = timed(lambda: eng.encode_digest_batch(ed, src, par, dig), reps)
    hsrc = src.cpu().numpy()
    hd, hp = dig.cpu().numpy().reshape(-1, 20), par.cpu().numpy()
    for i in (0, 1, nch * m - 1):  # a fast wrong digest is not a result
        c, j = divmod(i, m)
        piece = hsrc[c * n + j * B:c * n + (j + 1) * B] if j < k else hp[(c * (m - k) + j - k) * B:(c * (m - k) + j - k + 1) * B]
        assert hd[i].tobytes() == hashlib.sha1(piece.tobytes()).digest(), i
    hpar = np.empty(nch * (m - k) * B, dtype=np.uint8)
    hdig = np.empty(nch * m * 20, dtype=np.uint8)
    t_host = timed(lambda: eng.encode_digest_batch(ed, hsrc, hpar, hdig, host=True), 2)
    hashed = nch * m * B
    return {"pieces": nch * m, "piece_bytes": B, "sha1_ms": round(t_sha * 1e3, 3),
            "sha1_GBs": round(hashed / t_sha / 1e9, 1), "encode_ms": round(t_enc * 1e3, 3),
            "encode_plus_sha1_fused_ms": round(t_both * 1e3, 3),
            "e2e_host_encode_plus_sha1_gibs": round(nch * n / t_host / GIB, 2),
            "note": "wall time per call incl. launch + sync; SHA-1 is sequential per message: one lane per piece, or for few long pieces (as here) two waves per 64 pieces (schedule + rounds)"}


def host_case(eng, sizes, k, m, erased, reps=3, pinned=False):
    """End to end from host memory: pageable numpy buffers (staged through the library's pinned
    slabs) or, with pinned=True, Engine.host_empty buffers (the zero-copy path)."""
    total = int(np.sum(sizes))
    rng = np.random.default_rng(55)
    ed, B = enc_descs_var(sizes, k, m)
    nb = int(np.sum(B)) * (m - k)
    if pinned:
        host, par, out = eng.host_empty(total), eng.host_empty(nb), eng.host_empty(total)
        host[:] = rng.integers(0, 256, total, dtype=np.uint8)
    else:
        host = rng.integers(0, 256, total, dtype=np.uint8)
        par = np.empty(nb, dtype=np.uint8)
        out = np.empty_like(host)
    dd, sn, offs, av = dec_descs_var(sizes, k, m, B, host.ctypes.data, par.ctypes.data, erased)
    te = timed(lambda: eng.encode_batch(ed, host, par, host=True), reps)
    td = timed(lambda: eng.decode_batch(dd, sn, offs, 0, out, block_avail=av, host=True), reps)
    assert np.array_equal(out, host)
    return {"encode_gibs": round(total / te / GIB, 2), "decode_gibs": round(total / td / GIB, 2)}


def main():
    from storb_amd.engine import Engine

    eng = Engine(0)
    res = {}

    res["c2_c3_1024x1MiB_rs(4,2)"] = device_case(eng, [1 << 20] * 1024, 4, 6, (1, 3))
    res["c3_erasure_patterns_1024x1MiB_rs(4,2)"] = c3_patterns(eng)
    # the policy's shapes for large files at their own chunk sizes, 1 GiB each,
    # half as many data blocks lost as there are parity blocks
    for chunk, k, m in ((8 << 20, 16, 24), (32 << 20, 32, 48), (256 << 20, 64, 96)):
        res[f"policy_{chunk >> 20}MiB_chunks_zfec({k},{m})"] = device_case(
            eng, [chunk] * ((1 << 30) // chunk), k, m, tuple(range(0, m - k, 2)), reps=10)
    res["c4_8192x64KiB_rs(10,4)_per_gpu"] = device_case(eng, [65536] * 8192, 10, 14, (0, 2, 5, 7))
    sizes = c5_sizes()
    res["c5_mixed_4KiB-4MiB_rs(8,3)_device"] = device_case(eng, sizes, 8, 11, (1, 3, 5))
    res["c5_mixed_4KiB-4MiB_rs(8,3)_e2e_host"] = host_case(eng, sizes, 8, 11, (1, 3, 5))
    res["c5_mixed_4KiB-4MiB_rs(8,3)_e2e_host_pinned"] = host_case(eng, sizes, 8, 11, (1, 3, 5), pinned=True)
    res["c2_1024x1MiB_rs(4,2)_e2e_host"] = host_case(eng, [1 << 20] * 1024, 4, 6, (1, 3))
    res["c2_1024x1MiB_rs(4,2)_e2e_host_pinned"] = host_case(eng, [1 << 20] * 1024, 4, 6, (1, 3), pinned=True)
    res["f1_sha1_pieces_c2_device"] = sha1_case(eng)
    import hashlib
    blob = np.random.default_rng(3).integers(0, 256, 1 << 28, dtype=np.uint8).tobytes()
    t0 = time.perf_counter()
    hashlib.sha1(blob).digest()
    res["f1_cpu_hashlib_sha1_1thread_GBs"] = round(len(blob) / (time.perf_counter() - t0) / 1e9, 2)
    print(json.dumps(res, indent=1))
    eng.close()


if __name__ == "__main__":
    main()

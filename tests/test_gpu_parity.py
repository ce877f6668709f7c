"""GPU parity: the HIP kernels (through the C ABI) against the CPU oracle, bit-exact.

* golden fixtures (tests/golden/golden.json) and oracle/fec_oracle.c on seeded inputs at sizes
  the oracle finishes in seconds, covering aligned and unaligned block sizes, the zero-padded
  last block, tiny chunks, m == k, and row groups beyond 8 (p > 8, e > 8);
* BASELINE.json's full sizes (1024 x 1 MiB RS(4,2); RS(10,4) 64 KiB chunks; mixed RS(8,3))
  through size-independent properties — encode -> erase -> decode round trips over every
  chunk — plus oracle comparison on a sample of chunks.
"""

import hashlib
import itertools
import json
import os
import random

import numpy as np
import pytest

from oracle import cfec

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))

from storb_amd._lib import DEC_DTYPE, ENC_DTYPE  # noqa: E402


def sha(b):
    return hashlib.sha256(b).hexdigest()


def oracle_parity(data, k, m):
    return cfec.easy_encode(bytes(data), k, m)[k:]


# ---------------------------------------------------------------- host-mode path
def test_encode_golden(engine):
    ents = GOLDEN["encode"]
    chunks = [random.Random(e["seed"]).randbytes(e["n"]) for e in ents]
    par = engine.encode_host(chunks, [(e["k"], e["m"]) for e in ents])
    for e, p in zip(ents, par):
        assert [sha(b) for b in p] == e["blocks_sha256"][e["k"]:], (e["k"], e["m"], e["n"])


def test_decode_golden(engine):
    for e in GOLDEN["decode"]:
        k, m, sn = e["k"], e["m"], e["sharenums"]
        data = random.Random(e["seed"]).randbytes(e["n"])
        blocks = cfec.easy_encode(data, k, m)
        pad = len(blocks[0]) * k - len(data)
        got = engine.decode_host([(k, m, [blocks[s] for s in sn], sn, pad)])
        assert sha(got) == e["out_sha256"]


@pytest.mark.parametrize("k,m", [(1, 2), (2, 3), (3, 4), (4, 6), (5, 8), (8, 11), (10, 14), (8, 16), (12, 20),
                                 (16, 24), (20, 30), (32, 48), (64, 96), (4, 4), (7, 256),
                                 (128, 256), (255, 256)])
def test_encode_random_sizes_vs_oracle(engine, k, m):
    rng = random.Random(k * 1000 + m)
    sizes = [k, k * k, 4095, 4096 * k, 4096 * k + 1, 65536, 65536 + 7, 6554 * k - 3, 262144 + 13, 1 << 20]
    sizes += [rng.randrange(k * k, 300000) for _ in range(6)]
    sizes = [n for n in sizes if -(-n // k) * (k - 1) <= n]
    chunks = [rng.randbytes(n) for n in sizes]
    par = engine.encode_host(chunks, [(k, m)] * len(chunks))
    for c, p in zip(chunks, par):
        assert p == oracle_parity(c, k, m), (k, m, len(c))


def test_encode_mixed_shapes_one_batch(engine):
    rng = random.Random(5)
    shapes = [(1, 2), (2, 3), (4, 6), (8, 11), (10, 14), (16, 24), (3, 12)]
    chunks, km = [], []
    for i in range(60):
        k, m = shapes[i % len(shapes)]
        n = rng.randrange(max(k * k, 1), 200000)
        chunks.append(rng.randbytes(n))
        km.append((k, m))
    par = engine.encode_host(chunks, km)
    for c, (k, m), p in zip(chunks, km, par):
        assert p == oracle_parity(c, k, m)


@pytest.mark.parametrize("k,m", [(2, 3), (4, 6), (8, 11), (10, 14), (16, 24), (16, 40), (32, 48), (64, 96),
                                 (3, 256), (128, 256)])
def test_decode_erasures_vs_oracle(engine, k, m):
    rng = random.Random(k + 100 * m)
    items, expect = [], []
    for n in [k * k, 4096 * k - 5, 65536 + 3, 6554 * k, 300001]:
        if -(-n // k) * (k - 1) > n:
            continue
        data = rng.randbytes(n)
        blocks = cfec.easy_encode(data, k, m)
        B = len(blocks[0])
        for _ in range(4):
            sn = rng.sample(range(m), k)
            items.append((k, m, [blocks[s] for s in sn], sn, B * k - n))
            expect.append(data)
    got = engine.decode_host(items)
    assert got == b"".join(expect)
    # each case also equals the oracle's own decode (same bytes by construction)
    k0, m0, bl, sn, pad = items[-1]
    assert cfec.easy_decode(bl, sn, pad, k0, m0) == expect[-1]


def test_decode_every_pattern_rs42(engine):
    data = random.Random(9).randbytes(1 << 20)
    blocks = cfec.easy_encode(data, 4, 6)
    items = []
    for sub in itertools.combinations(range(6), 4):
        for order in (list(sub), list(reversed(sub))):
            items.append((4, 6, [blocks[s] for s in order], order, 0))
    got = engine.decode_host(items)
    assert got == data * len(items)


def test_empty_and_degenerate(engine):
    assert engine.encode_host([b""], [(4, 6)]) == [[b"", b""]]
    assert engine.encode_host([b"\x07"], [(1, 2)]) == [[b"\x07"]]  # zfec(1,2) parity = copy
    assert engine.encode_host([b"abcdefgh"], [(4, 4)]) == [[]]
    assert engine.decode_host([(1, 2, [b"\x07"], [1], 0)]) == b"\x07"


# ---------------------------------------------------------------- device-resident path
def _dev(nbytes, seed):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    return torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device="cuda", generator=g)


def _enc_descs(nchunks, n, k, m):
    B = -(-n // k)
    d = np.zeros(nchunks, dtype=ENC_DTYPE)
    d["in_off"] = np.arange(nchunks, dtype=np.uint64) * n
    d["n"] = n
    d["parity_off"] = np.arange(nchunks, dtype=np.uint64) * (m - k) * B
    d["parity_stride"] = B
    d["k"] = k
    d["m"] = m
    return d, B


def _dec_inputs(nchunks, n, k, m, B, erased, data_base, par_base):
    """Descriptors reading the surviving blocks straight from the encoded device buffers
    (an in-place last data block is short by padlen bytes, so it must be among the erased)."""
    assert B * k == n or (k - 1) in erased
    keep = [s for s in range(m) if s not in erased][:k]
    d = np.zeros(nchunks, dtype=DEC_DTYPE)
    d["out_off"] = np.arange(nchunks, dtype=np.uint64) * n
    d["B"] = B
    d["padlen"] = B * k - n
    d["slot0"] = np.arange(nchunks, dtype=np.uint64) * k
    d["k"] = k
    d["m"] = m
    sn = np.tile(np.array(keep, np.int32), nchunks)
    offs = np.zeros(nchunks * k, np.uint64)
    for j, s in enumerate(keep):
        ci = np.arange(nchunks, dtype=np.uint64)
        if s < k:
            offs[j::k] = data_base + ci * n + s * B
        else:
            offs[j::k] = par_base + ci * (m - k) * B + (s - k) * B
    return d, sn, offs


def _roundtrip_full(engine, nchunks, n, k, m, erased, sample):
    src = _dev(nchunks * n, seed=n + k)
    d, B = _enc_descs(nchunks, n, k, m)
    par = torch.empty(nchunks * (m - k) * B, dtype=torch.uint8, device="cuda")
    engine.encode_batch(d, src, par)
    # oracle on a sample of chunks
    src_h = src.cpu().numpy()
    par_h = par.cpu().numpy()
    for ci in sample:
        want = oracle_parity(src_h[ci * n:(ci + 1) * n].tobytes(), k, m)
        got = par_h[ci * (m - k) * B:(ci + 1) * (m - k) * B].tobytes()
        assert got == b"".join(want), ci
    # size-independent property over EVERY chunk: erase, decode, compare to the source
    out = torch.empty(nchunks * n, dtype=torch.uint8, device="cuda")
    dd, sn, offs = _dec_inputs(nchunks, n, k, m, B, erased, src.data_ptr(), par.data_ptr())
    engine.decode_batch(dd, sn, offs, 0, out)
    assert torch.equal(out, src)
    # linearity of the whole batch: parity(src ^ x) == parity(src) ^ parity(x)
    x = _dev(nchunks * n, seed=1234)
    px = torch.empty_like(par)
    pxs = torch.empty_like(par)
    engine.encode_batch(d, x, px)
    engine.encode_batch(d, src ^ x, pxs)
    assert torch.equal(pxs, par ^ px)


def test_c2_c3_full_size_rs42(engine):
    # BASELINE configs[1] / configs[2]: 1024 x 1 MiB, RS(4,2) = zfec(4,6), data shards {1,3} erased
    _roundtrip_full(engine, 1024, 1 << 20, 4, 6, erased={1, 3}, sample=[0, 1, 511, 1023])


def test_c4_shape_rs104_unaligned(engine):
    # BASELINE configs[3] per-GPU share at reduced count: 64 KiB chunks, RS(10,4): B = 6554 (unaligned)
    _roundtrip_full(engine, 1024, 65536, 10, 14, erased={0, 5, 9, 2}, sample=[0, 3, 777, 1023])


def test_decode_parity_only_and_more_than_8_missing(engine):
    # k=16 with 16 parity rows: decode from parity only (e = 16 > 8 -> two row groups)
    _roundtrip_full(engine, 16, 16 * 4096 * 3 + 5 * 16, 16, 32, erased=set(range(16)), sample=[0, 15])


def test_external_stream_async_and_timing(engine):
    n, k, m, nch = 1 << 20, 4, 6, 64
    src = _dev(nch * n, seed=3)
    d, B = _enc_descs(nch, n, k, m)
    par1 = torch.empty(nch * 2 * B, dtype=torch.uint8, device="cuda")
    par2 = torch.empty_like(par1)
    engine.encode_batch(d, src, par1)
    s = torch.cuda.Stream()
    engine.set_stream(s)
    engine.set_timing(True)
    try:
        engine.encode_batch(d, src, par2, asynchronous=True)
        s.synchronize()
        ms, launches = engine.collect_timing("encode")
        assert launches == 1 and ms > 0
    finally:
        engine.set_timing(False)
        engine.set_stream(None)
    assert torch.equal(par1, par2)


def test_c5_mixed_sizes_host_e2e(engine):
    # BASELINE configs[4] at reduced total: sizes log-uniform in [4 KiB, 4 MiB], RS(8,3) = zfec(8,11)
    rng = np.random.default_rng(5)
    sizes = np.exp(rng.uniform(np.log(4096), np.log(4 << 20), 48)).astype(int).tolist()
    chunks = [rng.integers(0, 256, s, dtype=np.uint8).tobytes() for s in sizes]
    par = engine.encode_host(chunks, [(8, 11)] * len(chunks))
    for c, p in zip(chunks, par):
        assert p == oracle_parity(c, 8, 11)
    items = []
    for i, (c, p) in enumerate(zip(chunks, par)):
        B = len(p[0])
        blocks = [c[j * B:(j + 1) * B].ljust(B, b"\0") for j in range(8)] + p
        sn = sorted(random.Random(i).sample(range(11), 8))
        items.append((8, 11, [blocks[s] for s in sn], sn, B * 8 - len(c)))
    assert engine.decode_host(items) == b"".join(chunks)


def test_decode_odd_padlen_and_tiny_blocks(engine):
    """padlen > B (several short output rows), B < 16 (tail-only chunks), valid < 16."""
    rng = random.Random(21)
    items, expect = [], []
    for k, m, n in [(4, 6, 4096), (10, 14, 100), (16, 24, 16 * 20), (3, 5, 7), (8, 11, 8 * 15 + 1), (5, 8, 5 * 17)]:
        data = rng.randbytes(n)
        blocks = cfec.easy_encode(data, k, m)
        B = len(blocks[0])
        for pad in sorted({B * k - n, min(B * k, B + 3), B * k}):
            sn = rng.sample(range(m), k)
            items.append((k, m, [blocks[s] for s in sn], sn, pad))
            expect.append(cfec.easy_decode([blocks[s] for s in sn], sn, pad, k, m))
    assert engine.decode_host(items) == b"".join(expect)


def test_encode_ragged_tails_many_shapes(engine):
    """Every padlen 0..k-1 for several k, block sizes around the 16-byte lane and 4 KiB tile edges."""
    rng = random.Random(22)
    chunks, km = [], []
    for k, m in [(3, 5), (10, 14), (16, 24), (64, 96)]:
        for B in (1, 15, 16, 17, 4095, 4096, 4097, 16384 + 5):
            for pad in range(0, k, max(1, k // 4)):
                n = B * k - pad
                if n <= 0 or -(-n // k) * (k - 1) > n:
                    continue
                chunks.append(rng.randbytes(n))
                km.append((k, m))
    par = engine.encode_host(chunks, km)
    for c, (k, m), p in zip(chunks, km, par):
        assert p == oracle_parity(c, k, m), (k, m, len(c))


def test_host_pipeline_many_slabs():
    """SEC_F_HOST batches cut into many 1 MiB slabs (chunks straddling slab limits, a chunk
    bigger than a slab, two pipeline slots cycling) — encode, decode and SHA-1."""
    import hashlib

    from storb_amd.engine import Engine

    eng = Engine(0, options={"SEC_SLAB_BYTES": 1 << 20, "SEC_SLAB_BYTES_DIGEST": 1 << 20})
    try:
        rng = random.Random(31)
        sizes = [rng.randrange(1000, 600000) for _ in range(30)] + [3 << 20, 5, 4096 * 10 + 3]
        chunks, km = [], []
        for i, n in enumerate(sizes):
            k, m = [(4, 6), (10, 14), (2, 3), (8, 11)][i % 4]
            if -(-n // k) * (k - 1) > n:
                k, m = 1, 2
            chunks.append(rng.randbytes(n))
            km.append((k, m))
        par, digs = eng.encode_host(chunks, km, digests=True)
        items = []
        for c, (k, m), p, d in zip(chunks, km, par, digs):
            blocks = cfec.easy_encode(c, k, m)
            assert p == blocks[k:]
            assert d == [hashlib.sha1(b).digest() for b in blocks]
            sn = rng.sample(range(m), k)
            items.append((k, m, [blocks[s] for s in sn], sn, len(blocks[0]) * k - len(c)))
        assert eng.decode_host(items) == b"".join(chunks)
        assert eng.sha1_host(chunks) == [hashlib.sha1(c).digest() for c in chunks]
    finally:
        eng.close()


def test_engines_in_threads():
    """One context per host thread (the C ABI's threading contract), running concurrently."""
    import threading

    from storb_amd.engine import get_engine

    errors = []

    def work(seed):
        try:
            rng = random.Random(seed)
            eng = get_engine(0)
            for _ in range(3):
                chunks = [rng.randbytes(rng.randrange(4096, 300000)) for _ in range(8)]
                par = eng.encode_host(chunks, [(4, 6)] * 8)
                for c, p in zip(chunks, par):
                    assert p == oracle_parity(c, 4, 6)
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    ts = [threading.Thread(target=work, args=(s,)) for s in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors


# ---------------------------------------------------------------- pinned host buffers (zero-copy)
def test_zero_copy_pinned_buffers_and_host_rewrites():
    """SEC_F_HOST on pinned buffers runs the kernels on host memory directly.  The host rewrites
    the same pinned input between calls: every call must see the new bytes (no stale device
    cache lines), and the parity / reassembled output must be visible to the host on return."""
    from storb_amd.engine import Engine

    eng = Engine(0)
    try:
        nch, n, k, m = 48, 65536 + 37, 4, 6  # ragged: padlen > 0, unaligned blocks
        B = -(-n // k)
        d = _enc_descs(nch, n, k, m)[0]
        hin, hpar, hout = eng.host_empty(nch * n), eng.host_empty(nch * (m - k) * B), eng.host_empty(nch * n)
        rng = np.random.default_rng(40)
        z0, r0, s0 = eng.host_paths()
        for rep in range(3):
            hin[:] = rng.integers(0, 256, hin.size, dtype=np.uint8)
            eng.encode_batch(d, hin, hpar, host=True)
            for ci in (0, 17, nch - 1):
                want = oracle_parity(hin[ci * n:(ci + 1) * n].tobytes(), k, m)
                assert hpar[ci * (m - k) * B:(ci + 1) * (m - k) * B].tobytes() == b"".join(want), (rep, ci)
            # decode from data blocks 0, 1 (in place) and both parity blocks: block 3 (short,
            # padded) and block 2 are erased
            keep = [0, 1, 4, 5]
            dd = np.zeros(nch, dtype=DEC_DTYPE)
            dd["out_off"] = np.arange(nch, dtype=np.uint64) * n
            dd["B"], dd["padlen"], dd["k"], dd["m"] = B, B * k - n, k, m
            dd["slot0"] = np.arange(nch, dtype=np.uint64) * k
            sn = np.tile(np.array(keep, np.int32), nch)
            offs = np.zeros(nch * k, np.uint64)
            ci = np.arange(nch, dtype=np.uint64)
            for j, s in enumerate(keep):
                offs[j::k] = (hin.ctypes.data + ci * n + s * B) if s < k else \
                    (hpar.ctypes.data + ci * (m - k) * B + (s - k) * B)
            hout[:] = 0
            eng.decode_batch(dd, sn, offs, 0, hout, host=True)
            assert np.array_equal(hout, hin), rep
        z1, r1, s1 = eng.host_paths()
        assert (z1 - z0, r1 - r0, s1 - s0) == (6, 0, 0)
        # pinned input, pageable output: not zero-copy on the caller's pins alone (the call
        # either locks the output pages itself or is staged); same bytes either way
        par2 = np.empty(hpar.size, dtype=np.uint8)
        eng.encode_batch(d, hin, par2, host=True)
        assert np.array_equal(par2, hpar)
        z2, r2, s2 = eng.host_paths()
        assert z2 == z1 and (r2 - r1) + (s2 - s1) == 1
    finally:
        eng.close()


def test_staged_flag_never_locks():
    """SEC_F_STAGED (engine staged=True): a large pageable call that would be page-locked is
    staged instead, pinned buffers stay zero-copy, the bytes are the same; the flag without
    SEC_F_HOST is rejected."""
    from storb_amd import _lib
    from storb_amd.engine import Engine

    eng = Engine(0)
    try:
        nch, n, k, m = 8, (1 << 20) + 11, 16, 24  # 8 MiB of pageable input: above SEC_REGISTER_MIN
        B = -(-n // k)
        d = _enc_descs(nch, n, k, m)[0]
        rng = np.random.default_rng(41)
        src = rng.integers(0, 256, nch * n, dtype=np.uint8)
        par_locked = np.zeros(nch * (m - k) * B, np.uint8)
        par_staged = np.zeros_like(par_locked)
        z0, r0, s0 = eng.host_paths()
        eng.encode_batch(d, src, par_locked, host=True)
        z1, r1, s1 = eng.host_paths()
        eng.encode_batch(d, src, par_staged, host=True, staged=True)
        z2, r2, s2 = eng.host_paths()
        assert (z2 - z1, r2 - r1, s2 - s1) == (0, 0, 1), ((z0, r0, s0), (z1, r1, s1), (z2, r2, s2))
        assert np.array_equal(par_locked, par_staged)
        want = oracle_parity(src[:n].tobytes(), k, m)
        assert par_staged[:(m - k) * B].tobytes() == b"".join(want)
        hin, hpar = eng.host_empty(nch * n), eng.host_empty(par_locked.size)
        hin[:] = src
        eng.encode_batch(d, hin, hpar, host=True, staged=True)  # pinned: still zero-copy
        assert eng.host_paths()[0] == z2 + 1 and np.array_equal(hpar, par_locked)
        dev = torch.zeros(16, dtype=torch.uint8, device="cuda")
        rc = eng.lib.sec_encode_batch(eng._ctx, d.ctypes.data, 1, dev.data_ptr(), dev.data_ptr(),
                                      _lib.SEC_F_STAGED)
        assert rc == _lib.SEC_EINVAL
    finally:
        eng.close()


def test_registered_buffer_host_path():
    """sec_host_register on an existing numpy buffer: results are exact whichever path the
    runtime's mapping allows (zero-copy needs device address == host address)."""
    from storb_amd.engine import Engine

    eng = Engine(0)
    try:
        nch, n, k, m = 16, 1 << 18, 8, 11
        B = n // k
        d = _enc_descs(nch, n, k, m)[0]
        src = np.random.default_rng(41).integers(0, 256, nch * n, dtype=np.uint8)
        par = np.zeros(nch * (m - k) * B, dtype=np.uint8)
        eng.register(src)
        eng.register(par)
        try:
            eng.encode_batch(d, src, par, host=True)
        finally:
            eng.unregister(src)
            eng.unregister(par)
        for ci in range(nch):
            want = oracle_parity(src[ci * n:(ci + 1) * n].tobytes(), k, m)
            assert par[ci * (m - k) * B:(ci + 1) * (m - k) * B].tobytes() == b"".join(want), ci
        z, r, s = eng.host_paths()
        print(f"registered buffers took the {'zero-copy' if z else 'staged'} path")
    finally:
        eng.close()


def test_pageable_large_calls_lock_pages_per_call():
    """Large host calls on pageable memory page-lock the caller's ranges for the call, run the
    kernels on them, and unlock them: results exact, the same buffers usable again (a second
    call locks them again), and SEC_REGISTER_MIN=0 forces the staged path with equal bytes."""
    from storb_amd.engine import Engine

    eng = Engine(0)
    try:
        nch, n, k, m = 24, (1 << 20) + 7, 4, 6  # ragged, 24 MiB in
        B = -(-n // k)
        d = _enc_descs(nch, n, k, m)[0]
        src = np.random.default_rng(43).integers(0, 256, nch * n, dtype=np.uint8)
        pars = []
        for rep in range(2):
            par = np.zeros(nch * (m - k) * B, dtype=np.uint8)
            eng.encode_batch(d, src, par, host=True)
            pars.append(par)
        z, r, s = eng.host_paths()
        assert r == 2 and z == 0 and s == 0, (z, r, s)
        for ci in (0, nch - 1):
            want = oracle_parity(src[ci * n:(ci + 1) * n].tobytes(), k, m)
            assert pars[0][ci * (m - k) * B:(ci + 1) * (m - k) * B].tobytes() == b"".join(want)
        assert np.array_equal(pars[0], pars[1])
        with eng.options(SEC_REGISTER_MIN=0):
            par3 = np.zeros_like(pars[0])
            eng.encode_batch(d, src, par3, host=True)
        assert np.array_equal(par3, pars[0])
        assert eng.host_paths() == (0, 2, 1)
        # decode from the (pageable) data + parity arrays, blocks 3 (short) and 1 erased
        keep = [0, 2, 4, 5]
        dd = np.zeros(nch, dtype=DEC_DTYPE)
        dd["out_off"] = np.arange(nch, dtype=np.uint64) * n
        dd["B"], dd["padlen"], dd["k"], dd["m"] = B, B * k - n, k, m
        dd["slot0"] = np.arange(nch, dtype=np.uint64) * k
        sn = np.tile(np.array(keep, np.int32), nch)
        offs = np.zeros(nch * k, np.uint64)
        ci = np.arange(nch, dtype=np.uint64)
        for j, sh in enumerate(keep):
            offs[j::k] = (src.ctypes.data + ci * n + sh * B) if sh < k else \
                (pars[0].ctypes.data + ci * (m - k) * B + (sh - k) * B)
        out = np.zeros_like(src)
        eng.decode_batch(dd, sn, offs, 0, out, host=True)
        assert np.array_equal(out, src)
        assert eng.host_paths() == (0, 3, 1)
        # pageable input, pinned output (Engine.encode_host's result scratch): locks the input only
        chunks = [src[ci * n:(ci + 1) * n] for ci in range(nch)]
        par4 = eng.encode_host(chunks, [(k, m)] * nch)
        assert b"".join(b"".join(p) for p in par4) == pars[0].tobytes()
        assert eng.host_paths() == (0, 4, 1)
    finally:
        eng.close()


def test_threads_pageable_locking_interleaved():
    """Per-call page locking under concurrent engines: big calls whose input and
    parity ranges are 2 MiB apart (locked as one registration, gap included) run beside calls
    whose buffers live in that gap.  A range touching another call's transient registration
    must never count as pinned for this call (it is staged instead), so every result is exact
    however the calls interleave, and the locked path does run."""
    import threading

    from storb_amd.engine import Engine

    MiB = 1 << 20
    big = np.random.default_rng(5).integers(0, 256, 64 * MiB, dtype=np.uint8)
    k, m = 4, 6
    errors, paths = [], []

    def run(lo_in, n_in, lo_par, iters, seed):
        try:
            eng = Engine(0, options={"SEC_REGISTER_MIN": MiB})
            try:
                nch = n_in // MiB
                d = np.zeros(nch, dtype=ENC_DTYPE)
                d["in_off"] = np.arange(nch, dtype=np.uint64) * MiB
                d["n"], d["parity_off"], d["parity_stride"] = MiB, np.arange(nch, dtype=np.uint64) * (MiB // 2), MiB // 4
                d["k"], d["m"] = k, m
                src = big[lo_in:lo_in + n_in]
                par = big[lo_par:lo_par + n_in // 2]
                rng = random.Random(seed)
                for _ in range(iters):
                    par[:] = 0
                    eng.encode_batch(d, src, par, host=True)
                    ci = rng.randrange(nch)
                    want = b"".join(oracle_parity(src[ci * MiB:(ci + 1) * MiB].tobytes(), k, m))
                    assert par[ci * MiB // 2:(ci + 1) * MiB // 2].tobytes() == want
                paths.append(eng.host_paths())
            finally:
                eng.close()
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    ts = []
    for t in range(2):
        base = 32 * MiB * t
        # big call: 8 MiB in at base, 4 MiB parity at base + 10 MiB (2 MiB gap between)
        ts.append(threading.Thread(target=run, args=(base, 8 * MiB, base + 10 * MiB, 12, t)))
        # small call inside that gap: 1 MiB in at base + 8 MiB, parity at base + 9 MiB
        ts.append(threading.Thread(target=run, args=(base + 8 * MiB, 1 * MiB, base + 9 * MiB, 30, 10 + t)))
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors
    assert sum(p[1] for p in paths) > 0, paths  # the locked (registered) path ran


def test_largest_block_size(engine):
    """B just under the 2^31-byte limit (u32 positions in the plan and kernels): zfec(2,3) on a
    4 GiB chunk, parity checked against the field arithmetic at the start, the middle and the
    end; B = 2^31 is refused with SEC_ESIZE as zfec-style precondition error."""
    from oracle import zfec_ref
    from storb_amd.engine import Error

    k, m = 2, 3
    B = (1 << 31) - 1
    n = 2 * B - 1  # padlen 1
    src = _dev(n, seed=31)
    d, B2 = _enc_descs(1, n, k, m)
    assert B2 == B
    par = torch.empty(B, dtype=torch.uint8, device="cuda")
    engine.encode_batch(d, src, par)
    c0, c1 = (int(c) for c in zfec_ref.parity_rows(k, m)[0])
    mul = zfec_ref.MUL
    for lo in (0, B // 2 - 4096, B - 8192):
        hi = min(lo + 8192, B)
        x0 = src[lo:hi].cpu().numpy()
        x1 = src[B + lo:min(B + hi, n)].cpu().numpy()
        x1 = np.concatenate([x1, np.zeros(hi - lo - len(x1), np.uint8)])  # the padded tail
        want = mul[c0][x0] ^ mul[c1][x1]
        assert par[lo:hi].cpu().numpy().tobytes() == want.tobytes(), lo
    del par, src
    d2, _ = _enc_descs(1, 2 * (1 << 31), k, m)
    with pytest.raises(Error):
        engine.encode_batch(d2, 1, 1)  # rejected before any address is touched


@pytest.mark.parametrize("bs", ["default", "off"])
def test_encode_wide_policy_shapes(bs):
    """The policy's wide shapes (64,96), (32,48), (16,24) (files of 1 GiB to 1 TiB, SURVEY
    Appendix B) through the default plan (the bit-sliced compile-time-matrix kernel) and with it
    off (SEC_BS=0: the v_perm rows), against the oracle: ragged tails, padded last blocks, tiny
    and unaligned B, mixed with other shapes in one batch."""
    from storb_amd.engine import Engine

    eng = Engine(0, options={"SEC_BS": 0} if bs == "off" else {})
    rng = random.Random(96)
    chunks, km = [], []
    for k, m in [(64, 96), (32, 48), (16, 24), (64, 96), (32, 48)]:
        for n in [k * k, 16 * k, 16 * k * 64 + 5, 4096 * k + 1, 65536 * k - 3, (1 << 20) + 17, rng.randrange(k * k, 900000)]:
            if -(-n // k) * (k - 1) > n:
                continue
            chunks.append(rng.randbytes(n))
            km.append((k, m))
    par = eng.encode_host(chunks, km)
    for c, (k, m), p in zip(chunks, km, par):
        assert p == oracle_parity(c, k, m), (bs, k, m, len(c))
    eng.close()

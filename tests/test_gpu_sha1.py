"""GPU: SHA-1 piece ids (piece_hash, /root/reference/storb/util/piece.py:54-68) computed by
sec_sha1_kernel, against hashlib — standalone, fused after encode, and through the piece API."""

import hashlib
import random

import numpy as np
import pytest

from oracle import cfec

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

from storb_amd._lib import ENC_DTYPE, MSG_DTYPE  # noqa: E402

LENGTHS = [0, 1, 3, 55, 56, 57, 63, 64, 65, 119, 120, 127, 128, 1000, 4096, 100001, 1 << 20]


def test_sha1_host_lengths(engine):
    rng = random.Random(1)
    datas = [rng.randbytes(n) for n in LENGTHS] + [rng.randbytes(rng.randrange(0, 70000)) for _ in range(200)]
    got = engine.sha1_host(datas)
    assert got == [hashlib.sha1(d).digest() for d in datas]


def test_sha1_device_with_zero_tail(engine):
    rng = np.random.default_rng(2)
    buf = torch.from_numpy(rng.integers(0, 256, 1 << 22, dtype=np.uint8)).cuda()
    host = buf.cpu().numpy().tobytes()
    msgs = np.zeros(64, dtype=MSG_DTYPE)
    expect = []
    for i in range(64):
        off = int(rng.integers(0, 1 << 21))
        ln = int(rng.integers(0, 300000))
        av = int(rng.integers(0, ln + 1)) if i % 2 else ln
        msgs[i] = (buf.data_ptr() + off, ln, av)
        expect.append(hashlib.sha1(host[off:off + av] + b"\0" * (ln - av)).digest())
    dig = torch.empty(64 * 20, dtype=torch.uint8, device="cuda")
    engine.sha1_batch(msgs, dig)
    got = dig.cpu().numpy().tobytes()
    assert [got[20 * i:20 * i + 20] for i in range(64)] == expect


@pytest.mark.parametrize("nmsgs", [65535, 70001])
def test_sha1_device_both_kernel_paths(engine, nmsgs):
    """Below 65536 messages the kernel prefetches each next block, from there on it does not
    (kernels.hip kSha1PrefetchMsgs): both paths, with zero tails, against hashlib on a sample."""
    rng = np.random.default_rng(nmsgs)
    buf = torch.from_numpy(rng.integers(0, 256, 1 << 20, dtype=np.uint8)).cuda()
    host = buf.cpu().numpy().tobytes()
    off = rng.integers(0, 1 << 19, nmsgs)
    ln = rng.integers(0, 1000, nmsgs)
    av = np.where(np.arange(nmsgs) % 3 == 0, rng.integers(0, 1000, nmsgs) % (ln + 1), ln)
    msgs = np.zeros(nmsgs, dtype=MSG_DTYPE)
    msgs["addr"] = buf.data_ptr() + off.astype(np.uint64)
    msgs["len"], msgs["avail"] = ln, av
    dig = torch.empty(nmsgs * 20, dtype=torch.uint8, device="cuda")
    engine.sha1_batch(msgs, dig)
    got = dig.cpu().numpy().reshape(-1, 20)
    for i in list(range(0, nmsgs, 97)) + [nmsgs - 1]:
        o, n, a = int(off[i]), int(ln[i]), int(av[i])
        assert got[i].tobytes() == hashlib.sha1(host[o:o + a] + b"\0" * (n - a)).digest(), i


@pytest.mark.parametrize("k,m", [(1, 2), (2, 3), (4, 6), (10, 14), (8, 11)])
def test_encode_digest_host_matches_hashlib(engine, k, m):
    rng = random.Random(k * 31 + m)
    chunks = [rng.randbytes(n) for n in (k * k, 4096 * k - 3, 65536, 6554 * k - 1, 262144 + 9)
              if -(-n // k) * (k - 1) <= n]
    par, digs = engine.encode_host(chunks, [(k, m)] * len(chunks), digests=True)
    for c, p, d in zip(chunks, par, digs):
        blocks = cfec.easy_encode(c, k, m)
        assert p == blocks[k:]
        assert d == [hashlib.sha1(b).digest() for b in blocks]


def test_encode_digest_device_c2_sample(engine):
    nch, n, k, m = 256, 1 << 20, 4, 6
    B = n // k
    src = torch.randint(0, 256, (nch * n,), dtype=torch.uint8, device="cuda")
    d = np.zeros(nch, dtype=ENC_DTYPE)
    d["in_off"] = np.arange(nch, dtype=np.uint64) * n
    d["n"], d["parity_stride"], d["k"], d["m"] = n, B, k, m
    d["parity_off"] = np.arange(nch, dtype=np.uint64) * 2 * B
    par = torch.empty(nch * 2 * B, dtype=torch.uint8, device="cuda")
    dig = torch.empty(nch * m * 20, dtype=torch.uint8, device="cuda")
    engine.encode_digest_batch(d, src, par, dig)
    sh, ph, gh = src.cpu().numpy(), par.cpu().numpy(), dig.cpu().numpy().tobytes()
    for c in (0, 17, 255):
        blocks = [sh[c * n + j * B:c * n + (j + 1) * B].tobytes() for j in range(k)]
        blocks += [ph[c * 2 * B + r * B:c * 2 * B + (r + 1) * B].tobytes() for r in range(2)]
        for j, b in enumerate(blocks):
            assert gh[(c * m + j) * 20:(c * m + j + 1) * 20] == hashlib.sha1(b).digest()


def test_piece_api_ids():
    from storb_amd.piece import encode_chunks, encode_chunks_with_ids, piece_hash, piece_hashes

    rng = random.Random(3)
    chunks = [rng.randbytes(rng.randrange(1, 3 << 20)) for _ in range(9)]
    enc, ids = encode_chunks_with_ids(chunks, 5)
    assert [e.model_dump() for e in enc] == [e.model_dump() for e in encode_chunks(chunks, 5)]
    assert ids == [[piece_hash(p.data) for p in e.pieces] for e in enc]
    datas = [p.data for e in enc for p in e.pieces]
    assert piece_hashes(datas) == [piece_hash(x) for x in datas]


@pytest.mark.parametrize("split", ["1", "0"])
def test_sha1_split_kernel_forced(split):
    """The two-wave SHA-1 kernel (schedule wave + rounds wave, kernels.hip
    sec_sha1_split_kernel), forced on (SEC_SHA1_SPLIT=1) and off, on messages of every length
    class: empty, sub-block, exact blocks, long, zero tails past avail, ragged workgroups (more
    and fewer than 64 messages, very unequal lengths in one workgroup), device buffers and the
    host path, and fused after an encode; against hashlib."""
    from storb_amd.engine import Engine

    eng = Engine(0, options={"SEC_SHA1_SPLIT": int(split)})
    rng = np.random.default_rng(11)
    buf = torch.from_numpy(rng.integers(0, 256, 1 << 22, dtype=np.uint8)).cuda()
    host = buf.cpu().numpy().tobytes()
    for nm in (1, 63, 64, 65, 200):
        msgs = np.zeros(nm, dtype=MSG_DTYPE)
        expect = []
        for i in range(nm):
            ln = int(rng.choice([0, 1, 55, 64, 65, 4096, int(rng.integers(0, 300000)), 1 << 20]))
            off = int(rng.integers(0, (1 << 22) - ln + 1))
            av = int(rng.integers(0, ln + 1)) if i % 3 == 1 else ln
            msgs[i] = (buf.data_ptr() + off, ln, av)
            expect.append(hashlib.sha1(host[off:off + av] + b"\0" * (ln - av)).digest())
        dig = torch.empty(nm * 20, dtype=torch.uint8, device="cuda")
        eng.sha1_batch(msgs, dig)
        got = dig.cpu().numpy().tobytes()
        assert [got[20 * i:20 * i + 20] for i in range(nm)] == expect, nm
    datas = [random.Random(5).randbytes(n) for n in (0, 70, 65536, 300001, 1 << 20, 123457)]
    assert eng.sha1_host(datas) == [hashlib.sha1(d).digest() for d in datas]
    chunks = [random.Random(6).randbytes(n) for n in (1 << 20, (4 << 20) + 3, 700001)]
    par, digs = eng.encode_host(chunks, [(4, 6)] * 3, digests=True)
    for c, p, ds in zip(chunks, par, digs):
        blocks = cfec.easy_encode(c, 4, 6)
        assert ds == [hashlib.sha1(b).digest() for b in blocks]
    eng.close()

"""GPU: APDP's 2048-bit arithmetic (bignum.hip through sec_bn_* / sec_apdp_tag_batch) against
Python's arbitrary-precision pow / % (oracle/apdp_ref.py), and storb_amd.apdp.ChallengeSystem
through the reference's own test scenarios (storb/challenge/challenge_test.py)."""

import os
import random

import numpy as np
import pytest

from oracle import apdp_ref

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

from storb_amd import apdp, bn  # noqa: E402
from storb_amd._lib import MSG_DTYPE  # noqa: E402
from storb_amd.engine import ECRuntimeError  # noqa: E402

R = 1 << 2048


@pytest.fixture(scope="module")
def key():
    return apdp_ref.test_key(11)


@pytest.fixture(scope="module")
def mk(key, engine):
    return bn.ModKey(key[0], engine)


def edge_moduli():
    return [R - 1, (1 << 2047) + 1, R - 2 ** 1024 - 1, apdp_ref.test_key(3)[0]]


def test_bad_moduli_rejected(engine):
    for n in (R - 2, (1 << 2047) - 1, 3):
        with pytest.raises(ValueError):
            bn.ModKey(n, engine)
    import ctypes
    h = ctypes.c_void_p()
    assert engine.lib.sec_bn_key_create(engine._ctx, (R - 2).to_bytes(256, "big"), ctypes.byref(h)) == -13
    assert engine.lib.sec_bn_key_create(engine._ctx, ((1 << 2047) - 1).to_bytes(256, "big"), ctypes.byref(h)) == -13


def test_reduce_lengths(mk, key):
    n = key[0]
    rng = random.Random(1)
    lens = [0, 1, 2, 3, 4, 5, 255, 256, 257, 511, 512, 513, 1000, 4096, 65537, 262144, 262147]
    datas = [rng.randbytes(ln) for ln in lens] + [rng.randbytes(rng.randrange(0, 9000)) for _ in range(100)]
    datas += [b"\xff" * 256, b"\xff" * 1024, n.to_bytes(256, "big"), (n - 1).to_bytes(256, "big"),
              (2 * n).to_bytes(257, "big"), b"\x00" * 300 + b"\x01"]
    assert mk.reduce(datas) == [int.from_bytes(d, "big") % n for d in datas]


def test_reduce_device_with_zero_tail(mk, key, engine):
    n = key[0]
    rng = np.random.default_rng(3)
    buf = torch.from_numpy(rng.integers(0, 256, 1 << 20, dtype=np.uint8)).cuda()
    host = buf.cpu().numpy().tobytes()
    cnt = 48
    msgs = np.zeros(cnt, dtype=MSG_DTYPE)
    expect = []
    for i in range(cnt):
        off = int(rng.integers(0, 1 << 19))
        ln = int(rng.integers(0, 20000))
        av = int(rng.integers(0, ln + 1)) if i % 2 else ln
        msgs[i] = (buf.data_ptr() + off, ln, av)
        expect.append(int.from_bytes(host[off:off + av] + b"\0" * (ln - av), "big") % n)
    out = torch.empty(cnt * 256, dtype=torch.uint8, device="cuda")
    mk.reduce_batch(msgs, out)
    assert bn.from_be(out.cpu().numpy()) == expect


@pytest.mark.parametrize("width", [1, 3, 32, 256, 288])
def test_powmod_random(mk, key, width):
    n = key[0]
    rng = random.Random(width)
    bases = [rng.randrange(R) for _ in range(40)] + [0, 1, 2, n - 1, n, n + 1, R - 1]
    exps = [rng.getrandbits(8 * width) for _ in range(len(bases))]
    exps[:4] = [0, 1, 2, (1 << (8 * width)) - 1]
    assert mk.powmod(bases, exps) == [pow(b, x, n) for b, x in zip(bases, exps)]


def test_powmod_and_mulmod_edge_moduli(engine):
    rng = random.Random(5)
    for n in edge_moduli():
        k = bn.ModKey(n, engine)
        bases = [rng.randrange(R) for _ in range(12)] + [n - 1, R - 1, 0]
        exps = [rng.getrandbits(2048) for _ in bases]
        assert k.powmod(bases, exps) == [pow(b, x, n) for b, x in zip(bases, exps)]
        a = [rng.randrange(R) for _ in range(20)] + [R - 1, n - 1, 0]
        b = [rng.randrange(R) for _ in range(20)] + [R - 1, n - 1, 5]
        assert k.mulmod(a, b) == [x * y % n for x, y in zip(a, b)]
        assert k.reduce([b"\xff" * 700]) == [int.from_bytes(b"\xff" * 700, "big") % n]


def test_tags_match_oracle(key, engine):
    n, e, d, p, q = key
    g = pow(987654321, 2, n)
    prf_key = b"x" * 44
    fdh = apdp_ref.full_domain_hash(n, apdp_ref.prf(prf_key, 0))
    k = bn.ModKey(n, engine)
    with pytest.raises(ECRuntimeError):
        k.tags([b"abc"])
    k.set_tag(g, fdh, d)
    rng = random.Random(9)
    datas = [rng.randbytes(ln) for ln in (1, 255, 256, 257, 1024, 65536 + 5)] + [b"\xff" * 512]
    assert k.tags(datas) == [apdp_ref.tag_value(n, g, d, prf_key, x) for x in datas]


def test_crt_powmod_matches_pow(key, engine):
    n, e, d, p, q = key
    k = bn.ModKey(n, engine)
    with pytest.raises(ECRuntimeError):
        k.crt_powmod([5], [3])
    k.set_crt(p, q)
    rng = random.Random(12)
    bases = [rng.randrange(R) for _ in range(30)] + [0, 1, n - 1, p, 2 * q, p * 7, R - 1]
    exps = [rng.getrandbits(2048) for _ in range(30)] + [0, 5, 1, p - 1, (p - 1) * (q - 1), 3, 65537]
    exps[:4] = [0, 1, p - 1, (p - 1) * 5]
    assert k.crt_powmod(bases, exps) == [pow(b, x, n) for b, x in zip(bases, exps)]
    # per-factor exponents directly: Fermat inverses
    dens = [rng.randrange(2, n) for _ in range(10)]
    inv = k.crt_powmod_pq(dens, [p - 2] * 10, [q - 2] * 10)
    assert inv == [pow(x, -1, n) for x in dens]


def test_crt_set_rejects_bad_factors(key, engine):
    n, e, d, p, q = key
    k = bn.ModKey(n, engine)
    with pytest.raises(ValueError):
        k.set_crt(p, q + 2)
    import ctypes
    bad = (p - 1).to_bytes(128, "big")  # even
    z = b"\0" * 256
    assert engine.lib.sec_bn_key_set_crt(engine._ctx, k._key, bad, q.to_bytes(128, "big"), z, z) == -13
    assert engine.lib.sec_apdp_gpow_batch(engine._ctx, k._key, z, 1, 1, ctypes.c_void_p(1), 1) == -14
    assert engine.lib.sec_bn_crt_modexp_batch(engine._ctx, k._key, z, z, z, 1, 1, ctypes.c_void_p(1), 1) == -15


@pytest.mark.parametrize("crt", [False, True])
def test_tags_and_gpow_fixed_base(key, engine, crt):
    n, e, d, p, q = key
    g = pow(1234567, 2, n)
    prf_key = b"y" * 44
    fdh = apdp_ref.full_domain_hash(n, apdp_ref.prf(prf_key, 0))
    k = bn.ModKey(n, engine)
    if crt:
        k.set_crt(p, q)
    k.set_tag(g, fdh, d)
    rng = random.Random(21 + crt)
    datas = [rng.randbytes(ln) for ln in (1, 2, 255, 256, 257, 3000, 65536)] + [b"\xff" * 256, b"\x00" * 300]
    assert k.tags(datas) == [apdp_ref.tag_value(n, g, d, prf_key, x) for x in datas]
    exps = [0, 1, 2, 255, 256, n - 1, R - 1] + [rng.randrange(n) for _ in range(20)] + [rng.getrandbits(40)]
    assert k.gpow(exps) == [pow(g, x, n) for x in exps]


def _system(key):
    n, e, d, p, q = key
    cs = apdp.ChallengeSystem()
    cs.key.rsa = apdp.RSAPrivateKey(p, q, e)
    cs.key.g = pow(31337, 2, n)
    cs.key.prf_key = b"prf-key-for-tests-0123456789abcdef0123456789="
    return cs


def test_challenge_system_against_oracle(key):
    n, e, d, p, q = key
    cs = _system(key)
    assert cs.key.rsa.private_numbers().d == d
    rng = random.Random(4)
    datas = [rng.randbytes(ln) for ln in (1, 100, 1024, 4096, 262144)]
    tags = cs.generate_tags(datas)
    for data, t in zip(datas, tags):
        assert t.tag_value == apdp_ref.tag_value(n, cs.key.g, d, cs.key.prf_key, data)
        assert t.prf_value == apdp_ref.prf(cs.key.prf_key, 0)
    chs = cs.issue_challenges(tags)
    for ch in chs:
        assert 2 <= ch.s <= n - 1 and ch.g_s == pow(cs.key.g, ch.s, n)
    proofs = cs.generate_proofs(list(zip(datas, tags, chs)), n)
    for data, t, ch, pr in zip(datas, tags, chs, proofs):
        agg_tag, agg_blocks, hashed = apdp_ref.proof(n, data, t.tag_value, ch.prf_key, ch.g_s)
        assert (pr.tag_value, pr.block_value, pr.hashed_result) == (agg_tag, agg_blocks, hashed)
        assert apdp_ref.verify(n, e, pr.tag_value, pr.hashed_result, ch.prf_key, t.prf_value, ch.s)
    assert cs.verify_proofs(list(zip(proofs, chs, tags)), n, e) == [True] * len(datas)
    bad = [p.model_copy(update={"tag_value": p.tag_value + 1}) for p in proofs]
    assert cs.verify_proofs(list(zip(bad, chs, tags)), n, e) == [False] * len(datas)


# -- the reference's own scenarios (storb/challenge/challenge_test.py), keys generated fresh
@pytest.fixture(scope="module")
def fresh():
    cs = apdp.ChallengeSystem()
    cs.initialize_keys()
    return cs


def test_reference_empty_data(fresh):  # challenge_test.py:40-47
    with pytest.raises(apdp.APDPError):
        fresh.generate_tag(b"")


def test_reference_uninitialized_proof(fresh):  # challenge_test.py:50-62
    tag = fresh.generate_tag(os.urandom(1024))
    with pytest.raises(apdp.APDPError):
        fresh.generate_proof(os.urandom(1024), tag, None)


def test_reference_challenge(fresh):  # challenge_test.py:65-82
    n = fresh.key.rsa.public_key().public_numbers().n
    assert n.bit_length() == 2048
    g = fresh.key.g
    assert g not in (0, 1) and 0 < g < n
    data = os.urandom(1024)
    tag = fresh.generate_tag(data)
    challenge = fresh.issue_challenge(tag)
    proof = fresh.generate_proof(data, tag, challenge)
    assert fresh.verify_proof(proof, challenge, tag)
    # as the miner and validator call them (miner.py:284-289, explicit n / e)
    proof2 = fresh.generate_proof(data=data, tag=tag, n=n, challenge=challenge)
    assert fresh.verify_proof(proof2, challenge, tag, n, 65537)


def test_reference_verification_failure(fresh):  # challenge_test.py:85-102
    data = os.urandom(1024)
    tag = fresh.generate_tag(data)
    challenge = fresh.issue_challenge(tag)
    proof = fresh.generate_proof(data, tag, challenge)
    proof.tag_value += 1
    assert not fresh.verify_proof(proof, challenge, tag)


def test_reference_verification_failure_invalid_data(fresh):  # challenge_test.py:105-122
    data = os.urandom(1024)
    tag = fresh.generate_tag(data)
    challenge = fresh.issue_challenge(tag)
    proof = fresh.generate_proof(os.urandom(1024), tag, challenge)
    assert not fresh.verify_proof(proof, challenge, tag)


def test_serialised_round_trip_verifies(fresh):
    data = os.urandom(5000)
    tag = apdp.APDPTag.model_validate_json(fresh.generate_tag(data).model_dump_json())
    ch = apdp.Challenge.model_validate_json(fresh.issue_challenge(tag.model_dump_json()).model_dump_json())
    pr = apdp.Proof.model_validate_json(fresh.generate_proof(data, ch.tag, ch).model_dump_json())
    assert fresh.verify_proof(pr, ch, tag)


def test_kernel_timing_covers_reduce_batches(mk, engine):
    """Kernel timing (Engine.set_timing / collect_timing("bignum")) measures the message-batch
    bignum launches (segment reduce + sum), which launch outside kernels.hip's event-carrying
    dispatch: 64 pieces of 256 KiB take well over 20 us of kernel time, not ~0."""
    rng = np.random.default_rng(9)
    buf = torch.from_numpy(rng.integers(0, 256, 64 << 18, dtype=np.uint8)).cuda()
    msgs = np.zeros(64, dtype=MSG_DTYPE)
    for i in range(64):
        msgs[i] = (buf.data_ptr() + i * (1 << 18), 1 << 18, 1 << 18)
    out = torch.empty(64 * 256, dtype=torch.uint8, device="cuda")
    mk.reduce_batch(msgs, out)  # warm (R^(32j) table growth)
    engine.sync()
    engine.collect_timing("bignum")
    engine.set_timing(True)
    mk.reduce_batch(msgs, out)
    engine.sync()
    engine.set_timing(False)
    ms, n = engine.collect_timing("bignum")
    assert n >= 1 and ms > 0.02, (ms, n)

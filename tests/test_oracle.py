"""CPU: the oracle (oracle/zfec_ref.py + oracle/fec_oracle.c) against the golden fixtures,
SURVEY.md Appendix A/B, and itself (two independent matrix constructions).

Parity status: unpinned against real zfec bytes (zfec 1.6.0.0 absent; the reference's tests
hold no known-answer vectors).  See oracle/fec_oracle.c header and DESIGN.md §Oracle.
"""

import hashlib
import json
import os
import random

import numpy as np
import pytest

from oracle import cfec, zfec_ref

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))


def sha(b):
    return hashlib.sha256(b).hexdigest()


@pytest.mark.parametrize("km", list(GOLDEN["matrices"]))
def test_matrices_two_constructions_and_golden(km):
    k, m = map(int, km.split(","))
    gj = zfec_ref.parity_rows(k, m)  # seed @ inv(top), Gauss-Jordan
    lag = cfec.encode_matrix(k, m)[k * k:]  # closed-form Lagrange basis (C)
    assert gj.tobytes() == lag
    assert [bytes(r).hex() for r in gj] == GOLDEN["matrices"][km]


def test_survey_appendix_a_rows():
    # rows restated in SURVEY.md Appendix A (an independent restatement, not zfec output)
    assert [bytes(r).hex() for r in zfec_ref.parity_rows(2, 3)] == ["0302"]
    assert [bytes(r).hex() for r in zfec_ref.parity_rows(4, 6)] == ["7740380e", "c7a70d6c"]
    assert [bytes(r).hex() for r in zfec_ref.parity_rows(8, 12)] == [
        "8918d07d92a4f5fe", "36f8d0ce2519fb16", "5fcda3405048f69e", "ed912490dc9057d2"]
    assert [bytes(r).hex() for r in zfec_ref.parity_rows(10, 14)] == [
        "42c15c2d722ceb841bd9", "a9155162f59532206599", "0f1f1be06bddd3634fa3", "fb4f95a62f7561260893"]
    assert zfec_ref.parity_rows(1, 2).tolist() == [[1]]  # zfec(1,2): parity is a copy


def test_gf_field():
    # 0x11D field, generator 2: multiplicative group of order 255
    assert zfec_ref.EXP[8] == 0x1D
    seen = {int(zfec_ref.EXP[e]) for e in range(255)}
    assert seen == set(range(1, 256))
    for a in (1, 2, 3, 0x53, 0xCA, 255):
        assert zfec_ref.gf_mul(a, int(zfec_ref.INV[a])) == 1
        assert cfec.lib().fo_gf_mul(a, int(zfec_ref.INV[a])) == 1


@pytest.mark.parametrize("ent", GOLDEN["encode"], ids=lambda e: f"k{e['k']}m{e['m']}n{e['n']}")
def test_encode_golden_both_oracles(ent):
    k, m, n = ent["k"], ent["m"], ent["n"]
    data = random.Random(ent["seed"]).randbytes(n)
    c = cfec.easy_encode(data, k, m)
    assert [sha(b) for b in c] == ent["blocks_sha256"]
    if n <= 70000:
        assert zfec_ref.easy_encode(data, k, m) == c
    if "parity_hex" in ent:
        assert [b.hex() for b in c[k:]] == ent["parity_hex"]
    # systematic: data blocks are the (padded) input slices
    assert b"".join(c[:k])[:n] == data


@pytest.mark.parametrize("ent", GOLDEN["decode"], ids=lambda e: f"k{e['k']}m{e['m']}-{e['sharenums']}")
def test_decode_golden_both_oracles(ent):
    k, m, sn = ent["k"], ent["m"], ent["sharenums"]
    _, idx = zfec_ref.normalise([b"x"] * k, sn, k, m)
    assert idx == ent["normalised"]
    assert [bytes(r).hex() for r in zfec_ref.decode_matrix(k, m, idx)] == ent["decode_matrix"]
    data = random.Random(ent["seed"]).randbytes(ent["n"])
    blocks = cfec.easy_encode(data, k, m)
    pad = len(blocks[0]) * k - len(data)
    got = cfec.easy_decode([blocks[s] for s in sn], sn, pad, k, m)
    assert sha(got) == ent["out_sha256"] and got == data
    assert zfec_ref.easy_decode([blocks[s] for s in sn], sn, pad, k, m) == data


def test_policy_table_appendix_b():
    for p in GOLDEN["policy"]:
        size = p["file_size"]
        assert zfec_ref.piece_length(size) == p["chunk"]
        assert zfec_ref.chunk_shape(min(p["chunk"], size)) == (p["k"], p["m"], p["B"], p["padlen"])
    # SURVEY Appendix B spot rows
    assert zfec_ref.chunk_shape(512 * 1024) == (4, 6, 131072, 0)
    assert zfec_ref.chunk_shape(256 * 1024) == (2, 3, 131072, 0)
    assert zfec_ref.chunk_shape(1 << 20) == (4, 6, 262144, 0)


def test_every_erasure_pattern_small():
    # exhaustive over all C(6,4) share subsets for zfec(4,6), both oracles
    import itertools
    data = random.Random(3).randbytes(1001)
    blocks = zfec_ref.easy_encode(data, 4, 6)
    pad = len(blocks[0]) * 4 - len(data)
    for sub in itertools.combinations(range(6), 4):
        for order in (list(sub), list(reversed(sub))):
            bl = [blocks[s] for s in order]
            assert zfec_ref.easy_decode(bl, order, pad, 4, 6) == data
            assert cfec.easy_decode(bl, order, pad, 4, 6) == data


def test_oracle_preconditions():
    with pytest.raises(ValueError):
        zfec_ref.encode_matrix(0, 1)
    with pytest.raises(ValueError):
        zfec_ref.encode_matrix(4, 257)
    with pytest.raises(ValueError):  # short middle slice: n=5, k=4 -> B=2, 3*2 > 5
        zfec_ref.easy_encode(b"12345", 4, 6)
    blocks = zfec_ref.easy_encode(b"abcdefgh", 4, 6)
    with pytest.raises(ValueError):
        zfec_ref.easy_decode(blocks[:4], [0, 1, 1, 2], 0, 4, 6)
    with pytest.raises(ValueError):
        zfec_ref.easy_decode(blocks[:4], [0, 1, 2, 6], 0, 4, 6)
    with pytest.raises(ValueError):
        zfec_ref.easy_decode(blocks[:3], [0, 1, 2], 0, 4, 6)


def test_linearity_property():
    # encode(a ^ b) == encode(a) ^ encode(b): the code is GF(2)-linear
    a = np.frombuffer(random.Random(1).randbytes(4096), np.uint8)
    b = np.frombuffer(random.Random(2).randbytes(4096), np.uint8)
    ea = cfec.easy_encode(a.tobytes(), 8, 12)
    eb = cfec.easy_encode(b.tobytes(), 8, 12)
    eab = cfec.easy_encode((a ^ b).tobytes(), 8, 12)
    for x, y, z in zip(ea, eb, eab):
        assert (np.frombuffer(x, np.uint8) ^ np.frombuffer(y, np.uint8)).tobytes() == z

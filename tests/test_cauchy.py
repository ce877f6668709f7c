"""The syndrome decode's Cauchy solve, restated on the host (no GPU).

kernels_bs.hip recovers the e lost data rows L from the syndromes of the e present parity rows
S as  d_l = z_l * XOR_{r in S} c[r][l] * (w_r * s_r)  (gf_host.hpp cauchy_scales), i.e. it
relies on  inv(c[S][L])[l][r] = z_l c[r][l] w_r  for zfec's parity rows c.  This checks that
identity against a Gauss-Jordan inverse (oracle/zfec_ref.py) for every bit-sliced shape and
random (S, L), and the bit-plane form of a scaling (scale_mask: byte s of the mask is
c * alpha^s; plane t of c * x = XOR of the planes s whose byte s has bit t set).
"""

import random

import numpy as np
import pytest

from oracle.zfec_ref import EXP, INV, MUL, encode_matrix, gf_invert

SHAPES = [(10, 14), (8, 12), (16, 24), (32, 48), (64, 96), (8, 11)]


def _pt(i):
    return 0 if i == 0 else int(EXP[(i - 1) % 255])


def _prod(vals):
    r = 1
    for v in vals:
        r = int(MUL[r, v])
    return r


def _div(a, b):
    return int(MUL[a, INV[b]])


def cauchy_scales(k, S, L):
    """w (per present parity row r in S) and z (per lost data row l in L), gf_host.hpp's formulas."""
    xs = [_pt(k + r) for r in S]
    ys = [_pt(l) for l in L]
    w = []
    for q, x in enumerate(xs):
        num = _prod(x ^ y for y in ys)
        den = _prod(x ^ x2 for q2, x2 in enumerate(xs) if q2 != q)
        a = _prod(x ^ _pt(i) for i in range(k))
        w.append(_div(_div(num, den), int(MUL[a, a])))
    z = []
    for t, (l, y) in enumerate(zip(L, ys)):
        num = _prod(x ^ y for x in xs)
        den = _prod(y ^ y2 for t2, y2 in enumerate(ys) if t2 != t)
        binv = _prod(y ^ _pt(i) for i in range(k) if i != l)
        z.append(int(MUL[_div(num, den), MUL[binv, binv]]))
    return w, z


@pytest.mark.parametrize("k,m", SHAPES)
def test_cauchy_inverse_matches_gauss_jordan(k, m):
    rng = random.Random(k * 131 + m)
    P = encode_matrix(k, m)[k:]
    p = m - k
    for e in sorted({1, 2, p // 2, p} | {rng.randint(1, p) for _ in range(4)}):
        for _ in range(3):
            S = sorted(rng.sample(range(p), e))
            L = sorted(rng.sample(range(k), e))
            want = gf_invert(P[np.ix_(S, L)])  # want[t][q]: lost row t from syndrome q
            w, z = cauchy_scales(k, S, L)
            got = np.array([[MUL[MUL[z[t], P[S[q], L[t]]], w[q]] for q in range(e)] for t in range(e)], np.uint8)
            assert np.array_equal(got, want), (k, m, S, L)


def _scale_mask(c):
    return sum(int(MUL[c, 1 << s]) << (8 * s) for s in range(8))


def _planes(x):
    """32 bytes -> 8 bit planes (plane t bit q = bit t of byte q)."""
    return [sum(((int(x[q]) >> t) & 1) << q for q in range(32)) for t in range(8)]


def _unplanes(pl):
    return np.array([sum(((pl[t] >> q) & 1) << t for t in range(8)) for q in range(32)], np.uint8)


def test_scale_mask_on_bit_planes():
    rng = np.random.default_rng(3)
    x = rng.integers(0, 256, 32, dtype=np.uint8)
    for c in [0, 1, 2, 3, 0x1D, 0x8E, 0xFF] + list(rng.integers(0, 256, 20)):
        m = _scale_mask(int(c))
        y = _planes(x)
        o = [0] * 8
        for s in range(8):
            for t in range(8):
                if (m >> (8 * s + t)) & 1:
                    o[t] ^= y[s]
        assert np.array_equal(_unplanes(o), MUL[int(c)][x]), c

"""GPU parity of the bit-sliced compile-time-matrix encode (storb_amd/csrc/kernels_bs.hip)
against the CPU oracle (oracle/fec_oracle.c), bit-exact.

The kernel serves zfec(10,14) (BASELINE C4), (8,11) (C5's RS(8,3)) and the policy's (8,12),
(16,24), (32,48), (64,96) for chunks with B >= 16 and covers every position [0, B) itself:
2 KiB wave spans, pieces past B moved back to end at B (overlapping a neighbour), block k-1's
zero padding read past `valid`.  Cases: B from 16 bytes to several tiles, B just under / at /
over one span, not a multiple of 16 or of the span, padlen 0 and k-1, mixed with shapes the
kernel does not serve in one batch, 64 / 128 / 256-lane tiles, (64,96)'s two row groups in one
two-wave workgroup per span sharing each block's plane subsets, host (staged) and
device-resident calls with a padded parity stride; "off" (SEC_BS=0) is the v_perm / xb path
for the same chunks.
"""

import random

import numpy as np
import pytest

from oracle import cfec

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from storb_amd._lib import ENC_DTYPE  # noqa: E402

BS_SHAPES = [(10, 14), (8, 11), (8, 12), (16, 24), (32, 48), (64, 96)]


def oracle_parity(data, k, m):
    return cfec.easy_encode(bytes(data), k, m)[k:]


def _sizes(k, rng):
    out = [2047 * k, 2048 * k, 2048 * k - (k - 1), 2048 * k + 1, 6554 * k - 4, 8192 * k, 8192 * k + 17,
           10240 * k - 3, 16 * 1024 * k + 2048 * k + 9, rng.randrange(2048 * k, 40000 * k)]
    return [n for n in out if -(-n // k) * (k - 1) < n]


MODES = {
    "default": {},  # the kernel for the shapes with >= 8 parity rows, v_perm / xb for the rest
    "all256": {"SEC_BS": 1},
    "all128": {"SEC_BS": 1, "SEC_BS_LANES": 128},
    "all64": {"SEC_BS": 1, "SEC_BS_LANES": 64},
    "off": {"SEC_BS": 0},
}


@pytest.mark.parametrize("mode", list(MODES))
def test_encode_bit_sliced_shapes_host(mode):
    from storb_amd.engine import Engine

    eng = Engine(0, options=MODES[mode])  # context options (sec_ctx_set_option)
    rng = random.Random(mode)
    chunks, km = [], []
    for k, m in BS_SHAPES + [(4, 6), (10, 14)]:
        for n in _sizes(k, rng):
            chunks.append(rng.randbytes(n))
            km.append((k, m))
    for k, m in [(16, 24), (64, 96), (32, 48)]:  # blocks of 16 .. 2047 bytes
        for n in [16 * k, 16 * k + 1, 100 * k - 7, 2000 * k]:
            if -(-n // k) * (k - 1) >= n:  # no zfec split (block k-1 would be empty)
                continue
            chunks.append(rng.randbytes(n))
            km.append((k, m))
    order = list(range(len(chunks)))
    rng.shuffle(order)  # shapes interleaved in one batch
    chunks = [chunks[i] for i in order]
    km = [km[i] for i in order]
    par = eng.encode_host(chunks, km)
    for c, (k, m), p in zip(chunks, km, par):
        assert p == oracle_parity(c, k, m), (mode, k, m, len(c))
    eng.close()


@pytest.mark.parametrize("k,m", BS_SHAPES)
def test_encode_bit_sliced_device_padded_stride(k, m):
    """Device-resident chunks back to back (unaligned block starts), parity blocks at a stride
    larger than B: the kernel writes exactly [0, B) of each parity block and nothing between."""
    from storb_amd.engine import Engine

    engine = Engine(0, options={"SEC_BS": 1})
    rng = random.Random(k * 7 + m)
    n = 4096 * k + 2 * k + 3 if k > 3 else 40000
    B = -(-n // k)
    nch = 24
    ps = B + 48
    g = torch.Generator(device="cuda")
    g.manual_seed(k + m)
    src = torch.randint(0, 256, (nch * n,), dtype=torch.uint8, device="cuda", generator=g)
    d = np.zeros(nch, dtype=ENC_DTYPE)
    d["in_off"] = np.arange(nch, dtype=np.uint64) * n
    d["n"] = n
    d["parity_off"] = np.arange(nch, dtype=np.uint64) * (m - k) * ps
    d["parity_stride"] = ps
    d["k"] = k
    d["m"] = m
    par = torch.full((nch * (m - k) * ps,), 0xA5, dtype=torch.uint8, device="cuda")
    engine.encode_batch(d, src, par)
    sh = src.cpu().numpy()
    ph = par.cpu().numpy().reshape(nch, m - k, ps)
    for ci in [0, 1, rng.randrange(2, nch - 1), nch - 1]:
        want = oracle_parity(sh[ci * n:(ci + 1) * n].tobytes(), k, m)
        for r in range(m - k):
            assert ph[ci, r, :B].tobytes() == want[r], (k, m, ci, r)
    assert (ph[:, :, B:] == 0xA5).all()  # the gaps between parity blocks are untouched
    engine.close()


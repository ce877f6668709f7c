"""GPU parity of the bit-sliced integer-MFMA encode (kernels_mfma.hip; k = 32 and 64, the
policy's shapes for >= 16 GiB files; an A/B path, on with SEC_MFMA=1,
since it measured slower than the v_perm kernels) against the oracle
(oracle/fec_oracle.c, zfec's fec_encode restated): every parity row count up to a row group
and beyond, 128-position groups whole and partial, block sizes below one group (no MFMA part),
unaligned blocks, padded last blocks, tiles spanning several 8192-position tiles; device and
host paths; and the same bytes as the v_perm kernels (SEC_MFMA=0)."""

import random

import numpy as np
import pytest

from oracle import cfec

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from storb_amd._lib import ENC_DTYPE  # noqa: E402


def _sizes(k, rng):
    out = [k * 100, k * 128, k * 128 * 3 + k, k * 8192 - 5, k * 8192 * 2 + 129 * k - 1, k * 20000 + 3,
           k * (1 << 15)]
    out += [rng.randrange(k * k, k * 30000) for _ in range(3)]
    return [n for n in out if -(-n // k) * (k - 1) <= n]


@pytest.fixture(scope="module")
def mfma_engine():
    """An engine whose plans use the MFMA encode (SEC_MFMA=1 is read when a plan is built)."""
    import os

    from storb_amd.engine import Engine

    old = os.environ.get("SEC_MFMA")
    os.environ["SEC_MFMA"] = "1"
    eng = Engine(0)
    yield eng
    eng.close()
    if old is None:
        os.environ.pop("SEC_MFMA", None)
    else:
        os.environ["SEC_MFMA"] = old


@pytest.mark.parametrize("k,m", [(32, 48), (32, 33), (32, 40), (32, 47), (32, 64), (64, 96), (64, 65), (64, 80)])
def test_mfma_encode_host_vs_oracle(mfma_engine, k, m, monkeypatch):
    monkeypatch.setenv("SEC_MFMA", "1")
    rng = random.Random(k * 1000 + m)
    chunks = [rng.randbytes(n) for n in _sizes(k, rng)]
    par = mfma_engine.encode_host(chunks, [(k, m)] * len(chunks))
    for c, p in zip(chunks, par):
        assert p == cfec.easy_encode(c, k, m)[k:], (k, m, len(c))


@pytest.mark.parametrize("k,m,n", [(32, 48, 1 << 20), (32, 48, (1 << 20) + 77), (64, 96, 1 << 21)])
def test_mfma_encode_device_matches_valu_kernels(k, m, n, monkeypatch):
    from storb_amd.engine import Engine

    nch = 16
    B = -(-n // k)
    src = torch.randint(0, 256, (nch * n,), dtype=torch.uint8, device="cuda")
    d = np.zeros(nch, dtype=ENC_DTYPE)
    d["in_off"] = np.arange(nch, dtype=np.uint64) * n
    d["n"], d["parity_off"], d["parity_stride"] = n, np.arange(nch, dtype=np.uint64) * (m - k) * B, B
    d["k"], d["m"] = k, m
    outs = []
    for flag in ("1", "0"):
        monkeypatch.setenv("SEC_MFMA", flag)
        eng = Engine(0)  # fresh plan with this setting
        try:
            par = torch.zeros(nch * (m - k) * B, dtype=torch.uint8, device="cuda")
            eng.encode_batch(d, src, par)
            outs.append(par)
        finally:
            eng.close()
    assert torch.equal(outs[0], outs[1])
    h, p = src.cpu().numpy(), outs[0].cpu().numpy()
    for ci in (0, nch - 1):
        want = b"".join(cfec.easy_encode(h[ci * n:(ci + 1) * n].tobytes(), k, m)[k:])
        assert p[ci * (m - k) * B:(ci + 1) * (m - k) * B].tobytes() == want

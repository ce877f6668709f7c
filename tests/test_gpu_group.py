"""GPU: the in-process multi-device path with REAL contexts — EngineGroup([0, 0]) puts two
libstorbec contexts (each on its own worker thread and streams) on the one GPU of the box, so
the split of a batch, the concurrent device calls and the reassembly in chunk order run through
the HIP kernels.  Every output is checked against the oracle (oracle/fec_oracle.c), not against
the one-device path.  The CPU twin with the oracle engine is tests/test_group.py."""

import random
import threading

import numpy as np
import pytest

from oracle import cfec

pytestmark = pytest.mark.gpu

from storb_amd import piece  # noqa: E402
from storb_amd.engine import EngineGroup  # noqa: E402


@pytest.fixture(scope="module")
def group():
    g = EngineGroup([0, 0])
    yield g
    g.close()


def _mixed_chunks(seed, n):
    """Sizes across the policy's shapes: zfec(1,2) tails up to zfec(8,12)-sized chunks."""
    rng = random.Random(seed)
    sizes = [rng.choice([1, 17, 4096, 16385, 70_000, 300_001, 1 << 20, (1 << 20) + 5, 3 << 20]) for _ in range(n)]
    return [rng.randbytes(s) for s in sizes]


def test_two_contexts_are_distinct(group):
    e0, e1 = group.engines
    assert e0 is not e1 and e0._ctx.value != e1._ctx.value
    assert e0.device == e1.device == 0


def test_encode_chunks_two_contexts_vs_oracle(group):
    chunks = _mixed_chunks(1, 24)
    out = piece.encode_chunks(chunks, first_chunk_idx=5, devices=group)
    assert [ec.chunk_idx for ec in out] == list(range(5, 29))
    for c, ec in zip(chunks, out):
        k, m, B, padlen = piece.chunk_shape(len(c))
        assert (ec.k, ec.m, ec.chunk_size, ec.padlen) == (k, m, B, padlen)
        assert [p.data for p in ec.pieces] == cfec.easy_encode(c, k, m)


def test_reconstruct_two_contexts_vs_oracle(group):
    chunks = _mixed_chunks(2, 20)
    ecs = piece.encode_chunks(chunks, devices=group)
    rng = random.Random(2)
    pieces = []
    for ec in ecs:  # every chunk loses as many pieces as it can, data pieces first
        lost = set(range(min(ec.m - ec.k, ec.k)))
        pieces += [p for p in ec.pieces if p.piece_idx not in lost]
    rng.shuffle(pieces)
    for ec in ecs:
        ec.pieces = None
    assert piece.reconstruct_data(pieces, ecs, devices=group) == b"".join(chunks)


def test_stream_two_contexts_order_and_error(group):
    chunks = _mixed_chunks(3, 30)
    ecs = piece.encode_chunks(chunks, devices=group)
    pieces = [p for ec in ecs for p in ec.pieces[-ec.k:] if ec.chunk_idx != 23]
    for ec in ecs:
        ec.pieces = None
    got = []
    with pytest.raises(ValueError, match="chunk 23"):
        for b in piece.reconstruct_data_stream(pieces, ecs, window_bytes=2 << 20, devices=group):
            got.append(b)
    assert got == chunks[:23]


def test_encode_stream_two_contexts_ids(group):
    chunks = _mixed_chunks(4, 16)
    outs = list(piece.encode_chunks_stream(chunks, 0, piece_ids=True, window_bytes=3 << 20, devices=group))
    for c, (ec, ids) in zip(chunks, outs):
        want = cfec.easy_encode(c, ec.k, ec.m)
        assert [p.data for p in ec.pieces] == want
        assert ids == [piece.piece_hash(bytes(w)) for w in want]


def test_concurrent_callers_share_group(group):
    """Two caller threads drive the same group at once (a validator serving two downloads)."""
    datas = [_mixed_chunks(10 + i, 10) for i in range(2)]
    ecs = [piece.encode_chunks(d, devices=group) for d in datas]
    res = [None, None]

    def run(i):
        pcs = [p for ec in ecs[i] for p in ec.pieces[1:]]  # piece 0 of every chunk lost
        res[i] = piece.reconstruct_data(pcs, ecs[i], devices=group)

    ts = [threading.Thread(target=run, args=(i,)) for i in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(120)
    assert res == [b"".join(d) for d in datas]


def test_device_batches_on_group_workers(group):
    """The bench's --in-process form: device-resident batches issued on each worker's engine."""
    import torch

    from storb_amd._lib import ENC_DTYPE

    nch, n, k, m = 16, 65536 + 3, 4, 6
    B = -(-n // k)
    rng = np.random.default_rng(9)
    host = rng.integers(0, 256, 2 * nch * n, dtype=np.uint8)

    def work(lo):
        src = torch.from_numpy(host[lo * nch * n:(lo + 1) * nch * n]).to("cuda:0")
        ed = np.zeros(nch, dtype=ENC_DTYPE)
        ed["in_off"] = np.arange(nch) * n
        ed["n"], ed["parity_stride"], ed["k"], ed["m"] = n, B, k, m
        ed["parity_off"] = np.arange(nch) * 2 * B
        par = torch.empty(nch * 2 * B, dtype=torch.uint8, device="cuda:0")
        from storb_amd.engine import get_engine

        get_engine().encode_batch(ed, src, par)
        return par.cpu().numpy()

    pars = [group.submit(i, work, i).result() for i in range(2)]
    for i, p in enumerate(pars):
        for c in range(nch):
            blob = host[(i * nch + c) * n:(i * nch + c + 1) * n].tobytes()
            assert p[c * 2 * B:(c + 1) * 2 * B].tobytes() == b"".join(cfec.easy_encode(blob, k, m)[k:])

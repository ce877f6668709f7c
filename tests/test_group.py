"""CPU: the in-process multi-device path (engine.EngineGroup, piece's ``devices=``) — the split of a
batch over the devices' workers, the reassembly in chunk order and the order of errors — with
tests/engine_stub.py's oracle engine in place of each device's HIP context.

The GPU twin (two real contexts on one GPU, checked against the oracle) is
tests/test_gpu_group.py."""

import random
import threading

import numpy as np
import pytest

from oracle import cfec
from storb_amd import piece
from storb_amd.engine import EngineGroup
from tests.engine_stub import OracleHostEngine


@pytest.fixture
def group3():
    g = EngineGroup([0, 0, 1], engine_factory=OracleHostEngine)
    yield g
    g.close()


def _chunks(seed, n, lo=1000, hi=300_000):
    rng = random.Random(seed)
    return [rng.randbytes(rng.randrange(lo, hi)) for _ in range(n)]


def _want_pieces(c):
    k, m, B, padlen = piece.chunk_shape(len(c))
    return cfec.easy_encode(c, k, m)


def test_group_workers_have_own_engines(group3):
    assert len(group3) == 3
    engs = group3.engines
    assert len({id(e) for e in engs}) == 3
    # get_engine() on a worker is that worker's engine
    from storb_amd.engine import get_engine

    for i, e in enumerate(engs):
        assert group3.submit(i, get_engine).result() is e


def test_encode_chunks_split_and_order(group3):
    chunks = _chunks(1, 23)
    out = piece.encode_chunks(chunks, first_chunk_idx=7, devices=group3)
    assert [ec.chunk_idx for ec in out] == list(range(7, 30))
    for c, ec in zip(chunks, out):
        want = _want_pieces(c)
        assert [p.data for p in ec.pieces] == want
        assert [p.piece_idx for p in ec.pieces] == list(range(ec.m))
        assert ec.original_chunk_size == len(c)
    counts = [e.chunks_encoded for e in group3.engines]
    assert sum(counts) == len(chunks) and all(x > 0 for x in counts)
    tids = [e.threads for e in group3.engines]
    assert all(len(t) == 1 for t in tids) and len(set().union(*tids)) == 3
    assert threading.get_ident() not in set().union(*tids)


def test_encode_chunks_empty_chunk_raises_before_work(group3):
    chunks = _chunks(2, 6)
    chunks[4] = b""
    with pytest.raises(ValueError):
        piece.encode_chunks(chunks, devices=group3)
    assert sum(e.chunks_encoded for e in group3.engines) == 0


def _erase(ecs, rng, keep_extra=0):
    pieces = []
    for ec in ecs:
        idx = list(range(ec.m))
        rng.shuffle(idx)
        for i in sorted(idx[:ec.k + keep_extra]):
            pieces.append(ec.pieces[i])
    rng.shuffle(pieces)
    return pieces


def test_reconstruct_data_split(group3):
    chunks = _chunks(3, 17)
    ecs = piece.encode_chunks(chunks, devices=group3)
    rng = random.Random(3)
    pieces = _erase(ecs, rng)
    for ec in ecs:
        ec.pieces = None
    before = [e.chunks_decoded for e in group3.engines]
    got = piece.reconstruct_data(pieces, ecs, devices=group3)
    assert got == b"".join(chunks)
    assert all(a > b for a, b in zip([e.chunks_decoded for e in group3.engines], before))


def test_decode_chunks_error_is_first_bad_chunk(group3):
    chunks = _chunks(4, 9)
    ecs = piece.encode_chunks(chunks, devices=group3)
    # chunk 6 (last share) gets a duplicate sharenum, chunk 2 (first share) a sharenum >= m
    ecs[6].pieces = [ecs[6].pieces[0]] * ecs[6].k
    bad = ecs[2].pieces[0].model_copy(update={"piece_idx": 999})
    ecs[2].pieces = [bad] + ecs[2].pieces[1:ecs[2].k]
    with pytest.raises(piece.Error, match="sharenum"):
        piece.decode_chunks(ecs, devices=group3)


def test_reconstruct_stream_order_and_late_error(group3):
    chunks = _chunks(5, 30, 4000, 60_000)
    ecs = piece.encode_chunks(chunks, devices=group3)
    rng = random.Random(5)
    pieces = _erase(ecs, rng, keep_extra=1)
    pieces = [p for p in pieces if p.chunk_idx != 21]  # chunk 21 has no pieces
    for ec in ecs:
        ec.pieces = None
    got = []
    with pytest.raises(ValueError, match="chunk 21"):
        for b in piece.reconstruct_data_stream(pieces, ecs, window_bytes=100_000, devices=group3):
            got.append(b)
    assert got == chunks[:21]


def test_encode_stream_split_and_ids(group3):
    chunks = _chunks(6, 20, 5000, 80_000)
    outs = list(piece.encode_chunks_stream(iter(chunks), 3, piece_ids=True, window_bytes=150_000, devices=group3))
    assert [ec.chunk_idx for ec, _ in outs] == list(range(3, 23))
    for c, (ec, ids) in zip(chunks, outs):
        want = _want_pieces(c)
        assert [p.data for p in ec.pieces] == want
        assert ids == [piece.piece_hash(bytes(w)) for w in want]
    assert sum(1 for e in group3.engines if e.chunks_encoded) == 3


def test_encode_stream_large_pieces_gpu_ids(group3):
    # pieces >= PARALLEL_COPY_MIN: the window's ids come from sec_encode_digest_batch
    rng = random.Random(7)
    chunks = [rng.randbytes(1 << 20) for _ in range(4)] + [rng.randbytes((1 << 20) + 3)]
    outs = list(piece.encode_chunks_stream(chunks, 0, piece_ids=True, window_bytes=2 << 20, devices=group3))
    for c, (ec, ids) in zip(chunks, outs):
        want = _want_pieces(c)
        assert [p.data for p in ec.pieces] == want
        assert ids == [piece.piece_hash(bytes(w)) for w in want]


def test_use_devices_default(group3):
    chunks = _chunks(8, 5)
    try:
        piece.use_devices(group3)
        out = piece.encode_chunks(chunks)
        assert sum(e.chunks_encoded for e in group3.engines) == 5
        assert piece.reconstruct_data([p for ec in out for p in ec.pieces], out) == b"".join(chunks)
    finally:
        piece.use_devices(None)
    from storb_amd import engine

    assert engine._spread["devices"] is None


def test_map_shares_runs_all_then_raises_first():
    g = EngineGroup([0, 1, 2, 3], engine_factory=OracleHostEngine)
    seen = []

    def fn(items, lo):
        seen.append(lo)
        if lo in (2, 6):
            raise KeyError(lo)
        return items

    try:
        with pytest.raises(KeyError) as ei:
            g.map_shares(fn, list(range(8)), [1] * 8)
        assert ei.value.args == (2,)
        assert sorted(seen) == [0, 2, 4, 6]
        assert g.map_shares(lambda it, lo: [x * 2 for x in it], list(range(5)), [1] * 5) == [[0, 2], [4], [6], [8]]
    finally:
        g.close()


def test_spread_threads_round_robin():
    from storb_amd import engine

    engine.spread_threads([3, 5])
    try:
        got = []
        ts = [threading.Thread(target=lambda: got.append(engine._thread_device())) for _ in range(4)]
        for t in ts:
            t.start()
            t.join()
        assert sorted(got) == [3, 3, 5, 5]
    finally:
        engine.spread_threads(None)
    assert engine._thread_device() is None


def test_decode_into_matches_join():
    e = OracleHostEngine()
    rng = np.random.default_rng(0)
    items = []
    want = b""
    for n, lost in ((5000, (1,)), (777, ()), (65536, (0, 2))):
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        blocks = cfec.easy_encode(data, 4, 6)
        keep = [s for s in range(6) if s not in lost][:4]
        items.append((4, 6, [blocks[s] for s in keep], keep, 4 * len(blocks[0]) - n))
        want += data
    dst = np.zeros(len(want), np.uint8)
    assert e.decode_host_into(items, dst) == len(want)
    assert dst.tobytes() == want == e.decode_host(items)
    with pytest.raises(ValueError):
        e.decode_host_into(items, np.zeros(len(want) - 1, np.uint8))

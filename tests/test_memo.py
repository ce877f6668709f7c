"""CPU: piece_hash's memo of encode_chunk's prefetched ids (storb_amd.piece._PieceIdMemo) — the
retention bounds the round-2 review asked for: entries leave on use, after `keep_calls` newer
calls, or past the byte cap; the same object put twice counts once; prefetching pauses after
`idle_calls` unused calls except for periodic probes, and resumes once an id is used."""

from concurrent.futures import Future

from storb_amd.piece import _PieceIdMemo


def _done(v):
    f = Future()
    f.set_result(v)
    return f


def test_memo_take_identity_and_bytes():
    m = _PieceIdMemo(max_bytes=1000, keep_calls=2)
    a, b = bytes(100), bytes(bytearray(100))
    c = m.begin(200)
    m.put(a, _done("A"), c)
    m.put(a, _done("A"), c)  # twice: counted once
    assert m.held_bytes() == 100
    m.put(b, _done("B"), c)
    assert m.take(bytes(bytearray(100))) is None  # equal, not identical
    assert m.take(a) == "A" and m.take(a) is None and m.take(b) == "B"
    assert m.held_bytes() == 0


def test_memo_keeps_only_recent_calls_and_cap():
    m = _PieceIdMemo(max_bytes=1000, keep_calls=2, idle_calls=100)
    objs = []
    for i in range(6):
        c = m.begin(300)
        o = bytes([i]) * 300
        objs.append(o)
        m.put(o, _done(i), c)
        assert m.held_bytes() <= 600  # this call and the one before
    assert m.take(objs[0]) is None and m.take(objs[5]) == 5
    assert m.begin(1001) is None  # larger than the cap: no prefetch
    c = m.begin(900)
    m.put(bytes(900), _done("x"), c)
    assert m.held_bytes() <= 1000


def test_memo_pauses_when_unused_and_resumes():
    m = _PieceIdMemo(max_bytes=10_000, keep_calls=1, idle_calls=3, probe_every=8)
    started = 0
    last = None
    for i in range(40):
        c = m.begin(10)
        if c is not None:
            started += 1
            last = bytes([i % 256]) * 10
            m.put(last, _done(i), c)
    assert started < 12  # 3-4 until paused, then one probe in 8 calls
    # the caller starts hashing: a probe call's id is taken, prefetch resumes for every call
    while True:
        c = m.begin(10)
        if c is not None:
            o = bytes(10)
            m.put(o, _done("p"), c)
            assert m.take(o) == "p"
            break
    assert all(m.begin(10) is not None for _ in range(5))


class _DeferringPool:
    """Runs the piece fills at once and holds every other task (the SHA-1s) until run_held()."""

    def __init__(self):
        self.held = []

    def submit(self, fn, *args):
        from storb_amd import piece as P
        f = Future()
        if fn is P._fill:
            fn(*args)
            f.set_result(None)
        else:
            self.held.append((f, fn, args))
        return f

    def run_held(self):
        for f, fn, args in self.held:
            f.set_result(fn(*args))


class _OracleRawEngine:
    """encode_host_raw through the CPU oracle (test infrastructure only)."""

    def encode_host_raw(self, chunks, shapes, digests=False, staged=False):
        import numpy as np
        from oracle import cfec
        bufs, layout, o = [], [], 0
        for c, (k, m) in zip(chunks, shapes):
            blocks = cfec.easy_encode(bytes(c), k, m)
            B = len(blocks[0])
            bufs.extend(blocks[k:])
            layout.append((o, B, m - k))
            o += (m - k) * B
        return np.frombuffer(b"".join(bufs) or b"\0", dtype=np.uint8).copy(), layout


def test_hash_tasks_keep_their_pieces_alive(monkeypatch):
    """a queued or running SHA-1 of encode_chunk's pieces must hold the piece
    object itself, not only a raw view of its buffer, so neither the memo's eviction nor the caller
    dropping the piece can free the bytes under the hash."""
    import gc
    import hashlib
    import random
    import sys

    from storb_amd import piece as P

    pool = _DeferringPool()
    monkeypatch.setattr(P, "_pool", lambda name: pool)
    monkeypatch.setattr(P, "get_engine", lambda: _OracleRawEngine())
    chunk = random.Random(7).randbytes(3 * 300_000 + 11)
    k, m, B, padlen = 4, 6, -(-len(chunk) // 4), 4 * (-(-len(chunk) // 4)) - len(chunk)
    pieces, futs = P._pieces_parallel([chunk], [(k, m, B, padlen)], hash_ids=True)
    ps, fs = pieces[0], futs[0]
    assert len(ps) == m and len(pool.held) == m
    want = [hashlib.sha1(p).hexdigest() for p in ps]
    for p, (_, fn, args) in zip(ps, pool.held):
        assert any(a is p for a in args), "hash task does not hold its piece"
    # the caller and the memo drop every piece while the hashes are still queued
    refs = [sys.getrefcount(p) for p in ps]
    del pieces, ps, p
    gc.collect()
    assert all(r >= 3 for r in refs)
    pool.run_held()
    assert [f.result() for f in fs] == want

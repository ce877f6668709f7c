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

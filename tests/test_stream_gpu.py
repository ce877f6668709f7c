"""GPU: the streamed upload / download pipelines at the API storb calls.

* reconstruct_data_stream (/root/reference/storb/util/piece.py:239-263, consumed chunk by
  chunk into the HTTP response at validator.py:1630-1638): >= 64 chunks of mixed sizes and
  shapes, some with lost data pieces (GPU recovery), some complete (joined), decoded in many
  small windows so window w+1 runs on the worker while window w is consumed; bytes checked
  against the source and the oracle's decode; the "Not enough pieces" ValueError surfaces in
  order, after every earlier chunk;
* encode_chunks_stream (the upload loop's produce/consume, validator.py:1338-1446): the same
  EncodedChunks as per-chunk encode_chunk, parity equal to the oracle's, piece ids equal to
  hashlib's;
* piece_hash's memo of encode_chunk's prefetched ids: identity hits, equal-but-distinct
  objects hashed afresh, disabled mode;
* the reassemble kernel's pure-copy form (R = 0: every primary present), which the host
  decode path no longer sends to the GPU, through the device ABI.
"""

import hashlib
import random

import numpy as np
import pytest

from oracle import cfec

pytestmark = pytest.mark.gpu

from storb_amd import piece  # noqa: E402


def _encode_file(data, chunk_size):
    chunks, pieces = [], []
    for ci in range(0, len(data), chunk_size):
        info = piece.encode_chunk(data[ci:ci + chunk_size], ci // chunk_size)
        chunks.append(info.model_copy(update={"pieces": None}))
        pieces.extend(info.pieces)
    return chunks, pieces


def _mixed_objects(seed, count):
    rng = random.Random(seed)
    out = []
    for _ in range(count):
        n = int(np.exp(rng.uniform(np.log(300), np.log(3 << 20))))
        out.append(rng.randbytes(n))
    return out


def test_reconstruct_stream_mixed_chunks_many_windows():
    rng = random.Random(64)
    objs = _mixed_objects(64, 80)  # 80 chunks, sizes 300 B .. 3 MiB -> k from 1 to 8
    encoded = [piece.encode_chunk(o, i) for i, o in enumerate(objs)]
    chunks = [e.model_copy(update={"pieces": None}) for e in encoded]
    pieces, expect = [], []
    for i, e in enumerate(encoded):
        ps = list(e.pieces)
        if i % 3:  # lose up to m-k pieces, data pieces first when possible
            lose = min(e.m - e.k, max(1, e.k // 2))
            drop = set(rng.sample(range(e.k), min(lose, e.k)))
            ps = [p for p in ps if p.piece_idx not in drop]
        pieces.extend(ps)
        # the oracle's decode of the pieces reconstruct will use (first k by piece_idx)
        use = sorted(ps, key=lambda p: p.piece_idx)[:e.k]
        expect.append(cfec.easy_decode([p.data for p in use], [p.piece_idx for p in use], e.padlen, e.k, e.m))
    assert expect == objs
    rng.shuffle(pieces)
    got = list(piece.reconstruct_data_stream(pieces, chunks, window_bytes=2 << 20))
    assert len(got) == len(objs)
    for i, (g, o) in enumerate(zip(got, objs)):
        assert type(g) is bytes and g == o, i
    assert piece.reconstruct_data(pieces, chunks) == b"".join(objs)


def test_reconstruct_stream_error_in_order():
    data = random.Random(5).randbytes(48 << 20)  # 48 MiB -> chunk 2 MiB (piece_length), 24 chunks
    cs = piece.piece_length(len(data))
    chunks, pieces = _encode_file(data, cs)
    bad = 13
    k = chunks[bad].k
    survivors = [p for p in pieces if p.chunk_idx != bad or p.piece_idx < k - 1]  # k-1 pieces left
    it = piece.reconstruct_data_stream(survivors, chunks, window_bytes=5 << 20)
    got = []
    with pytest.raises(ValueError, match=f"Not enough pieces to reconstruct chunk {bad}"):
        for b in it:
            got.append(b)
    assert b"".join(got) == data[:bad * cs]


def test_encode_stream_matches_per_chunk_and_oracle():
    objs = _mixed_objects(7, 70)

    def gen():  # a one-pass producer, as the upload loop's queue
        yield from objs

    ref = [piece.encode_chunk(o, 100 + i) for i, o in enumerate(objs)]
    got = list(piece.encode_chunks_stream(gen(), 100, window_bytes=3 << 20))
    assert [e.model_dump() for e in got] == [e.model_dump() for e in ref]
    withids = list(piece.encode_chunks_stream(iter(objs), 100, piece_ids=True, window_bytes=8 << 20))
    for (ec, ids), o, r in zip(withids, objs, ref):
        assert ec.model_dump() == r.model_dump()
        blocks = cfec.easy_encode(o, ec.k, ec.m)
        assert [p.data for p in ec.pieces] == blocks
        assert ids == [hashlib.sha1(b).hexdigest() for b in blocks]
    assert list(piece.encode_chunks_stream(iter([]))) == []


def test_piece_hash_memo_identity():
    chunk = random.Random(9).randbytes(700_000)
    info = piece.encode_chunk(chunk, 0)
    want = [hashlib.sha1(p.data).hexdigest() for p in info.pieces]
    # an equal but distinct object is hashed afresh (no memo hit), and gives the same digest
    assert piece.piece_hash(bytes(bytearray(info.pieces[0].data))) == want[0]
    assert [piece.piece_hash(p.data) for p in info.pieces] == want
    assert [piece.piece_hash(p.data) for p in info.pieces] == want  # second call: hashlib
    old = piece.PREFETCH_PIECE_IDS
    piece.PREFETCH_PIECE_IDS = False
    try:
        info2 = piece.encode_chunk(chunk, 0)
        assert info2.model_dump() == info.model_dump()
        assert [piece.piece_hash(p.data) for p in info2.pieces] == want
    finally:
        piece.PREFETCH_PIECE_IDS = old


def test_reassemble_kernel_pure_copy_through_abi(engine):
    """Every primary present (e = 0): the device decode is the R = 0 copy kernel; host-side
    decode_host joins such chunks without the GPU, so the kernel is exercised here directly."""
    from storb_amd._lib import DEC_DTYPE

    rng = random.Random(3)
    cases = [(4, 6, 1 << 20), (10, 14, 65536), (8, 11, 4096 * 8 + 5), (3, 5, 100), (16, 24, 16 * 4099)]
    for k, m, n in cases:
        data = rng.randbytes(n)
        blocks = cfec.easy_encode(data, k, m)
        B = len(blocks[0])
        order = list(range(k))
        rng.shuffle(order)
        buf = np.frombuffer(b"".join(blocks[s] for s in order), np.uint8).copy()
        d = np.zeros(1, dtype=DEC_DTYPE)
        d["B"], d["padlen"], d["k"], d["m"], d["slot0"], d["out_off"] = B, B * k - n, k, m, 0, 0
        offs = np.arange(k, dtype=np.uint64) * B
        out = np.zeros(n, np.uint8)
        engine.decode_batch(d, np.array(order, np.int32), offs, buf, out, host=True)
        assert out.tobytes() == data, (k, m, n)


@pytest.mark.parametrize("gpu_ids", [True, False])
def test_encode_stream_piece_ids_large_pieces(gpu_ids, monkeypatch):
    """Upload stream with piece ids over chunks whose pieces are all >= PARALLEL_COPY_MIN (the
    GPU SHA-1 path when GPU_PIECE_IDS, hashlib on the pool otherwise): ragged chunk sizes,
    several windows, the last chunk short; pieces against the oracle and ids against hashlib."""
    monkeypatch.setattr(piece, "GPU_PIECE_IDS", gpu_ids)
    rng = random.Random(31)
    # >= 2.5 MiB: 512 KiB pieces (piece_length), so every block is >= 256 KiB even when ragged
    objs = [rng.randbytes(rng.randrange(5 << 19, 6 << 20)) for _ in range(9)] + [rng.randbytes(3 << 20)]
    got = list(piece.encode_chunks_stream(iter(objs), 7, piece_ids=True, window_bytes=12 << 20))
    assert len(got) == len(objs)
    for i, ((ec, ids), o) in enumerate(zip(got, objs)):
        assert ec.chunk_idx == 7 + i
        blocks = cfec.easy_encode(o, ec.k, ec.m)
        assert min(len(b) for b in blocks) >= piece.PARALLEL_COPY_MIN
        assert [p.data for p in ec.pieces] == blocks
        assert ids == [hashlib.sha1(b).hexdigest() for b in blocks]


def test_validator_bytearray_chunks():
    """The validator hands encode_chunk a bytearray: `copy.copy(buffer[:chunk_size])` of its
    read buffer (/root/reference/storb/validator/validator.py:1356-1380).  The same objects
    through encode_chunk, encode_chunks and encode_chunks_stream (with and without ids), small
    and large pieces: pieces against the oracle, ids against hashlib."""
    import copy

    rng = random.Random(1356)
    buffer = bytearray(rng.randbytes(12 << 20))
    sizes = [4096 + 3, 256 << 10, 700_000, 1 << 20, 3 << 20, (5 << 20) + 17]
    chunks, off = [], 0
    for n in sizes:
        chunks.append(copy.copy(buffer[off:off + n]))
        off += n
    assert all(type(c) is bytearray for c in chunks)
    want = []
    for c in chunks:
        k, m, _, _ = piece.chunk_shape(len(c))
        want.append(cfec.easy_encode(bytes(c), k, m))
    for i, c in enumerate(chunks):
        ec = piece.encode_chunk(c, i)
        assert [p.data for p in ec.pieces] == want[i], i
        assert all(type(p.data) is bytes for p in ec.pieces)
        assert [piece.piece_hash(p.data) for p in ec.pieces] == [hashlib.sha1(b).hexdigest() for b in want[i]]
    for i, ec in enumerate(piece.encode_chunks(chunks)):
        assert ec.chunk_idx == i and [p.data for p in ec.pieces] == want[i], i
    for i, ec in enumerate(piece.encode_chunks_stream(iter(chunks), window_bytes=4 << 20)):
        assert [p.data for p in ec.pieces] == want[i], i
    got = list(piece.encode_chunks_stream(iter(chunks), piece_ids=True, window_bytes=6 << 20))
    for i, (ec, ids) in enumerate(got):
        assert [p.data for p in ec.pieces] == want[i], i
        assert ids == [hashlib.sha1(b).hexdigest() for b in want[i]], i
    # decoding the bytearray-born pieces with data pieces lost gives the bytearray's bytes back
    ecs = piece.encode_chunks(chunks)
    pieces = [p for ec in ecs for p in ec.pieces if p.piece_idx != 0 or ec.k == 1]
    metas = [ec.model_copy(update={"pieces": None}) for ec in ecs]
    assert piece.reconstruct_data(pieces, metas) == b"".join(bytes(c) for c in chunks)


def _stream_fixture(seed, n_chunks=10, size=600_000):
    rng = random.Random(seed)
    objs = [rng.randbytes(size + 97 * i) for i in range(n_chunks)]
    encoded = [piece.encode_chunk(o, i) for i, o in enumerate(objs)]
    chunks = [e.model_copy(update={"pieces": None}) for e in encoded]
    return objs, encoded, chunks


@pytest.mark.parametrize("fault", ["duplicate_idx", "truncated_piece", "bad_sharenum", "bad_sharenum_spare"])
def test_reconstruct_stream_precondition_error_after_prefix(fault):
    """A zfec precondition failure in the middle of a window: every chunk before
    the bad one is still yielded, then the error is raised, as the reference's per-chunk loop
    does (piece.py:246-263)."""
    objs, encoded, chunks = _stream_fixture(11)
    bad = 6
    pieces = []
    for e in encoded:
        ps = [p for p in e.pieces if p.piece_idx != 0]  # data piece 0 lost: GPU recovery everywhere
        if e.chunk_idx == bad:
            if fault == "duplicate_idx":
                ps = [ps[0].model_copy(), *ps[:e.k - 1]]  # k pieces, two with the same piece_idx
            elif fault == "truncated_piece":
                ps[1] = ps[1].model_copy(update={"data": ps[1].data[:-1]})
            elif fault == "bad_sharenum":  # exactly k pieces, one of them with sharenum -1
                ps = ps[:e.k]
                ps[1] = ps[1].model_copy(update={"piece_idx": -1})
            else:  # bad_sharenum_spare: a spare valid piece beside it, which the chooser uses
                ps[1] = ps[1].model_copy(update={"piece_idx": -1})
        pieces.extend(ps)
    got = []
    if fault == "bad_sharenum_spare":  # sec_decode_choose never picks an invalid sharenum
        assert b"".join(piece.reconstruct_data_stream(pieces, chunks, window_bytes=64 << 20)) == b"".join(objs)
        return
    with pytest.raises((piece.Error, ValueError)):
        for b in piece.reconstruct_data_stream(pieces, chunks, window_bytes=64 << 20):  # one window
            got.append(b)
    assert got == objs[:bad]


def test_encode_stream_error_after_prefix():
    rng = random.Random(12)
    objs = [rng.randbytes(300_000 + i) for i in range(7)]
    objs[4] = b""  # piece_length(0): the reference's ValueError (math domain error)
    got = []
    with pytest.raises(ValueError):
        for ec in piece.encode_chunks_stream(iter(objs), window_bytes=64 << 20):
            got.append(ec)
    assert [len(ec.pieces) for ec in got] == [piece.chunk_shape(len(o))[1] for o in objs[:4]]
    for ec, o in zip(got, objs):
        assert [p.data for p in ec.pieces] == cfec.easy_encode(o, ec.k, ec.m)


def test_streams_closed_early_and_concurrent():
    """Consumers that stop early (client disconnect) do not hold up other streams, and several
    streams on request threads run side by side."""
    import threading

    objs, encoded, chunks = _stream_fixture(13, n_chunks=24, size=1 << 20)
    pieces = [p for e in encoded for p in e.pieces if p.piece_idx != 1]
    for _ in range(3):
        it = piece.reconstruct_data_stream(pieces, chunks, window_bytes=2 << 20)
        assert next(it) == objs[0]
        it.close()
        it2 = piece.encode_chunks_stream(iter(objs), window_bytes=2 << 20)
        assert next(it2).model_dump() == encoded[0].model_dump()
        it2.close()
    results, errs = {}, []

    def run(t):
        try:
            results[t] = b"".join(piece.reconstruct_data_stream(pieces, chunks, window_bytes=3 << 20))
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    ts = [threading.Thread(target=run, args=(t,)) for t in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(120)
    assert not errs and len(results) == 4
    assert all(v == b"".join(objs) for v in results.values())


def test_piece_id_memo_bounded_without_piece_hash():
    """A caller that never asks for piece ids (ADVICE / VERDICT r02): encode_chunk keeps at most
    the memo's cap (and its last `keep_calls` calls) of piece bytes alive, and stops prefetching
    once whole calls go unused; the ids are right again as soon as the caller hashes."""
    memo = piece._memo
    chunk_objs = [random.Random(40 + i).randbytes(1 << 20) for i in range(3)]
    per_call = sum(len(p.data) for p in piece.encode_chunk(chunk_objs[0], 0).pieces)
    for i in range(40):
        piece.encode_chunk(chunk_objs[i % 3], i)
        held = memo.held_bytes()
        assert held <= memo.max_bytes and held <= memo.keep_calls * per_call, (i, held)
    assert memo._idle >= memo.idle_calls  # prefetch paused
    info = piece.encode_chunk(chunk_objs[0], 0)
    assert [piece.piece_hash(p.data) for p in info.pieces] == [hashlib.sha1(p.data).hexdigest() for p in info.pieces]

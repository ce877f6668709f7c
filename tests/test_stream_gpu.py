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

"""The reference's own hot-path tests (/root/reference/storb/util/piece_test.py) run against the
drop-in ``storb_amd.piece``, plus the cases the reference lacks: a deterministic parity-based
recovery, the reference's positional-sharenum behaviour reproduced on request, batching, and
oracle-checked pieces.  The reference draws unseeded ``randbytes``; here inputs are seeded."""

import math
import random
from io import BytesIO

import pytest

from oracle import cfec

pytestmark = pytest.mark.gpu

from storb_amd.piece import (  # noqa: E402
    EncodedChunk,
    Piece,
    PieceType,
    decode_chunk,
    decode_chunks,
    encode_chunk,
    encode_chunks,
    piece_hash,
    piece_length,
    reconstruct_data,
    reconstruct_data_stream,
)

TEST_FILE_SIZE = 1024 * 1024  # piece_test.py:15


def _encode_file(data):
    """piece_test.py:24-37: stream the file in piece_length(file) chunks through encode_chunk."""
    f = BytesIO(data)
    chunk_size = piece_length(len(data))
    chunks, pieces, expected = [], [], 0
    for chunk_idx, chunk in enumerate(iter(lambda: f.read(chunk_size), b"")):
        info = encode_chunk(chunk, chunk_idx)
        chunks.append(info.model_copy(update={"pieces": None}))
        piece_size = piece_length(info.original_chunk_size)
        expected += info.m * math.ceil(info.chunk_size / piece_size)
        pieces.extend(info.pieces)
    return chunk_size, chunks, pieces, expected


def test_split_data():  # piece_test.py:18-45
    data = random.Random(18).randbytes(TEST_FILE_SIZE)
    chunk_size, chunks, pieces, expected = _encode_file(data)
    assert len(chunks) == math.ceil(TEST_FILE_SIZE / chunk_size)
    assert len(pieces) == expected == 12  # 4 chunks x zfec(2,3)


def test_reconstruct_data():  # piece_test.py:48-80
    data = random.Random(48).randbytes(TEST_FILE_SIZE)
    _, chunks, pieces, _ = _encode_file(data)
    random.Random(1).shuffle(pieces)
    assert reconstruct_data(pieces, chunks) == data


def test_reconstruct_data_corrupted():  # piece_test.py:83-125, seeded; drop loop as the reference
    rng = random.Random(83)
    data = rng.randbytes(TEST_FILE_SIZE)
    _, chunks, pieces, _ = _encode_file(data)
    for _ in list(pieces):
        max_pieces_to_lose = math.ceil(len(pieces) * 0.3)
        keep = rng.sample(pieces, len(pieces) - max_pieces_to_lose)
        keep_blocks = [p.piece_idx for p in keep]
        pieces = [p for p in pieces if p.piece_idx in keep_blocks]
    rng.shuffle(pieces)
    # with true sharenums any surviving k-subset decodes (the reference fails ~4.5% of runs)
    assert reconstruct_data(pieces, chunks) == data


def test_parity_recovery_every_chunk():
    """Deterministic erasure the reference never exercises: drop data piece 0 of every chunk."""
    data = random.Random(7).randbytes(4 * 1024 * 1024)  # 8 chunks x zfec(4,6)
    _, chunks, pieces, _ = _encode_file(data)
    assert {(c.k, c.m) for c in chunks} == {(4, 6)}
    survivors = [p for p in pieces if p.piece_idx not in (0, 2)]
    assert reconstruct_data(survivors, chunks) == data
    assert b"".join(reconstruct_data_stream(survivors, chunks)) == data


def test_pieces_match_oracle_and_types():
    chunk = random.Random(11).randbytes(512 * 1024 + 333)
    info = encode_chunk(chunk, 3)
    blocks = cfec.easy_encode(chunk, info.k, info.m)
    assert [p.data for p in info.pieces] == blocks
    assert [p.piece_type for p in info.pieces] == [PieceType.Data] * info.k + [PieceType.Parity] * (info.m - info.k)
    assert info.padlen == info.chunk_size * info.k - len(chunk)
    assert all(p.chunk_idx == 3 for p in info.pieces)
    assert piece_hash(info.pieces[0].data) == __import__("hashlib").sha1(blocks[0]).hexdigest()


def test_positional_sharenums_reproduces_reference():
    chunk = random.Random(12).randbytes(1 << 20)
    info = encode_chunk(chunk, 0)  # zfec(4,6)
    k = info.k
    # pieces 0..k-1 present: reference (positional) and drop-in agree
    info.pieces = sorted(info.pieces, key=lambda p: p.piece_idx)
    assert decode_chunk(info) == decode_chunk(info, positional_sharenums=True) == chunk
    # piece 1 missing: the reference's positional sharenums give the oracle's wrong bytes
    info.pieces = [p for p in info.pieces if p.piece_idx != 1]
    blocks = [p.data for p in info.pieces[:k]]
    assert decode_chunk(info, positional_sharenums=True) == cfec.easy_decode(blocks, list(range(k)), info.padlen,
                                                                             k, info.m)
    assert decode_chunk(info) == chunk


def test_batched_entry_points():
    rng = random.Random(13)
    chunks = [rng.randbytes(rng.randrange(1, 3 << 20)) for _ in range(12)]
    one = [encode_chunk(c, i) for i, c in enumerate(chunks)]
    many = encode_chunks(chunks)
    assert [e.model_dump() for e in one] == [e.model_dump() for e in many]
    assert decode_chunks(many) == b"".join(chunks)


def test_errors():
    with pytest.raises(ValueError):
        encode_chunk(b"", 0)  # math.log2(0), as the reference
    data = random.Random(14).randbytes(TEST_FILE_SIZE)
    _, chunks, pieces, _ = _encode_file(data)
    with pytest.raises(ValueError, match="Not enough pieces"):
        reconstruct_data([p for p in pieces if p.chunk_idx != 2 or p.piece_idx == 0], chunks)


def test_models_roundtrip_json():
    info = encode_chunk(b"hello world" * 100, 0)
    again = EncodedChunk.model_validate_json(info.model_dump_json())
    assert again == info
    assert Piece(chunk_idx=0, piece_idx=1, piece_type=1, data=b"x").piece_type == 1

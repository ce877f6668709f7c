"""Drop-in for /root/reference/storb/util/piece.py on the MI355X engine.

Same names, models, signatures and error behaviour as the reference module; the
Reed–Solomon arithmetic runs in libstorbec.so's HIP kernels instead of zfec.

Deliberate differences (documented in DESIGN.md §Boundary):

* ``decode_chunk`` passes each piece's true ``piece_idx`` as its zfec sharenum.  The
  reference passes list positions (piece.py:189-194), which returns wrong bytes whenever
  the pieces handed over are not exactly blocks 0..k-1.  On every input where the reference
  is correct both give identical bytes.  ``decode_chunk(..., positional_sharenums=True)``
  reproduces the reference's behaviour exactly.
* ``reconstruct_data`` decodes all chunks in ONE batched GPU call instead of one zfec call
  per chunk (same output; the "not enough pieces" ValueError is raised before any decode).
* the two ``print()`` calls per piece in ``encode_chunk`` (piece.py:140,151) are debug
  logs here.
* extra batch entry points ``encode_chunks`` / ``decode_chunks`` for callers that can hand
  over many chunks at once (the validator's upload loop, validator.py:1352-1431).
"""

from __future__ import annotations

import hashlib
import logging
import math
import typing
from collections.abc import Iterator
from enum import IntEnum

from pydantic import BaseModel, ConfigDict, Field

from .constants import MAX_PIECE_SIZE, MIN_PIECE_SIZE, PIECE_LENGTH_OFFSET, PIECE_LENGTH_SCALING
from .easyfec import Decoder, Encoder, Error
from .engine import get_engine

logger = logging.getLogger(__name__)

__all__ = [
    "PieceType", "Piece", "EncodedChunk", "ProcessedPieceInfo", "EncodedPieces", "piece_hash", "piece_length",
    "encode_chunk", "decode_chunk", "reconstruct_data", "reconstruct_data_stream", "encode_chunks",
    "decode_chunks", "chunk_shape", "piece_hashes", "encode_chunks_with_ids", "Encoder", "Decoder", "Error",
]


class PieceType(IntEnum):  # piece.py:21-23
    Data = 0
    Parity = 1


class Piece(BaseModel):  # piece.py:26-33
    model_config = ConfigDict(use_enum_values=True)

    chunk_idx: int
    piece_idx: int
    piece_type: PieceType
    data: bytes


class EncodedChunk(BaseModel):  # piece.py:36-43
    pieces: list[Piece] = Field(default=None)
    chunk_idx: int
    k: int  # Number of data blocks
    m: int  # Total blocks (data + parity)
    chunk_size: int
    padlen: int
    original_chunk_size: int


class ProcessedPieceInfo(Piece):  # piece.py:46-47
    piece_id: typing.Optional[str] = Field(default=None)


class EncodedPieces(BaseModel):  # piece.py:50-51
    pieces: list[Piece]


def piece_hash(data: bytes) -> str:
    """SHA-1 hex digest of a piece (piece.py:54-68)."""
    return hashlib.sha1(data).hexdigest()


def piece_hashes(datas: typing.Sequence[bytes]) -> list[str]:
    """``[piece_hash(d) for d in datas]`` computed by the GPU SHA-1 kernel in one call."""
    if not datas:
        return []
    return [d.hex() for d in get_engine().sha1_host(list(datas))]


def piece_length(content_length: int, min_size: int = MIN_PIECE_SIZE, max_size: int = MAX_PIECE_SIZE) -> int:
    """Piece size for a content length, clamped to [min_size, max_size] (piece.py:71-100)."""
    exponent = int((math.log2(content_length) * PIECE_LENGTH_SCALING) + PIECE_LENGTH_OFFSET)
    length = 1 << exponent
    if length < min_size:
        return min_size
    elif length > max_size:
        return max_size
    return length


def chunk_shape(chunk_size: int) -> tuple[int, int, int, int]:
    """(k, m, B, padlen) encode_chunk uses for a chunk of `chunk_size` bytes (piece.py:116-134)."""
    piece_size = piece_length(chunk_size)
    expected_data_pieces = math.ceil(chunk_size / piece_size)
    expected_parity_pieces = math.ceil(expected_data_pieces / 2)
    k = expected_data_pieces
    m = k + expected_parity_pieces
    zfec_chunk_size = (chunk_size + (k - 1)) // k
    padlen = (zfec_chunk_size * k) - chunk_size
    return k, m, zfec_chunk_size, padlen


def _split(chunk, k: int, B: int) -> list[bytes]:
    mv = memoryview(chunk).cast("B")
    prim = [bytes(mv[i * B:(i + 1) * B]) for i in range(k)]
    if len(prim[-1]) != B:
        prim[-1] = prim[-1] + b"\x00" * (B - len(prim[-1]))
    return prim


def _build(chunk_idx: int, k: int, m: int, B: int, padlen: int, n: int, blocks: list[bytes]) -> EncodedChunk:
    pieces = []
    for i, block in enumerate(blocks):
        piece_type = PieceType.Data if i < k else PieceType.Parity
        logger.debug("Encoding piece %d with length %d", i, len(block))
        pieces.append(Piece(piece_type=piece_type, data=block, chunk_idx=chunk_idx, piece_idx=i))
    return EncodedChunk(pieces=pieces, chunk_idx=chunk_idx, k=k, m=m, chunk_size=B, padlen=padlen,
                        original_chunk_size=n)


def encode_chunk(chunk: bytes, chunk_idx: int) -> EncodedChunk:
    """Encode one chunk into k data + ceil(k/2) parity pieces (piece.py:103-166)."""
    chunk_size = len(chunk)
    piece_size = piece_length(chunk_size)  # ValueError for an empty chunk, as the reference
    logger.debug("[encode_chunk] chunk %d: %d bytes, piece_size = %d", chunk_idx, chunk_size, piece_size)
    k, m, B, padlen = chunk_shape(chunk_size)
    encoded_pieces = Encoder(k, m).encode(chunk)
    enc = _build(chunk_idx, k, m, B, padlen, chunk_size, encoded_pieces)
    logger.debug("[encode_chunk] chunk %d: k=%d, m=%d, encoded %d blocks", chunk_idx, k, m, len(enc.pieces))
    return enc


def encode_chunks(chunks: typing.Sequence[bytes], first_chunk_idx: int = 0) -> list[EncodedChunk]:
    """Batched ``encode_chunk`` over many chunks in ONE GPU call; chunk i gets index first+i."""
    shapes = []
    for c in chunks:
        n = len(c)
        piece_length(n)  # same ValueError as encode_chunk for n == 0
        shapes.append(chunk_shape(n))
    parity = get_engine().encode_host(list(chunks), [(k, m) for (k, m, _, _) in shapes]) if chunks else []
    out = []
    for i, (c, (k, m, B, padlen), par) in enumerate(zip(chunks, shapes, parity)):
        out.append(_build(first_chunk_idx + i, k, m, B, padlen, len(c), _split(c, k, B) + par))
    return out


def encode_chunks_with_ids(chunks: typing.Sequence[bytes],
                           first_chunk_idx: int = 0) -> tuple[list[EncodedChunk], list[list[str]]]:
    """``encode_chunks`` plus every piece's id (``piece_hash``, the SHA-1 the validator computes
    right after encoding, validator.py:1081), hashed on the GPU while the pieces are still there."""
    shapes = []
    for c in chunks:
        n = len(c)
        piece_length(n)
        shapes.append(chunk_shape(n))
    if not chunks:
        return [], []
    parity, digs = get_engine().encode_host(list(chunks), [(k, m) for (k, m, _, _) in shapes], digests=True)
    out = []
    for i, (c, (k, m, B, padlen), par) in enumerate(zip(chunks, shapes, parity)):
        out.append(_build(first_chunk_idx + i, k, m, B, padlen, len(c), _split(c, k, B) + par))
    return out, [[d.hex() for d in ds] for ds in digs]


def _sharenums(encoded_chunk: EncodedChunk, positional: bool):
    k = encoded_chunk.k
    pieces = encoded_chunk.pieces
    if positional:  # the reference's own behaviour, piece.py:189-194
        if len(pieces) > k:
            use = pieces[:k]
            return [p.data for p in use], list(range(k))
        return [p.data for p in pieces], list(range(len(pieces)))
    use = pieces[:k] if len(pieces) > k else pieces
    return [p.data for p in use], [p.piece_idx for p in use]


def decode_chunk(encoded_chunk: EncodedChunk, *, positional_sharenums: bool = False) -> bytes:
    """Decode one chunk from its pieces (piece.py:169-198); see module doc for sharenums."""
    blocks, sharenums = _sharenums(encoded_chunk, positional_sharenums)
    decoder = Decoder(encoded_chunk.k, encoded_chunk.m)
    return decoder.decode(blocks, sharenums, encoded_chunk.padlen)


def decode_chunks(encoded_chunks: typing.Sequence[EncodedChunk], *, positional_sharenums: bool = False) -> bytes:
    """Batched ``decode_chunk``: the concatenation of every chunk's bytes, one GPU call."""
    items = []
    for ch in encoded_chunks:
        if not (1 <= ch.k <= ch.m <= 256):
            raise Error(f"Precondition violation: 1 <= k <= m <= 256 required (k={ch.k}, m={ch.m})")
        blocks, sharenums = _sharenums(ch, positional_sharenums)
        B = len(blocks[0]) if blocks else 0
        if not (0 <= ch.padlen <= ch.k * B):
            # out-of-range padlen: keep easyfec's slicing semantics on the per-chunk path
            return b"".join(decode_chunk(c, positional_sharenums=positional_sharenums) for c in encoded_chunks)
        items.append((ch.k, ch.m, blocks, sharenums, ch.padlen))
    return get_engine().decode_host(items) if items else b""


def _relevant(pieces: list[Piece], chunk: EncodedChunk) -> list[Piece]:
    relevant = [piece for piece in pieces if piece.chunk_idx == chunk.chunk_idx]
    relevant.sort(key=lambda p: p.piece_idx)
    if len(relevant) < chunk.k:
        raise ValueError(f"Not enough pieces to reconstruct chunk {chunk.chunk_idx}")
    return relevant


def reconstruct_data(pieces: list[Piece], chunks: list[EncodedChunk]) -> bytes:
    """Reconstruct the original bytes from pieces (piece.py:201-236), one batched decode."""
    by_chunk: dict[int, list[Piece]] = {}
    for p in pieces:
        by_chunk.setdefault(p.chunk_idx, []).append(p)
    for chunk in chunks:
        relevant = sorted(by_chunk.get(chunk.chunk_idx, []), key=lambda p: p.piece_idx)
        if len(relevant) < chunk.k:
            raise ValueError(f"Not enough pieces to reconstruct chunk {chunk.chunk_idx}")
        chunk.pieces = relevant
    return decode_chunks(chunks)


def reconstruct_data_stream(pieces: list[Piece], chunks: list[EncodedChunk]) -> Iterator[bytes]:
    """Yield the reconstructed bytes chunk by chunk (piece.py:239-263)."""
    for chunk in chunks:
        chunk.pieces = _relevant(pieces, chunk)
        yield decode_chunk(chunk)

"""CPU: the PRODUCT's policy functions (storb_amd.piece.piece_length / chunk_shape) pinned to
the committed policy table (tests/golden/golden.json "policy") and to
the reference's formula at every power-of-two boundary from 1 B to 1 TiB.

Reference: /root/reference/storb/util/piece.py:71-100 (piece_length), :116-134 (k, m, B,
padlen inside encode_chunk); the validator picks the chunk size with the same function
(/root/reference/storb/validator/validator.py:1324).
"""

import json
import math
import os

import pytest

from oracle import zfec_ref
from storb_amd import piece

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))

KIB, MIB, GIB, TIB = 1 << 10, 1 << 20, 1 << 30, 1 << 40

# file size -> (chunk, #chunks, piece, k, m, B)
APPENDIX_B = [
    (4 * KIB, 16 * KIB, 1, 16 * KIB, 1, 2, 4096),
    (256 * KIB, 128 * KIB, 2, 64 * KIB, 2, 3, 65536),
    (1 * MIB, 256 * KIB, 4, 128 * KIB, 2, 3, 131072),
    (4 * MIB, 512 * KIB, 8, 128 * KIB, 4, 6, 131072),
    (16 * MIB, 1 * MIB, 16, 256 * KIB, 4, 6, 262144),
    (64 * MIB, 2 * MIB, 32, 256 * KIB, 8, 12, 262144),
    (256 * MIB, 4 * MIB, 64, 512 * KIB, 8, 12, 524288),
    (1 * GIB, 8 * MIB, 128, 512 * KIB, 16, 24, 524288),
    (16 * GIB, 32 * MIB, 512, 1 * MIB, 32, 48, 1048576),
    (1 * TIB, 256 * MIB, 4096, 4 * MIB, 64, 96, 4194304),
]


@pytest.mark.parametrize("row", GOLDEN["policy"], ids=lambda p: str(p["file_size"]))
def test_product_policy_matches_golden_table(row):
    size = row["file_size"]
    chunk = piece.piece_length(size)
    assert chunk == row["chunk"]
    assert math.ceil(size / chunk) == row["chunks"]
    first = min(chunk, size)  # the first chunk's byte count
    assert piece.piece_length(first) == row["piece"]
    assert piece.chunk_shape(first) == (row["k"], row["m"], row["B"], row["padlen"])


@pytest.mark.parametrize("row", APPENDIX_B, ids=lambda r: str(r[0]))
def test_product_policy_matches_survey_appendix_b(row):
    size, chunk, nchunks, pce, k, m, B = row
    assert piece.piece_length(size) == chunk
    assert math.ceil(size / chunk) == nchunks
    first = min(chunk, size)  # a 4 KiB file is one 4 KiB chunk
    assert piece.piece_length(first) == pce
    assert piece.chunk_shape(first) == (k, m, B, 0)


def _boundary_sizes():
    out = set()
    for e in range(0, 41):  # 1 B .. 1 TiB
        for d in (-1, 0, 1):
            if (1 << e) + d >= 1:
                out.add((1 << e) + d)
    return sorted(out)


def test_product_policy_equals_reference_formula_at_every_boundary():
    # both restate piece.py:71-100's double expression; this checks the product function
    # itself (not only the oracle) at every 2^e - 1, 2^e, 2^e + 1 up to 1 TiB, where the
    # truncated log2 changes value
    for n in _boundary_sizes():
        assert piece.piece_length(n) == zfec_ref.piece_length(n), n
        assert piece.chunk_shape(n) == zfec_ref.chunk_shape(n), n
    # the clamps: 16 KiB floor, 256 MiB ceiling
    assert piece.piece_length(1) == 16 * KIB
    assert piece.piece_length(1 << 62) == 256 * MIB


def test_product_policy_custom_clamps_and_empty():
    assert piece.piece_length(1 << 20, min_size=1 << 19) == 1 << 19
    assert piece.piece_length(1 << 20, max_size=1 << 16) == 1 << 16
    with pytest.raises(ValueError):  # math.log2(0), as the reference
        piece.piece_length(0)


def test_new_bytes_fill_in_place():
    # storb_amd.piece._new_bytes: a fresh bytes object filled through its buffer before it is
    # shared (the parallel piece copies); it must behave as any other bytes afterwards
    from storb_amd.piece import _fill, _new_bytes
    import numpy as np

    b, v = _new_bytes(1000)
    _fill(v, np.arange(700, dtype=np.uint8))
    want = bytes(np.arange(700, dtype=np.uint8)) + bytes(300)
    assert type(b) is bytes and b == want and hash(b) == hash(want)
    e, ev = _new_bytes(0)
    assert e == b"" and ev.size == 0

"""zfec.easyfec-compatible ``Encoder`` / ``Decoder`` running on the MI355X kernels.

Drop-in for the import at /root/reference/storb/util/piece.py:8
(``from zfec.easyfec import Decoder, Encoder``, zfec 1.6.0.0):

* ``Encoder(k, m).encode(data)`` -> list of m blocks of B = ceil(len/k) bytes: the k
  data slices (the last zero-padded) followed by the m-k parity blocks (piece.py:129-130).
* ``Decoder(k, m).decode(blocks, sharenums, padlen)`` -> the joined k primaries with
  ``padlen`` bytes stripped (piece.py:196-197).

Preconditions raise :class:`Error` (zfec raises ``zfec.Error``) for: k < 1, m < k, m > 256,
unequal block lengths (including easyfec's short middle slice when len < (k-1)*B), a block
count other than k, a sharenum outside [0, m) and duplicate sharenums.
"""

from __future__ import annotations

from . import _lib
from .engine import Error, get_engine

__all__ = ["Encoder", "Decoder", "Error"]


def _check_km(k: int, m: int) -> None:
    if not (1 <= k <= m <= 256):
        raise Error(_lib.strerror(_lib.SEC_EKM) + f" (k={k}, m={m})")


class Encoder:
    def __init__(self, k: int, m: int):
        _check_km(k, m)
        self.k = k
        self.m = m

    def encode(self, data) -> list[bytes]:
        k, m = self.k, self.m
        n = len(data)
        B = -(-n // k)
        if k > 1 and (k - 1) * B > n:
            raise Error(_lib.strerror(_lib.SEC_EBLOCKLEN))
        mv = memoryview(data).cast("B")
        primaries = [bytes(mv[i * B:(i + 1) * B]) for i in range(k)]
        if len(primaries[-1]) != B:
            primaries[-1] = primaries[-1] + b"\x00" * (B - len(primaries[-1]))
        if m == k or B == 0:
            return primaries + [b""] * (m - k) if B == 0 else primaries
        return primaries + self.encode_parity(mv)

    def encode_parity(self, data) -> list[bytes]:
        """The m - k secondary blocks of ``encode(data)`` alone (no primary copies)."""
        k, m = self.k, self.m
        n = len(data)
        B = -(-n // k)
        if k > 1 and (k - 1) * B > n:
            raise Error(_lib.strerror(_lib.SEC_EBLOCKLEN))
        if m == k or B == 0:
            return [b""] * (m - k)
        return get_engine().encode_host([memoryview(data).cast("B")], [(k, m)])[0]


class Decoder:
    def __init__(self, k: int, m: int):
        _check_km(k, m)
        self.k = k
        self.m = m

    def decode(self, blocks, sharenums, padlen: int) -> bytes:
        k, m = self.k, self.m
        blocks = list(blocks)
        sharenums = [int(s) for s in sharenums]
        if len(blocks) != k or len(sharenums) != k:
            raise Error(_lib.strerror(_lib.SEC_ENBLOCKS) + f" (got {len(blocks)} blocks, {len(sharenums)} sharenums)")
        B = len(blocks[0])
        total = k * B
        if 0 <= padlen <= total:
            return get_engine().decode_host([(k, m, blocks, sharenums, padlen)])
        # easyfec strips with data[:-padlen]; keep Python's slicing for out-of-range padlen
        data = get_engine().decode_host([(k, m, blocks, sharenums, 0)])
        return data[:-padlen] if padlen else data

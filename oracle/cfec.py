"""ctypes wrapper of oracle/fec_oracle.c — TEST INFRASTRUCTURE ONLY (checker + CPU baseline).

Restates zfec.easyfec.Encoder/Decoder (called at /root/reference/storb/util/piece.py:129-130
and :196-197).  Parity unpinned against real zfec bytes (see fec_oracle.c header).
"""

from __future__ import annotations

import ctypes
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "build", "libfec_oracle.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _SO


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = ctypes.CDLL(_SO)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.fo_init.restype = None
        L.fo_encode_matrix.argtypes = [ctypes.c_int, ctypes.c_int, u8p]
        L.fo_invert.argtypes = [u8p, ctypes.c_int]
        L.fo_easy_encode.restype = ctypes.c_long
        L.fo_easy_encode.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t, u8p]
        L.fo_easy_decode.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_char_p),
                                     ctypes.POINTER(ctypes.c_int), ctypes.c_size_t, ctypes.c_size_t, u8p]
        L.fo_gf_mul.restype = ctypes.c_uint8
        L.fo_gf_mul.argtypes = [ctypes.c_uint8, ctypes.c_uint8]
        L.fo_init()
        _lib = L
    return _lib


def _u8(buf):
    return (ctypes.c_uint8 * len(buf)).from_buffer(buf)


def encode_matrix(k: int, m: int) -> bytes:
    out = bytearray(m * k)
    if lib().fo_encode_matrix(k, m, _u8(out)):
        raise ValueError(f"bad (k, m) = ({k}, {m})")
    return bytes(out)


def easy_encode(data: bytes, k: int, m: int) -> list[bytes]:
    n = len(data)
    B = -(-n // k) if k > 0 else 0
    out = bytearray(max(m * B, 1))
    rc = lib().fo_easy_encode(k, m, bytes(data), n, _u8(out))
    if rc < 0:
        raise ValueError(f"fo_easy_encode rc={rc}")
    return [bytes(out[i * B:(i + 1) * B]) for i in range(m)]


def easy_decode(blocks, sharenums, padlen: int, k: int, m: int) -> bytes:
    if len(blocks) != k or len(sharenums) != k:
        raise ValueError("exactly k blocks required")
    B = len(blocks[0])
    if any(len(b) != B for b in blocks):
        raise ValueError("unequal block lengths")
    arr = (ctypes.c_char_p * k)(*[bytes(b) for b in blocks])
    sn = (ctypes.c_int * k)(*sharenums)
    out = bytearray(max(k * B - padlen, 1))
    rc = lib().fo_easy_decode(k, m, arr, sn, B, padlen, _u8(out))
    if rc:
        raise ValueError(f"fo_easy_decode rc={rc}")
    return bytes(out[: k * B - padlen])

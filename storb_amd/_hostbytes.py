"""New bytes objects filled in place before anyone else sees them (the pieces and reassembled
chunks the drop-in returns), as a C extension does with PyBytes_FromStringAndSize(NULL, n): the
library (or numpy copies, which release the GIL) writes straight into the object's buffer.
"""

from __future__ import annotations

import ctypes
import platform

import numpy as np

# This relies on CPython's PyBytesObject layout (the buffer at offsetof(ob_sval) =
# bytes.__basicsize__ - 1) and on id() being the object's address.  It is used only on CPython
# and only after a self-test at import time confirms both (a pattern written through the view
# reads back through the bytes object); anywhere else the pieces are filled into a bytearray and
# converted with one copy (_FILL_IN_PLACE False).
def _bytes_view_self_test() -> bool:
    if platform.python_implementation() != "CPython":
        return False
    try:
        new = ctypes.pythonapi.PyBytes_FromStringAndSize
        new.restype = ctypes.py_object
        new.argtypes = [ctypes.c_void_p, ctypes.c_ssize_t]
        off = bytes.__basicsize__ - 1  # offsetof(PyBytesObject, ob_sval)
        pat = bytes(range(251)) * 3
        b = new(None, len(pat))
        if not isinstance(b, bytes) or len(b) != len(pat):
            return False
        ctypes.memmove(id(b) + off, pat, len(pat))
        return b == pat and b[len(pat):len(pat) + 1] == b""
    except Exception:  # noqa: BLE001 - any surprise: use the portable path
        return False


_FILL_IN_PLACE = _bytes_view_self_test()
if _FILL_IN_PLACE:
    _PyBytes_New = ctypes.pythonapi.PyBytes_FromStringAndSize
    _BYTES_DATA = bytes.__basicsize__ - 1


class _PendingBytes:
    """Portable stand-in: a bytearray filled by the pool, turned into bytes by finalize()."""

    __slots__ = ("buf",)

    def __init__(self, n: int):
        self.buf = bytearray(n)


def _new_bytes(n: int):
    """(a new unshared bytes object of n bytes, or a _PendingBytes off CPython; a writable uint8
    view of its buffer)."""
    if not _FILL_IN_PLACE:
        p = _PendingBytes(n)
        return p, np.frombuffer(p.buf, dtype=np.uint8) if n else np.empty(0, np.uint8)
    b = _PyBytes_New(None, n)
    if n == 0:
        return b, np.empty(0, np.uint8)
    return b, np.frombuffer((ctypes.c_char * n).from_address(id(b) + _BYTES_DATA), dtype=np.uint8)


def _finalize(piece):
    return bytes(piece.buf) if type(piece) is _PendingBytes else piece



"""Debug: what the HIP runtime reports for pinned / pageable pointers (zero-copy path checks)."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401

from storb_amd.engine import Engine  # noqa: E402

eng = Engine(0)
hip = ctypes.CDLL("libamdhip64.so.7")  # the runtime libstorbec (and torch) already loaded


class Attr(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("device", ctypes.c_int), ("devicePointer", ctypes.c_void_p),
                ("hostPointer", ctypes.c_void_p), ("isManaged", ctypes.c_int), ("allocationFlags", ctypes.c_uint)]


def q(name, p):
    a = Attr()
    rc = hip.hipPointerGetAttributes(ctypes.byref(a), ctypes.c_void_p(p))
    start = ctypes.c_void_p()
    size = ctypes.c_size_t()
    # HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR / RANGE_SIZE enum values from driver_types.h
    r1 = hip.hipPointerGetAttribute(ctypes.byref(start), ctypes.c_int(RS), ctypes.c_void_p(p))
    r2 = hip.hipPointerGetAttribute(ctypes.byref(size), ctypes.c_int(RS + 1), ctypes.c_void_p(p))
    print(name, hex(p), "rc", rc, "type", a.type, "dev", hex(a.devicePointer or 0), "host", hex(a.hostPointer or 0),
          "| range rc", r1, r2, hex(start.value or 0), size.value)
    hip.hipGetLastError()


RS = int(sys.argv[1]) if len(sys.argv) > 1 else 0
n = 48 * (65536 + 37)
a = eng.host_empty(n)
b = eng.host_empty(4096)
q("pinned start", a.ctypes.data)
q("pinned mid", a.ctypes.data + n // 2)
q("pinned end-1", a.ctypes.data + n - 1)
q("pinned small", b.ctypes.data)
c = np.zeros(1 << 20, np.uint8)
q("pageable", c.ctypes.data)
eng.register(c)
q("registered", c.ctypes.data)
q("registered mid", c.ctypes.data + 12345)
eng.unregister(c)

"""Debug: which host path each call of the zero-copy test takes."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401

from storb_amd._lib import DEC_DTYPE  # noqa: E402
from storb_amd.engine import Engine  # noqa: E402
from tests.test_gpu_parity import _enc_descs  # noqa: E402

eng = Engine(0)
nch, n, k, m = 48, 65536 + 37, 4, 6
B = -(-n // k)
d = _enc_descs(nch, n, k, m)[0]
hin, hpar, hout = eng.host_empty(nch * n), eng.host_empty(nch * (m - k) * B), eng.host_empty(nch * n)
hin[:] = np.random.default_rng(1).integers(0, 256, hin.size, dtype=np.uint8)
eng.encode_batch(d, hin, hpar, host=True)
print("after encode", eng.host_paths())
keep = [0, 1, 4, 5]
dd = np.zeros(nch, dtype=DEC_DTYPE)
dd["out_off"] = np.arange(nch, dtype=np.uint64) * n
dd["B"], dd["padlen"], dd["k"], dd["m"] = B, B * k - n, k, m
dd["slot0"] = np.arange(nch, dtype=np.uint64) * k
sn = np.tile(np.array(keep, np.int32), nch)
offs = np.zeros(nch * k, np.uint64)
ci = np.arange(nch, dtype=np.uint64)
for j, s in enumerate(keep):
    offs[j::k] = (hin.ctypes.data + ci * n + s * B) if s < k else (hpar.ctypes.data + ci * (m - k) * B + (s - k) * B)
eng.decode_batch(dd, sn, offs, 0, hout, host=True)
print("after decode", eng.host_paths(), np.array_equal(hout, hin))
print("hin", hex(hin.ctypes.data), "hpar", hex(hpar.ctypes.data), "hout", hex(hout.ctypes.data))
print("offs[:8]", [hex(int(x)) for x in offs[:8]])

"""TEST INFRASTRUCTURE: the oracle behind storb_amd.engine.Engine's interface, on host memory.

bench.py runs its ranks with this engine when STORB_BENCH_ENGINE=tests.bench_stub:OracleEngine
(CPU tensors, gloo), so `python bench.py --gpus 2` — the launch, the partition, the
descriptors the bench builds and the max / sum reductions — is tested on a machine with no
GPU.  Every call really encodes / decodes with oracle/fec_oracle.c through the same
descriptor arrays and addresses the HIP library would get, so the bench's own round-trip
checks pass only if its descriptors are right.  Never used by the product or by a GPU run.
"""

from __future__ import annotations

import contextlib
import ctypes
import os
import time

import numpy as np

from oracle import cfec


def _addr(obj) -> int:
    if obj is None:
        return 0
    if isinstance(obj, int):
        return obj
    if hasattr(obj, "data_ptr"):
        return int(obj.data_ptr())
    return int(obj.ctypes.data)


class OracleEngine:
    def __init__(self):
        # STORB_STUB_SLOW_RANK=r: rank r sleeps 50 ms in every encode call, so a test can tell the
        # max-over-ranks time from rank 0's own
        self._slow = os.environ.get("STORB_STUB_SLOW_RANK") == os.environ.get("RANK", "0")
        self._timing = False
        self._ms = {"encode": 0.0, "decode": 0.0}
        self._n = {"encode": 0, "decode": 0}
        self.calls = {"encode": 0, "decode": 0}

    def _record(self, kind, t0):
        self.calls[kind] += 1
        if self._timing:
            self._ms[kind] += (time.perf_counter() - t0) * 1e3
            self._n[kind] += 1

    def encode_batch(self, descs, src, parity, *, host=False, asynchronous=False):
        t0 = time.perf_counter()
        s, p = _addr(src), _addr(parity)
        for d in descs:
            n, k, m = int(d["n"]), int(d["k"]), int(d["m"])
            B = -(-n // k)
            blocks = cfec.easy_encode(ctypes.string_at(s + int(d["in_off"]), n), k, m)
            for r in range(m - k):
                ctypes.memmove(p + int(d["parity_off"]) + r * int(d["parity_stride"]), blocks[k + r], B)
        if self._slow:
            time.sleep(0.05)
        self._record("encode", t0)

    def decode_batch(self, descs, sharenums, block_offs, blocks, out, *, block_avail=None, recover_only=False,
                     host=False, asynchronous=False):
        t0 = time.perf_counter()
        base, o = _addr(blocks), _addr(out)
        for d in descs:
            k, m, B, padlen = int(d["k"]), int(d["m"]), int(d["B"]), int(d["padlen"])
            s0 = int(d["slot0"])
            sn = [int(x) for x in sharenums[s0:s0 + k]]
            blks = []
            for q in range(k):
                av = B if block_avail is None else int(block_avail[s0 + q])
                blks.append(ctypes.string_at(base + int(block_offs[s0 + q]), min(av, B)).ljust(B, b"\0"))
            full = cfec.easy_decode(blks, sn, 0, k, m)
            if recover_only:
                rows = [j for j in range(k) if j not in sn]
                data = b"".join(full[j * B:(j + 1) * B] for j in rows)
            else:
                data = full[:k * B - padlen]
            ctypes.memmove(o + int(d["out_off"]), data, len(data))
        self._record("decode", t0)

    def option(self, name):
        return -1 if name in ("SEC_BS", "SEC_SYN") else 0

    @contextlib.contextmanager
    def options(self, **opts):  # the oracle has no plan choices to force
        yield self

    def host_empty(self, nbytes):
        return np.empty(int(nbytes), dtype=np.uint8)

    def sync(self):
        pass

    def set_timing(self, on):
        self._timing = bool(on)

    def collect_timing(self, kind):
        r = (self._ms.get(kind, 0.0), self._n.get(kind, 0))
        if kind in self._ms:
            self._ms[kind], self._n[kind] = 0.0, 0
        return r

    def close(self):
        pass

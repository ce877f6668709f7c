"""TEST INFRASTRUCTURE: storb_amd.engine.Engine with the oracle behind its batch calls, on host
memory, so the host-side logic above them (encode_host*, decode_host*, the piece drop-in and
EngineGroup's split / reassembly) runs on a machine with no GPU.  Only the four device calls
are replaced (sec_encode_batch, sec_decode_batch_ex, sec_encode_digest_batch, sec_host_alloc);
each one really encodes / decodes with oracle/fec_oracle.c through the same descriptor arrays
and absolute addresses the HIP library would get.  Never used by the product or a GPU run.
"""

from __future__ import annotations

import ctypes
import hashlib
import threading

import numpy as np

from storb_amd.engine import Engine
from tests.bench_stub import OracleEngine


class OracleHostEngine(Engine):
    def __init__(self, device: int = 0):  # no libstorbec context
        self.lib = None
        self._ctx = None
        self.device = int(device)
        self._oracle = OracleEngine()
        self.chunks_encoded = 0
        self.chunks_decoded = 0
        self.threads = set()

    def close(self) -> None:
        pass

    def host_empty(self, nbytes: int) -> np.ndarray:
        return np.empty(max(int(nbytes), 0), dtype=np.uint8)

    def encode_batch(self, descs, src, parity, *, host=False, asynchronous=False, staged=False):
        self.threads.add(threading.get_ident())
        self.chunks_encoded += len(descs)
        self._oracle.encode_batch(descs, src, parity)

    def decode_batch(self, descs, sharenums, block_offs, blocks, out, *, block_avail=None, recover_only=False,
                     host=False, asynchronous=False, staged=False):
        self.threads.add(threading.get_ident())
        self.chunks_decoded += len(descs)
        self._oracle.decode_batch(descs, sharenums, block_offs, blocks, out, block_avail=block_avail,
                                  recover_only=recover_only)

    def encode_digest_batch(self, descs, src, parity, digests, *, host=False, asynchronous=False):
        self.encode_batch(descs, src, parity)
        s = 0 if src is None or isinstance(src, int) and src == 0 else int(np.asarray(src).ctypes.data)
        p = int(parity.ctypes.data)
        d = digests
        j = 0
        for c in descs:
            n, k, m = int(c["n"]), int(c["k"]), int(c["m"])
            B = -(-n // k)
            data = ctypes.string_at(s + int(c["in_off"]), n) + b"\0" * (k * B - n)
            for i in range(m):
                blk = data[i * B:(i + 1) * B] if i < k else ctypes.string_at(
                    p + int(c["parity_off"]) + (i - k) * int(c["parity_stride"]), B)
                d[20 * j:20 * (j + 1)] = np.frombuffer(hashlib.sha1(blk).digest(), np.uint8)
                j += 1

    def encode_pieces_into(self, chunks, shapes, piece_addrs, digests=None, staged=False, gpu_parity_ids=False):
        """sec_encode_pieces on the oracle: every piece written to its address, its SHA-1 beside."""
        from oracle import cfec

        self.threads.add(threading.get_ident())
        self.chunks_encoded += len(chunks)
        j = 0
        for c, (k, m) in zip(chunks, shapes):
            for b in cfec.easy_encode(bytes(c), k, m):
                if b:
                    ctypes.memmove(int(piece_addrs[j]), b, len(b))
                if digests is not None:
                    digests[20 * j:20 * (j + 1)] = np.frombuffer(hashlib.sha1(b).digest(), np.uint8)
                j += 1

    def _join_into(self, views, base):
        """sec_host_copy on the host: the views back to back at `base`."""
        off = 0
        for v in views:
            b = bytes(v)
            ctypes.memmove(base + off, b, len(b))
            off += len(b)
        return off

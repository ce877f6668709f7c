"""Host-side engine over libstorbec.so: one HIP context per (device, thread).

Two ways in:
  * device-resident batches (``encode_batch`` / ``decode_batch``): descriptor arrays +
    device addresses (torch tensors, or any integer address) — the bench and the GPU parity
    tests use these;
  * host batches (``encode_host`` / ``decode_host``): lists of bytes-like objects; the
    library gathers them into pinned staging, runs the kernels and copies results back —
    this is what the easyfec-compatible layer and the ``piece`` drop-in use.

There is no CPU compute path: every call goes to the HIP kernels; construction raises
``ECRuntimeError`` when no device is present.
"""

from __future__ import annotations

import contextlib
import ctypes
import os
import threading
import weakref

import numpy as np

from . import _lib
from ._lib import (COPY_DTYPE, DEC_DTYPE, ENC_DTYPE, MSG_DTYPE, SEC_F_ASYNC, SEC_F_GPU_PARITY_IDS, SEC_F_HOST,
                   SEC_F_RECOVER, SEC_F_STAGED)


class Error(Exception):
    """A zfec precondition violation (zfec raises ``zfec.Error`` for the same cases)."""


class ECRuntimeError(RuntimeError):
    """Device / runtime failure (no GPU, HIP error, out of memory)."""


def check(rc: int, lib=None) -> None:
    if rc == 0:
        return
    msg = _lib.strerror(rc, lib)
    if rc in _lib.PRECONDITION_CODES:
        raise Error(msg)
    raise ECRuntimeError(f"libstorbec: {msg} (status {rc})")


def addr(obj) -> tuple[int, object]:
    """(address, keep-alive) of a buffer: int, torch tensor, numpy array or bytes-like."""
    if obj is None:
        return 0, None
    if isinstance(obj, int):
        return obj, None
    if hasattr(obj, "data_ptr"):  # torch.Tensor (device or host)
        return int(obj.data_ptr()), obj
    if isinstance(obj, np.ndarray):
        return int(obj.ctypes.data), obj
    arr = np.frombuffer(obj, dtype=np.uint8)
    return (int(arr.ctypes.data) if arr.size else 0), arr


def _ptr(a: np.ndarray) -> int:
    return int(a.ctypes.data) if a.size else 0


def default_device() -> int:
    for var in ("STORB_EC_DEVICE", "LOCAL_RANK"):
        v = os.environ.get(var)
        if v is not None and v.strip().lstrip("-").isdigit():
            return int(v)
    return 0


def device_count() -> int:
    lib = _lib.load()
    n = ctypes.c_int(0)
    rc = lib.sec_device_count(ctypes.byref(n))
    return n.value if rc == 0 else 0


_TIMING_KINDS = {"encode": 0, "decode": 1, "sha1": 2, "bignum": 3}


class Engine:
    """A libstorbec context on one device.  Not thread-safe; use ``get_engine()`` per thread."""

    def __init__(self, device: int | None = None, lib_path: str | None = None, options: dict | None = None):
        self.lib = _lib.load(lib_path)
        self.device = default_device() if device is None else int(device)
        h = ctypes.c_void_p()
        rc = self.lib.sec_ctx_create(self.device, ctypes.byref(h))
        if rc:
            raise ECRuntimeError(f"cannot create HIP context on device {self.device}: {_lib.strerror(rc)}")
        self._ctx = h
        try:
            for k, v in (options or {}).items():  # sec_ctx_set_option: forced plan choices (tests, A/B)
                self.set_option(k, int(v))
        except BaseException:  # an unknown option or a bad value: no context left behind
            self.close()
            raise

    def _check(self, rc: int) -> None:
        check(rc, self.lib)

    # -- lifecycle / stream / timing ----------------------------------------
    def close(self) -> None:
        if self._ctx:
            self.lib.sec_ctx_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, stream) -> None:
        """Launch on an external hipStream_t (int handle or torch.cuda.Stream); None = own."""
        h = getattr(stream, "cuda_stream", stream)
        self._check(self.lib.sec_ctx_set_stream(self._ctx, h or None))

    def sync(self) -> None:
        self._check(self.lib.sec_sync(self._ctx))

    def set_timing(self, enable: bool) -> None:
        self._check(self.lib.sec_ctx_set_timing(self._ctx, int(bool(enable))))

    def collect_timing(self, kind: str) -> tuple[float, int]:
        """(summed kernel ms, launch count) recorded since the last collect;
        kind 'encode' | 'decode' | 'sha1' | 'bignum'."""
        ms = ctypes.c_double(0)
        n = ctypes.c_int64(0)
        self._check(self.lib.sec_timing_collect(self._ctx, _TIMING_KINDS[kind], ctypes.byref(ms),
                                          ctypes.byref(n)))
        return ms.value, n.value

    # -- context options (sec_ctx_set_option) ----------------------------------
    def set_option(self, name: str, value: int) -> None:
        """Force a plan choice on this context (tests, A/B tools); see include/storb_ec.h.
        The library reads no environment variable: an option holds only for this engine."""
        self._check(self.lib.sec_ctx_set_option(self._ctx, name.encode(), int(value)))

    def option(self, name: str) -> int:
        v = ctypes.c_int64(0)
        self._check(self.lib.sec_ctx_get_option(self._ctx, name.encode(), ctypes.byref(v)))
        return v.value

    @contextlib.contextmanager
    def options(self, **opts):
        """``with eng.options(SEC_SYN=0): ...``: the options set for the block, restored after."""
        old = {k: self.option(k) for k in opts}
        try:
            for k, v in opts.items():
                self.set_option(k, v)
            yield self
        finally:
            for k, v in old.items():
                self.set_option(k, v)

    # -- device-resident batches --------------------------------------------
    def encode_batch(self, descs: np.ndarray, src, parity, *, host: bool = False, asynchronous: bool = False,
                     staged: bool = False) -> None:
        """sec_encode_batch.  staged (host only): never page-lock pageable buffers for the call
        (SEC_F_STAGED), for callers whose other threads fault in memory meanwhile."""
        descs = np.ascontiguousarray(descs, dtype=ENC_DTYPE)
        s, _ks = addr(src)
        p, _kp = addr(parity)
        flags = (SEC_F_HOST if host else 0) | (SEC_F_ASYNC if asynchronous else 0) | (SEC_F_STAGED if staged else 0)
        self._check(self.lib.sec_encode_batch(self._ctx, _ptr(descs), len(descs), s or None, p or None, flags))

    def decode_batch(self, descs: np.ndarray, sharenums: np.ndarray, block_offs: np.ndarray, blocks, out, *,
                     block_avail: np.ndarray | None = None, recover_only: bool = False, host: bool = False,
                     asynchronous: bool = False, staged: bool = False) -> None:
        """sec_decode_batch_ex.  block_avail (per slot, optional): bytes of the block that exist,
        the rest read as zero (zfec's padded last data block read in place: B - padlen).
        recover_only: write just the missing primaries (SEC_F_RECOVER), e*B bytes per chunk.
        staged: as encode_batch."""
        descs = np.ascontiguousarray(descs, dtype=DEC_DTYPE)
        sn = np.ascontiguousarray(sharenums, dtype=np.int32)
        bo = np.ascontiguousarray(block_offs, dtype=np.uint64)
        av = None if block_avail is None else np.ascontiguousarray(block_avail, dtype=np.uint64)
        if av is not None and av.size < bo.size:
            raise ValueError("block_avail needs one entry per slot")
        b, _kb = addr(blocks)
        o, _ko = addr(out)
        flags = ((SEC_F_HOST if host else 0) | (SEC_F_ASYNC if asynchronous else 0) |
                 (SEC_F_RECOVER if recover_only else 0) | (SEC_F_STAGED if staged else 0))
        self._check(self.lib.sec_decode_batch_ex(self._ctx, _ptr(descs), len(descs), _ptr(sn), _ptr(bo),
                                                 None if av is None else _ptr(av), b or None, o or None, flags))

    def encode_digest_batch(self, descs: np.ndarray, src, parity, digests, *, host: bool = False,
                            asynchronous: bool = False) -> None:
        """Encode + SHA-1 of every block (20 B per block, chunk-major) — sec_encode_digest_batch."""
        descs = np.ascontiguousarray(descs, dtype=ENC_DTYPE)
        s, _ks = addr(src)
        p, _kp = addr(parity)
        g, _kg = addr(digests)
        flags = (SEC_F_HOST if host else 0) | (SEC_F_ASYNC if asynchronous else 0)
        self._check(self.lib.sec_encode_digest_batch(self._ctx, _ptr(descs), len(descs), s or None, p or None,
                                                     g or None, flags))

    def sha1_batch(self, msgs: np.ndarray, digests, *, host: bool = False, asynchronous: bool = False) -> None:
        """SHA-1 of each (addr, len, avail) message into 20-byte digests — sec_sha1_batch."""
        msgs = np.ascontiguousarray(msgs, dtype=MSG_DTYPE)
        g, _kg = addr(digests)
        flags = (SEC_F_HOST if host else 0) | (SEC_F_ASYNC if asynchronous else 0)
        self._check(self.lib.sec_sha1_batch(self._ctx, _ptr(msgs), len(msgs), g or None, flags))

    # -- pinned host memory: the zero-copy host path ----------------------------
    def host_empty(self, nbytes: int) -> np.ndarray:
        """A page-locked uint8 host array (sec_host_alloc).  ``host=True`` calls whose buffers
        are all pinned run the kernels on them directly over PCIe, with no staging copy.
        Freed when the array and every view of it are gone."""
        n = int(nbytes)
        p = ctypes.c_void_p()
        self._check(self.lib.sec_host_alloc(self._ctx, max(n, 1), ctypes.byref(p)))
        raw = (ctypes.c_uint8 * max(n, 1)).from_address(p.value)
        weakref.finalize(raw, self.lib.sec_host_free, None, p.value).atexit = False  # the OS reclaims at exit
        return np.frombuffer(raw, dtype=np.uint8, count=n)

    def register(self, buf) -> None:
        """Page-lock an existing writable host buffer (hipHostRegister) so ``host=True`` calls
        on it take the zero-copy path.  Call ``unregister`` before the buffer is freed."""
        a, keep = addr(buf)
        self._check(self.lib.sec_host_register(self._ctx, a, keep.nbytes if keep is not None else len(buf)))

    def unregister(self, buf) -> None:
        a, _ = addr(buf)
        self._check(self.lib.sec_host_unregister(None, a))

    def host_paths(self) -> tuple[int, int, int]:
        """(zero-copy on pinned buffers, zero-copy on pages locked for the call, staged) counts
        of the ``host=True`` encode / decode calls so far."""
        z, r, st = ctypes.c_int64(0), ctypes.c_int64(0), ctypes.c_int64(0)
        self._check(self.lib.sec_ctx_host_paths(self._ctx, ctypes.byref(z), ctypes.byref(r), ctypes.byref(st)))
        return z.value, r.value, st.value

    def decode_paths(self) -> tuple[int, int]:
        """(syndrome, direct): chunks with a lost data block decoded so far, by method."""
        syn, direct = ctypes.c_int64(0), ctypes.c_int64(0)
        self._check(self.lib.sec_ctx_decode_paths(self._ctx, ctypes.byref(syn), ctypes.byref(direct)))
        return syn.value, direct.value

    def decode_methods(self) -> tuple[int, int, int, int]:
        """(fused one-wave syndrome kernel, two-wave kernel, two syndrome kernels, direct): chunks
        with a lost data block decoded so far, by kernel."""
        f, p, t, d = (ctypes.c_int64(0) for _ in range(4))
        self._check(self.lib.sec_ctx_decode_methods(self._ctx, ctypes.byref(f), ctypes.byref(p), ctypes.byref(t),
                                                    ctypes.byref(d)))
        return f.value, p.value, t.value, d.value

    _SCRATCH_CAP = 256 << 20  # largest result staged in the reusable pinned scratch

    def _out_buffer(self, nbytes: int) -> np.ndarray:
        """Result buffer of encode_host / decode_host: a reusable pinned scratch (so a call on
        pinned inputs stays zero-copy end to end; results are copied out before returning), or
        plain memory past _SCRATCH_CAP."""
        n = max(int(nbytes), 1)
        if n > self._SCRATCH_CAP:
            return np.empty(n, dtype=np.uint8)
        cur = getattr(self, "_scratch", None)
        if cur is None or cur.size < n:
            cur = self._scratch = self.host_empty(max(n, 2 * (cur.size if cur is not None else 0), 1 << 20))
        return cur[:n]

    # -- host batches ---------------------------------------------------------
    def sha1_host(self, datas) -> list[bytes]:
        """SHA-1 digests (20 bytes each) of host byte strings, hashed on the GPU."""
        msgs = np.zeros(len(datas), dtype=MSG_DTYPE)
        keep = []
        for i, d in enumerate(datas):
            a, kp = addr(d)
            keep.append(kp)
            ln = len(kp) if isinstance(kp, np.ndarray) else len(d)
            msgs[i] = (a, ln, ln)
        out = np.empty(max(20 * len(datas), 1), dtype=np.uint8)
        self.sha1_batch(msgs, out, host=True)
        mv = memoryview(out)
        return [bytes(mv[20 * i:20 * (i + 1)]) for i in range(len(datas))]

    def encode_host_raw(self, chunks, shapes, digests: bool = False, staged: bool = False):
        """``encode_host`` without the per-block ``bytes``: returns (buf, layout) where buf is
        this engine's pinned result scratch and layout[i] = (offset, B, m - k) of chunk i's
        parity blocks in it, back to back.  buf is reused by the engine's next call.  With
        ``digests=True``: (buf, layout, dig), dig = the SHA-1 of every chunk's m blocks in order,
        20 bytes each (GPU-computed after the encode, sec_encode_digest_batch).  staged: as
        encode_batch."""
        n = len(chunks)
        descs = np.zeros(n, dtype=ENC_DTYPE)
        keep = []
        layout = []
        total = 0
        for i, (c, (k, m)) in enumerate(zip(chunks, shapes)):
            a, kp = addr(c)
            keep.append(kp)
            ln = len(kp) if isinstance(kp, np.ndarray) else len(c)
            B = -(-ln // k) if ln else 0
            descs[i] = (a, ln, total, max(B, 1), k, m)
            layout.append((total, B, m - k))
            total += (m - k) * B
        out = self._out_buffer(total)
        if digests:
            dig = np.empty(max(20 * sum(m for (_, m) in shapes), 1), dtype=np.uint8)
            if n:
                self.encode_digest_batch(descs, 0, out, dig, host=True)
            return out, layout, dig
        if n:
            self.encode_batch(descs, 0, out, host=True, staged=staged)
        return out, layout

    def encode_pieces_into(self, chunks, shapes, piece_addrs, digests: np.ndarray | None = None,
                           staged: bool = False, gpu_parity_ids: bool = False) -> None:
        """easyfec's Encoder.encode output for every chunk written to caller buffers
        (sec_encode_pieces): piece_addrs[M_c + j] = the address of a writable B-byte buffer for
        piece j of chunk c (M_c = sum of m over the chunks before c); digests (optional, a
        writable uint8 array of 20 bytes per piece) receives each piece's SHA-1, computed on the
        library's host threads while the GPU encodes (``gpu_parity_ids``: the parity pieces' on
        the GPU, SEC_F_GPU_PARITY_IDS).  shapes: [(k, m)] per chunk."""
        n = len(chunks)
        descs = np.zeros(n, dtype=ENC_DTYPE)
        keep = []
        for i, (c, (k, m)) in enumerate(zip(chunks, shapes)):
            a, kp = addr(c)
            keep.append(kp)
            ln = len(kp) if isinstance(kp, np.ndarray) else len(c)
            B = -(-ln // k) if ln else 0
            descs[i] = (a, ln, 0, max(B, 1), k, m)
        pa = np.ascontiguousarray(piece_addrs, dtype=np.uint64)
        if pa.size != sum(m for (_, m) in shapes):
            raise ValueError("encode_pieces_into: one piece address per piece")
        if digests is not None and digests.size < 20 * pa.size:
            raise ValueError("encode_pieces_into: digests needs 20 bytes per piece")
        flags = SEC_F_HOST | (SEC_F_STAGED if staged else 0) | (SEC_F_GPU_PARITY_IDS if gpu_parity_ids else 0)
        if n:
            self._check(self.lib.sec_encode_pieces(self._ctx, _ptr(descs), n, None, _ptr(pa),
                                                   None if digests is None else _ptr(digests), flags))

    def encode_host(self, chunks, shapes, digests: bool = False):
        """Parity blocks for each chunk.  chunks: bytes-like list; shapes: [(k, m)] per chunk.

        Returns, per chunk, the m-k secondary blocks (block numbers k..m-1) as bytes; with
        ``digests=True`` also, per chunk, the SHA-1 digests of all m blocks (GPU-computed).
        """
        n = len(chunks)
        descs = np.zeros(n, dtype=ENC_DTYPE)
        keep = []
        blocks = []
        total = 0
        for i, (c, (k, m)) in enumerate(zip(chunks, shapes)):
            a, kp = addr(c)
            keep.append(kp)
            ln = len(kp) if isinstance(kp, np.ndarray) else len(c)
            B = -(-ln // k) if ln else 0
            descs[i] = (a, ln, total, max(B, 1), k, m)
            blocks.append((total, B, m - k))
            total += (m - k) * B
        out = self._out_buffer(total)
        if not digests:
            self.encode_batch(descs, 0, out, host=True)
            mv = memoryview(out)
            return [[bytes(mv[o + r * B:o + (r + 1) * B]) for r in range(p)] for (o, B, p) in blocks]
        ms = [m for (_, m) in shapes]
        dig = np.empty(max(20 * sum(ms), 1), dtype=np.uint8)
        self.encode_digest_batch(descs, 0, out, dig, host=True)
        mv, dv = memoryview(out), memoryview(dig)
        par = [[bytes(mv[o + r * B:o + (r + 1) * B]) for r in range(p)] for (o, B, p) in blocks]
        first = np.concatenate([[0], np.cumsum(ms)[:-1]]).astype(int) if ms else []
        digs = [[bytes(dv[20 * (f + j):20 * (f + j + 1)]) for j in range(m)] for f, m in zip(first, ms)]
        return par, digs

    # joins of at least this many bytes go to the library's copy threads (sec_host_copy) instead
    # of a single-threaded b"".join under the GIL
    NATIVE_JOIN_MIN = 1 << 20

    def _join_into(self, views, base: int) -> int:
        """Copy `views` back to back to the host address `base` on the copy threads; returns the
        bytes written."""
        jobs = np.zeros(len(views), dtype=COPY_DTYPE)
        off = 0
        keep = []
        for i, v in enumerate(views):
            a = np.frombuffer(v, dtype=np.uint8)
            keep.append(a)
            n = a.size
            jobs[i] = (base + off, a.ctypes.data if n else 0, n)
            off += n
        if len(views):
            self._check(self.lib.sec_host_copy(self._ctx, _ptr(jobs), len(views)))
        return off

    def _joined(self, views) -> bytes:
        from ._hostbytes import _finalize, _new_bytes

        total = sum(len(v) for v in views)
        if total < self.NATIVE_JOIN_MIN:
            return b"".join(views)
        b, dst = _new_bytes(total)
        self._join_into(views, dst.ctypes.data)
        return _finalize(b)

    # A host reassembly in ONE library call (sec_decode_batch_ex's host join, api.cpp decode_core
    # / join_staged): chunks with every data piece present are copied by the library's task
    # threads and never reach the GPU; the others are recovered on the GPU beside those copies,
    # only the recovered rows crossing PCIe.  False: round 4's form (a recover-only call into a
    # pinned scratch, then the join; A/B in tools/stream_rate.py).
    LIBRARY_JOIN = True

    def _reassemble(self, items, outs) -> None:
        """Every chunk's k*B - padlen bytes written to the host address outs[i], one call."""
        for it in items:
            check_decode_item(*it)
        n = len(items)
        descs = np.zeros(n, dtype=DEC_DTYPE)
        nslots = sum(it[0] for it in items)
        sn = np.zeros(max(nslots, 1), dtype=np.int32)
        bo = np.zeros(max(nslots, 1), dtype=np.uint64)
        keep = []
        slot = 0
        for j, (k, m, blocks, sharenums, padlen) in enumerate(items):
            B = len(blocks[0])
            for q, b in enumerate(blocks):
                a, kp = addr(b)
                keep.append(kp)
                bo[slot + q] = a
                sn[slot + q] = int(sharenums[q])
            descs[j] = (int(outs[j]), B, padlen, slot, k, m)
            slot += k
        if n:
            # (not staged=True: when the pieces are too scattered to page-lock, the library
            # copies the present ones into the output first and a large call's kernels read
            # them back from there, the output page-locked for the call)
            self.decode_batch(descs, sn, bo, 0, 0, host=True)

    def decode_host(self, items) -> bytes:
        """Reassemble chunks from host blocks, concatenated in order.

        items: [(k, m, blocks, sharenums, padlen)] with exactly k equal-length blocks each.
        Returns the concatenation of every chunk's k*B - padlen bytes.
        """
        if not self.LIBRARY_JOIN:
            return self._joined(self._decode_parts(items, per_chunk=False))
        from ._hostbytes import _finalize, _new_bytes

        lens = [it[0] * len(it[2][0]) - it[4] for it in items]
        b, dst = _new_bytes(sum(lens))
        if dst.size:
            starts = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64) if lens else []
            self._reassemble(items, [dst.ctypes.data + int(o) for o in starts])
        return _finalize(b)

    def decode_host_into(self, items, dst: np.ndarray) -> int:
        """``decode_host`` written into `dst` (a writable uint8 array) instead of a new bytes
        object: the output of a share of a multi-device call lands straight in the caller's
        result.  Returns the bytes written; ValueError when `dst` is too small."""
        if not self.LIBRARY_JOIN:
            views = self._decode_parts(items, per_chunk=False)
            if sum(len(v) for v in views) > dst.size:
                raise ValueError("decode_host_into: destination too small")
            return self._join_into(views, dst.ctypes.data) if dst.size else 0
        lens = [it[0] * len(it[2][0]) - it[4] for it in items]
        total = sum(lens)
        if total > dst.size:
            raise ValueError("decode_host_into: destination too small")
        if total:
            starts = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
            self._reassemble(items, [dst.ctypes.data + int(o) for o in starts])
        return total

    def decode_host_chunks(self, items) -> list[bytes]:
        """``decode_host``, one bytes object per chunk."""
        if not self.LIBRARY_JOIN:
            return [self._joined(p) for p in self._decode_parts(items, per_chunk=True, views=True)]
        from ._hostbytes import _finalize, _new_bytes

        objs = [_new_bytes(it[0] * len(it[2][0]) - it[4]) for it in items]
        live = [(it, v.ctypes.data) for it, (_, v) in zip(items, objs) if v.size]
        if live:
            self._reassemble([it for it, _ in live], [a for _, a in live])
        return [_finalize(b) for b, _ in objs]

    def _decode_parts(self, items, per_chunk: bool, views: bool = False) -> list:
        """Chunks with a missing primary go to the GPU in ONE sec_decode_batch_ex call (recover-only);
        a chunk whose k blocks are its k primaries needs no field arithmetic at all (zfec's fec_decode writes
        nothing for present primaries and easyfec joins them, /root/reference/storb/util/
        piece.py:196-197), so it is the join of its blocks, taken as views with no staging or
        PCIe round trip.  Returns per chunk either that chunk's bytes (per_chunk; with `views`
        the list of its buffers instead) or a list of buffers whose concatenation is the output."""
        n = len(items)
        as_views = views
        gpu = []  # indices of chunks with a missing primary
        for i, item in enumerate(items):
            check_decode_item(*item)
            k, sharenums = item[0], item[3]
            if any(int(x) >= k for x in sharenums):
                gpu.append(i)
        # The GPU only recovers (SEC_F_RECOVER: zfec fec_decode's own output, the e missing
        # primaries, B bytes each, in primary order); the chunk is then the join of its present
        # primaries and those rows, so only e * B bytes per chunk come back over PCIe instead of
        # the whole reassembled chunk.
        rec = {}
        if gpu:
            descs = np.zeros(len(gpu), dtype=DEC_DTYPE)
            nslots = sum(items[i][0] for i in gpu)
            sn_arr = np.zeros(nslots, dtype=np.int32)
            bo = np.zeros(nslots, dtype=np.uint64)
            keep = []
            slot = total = 0
            for j, i in enumerate(gpu):
                k, m, blocks, sharenums, padlen = items[i]
                B = len(blocks[0])
                for q, b in enumerate(blocks):
                    a, kp = addr(b)
                    keep.append(kp)
                    bo[slot + q] = a
                    sn_arr[slot + q] = int(sharenums[q])
                e = sum(1 for x in sharenums if int(x) >= k)
                descs[j] = (total, B, padlen, slot, k, m)
                rec[i] = total
                slot += k
                total += e * B
            buf = self._out_buffer(total)
            self.decode_batch(descs, sn_arr, bo, 0, buf, host=True, recover_only=True)
            mv = memoryview(buf)
        parts = []
        for i in range(n):
            k, m, blocks, sharenums, padlen = items[i]
            B = len(blocks[0])
            prim = {int(x): q for q, x in enumerate(sharenums) if int(x) < k}  # primary -> its block
            o = rec.get(i)
            left = k * B - padlen
            views = []
            for j in range(k):
                if left <= 0:
                    break
                if j in prim:
                    v = memoryview(blocks[prim[j]]).cast("B")
                else:  # the next recovered row (rows come in primary order)
                    v = mv[o:o + B]
                    o += B
                views.append(v[:left] if left < B else v)
                left -= B
            if per_chunk:
                parts.append(views if as_views else b"".join(views))
            else:
                parts.extend(views)
        return parts


def check_decode_item(k: int, m: int, blocks, sharenums, padlen: int) -> None:
    """zfec's decode preconditions for one chunk (the library's own checks, raised before any
    GPU work): exactly k blocks and sharenums, equal lengths, 1 <= k <= m <= 256, sharenums in
    [0, m) and distinct, 0 <= padlen <= k*B.  Raises Error."""
    if len(blocks) != k or len(sharenums) != k:
        raise Error(_lib.strerror(_lib.SEC_ENBLOCKS))
    B = len(blocks[0]) if blocks else 0
    for b in blocks:
        if len(b) != B:
            raise Error(_lib.strerror(_lib.SEC_EBLOCKLEN))
    sn = [int(x) for x in sharenums]
    if not (1 <= k <= m <= 256):
        raise Error(_lib.strerror(_lib.SEC_EKM))
    if any(x < 0 or x >= m for x in sn):
        raise Error(_lib.strerror(_lib.SEC_ESHARENUM))
    if len(set(sn)) != k:
        raise Error(_lib.strerror(_lib.SEC_EDUPSHARE))
    if not (0 <= padlen <= k * B):
        raise Error(_lib.strerror(_lib.SEC_EPADLEN))


# -- matrices (host arithmetic; no device needed) ------------------------------
def encode_matrix(k: int, m: int) -> bytes:
    """Rows k..m-1 of zfec's systematic encode matrix, as produced by libstorbec."""
    lib = _lib.load()
    out = np.zeros(max((m - k) * k, 1), dtype=np.uint8)
    check(lib.sec_encode_matrix(k, m, _ptr(out)))
    return out[: (m - k) * k].tobytes()


def choose_blocks(k: int, m: int, sharenums) -> list[int] | None:
    """Positions (ascending sharenum) of the k blocks to decode from when more are at hand
    (sec_decode_choose: every present primary, then parity rows from as few of the decode
    kernels' row groups as possible), or None when fewer than k distinct valid sharenums."""
    lib = _lib.load()
    sn = np.ascontiguousarray([int(x) for x in sharenums], dtype=np.int32)
    pick = np.zeros(max(k, 1), dtype=np.int32)
    rc = lib.sec_decode_choose(int(k), int(m), sn.size, _ptr(sn), _ptr(pick))
    if rc == _lib.SEC_ENBLOCKS:
        return None
    check(rc, lib)
    return pick[:k].tolist()


def pinned_bytes() -> tuple[int, int]:
    """(loaned, idle): the process's pinned staging memory lent to host-mode calls in progress,
    and kept idle for the next call (sec_host_pinned_bytes; contexts hold none between calls)."""
    lib = _lib.load()
    a, b = ctypes.c_int64(0), ctypes.c_int64(0)
    rc = lib.sec_host_pinned_bytes(ctypes.byref(a), ctypes.byref(b))
    if rc:
        raise ECRuntimeError(f"sec_host_pinned_bytes: {rc}")
    return a.value, b.value


def option_names() -> list[str]:
    """Every context option the library knows (sec_option_name)."""
    lib = _lib.load()
    out, i = [], 0
    while (n := lib.sec_option_name(i)) is not None:
        out.append(n.decode())
        i += 1
    return out


def option_default(name: str) -> int:
    lib = _lib.load()
    v = ctypes.c_int64(0)
    check(lib.sec_ctx_get_option(None, name.encode(), ctypes.byref(v)))
    return v.value


def decode_matrix(k: int, m: int, sharenums) -> tuple[bytes, list[int]]:
    lib = _lib.load()
    sn = np.ascontiguousarray(sharenums, dtype=np.int32)
    if sn.size != k:
        raise Error(_lib.strerror(_lib.SEC_ENBLOCKS))
    out = np.zeros(k * k, dtype=np.uint8)
    idx = np.zeros(k, dtype=np.int32)
    check(lib.sec_decode_matrix(k, m, _ptr(sn), _ptr(out), _ptr(idx)))
    return out.tobytes(), idx.tolist()


_tls = threading.local()
_spread = {"devices": None, "next": 0}
_spread_lock = threading.Lock()


def spread_threads(devices) -> None:
    """Give each host thread that first asks for an engine without naming a device (and is not
    an EngineGroup worker) the next device of `devices`, round robin; None: every thread uses
    default_device().  A multi-threaded caller (the validator serves uploads and downloads on
    executor threads) then spreads its per-chunk calls over the GPUs.  A thread keeps the
    device it was given."""
    with _spread_lock:
        _spread["devices"] = None if devices is None else [int(d) for d in devices]
        _spread["next"] = 0


def _thread_device():
    devs = _spread["devices"]
    if devs is None:
        return None
    mine = getattr(_tls, "spread", None)
    if mine is not None and mine[0] is devs:
        return mine[1]
    with _spread_lock:
        d = devs[_spread["next"] % len(devs)]
        _spread["next"] += 1
    _tls.spread = (devs, d)
    return d


def get_engine(device: int | None = None) -> Engine:
    """The calling thread's engine for `device` (default: the engine of the EngineGroup worker
    this thread is, else STORB_EC_DEVICE / LOCAL_RANK / 0)."""
    if device is None:
        bound = getattr(_tls, "bound", None)
        if bound is not None:
            return bound
        device = _thread_device()
    dev = default_device() if device is None else int(device)
    engines = getattr(_tls, "engines", None)
    if engines is None:
        engines = _tls.engines = {}
    eng = engines.get(dev)
    if eng is None:
        eng = engines[dev] = Engine(dev)
    return eng


class EngineGroup:
    """Several devices driven from ONE process: one worker thread per
    entry of `devices`, each holding its own Engine (its own libstorbec context and streams on
    that device).  Chunks are independent (/root/reference/storb/validator/validator.py:1352-1431
    handles them one by one), so a batch is split into contiguous ranges balanced by bytes
    (``dist.partition``), each range runs on its worker, and the results come back in chunk
    order.  No collective and no peer traffic: every device reads and writes only its own share.

    ``devices=None`` uses every visible device.  An entry may repeat (``[0, 0]``: two contexts
    on one GPU, each with its own worker), so the split, the threads and the reassembly can be
    tested on a one-GPU box.  Inside a worker, ``get_engine()`` (no argument) returns that
    worker's engine, so the piece-level batch functions run unchanged on each share.

    ``engine_factory(device)`` (tests only) builds the per-worker engine instead of Engine.
    """

    def __init__(self, devices=None, engine_factory=None):
        from concurrent.futures import ThreadPoolExecutor

        if devices is None:
            devices = list(range(device_count()))
        self.devices = [int(d) for d in devices]
        if not self.devices:
            raise ECRuntimeError("EngineGroup: no HIP device available")
        make = engine_factory or (lambda d: Engine(d))
        self._workers = []
        self._engines = []
        try:
            for i, d in enumerate(self.devices):
                w = ThreadPoolExecutor(1, thread_name_prefix=f"storb_amd_dev{d}_{i}")
                self._workers.append(w)
                # the engine is created on its own worker thread and bound there
                self._engines.append(w.submit(self._bind, make, d).result())
        except BaseException:
            self.close()
            raise

    @staticmethod
    def _bind(make, d):
        eng = make(d)
        _tls.bound = eng
        return eng

    def __len__(self) -> int:
        return len(self.devices)

    @property
    def engines(self) -> list:
        return list(self._engines)

    def submit(self, i: int, fn, *args, **kw):
        """Run fn(*args, **kw) on worker i (whose ``get_engine()`` is engine i); a Future."""
        return self._workers[i].submit(fn, *args, **kw)

    def shares(self, sizes) -> list[tuple[int, int]]:
        """Contiguous [lo, hi) ranges of the items, one per worker, balanced by `sizes`."""
        from .dist import partition

        return partition(sizes, len(self.devices))

    def map_shares(self, fn, items, sizes) -> list:
        """fn(items[lo:hi], lo) on every worker's share at once; returns the per-share results
        in share (= item) order.  Every share runs to completion; then the error of the FIRST
        failing share (the one holding the earliest chunk) is raised, as a single-device call
        over the whole batch would raise for that chunk."""
        futs = [(self.submit(i, fn, items[lo:hi], lo) if hi > lo else None)
                for i, (lo, hi) in enumerate(self.shares(sizes))]
        res, err = [], None
        for f in futs:
            if f is None:
                res.append(None)
                continue
            try:
                res.append(f.result())
            except BaseException as e:  # noqa: BLE001 - re-raised below, in chunk order
                res.append(None)
                if err is None:
                    err = e
        if err is not None:
            raise err
        return res

    def sync(self) -> None:
        for f in [self.submit(i, e.sync) for i, e in enumerate(self._engines)]:
            f.result()

    def close(self) -> None:
        for i, w in enumerate(self._workers):
            eng = self._engines[i] if i < len(self._engines) else None
            if eng is not None:
                try:
                    w.submit(eng.close).result()
                except Exception:  # noqa: BLE001 - closing: best effort
                    pass
            w.shutdown(wait=True)
        self._workers, self._engines = [], []

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

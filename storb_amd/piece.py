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
* handed more than k pieces, ``decode_chunk`` decodes from the k the library picks
  (``sec_decode_choose``: every present primary, then parity pieces from as few of the decode
  kernels' row groups as possible) instead of the first k (piece.py:189-191); any k distinct
  pieces give the same bytes, the choice only sets the decode's cost.
* the two ``print()`` calls per piece in ``encode_chunk`` (piece.py:140,151) are debug
  logs here.
* extra batch entry points ``encode_chunks`` / ``decode_chunks`` for callers that can hand
  over many chunks at once (the validator's upload loop, validator.py:1352-1431).
* ``reconstruct_data_stream`` decodes window w+1 on a worker thread (its own HIP context)
  while the caller consumes window w's chunks; ``encode_chunks_stream`` does the same for the
  upload loop's produce/consume pattern (validator.py:1338-1446, 1630-1638).
* ``encode_chunk`` starts the SHA-1 of its pieces on a small thread pool (hashlib, as
  ``piece_hash``), data pieces while the parity is on the GPU; ``piece_hash(data)`` returns
  that digest when ``data`` is one of those very piece objects (identity, not equality), so
  the validator's ``piece_hash`` right after ``encode_chunk`` (validator.py:1081) does not
  hash serially.  Same digests either way; ``PREFETCH_PIECE_IDS = False`` turns it off.
* several GPUs in one process: the batch and stream functions take ``devices=`` (or the
  module default ``use_devices(...)``) and split their chunks over those devices
  (``engine.EngineGroup``: one worker thread and HIP context per device, chunks partitioned
  by bytes, results in chunk order).  Same bytes as one device.
"""

from __future__ import annotations

import ctypes
import hashlib
import logging
import math
import os
import platform
import threading
import typing
from collections import OrderedDict, deque
from collections.abc import Iterable, Iterator
from concurrent.futures import Future, ThreadPoolExecutor
from enum import IntEnum

import numpy as np
from pydantic import BaseModel, ConfigDict, Field

from .constants import MAX_PIECE_SIZE, MIN_PIECE_SIZE, PIECE_LENGTH_OFFSET, PIECE_LENGTH_SCALING
from .easyfec import Decoder, Encoder, Error
from .engine import EngineGroup, check_decode_item, choose_blocks, device_count, get_engine, spread_threads

logger = logging.getLogger(__name__)

__all__ = [
    "PieceType", "Piece", "EncodedChunk", "ProcessedPieceInfo", "EncodedPieces", "piece_hash", "piece_length",
    "encode_chunk", "decode_chunk", "reconstruct_data", "reconstruct_data_stream", "encode_chunks",
    "decode_chunks", "chunk_shape", "piece_hashes", "encode_chunks_with_ids", "encode_chunks_stream", "Encoder",
    "Decoder", "Error", "use_devices",
]

PREFETCH_PIECE_IDS = True  # encode_chunk hashes its pieces on a thread pool (see module doc)
# decode_chunk & co. handed more than k pieces decode from the k that sec_decode_choose picks
# (False: the first k in piece order, as the reference's piece.py:189-191; same bytes either way)
CHOOSE_BLOCKS = True
# ... for chunks of at least this many bytes.  The validator's pattern (encode_chunk, then
# piece_hash of every piece; tools/prefetch_study.py, profiles/r02_prefetch_study.json), us per
# chunk without / with: 256 KiB 217 / 217, 512 KiB 395 / 303, 1 MiB 744 / 411, 4 MiB 2754 / 918.
# Below 512 KiB each hand-off to a hashing thread (GIL + wake-up) costs what the hash saves.
PREFETCH_MIN_CHUNK = 512 << 10
# Pieces of at least this many bytes are copied on the thread pool too (_pieces_parallel):
# 8 MiB chunks (512 KiB pieces) 1.79 -> 2.1-2.7 GiB/s per chunk, 3.47 -> 4.1-5.3 streamed
# (tools/stream_rate.py); with 128 KiB pieces the hand-offs cost more than the copies (C1's
# 4 MiB object fell from 1236-1289 to 811 MiB/s per chunk, 1327-1469 to 868 streamed).
PARALLEL_COPY_MIN = 256 << 10
HASH_ON_FILL = True  # encode_chunk: each large piece's id hashing starts as soon as that piece is filled
# The pieces (easyfec's k slices + the parity) and their SHA-1 ids made by the library in one call
# (sec_encode_pieces: copies and OpenSSL SHA-1 on its own host threads, the data pieces while
# the GPU encodes), instead of Python slicing / numpy fills and hashlib on the thread pool.
# False: the round-4 paths (A/B: tools/c1_loopback.py, tools/small_call_profile.py).
HOST_PIECES = True

# The library never retunes the host process's allocator.  A validator that drops each chunk's
# pieces after sending them can keep glibc from trimming the freed heap back to the kernel (so the
# next chunk's pieces do not fault their pages in again) by starting the process with
# MALLOC_MMAP_THRESHOLD_=33554432 MALLOC_TRIM_THRESHOLD_=268435456 ("Host
# allocator"; measured in DESIGN.md §5 Round 4).
STREAM_WINDOW_BYTES = 64 << 20  # chunk bytes per GPU call in the *_stream pipelines
# encode_chunks_stream(piece_ids=True) over windows whose pieces are all >= PARALLEL_COPY_MIN:
# the ids come from the GPU SHA-1 kernel, fused after the window's encode, instead of hashlib
# on the thread pool, in windows of STREAM_WINDOW_IDS_BYTES (when window_bytes is not given).
# The kernel is one lane per piece, so a window's hashing takes about one piece's chain
# whatever the window size: 1 GiB object, 8 MiB chunks, zfec(16,24): 7.1 / 9.1 GiB/s with
# 256 / 512 MiB windows against 3.2-5.3 hashing on the host (profiles/r02_stream_rate.json).
# Round 5: the host ids from sec_encode_pieces (OpenSSL on the library's threads, HOST_PIECES)
# beat them at every window: 8.1-8.3 GiB/s at 64-256 MiB against 4.6-7.1 for GPU ids
# (profiles/r05_stream_rate.json), at the 64 MiB window (lower latency to the first chunk), so
# the GPU ids are off by default.
GPU_PIECE_IDS = False
STREAM_WINDOW_IDS_BYTES = 256 << 20
# Round 6: with the host ids, the parity pieces' ids from the GPU instead
# (sec_encode_pieces SEC_F_GPU_PARITY_IDS: the SHA-1 kernel on the device-resident parity, one
# lane per piece, while the library's host threads hash only the data pieces), in windows of
# STREAM_WINDOW_PARITY_IDS_BYTES so that hundreds of parity pieces share one chain time.
# Measured on the 1 GiB upload (8 MiB chunks, zfec(16,24); profiles/r06_parity_ids.json): 3.96 /
# 6.21 / 6.70 / 7.13 GiB/s at 64 / 256 / 512 / 1024 MiB windows against 5.97 / 6.82 / 6.82 / 6.91
# with every id on the host threads.  Taking a third of the hashing off the host buys nothing:
# the upload is bound by the host's memory work on the fresh piece buffers (first touch, copies),
# and the GPU path adds a staged 512 MiB slab per window.  Off (F1 closed as host-only for the
# upload; the flag stays in the ABI, tested).
GPU_PARITY_IDS = False
STREAM_WINDOW_PARITY_IDS_BYTES = 512 << 20
STREAM_WORKERS = 4  # single-thread workers (one engine each) the *_stream pipelines are spread over


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


_pools: dict = {}
_pools_lock = threading.Lock()
# at most this many hash-pool threads (piece copies and hashlib SHA-1); STORB_HASH_WORKERS overrides
HASH_WORKERS = int(os.environ.get("STORB_HASH_WORKERS", "16") or 16)


def _cgroup_cpus() -> int | None:
    """The CPU quota of this process's cgroup (cgroup v2 cpu.max "quota period"), rounded up, or
    None when unlimited or unknown: a container's CPU share is often a quota, not an affinity
    mask, and threads beyond it are throttled rather than run."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota == "max":
            return None
        return max(1, -(-int(quota) // int(period)))
    except (OSError, ValueError):
        return None


def _usable_cpus() -> int:
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 2
    q = _cgroup_cpus()
    return min(n, q) if q else n


def _pool(name: str) -> ThreadPoolExecutor:
    """Module thread pools: "hash" (piece copies and hashlib SHA-1, which release the GIL) and
    "stream<i>" (_stream_pool)."""
    with _pools_lock:
        p = _pools.get(name)
        if p is None:
            # half the CPUs: SHA-1 on 8 threads of a 16-CPU quota ran at 15.3 GB/s, on 16 at 14.1, and
            # the per-chunk upload at 4.9 against 3.4 GiB/s (r03_upload_ab.jsonl)
            n = 1 if name.startswith("stream") else max(1, min(HASH_WORKERS, _usable_cpus() // 2))
            p = _pools[name] = ThreadPoolExecutor(n, thread_name_prefix=f"storb_amd_{name}")
        return p


_stream_rr = [0]


def _stream_pool() -> ThreadPoolExecutor:
    """The worker a new *_stream pipeline runs its GPU calls on: one of STREAM_WORKERS
    single-thread workers (each with its own engine), round robin.  A stream keeps its windows
    on its one worker (window w + 1 decodes while the caller consumes window w), and concurrent
    streams (downloads served on several request threads) do not queue behind one another.
    (All windows of one stream on 4 shared workers measured 2-7 % slower: tools/stream_rate.py
    --ab, profiles/r03_stream_ab.json.)"""
    with _pools_lock:
        i = _stream_rr[0] % max(1, STREAM_WORKERS)
        _stream_rr[0] += 1
    return _pool(f"stream{i}")


_ONE = "one"  # devices=_ONE: the calling thread's own engine (inside an EngineGroup worker: its device)
_default_devices = None  # use_devices()
_groups: dict = {}


def use_devices(devices) -> None:
    """Module default of the batch and stream functions' ``devices=``: None (one device, the
    calling thread's engine: the default), "all" (every visible device), a list of device ids,
    or an EngineGroup.  A single-process validator (/root/reference/storb/validator/
    __main__.py:10-24) calls this once at start-up and then drives every GPU through the
    unchanged names: encode_chunks / decode_chunks / reconstruct_data split each batch by bytes
    over the devices, the *_stream pipelines send windows round robin to them, and the per-chunk
    calls (encode_chunk, decode_chunk) of different host threads are spread over them
    (engine.spread_threads)."""
    global _default_devices
    grp = _group(devices) if devices is not None else None
    _default_devices = grp
    spread_threads(grp.devices if grp is not None else None)


def _group(devices):
    """The EngineGroup for a ``devices=`` argument (None: the module default), or None for the
    one-device path.  Groups are created once per device list and kept (each holds a HIP
    context and a worker thread per device)."""
    if devices is _ONE:
        return None
    if devices is None:
        devices = _default_devices
        if devices is None:
            return None
    if isinstance(devices, EngineGroup):
        return devices
    key = "all" if isinstance(devices, str) and devices == "all" else tuple(int(d) for d in devices)
    with _pools_lock:
        g = _groups.get(key)
        if g is None:
            g = _groups[key] = EngineGroup(list(range(device_count())) if key == "all" else list(key))
    return g


def _sha1_hex(b) -> str:
    return hashlib.sha1(b).hexdigest()


class _PieceIdMemo:
    """Digests encode_chunk started for its pieces, keyed by the piece's bytes object.  A hit
    requires the very object (``is``), which the memo keeps alive while it holds it, so an id
    cannot be reused under it.

    Retention is bounded (the validator hashes a chunk's pieces right after its encode_chunk,
    validator.py:1380 -> 1081, so nothing older is ever asked for): entries leave on first use,
    when they belong to an encode_chunk call more than `keep_calls` calls ago, or oldest-first
    past `max_bytes`.  A call whose pieces alone exceed `max_bytes` is not prefetched.  When
    `idle_calls` calls in a row were evicted with none of their ids asked for (a caller that
    does not hash, or hashes copies), prefetching pauses, except for one probe call in every
    `probe_every`, so a caller that does not use the ids costs almost no hashing."""

    def __init__(self, max_bytes: int = 128 << 20, keep_calls: int = 2, idle_calls: int = 4, probe_every: int = 64):
        self.max_bytes = max_bytes
        self.keep_calls = keep_calls
        self.idle_calls = idle_calls
        self.probe_every = probe_every
        self._d: OrderedDict = OrderedDict()  # id -> (obj, future, call number)
        self._bytes = 0
        self._call = 0
        self._calls: dict[int, list[int]] = {}  # call number -> [entries held, ids taken]
        self._idle = 0  # consecutive evicted calls with no id taken
        self._lock = threading.Lock()

    def _drop(self, c: int, taken: bool) -> None:
        st = self._calls.get(c)
        if st is None:
            return
        st[0] -= 1
        st[1] += taken
        if st[0] <= 0:  # that call's last entry
            del self._calls[c]
            self._idle = 0 if st[1] else self._idle + 1

    def _evict_oldest(self) -> None:
        _, (o, f, c) = self._d.popitem(last=False)
        self._bytes -= len(o)
        f.cancel()  # not started yet: no hashing for an id nobody will ask for
        self._drop(c, False)

    def begin(self, nbytes: int) -> int | None:
        """Start an encode_chunk call's prefetch of `nbytes` of pieces: its call number, or None
        when it should not prefetch."""
        with self._lock:
            self._call += 1
            c = self._call
            if nbytes > self.max_bytes:
                return None
            if self._idle >= self.idle_calls and c % self.probe_every:
                return None
            while self._d and (next(iter(self._d.values()))[2] <= c - self.keep_calls
                               or self._bytes + nbytes > self.max_bytes):
                self._evict_oldest()
            return c

    def put(self, obj: bytes, fut: Future, call: int) -> None:
        with self._lock:
            old = self._d.pop(id(obj), None)
            if old is not None:  # the same object twice: counted once
                self._bytes -= len(old[0])
                self._drop(old[2], False)
            self._d[id(obj)] = (obj, fut, call)
            self._bytes += len(obj)
            self._calls.setdefault(call, [0, 0])[0] += 1
            while self._bytes > self.max_bytes and self._d:
                self._evict_oldest()

    def take(self, obj):
        with self._lock:
            e = self._d.get(id(obj))
            if e is None or e[0] is not obj:
                return None
            del self._d[id(obj)]
            self._bytes -= len(obj)
            self._idle = 0
            self._drop(e[2], True)
        try:
            return e[1].result()
        except Exception:  # noqa: BLE001 - cancelled or failed: hash here instead
            return None

    def held_bytes(self) -> int:
        with self._lock:
            return self._bytes


_memo = _PieceIdMemo()


def piece_hash(data: bytes) -> str:
    """SHA-1 hex digest of a piece (piece.py:54-68)."""
    d = _memo.take(data) if type(data) is bytes else None
    return d if d is not None else hashlib.sha1(data).hexdigest()


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


# New bytes objects filled in place before anyone else sees them: storb_amd/_hostbytes.py.
from ._hostbytes import _FILL_IN_PLACE, _PendingBytes, _finalize, _new_bytes  # noqa: E402,F401


def _fill(dst: np.ndarray, src: np.ndarray) -> None:
    dst[:len(src)] = src
    if len(src) < len(dst):
        dst[len(src):] = 0


def _hash_filled(fill: Future | None, view: np.ndarray, piece) -> str:
    """SHA-1 hex of a piece once its fill (an earlier task of the same FIFO pool) is done.

    `piece` is the bytes object (or _PendingBytes) `view` looks into.  The task holds it so the
    piece outlives the hash: on CPython `view` is a raw view of the object's buffer with no
    reference to it, and the memo may drop its own reference (eviction) while this task is
    queued or running, after the caller dropped the piece too."""
    if fill is not None:
        fill.result()
    assert piece is not None
    return hashlib.sha1(view).hexdigest()


def _pieces_parallel(chunks: list, shapes: list, digests: bool = False, hash_ids: bool = False):
    """Every chunk's m pieces as bytes (k zero-padded data slices, then the parity): one GPU
    call for all chunks; the piece copies run on the hash pool, the data slices beside the GPU
    call.  Returns once every piece is filled.  ``digests=True``: (pieces, ids), ids[i] = the
    piece ids (SHA-1 hex) of chunk i's m pieces, hashed on the GPU after the encode.
    ``hash_ids=True``: (pieces, futures), futures[i][j] = the hashlib SHA-1 hex of piece j of
    chunk i, each started as soon as that piece is filled (data pieces beside the GPU call) and
    still running when this returns."""
    hp = _pool("hash")
    out, jobs, hfut = [], [], []
    for c, (k, m, B, _) in zip(chunks, shapes):
        if k > 1 and (k - 1) * B > len(c):  # easyfec's short middle slice, as Encoder.encode
            raise Error("Precondition violation: Input blocks are required to be all the same length.")
        src = np.frombuffer(memoryview(c).cast("B"), dtype=np.uint8)
        ps, views = [], []
        for j in range(k):
            b, v = _new_bytes(B)
            ps.append(b)
            views.append(v)
            jobs.append(hp.submit(_fill, v, src[j * B:min((j + 1) * B, len(src))]))
        out.append(ps)
        if hash_ids:  # queued behind this chunk's data fills (FIFO), so they never wait long
            hfut.append([hp.submit(_hash_filled, f, v, b) for f, v, b in zip(jobs[-k:], views, ps)])
    # staged, not page-locked: the pool is faulting in the new pieces meanwhile, and locking
    # waits on the same memory-map lock (6.4 against 0.55 ms for one 8 MiB chunk on MI355X,
    # profiles/r03_upload_ab.jsonl)
    res = get_engine().encode_host_raw(list(chunks), [(k, m) for (k, m, _, _) in shapes], digests=digests,
                                       staged=True)
    buf, layout = res[0], res[1]
    for i, (ps, (o, B, p)) in enumerate(zip(out, layout)):
        pj = []
        for r in range(p):
            b, v = _new_bytes(B)
            ps.append(b)
            if hash_ids:  # the pool's queue holds the data pieces' hashes: the caller, idle
                # until its pieces exist, copies the parity itself (r03_upload_timeline.json)
                _fill(v, buf[o + r * B:o + (r + 1) * B])
                hfut[i].append(hp.submit(_hash_filled, None, v, b))
            else:
                jobs.append(hp.submit(_fill, v, buf[o + r * B:o + (r + 1) * B]))
                pj.append((jobs[-1], v))
    ids = None
    if digests:
        hx, ids, f = res[2].tobytes().hex(), [], 0
        for (_, m, _, _) in shapes:
            ids.append([hx[40 * (f + j):40 * (f + j + 1)] for j in range(m)])
            f += m
    for f in jobs:  # the pieces must be complete before anyone sees them (and buf is reused)
        f.result()
    if not _FILL_IN_PLACE:
        out = [[_finalize(p) for p in ps] for ps in out]
    if hash_ids:
        return out, hfut
    return (out, ids) if digests else out


class _Done:
    """A finished result in the memo's future slot (the library computed the digest already)."""

    __slots__ = ("v",)

    def __init__(self, v):
        self.v = v

    def result(self):
        return self.v

    def cancel(self):
        return False


def _encode_pieces(chunks: list, shapes: list, ids: bool, gpu_parity_ids: bool = False):
    """Every chunk's m pieces as new bytes objects, filled by the library (sec_encode_pieces:
    the k data slices, zero-padded, then the parity), and with `ids` each piece's SHA-1 hex
    (the library's host threads, OpenSSL: hashlib's bytes; with `gpu_parity_ids` the parity
    pieces' from the GPU SHA-1 kernel).  Returns (pieces, ids or None)."""
    objs, addrs = [], []
    for (k, m, B, _) in shapes:
        row = []
        for _ in range(m):
            b, v = _new_bytes(B)
            row.append((b, v))
            addrs.append(v.ctypes.data if B else 0)
        objs.append(row)
    dig = np.empty(max(20 * len(addrs), 1), dtype=np.uint8) if ids else None
    # staged, not page-locked: the library's threads fault in the new pieces meanwhile, and locking
    # waits on the same memory-map lock (6.4 against 0.55 ms for one 8 MiB chunk on MI355X,
    # profiles/r03_upload_ab.jsonl)
    get_engine().encode_pieces_into(chunks, [(k, m) for (k, m, _, _) in shapes], addrs, dig, staged=True,
                                    gpu_parity_ids=ids and gpu_parity_ids)
    pieces = [[_finalize(b) for b, _ in row] for row in objs]
    hexes = None
    if ids:
        hx, hexes, f = dig.tobytes().hex(), [], 0
        for (_, m, _, _) in shapes:
            hexes.append([hx[40 * (f + j):40 * (f + j + 1)] for j in range(m)])
            f += m
    return pieces, hexes


def _short_middle(shapes, chunks) -> None:
    for c, (k, m, B, _) in zip(chunks, shapes):
        if k > 1 and (k - 1) * B > len(c):  # easyfec's short middle slice, as Encoder.encode
            raise Error("Precondition violation: Input blocks are required to be all the same length.")


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
    enc_ = Encoder(k, m)
    if HOST_PIECES:  # pieces and (prefetched) ids from the library in one call
        call = _memo.begin(m * B) if PREFETCH_PIECE_IDS else None
        _short_middle([(k, m, B, padlen)], [chunk])
        pieces, ids = _encode_pieces([chunk], [(k, m, B, padlen)], call is not None)
        if call is not None:
            for b, h in zip(pieces[0], ids[0]):
                _memo.put(b, _Done(h), call)
        return _build(chunk_idx, k, m, B, padlen, chunk_size, pieces[0])
    call = _memo.begin(m * B) if PREFETCH_PIECE_IDS and chunk_size >= PREFETCH_MIN_CHUNK else None
    if call is None:
        encoded_pieces = enc_.encode(chunk)
    else:  # piece ids hashed on the pool: data pieces beside the GPU call, parity right after
        hp = _pool("hash")
        if B >= PARALLEL_COPY_MIN and HASH_ON_FILL:  # large pieces: copies on the pool too, each hashed once filled
            pieces, hf = _pieces_parallel([chunk], [(k, m, B, padlen)], hash_ids=True)
            encoded_pieces, futs = pieces[0], hf[0]
        elif B >= PARALLEL_COPY_MIN:  # (A/B: every piece hashed after all are filled)
            encoded_pieces = _pieces_parallel([chunk], [(k, m, B, padlen)])[0]
            futs = [hp.submit(_sha1_hex, b) for b in encoded_pieces]
        else:
            prim = _split(chunk, k, B)
            futs = [hp.submit(_sha1_hex, b) for b in prim]
            parity = enc_.encode_parity(chunk) if m > k and B else [b""] * (m - k)
            futs += [hp.submit(_sha1_hex, b) for b in parity]
            encoded_pieces = prim + parity
        for b, f in zip(encoded_pieces, futs):
            _memo.put(b, f, call)
    enc = _build(chunk_idx, k, m, B, padlen, chunk_size, encoded_pieces)
    logger.debug("[encode_chunk] chunk %d: k=%d, m=%d, encoded %d blocks", chunk_idx, k, m, len(enc.pieces))
    return enc


def encode_chunks(chunks: typing.Sequence[bytes], first_chunk_idx: int = 0, *, devices=None) -> list[EncodedChunk]:
    """Batched ``encode_chunk`` over many chunks in ONE GPU call; chunk i gets index first+i.

    devices (or the module default set by ``use_devices``): the chunks are split by bytes over
    those devices' workers (``EngineGroup``), one GPU call per device, results in chunk order."""
    shapes = []
    for c in chunks:
        n = len(c)
        piece_length(n)  # same ValueError as encode_chunk for n == 0
        shapes.append(chunk_shape(n))
    if not chunks:
        return []
    grp = _group(devices)
    if grp is not None:
        parts = grp.map_shares(lambda share, lo: encode_chunks(share, first_chunk_idx + lo, devices=_ONE),
                               list(chunks), [len(c) for c in chunks])
        return [ec for p in parts if p for ec in p]
    if HOST_PIECES:
        _short_middle(shapes, chunks)
        pieces, _ = _encode_pieces(list(chunks), shapes, False)
        return [_build(first_chunk_idx + i, k, m, B, padlen, len(c), ps)
                for i, (c, (k, m, B, padlen), ps) in enumerate(zip(chunks, shapes, pieces))]
    if min(B for (_, _, B, _) in shapes) >= PARALLEL_COPY_MIN:  # piece copies in parallel
        pieces = _pieces_parallel(list(chunks), shapes)
        return [_build(first_chunk_idx + i, k, m, B, padlen, len(c), ps)
                for i, (c, (k, m, B, padlen), ps) in enumerate(zip(chunks, shapes, pieces))]
    parity = get_engine().encode_host(list(chunks), [(k, m) for (k, m, _, _) in shapes])
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
    if len(pieces) > k and CHOOSE_BLOCKS:
        # the validator hands over every piece it fetched (validator.py:1556-1604, 1631): decode
        # from the k the library picks (every present primary, then parity rows of one decode
        # row group where possible: the fused syndrome kernel), not the first k; same bytes
        pick = choose_blocks(k, encoded_chunk.m, [p.piece_idx for p in pieces])
        if pick is not None:
            use = [pieces[i] for i in pick]
            return [p.data for p in use], [p.piece_idx for p in use]
    use = pieces[:k] if len(pieces) > k else pieces
    return [p.data for p in use], [p.piece_idx for p in use]


def decode_chunk(encoded_chunk: EncodedChunk, *, positional_sharenums: bool = False) -> bytes:
    """Decode one chunk from its pieces (piece.py:169-198); see module doc for sharenums."""
    blocks, sharenums = _sharenums(encoded_chunk, positional_sharenums)
    decoder = Decoder(encoded_chunk.k, encoded_chunk.m)
    return decoder.decode(blocks, sharenums, encoded_chunk.padlen)


def decode_chunks(encoded_chunks: typing.Sequence[EncodedChunk], *, positional_sharenums: bool = False,
                  devices=None) -> bytes:
    """Batched ``decode_chunk``: the concatenation of every chunk's bytes, one GPU call.

    devices (or the module default set by ``use_devices``): the chunks are split by bytes over
    those devices' workers, each share decoded by its own device straight into its slice of the
    result (one copy, as on one device)."""
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
    if not items:
        return b""
    grp = _group(devices)
    if grp is None:
        return get_engine().decode_host(items)
    for it in items:  # zfec's preconditions for every chunk before any device starts
        check_decode_item(*it)
    lens = [k * len(blocks[0]) - padlen for (k, _, blocks, _, padlen) in items]
    starts = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    out, view = _new_bytes(int(starts[-1]))

    def share(its, lo):
        return get_engine().decode_host_into(its, view[starts[lo]:starts[lo + len(its)]])

    grp.map_shares(share, items, lens)
    return _finalize(out)


def _relevant(pieces: list[Piece], chunk: EncodedChunk) -> list[Piece]:
    relevant = [piece for piece in pieces if piece.chunk_idx == chunk.chunk_idx]
    relevant.sort(key=lambda p: p.piece_idx)
    if len(relevant) < chunk.k:
        raise ValueError(f"Not enough pieces to reconstruct chunk {chunk.chunk_idx}")
    return relevant


def reconstruct_data(pieces: list[Piece], chunks: list[EncodedChunk], *, devices=None) -> bytes:
    """Reconstruct the original bytes from pieces (piece.py:201-236), one batched decode (per
    device with `devices` / ``use_devices``: see decode_chunks)."""
    by_chunk: dict[int, list[Piece]] = {}
    for p in pieces:
        by_chunk.setdefault(p.chunk_idx, []).append(p)
    for chunk in chunks:
        relevant = sorted(by_chunk.get(chunk.chunk_idx, []), key=lambda p: p.piece_idx)
        if len(relevant) < chunk.k:
            raise ValueError(f"Not enough pieces to reconstruct chunk {chunk.chunk_idx}")
        chunk.pieces = relevant
    return decode_chunks(chunks, devices=devices)


def _windows(chunks, nbytes, size_of) -> Iterator[list]:
    """Consecutive groups of chunks totalling at most `nbytes` (at least one chunk each)."""
    win, acc = [], 0
    for c in chunks:
        sz = size_of(c)
        if win and acc + sz > nbytes:
            yield win
            win, acc = [], 0
        win.append(c)
        acc += sz
    if win:
        yield win


def _decode_window(window: list, by_chunk: dict):
    """Worker side of reconstruct_data_stream: (per-chunk bytes, error) for one window.  The
    window's chunks up to the first one that cannot be decoded are decoded (one GPU call for
    those with a missing primary); that chunk's error is returned, to be raised in order."""
    items, err = [], None
    for chunk in window:
        try:
            relevant = sorted(by_chunk.get(chunk.chunk_idx, []), key=lambda p: p.piece_idx)
            if len(relevant) < chunk.k:
                raise ValueError(f"Not enough pieces to reconstruct chunk {chunk.chunk_idx}")
            chunk.pieces = relevant
            blocks, sharenums = _sharenums(chunk, False)
            B = len(blocks[0]) if blocks else 0
            if not (1 <= chunk.k <= chunk.m <= 256) or not (0 <= chunk.padlen <= chunk.k * B):
                # easyfec's own slicing semantics: the per-chunk path, decoded here
                items.append(("bytes", decode_chunk(chunk)))
                continue
            item = (chunk.k, chunk.m, blocks, sharenums, chunk.padlen)
            check_decode_item(*item)  # zfec's preconditions, before any chunk of the window decodes
        except Exception as e:  # noqa: BLE001 - re-raised on the caller's thread after the chunks before it
            err = e
            break
        items.append(item)
    try:
        batch = [it for it in items if it[0] != "bytes"]
        outs = iter(get_engine().decode_host_chunks(batch) if batch else [])
        res = [it[1] if it[0] == "bytes" else next(outs) for it in items]
    except Exception as e:  # noqa: BLE001 - a device failure: nothing of the window is trusted
        return [], e
    return res, err


def reconstruct_data_stream(pieces: list[Piece], chunks: list[EncodedChunk], *,
                            window_bytes: int | None = None, devices=None) -> Iterator[bytes]:
    """Yield the reconstructed bytes chunk by chunk (piece.py:239-263).

    Chunks go in windows of about `window_bytes` (default STREAM_WINDOW_BYTES) of output; each
    window is one batched decode on a worker thread, and window w+1's decode runs while the
    caller consumes window w (the validator streams them into the HTTP response,
    validator.py:1630-1638).  With `devices` (or ``use_devices``) the windows go round robin to
    those devices' workers, two per device in flight.  Chunks come out in order; a chunk without
    enough pieces raises the reference's ValueError when the stream reaches it, after every
    earlier chunk."""
    by_chunk: dict[int, list[Piece]] = {}
    for p in pieces:
        by_chunk.setdefault(p.chunk_idx, []).append(p)
    wb = STREAM_WINDOW_BYTES if window_bytes is None else window_bytes
    wins = _windows(chunks, wb, lambda c: max(c.original_chunk_size, 1))
    for outs, err in _pipeline(wins, _decode_window, (by_chunk,), _group(devices)):
        yield from outs
        if err is not None:
            raise err


def _pipeline(windows: Iterator[list], fn, args: tuple, grp) -> Iterator:
    """fn(window, *args) of each window on the stream workers, results in window order.

    One device (grp None): one _stream_pool worker, window w + 1 running while the caller
    consumes window w.  EngineGroup: window i on worker i mod D, 2 D windows in flight.  Windows
    are pulled from `windows` (on the caller's thread) only as slots free up; an error, or the
    consumer closing the stream early, cancels the windows not yet started."""
    if grp is None:
        pool = _stream_pool()
        depth, submit = 2, (lambda i, w: pool.submit(fn, w, *args))
    else:
        depth, submit = 2 * len(grp), (lambda i, w: grp.submit(i % len(grp), fn, w, *args))
    q: deque = deque()
    nxt = [0]

    def fill():
        while len(q) < depth:
            w = next(windows, None)
            if w is None:
                return
            q.append(submit(nxt[0], w))
            nxt[0] += 1

    try:
        fill()
        while q:
            fut = q.popleft()
            res = fut.result()
            yield res
            fill()
    finally:
        for f in q:
            f.cancel()


def _window_shapes(window: list):
    """(shapes of the window's chunks up to the first one encode_chunk would reject, that
    chunk's error or None): piece_length's ValueError for an empty chunk, easyfec's short middle
    slice (zfec Error)."""
    shapes = []
    for c in window:
        try:
            n = len(c)
            piece_length(n)
            k, m, B, padlen = chunk_shape(n)
            if k > 1 and (k - 1) * B > n:
                raise Error("Precondition violation: Input blocks are required to be all the same length.")
        except Exception as e:  # noqa: BLE001 - raised on the caller's thread after the chunks before it
            return shapes, e
        shapes.append((k, m, B, padlen))
    return shapes, None


def _encode_window(window: list, first_idx: int, piece_ids: bool):
    """Worker side of encode_chunks_stream: one batched GPU encode for the window (+ SHA-1 piece
    ids: on the GPU for large pieces, else on the hash pool, data pieces starting before the GPU
    call and parity pieces after it).  Returns (results, error): a chunk encode_chunk would
    reject ends the window there, and the chunks before it are still encoded and returned."""
    shapes, err = _window_shapes(window)
    window = window[:len(shapes)]
    if not window:
        return [], err
    try:
        if not piece_ids:
            return [(c, None) for c in encode_chunks(window, first_idx)], err
        hp = _pool("hash")
        if GPU_PIECE_IDS and min(B for (_, _, B, _) in shapes) >= PARALLEL_COPY_MIN:
            pieces, ids = _pieces_parallel(window, shapes, digests=True)
            out = [_build(first_idx + i, k, m, B, padlen, len(c), ps)
                   for i, (c, (k, m, B, padlen), ps) in enumerate(zip(window, shapes, pieces))]
            return list(zip(out, ids)), err
        if HOST_PIECES:  # ids by the library's host threads (OpenSSL; parity ids on the GPU), pieces in the same call
            pieces, ids = _encode_pieces(list(window), shapes, True, GPU_PARITY_IDS)
            out = [_build(first_idx + i, k, m, B, padlen, len(c), ps)
                   for i, (c, (k, m, B, padlen), ps) in enumerate(zip(window, shapes, pieces))]
            return list(zip(out, ids)), err
        if min(B for (_, _, B, _) in shapes) >= PARALLEL_COPY_MIN:
            pieces = _pieces_parallel(window, shapes)
            futs = [[hp.submit(_sha1_hex, b) for b in ps] for ps in pieces]
        else:  # small pieces: caller-thread copies; data pieces hash while the GPU runs
            prims = [_split(c, k, B) for c, (k, _, B, _) in zip(window, shapes)]
            futs = [[hp.submit(_sha1_hex, b) for b in prim] for prim in prims]
            parity = get_engine().encode_host(list(window), [(k, m) for (k, m, _, _) in shapes])
            pieces = [prim + par for prim, par in zip(prims, parity)]
            for fs, par in zip(futs, parity):
                fs.extend(hp.submit(_sha1_hex, b) for b in par)
        out = [_build(first_idx + i, k, m, B, padlen, len(c), ps)
               for i, (c, (k, m, B, padlen), ps) in enumerate(zip(window, shapes, pieces))]
        return [(ec, [f.result() for f in fs]) for ec, fs in zip(out, futs)], err
    except Exception as e:  # noqa: BLE001 - a device failure: nothing of the window is trusted
        return [], e


def encode_chunks_stream(chunks: Iterable[bytes], first_chunk_idx: int = 0, *, piece_ids: bool = False,
                         window_bytes: int | None = None, devices=None) -> Iterator:
    """``encode_chunk`` over a stream of chunks (the validator's upload loop: chunks read from
    the request, encoded, handed to the miners, validator.py:1338-1446), pipelined.

    Chunks are pulled from `chunks` on the caller's thread into windows of about
    `window_bytes` (default STREAM_WINDOW_BYTES); each window is one batched GPU encode on a
    worker thread, running while the caller consumes the previous window's results (with
    `devices` / ``use_devices``: windows round robin over those devices, two per device in
    flight).  Yields ``EncodedChunk`` per chunk in order (chunk i gets index first_chunk_idx + i),
    or with ``piece_ids=True`` ``(EncodedChunk, [piece_hash of each of its m pieces])``; those ids
    come from the library's host threads for the data pieces and from the GPU for the parity
    pieces (GPU_PARITY_IDS; default window STREAM_WINDOW_PARITY_IDS_BYTES), or all from the GPU
    (GPU_PIECE_IDS) for windows of large pieces, whose default window is then
    STREAM_WINDOW_IDS_BYTES."""
    wb = window_bytes
    if wb is None:
        wb = (STREAM_WINDOW_IDS_BYTES if piece_ids and GPU_PIECE_IDS else
              STREAM_WINDOW_PARITY_IDS_BYTES if piece_ids and HOST_PIECES and GPU_PARITY_IDS else STREAM_WINDOW_BYTES)

    def numbered():  # (window, index of its first chunk)
        idx = first_chunk_idx
        for win in _windows(chunks, wb, lambda c: max(len(c), 1)):
            yield win, idx
            idx += len(win)

    def run(wi, pid):
        return _encode_window(wi[0], wi[1], pid)

    for outs, err in _pipeline(numbered(), run, (piece_ids,), _group(devices)):
        for ec, ids in outs:
            yield (ec, ids) if piece_ids else ec
        if err is not None:
            raise err

"""GPU: sec_encode_pieces — easyfec's Encoder.encode output written straight into the caller's
piece buffers, with each piece's SHA-1 from the library's host threads (VERDICT r04 next #7:
the per-call floor at storb's granularity).  Every piece is compared with the oracle's
(oracle/fec_oracle.c easy_encode) and every digest with hashlib; the drop-in's encode_chunk /
encode_chunks / encode_chunks_stream give the same pieces and ids with the library path on and
off (piece.HOST_PIECES)."""

import ctypes
import hashlib
import random

import numpy as np
import pytest

from oracle import cfec

pytestmark = pytest.mark.gpu

from storb_amd import piece  # noqa: E402
from storb_amd.engine import ECRuntimeError, Error, get_engine  # noqa: E402


def _shapes_and_chunks(rng):
    out = []
    for n in (1, 2, 17, 4096, 16384, 16385, 70_000, 256 << 10, (256 << 10) + 1, 1 << 20, 3 << 20, (8 << 20) + 5):
        out.append((piece.chunk_shape(n), rng.randbytes(n)))
    for k, m, n in ((1, 2, 999), (4, 6, 6554 * 4 - 3), (10, 14, 65536), (8, 11, 300_007), (16, 24, 2 << 20),
                    (64, 96, 1 << 20), (3, 3, 5000)):
        B = -(-n // k)
        out.append(((k, m, B, k * B - n), rng.randbytes(n)))
    return out


def _run(cases, digests=True, gpu_parity_ids=False):
    eng = get_engine()
    bufs, addrs = [], []
    for (k, m, B, _), _ in cases:
        row = [np.empty(B, np.uint8) for _ in range(m)]
        bufs.append(row)
        addrs += [a.ctypes.data for a in row]
    dig = np.zeros(20 * len(addrs), np.uint8) if digests else None
    eng.encode_pieces_into([c for _, c in cases], [(k, m) for (k, m, _, _), _ in cases], addrs, dig,
                           gpu_parity_ids=gpu_parity_ids)
    return bufs, dig


@pytest.mark.parametrize("gpu_parity_ids", [False, True])
def test_pieces_and_ids_vs_oracle(gpu_parity_ids):
    """Every piece against the oracle, every id against hashlib; with gpu_parity_ids the parity
    pieces' ids come from the GPU SHA-1 kernel (SEC_F_GPU_PARITY_IDS), the data pieces' from the
    host threads, in one call over every shape (including m == k and an empty chunk)."""
    rng = random.Random(1)
    cases = _shapes_and_chunks(rng)
    if gpu_parity_ids:
        cases.append(((2, 3, 0, 0), b""))  # B = 0: every piece b"", ids sha1(b"")
    rng.shuffle(cases)  # shapes interleaved in one call
    bufs, dig = _run(cases, gpu_parity_ids=gpu_parity_ids)
    j = 0
    for ((k, m, B, padlen), c), row in zip(cases, bufs):
        want = cfec.easy_encode(c, k, m) if c else [b""] * m
        assert [r.tobytes() for r in row] == want, (k, m, len(c))
        for w in want:
            assert dig[20 * j:20 * (j + 1)].tobytes() == hashlib.sha1(w).digest(), (k, m, len(c), j)
            j += 1


def test_gpu_parity_ids_many_sub_batches():
    """SEC_F_GPU_PARITY_IDS over more parity than one SEC_SLAB_BYTES_DIGEST sub-batch (the option
    lowered to 1 MiB on a fresh engine): ids still land in each piece's own slot."""
    from storb_amd.engine import Engine

    rng = random.Random(5)
    eng = Engine(0, options={"SEC_SLAB_BYTES_DIGEST": 1 << 20})
    try:
        cases = [(piece.chunk_shape(n), rng.randbytes(n)) for n in [(1 << 20) + 7, 600_001, 2 << 20, 1 << 20, 99_999]]
        bufs, addrs = [], []
        for (k, m, B, _), _ in cases:
            row = [np.empty(B, np.uint8) for _ in range(m)]
            bufs.append(row)
            addrs += [a.ctypes.data for a in row]
        dig = np.zeros(20 * len(addrs), np.uint8)
        eng.encode_pieces_into([c for _, c in cases], [(k, m) for (k, m, _, _), _ in cases], addrs, dig,
                               gpu_parity_ids=True)
        j = 0
        for ((k, m, B, _), c), row in zip(cases, bufs):
            want = cfec.easy_encode(c, k, m)
            assert [r.tobytes() for r in row] == want
            for w in want:
                assert dig[20 * j:20 * (j + 1)].tobytes() == hashlib.sha1(w).digest(), (k, m, len(c), j)
                j += 1
    finally:
        eng.close()


def test_pieces_without_ids_and_repeat_calls():
    rng = random.Random(2)
    cases = _shapes_and_chunks(rng)[:8]
    for _ in range(3):  # the pinned parity scratch and the task pool reused across calls
        bufs, dig = _run(cases, digests=False)
        assert dig is None
        for ((k, m, _, _), c), row in zip(cases, bufs):
            assert [r.tobytes() for r in row] == cfec.easy_encode(c, k, m)


def test_pieces_errors():
    eng = get_engine()
    with pytest.raises(Error):  # easyfec's short middle slice (k = 4, n = 5: B = 2, 3 * 2 > 5)
        eng.encode_pieces_into([b"12345"], [(4, 6)], [np.empty(2, np.uint8).ctypes.data] * 6)
    with pytest.raises(ECRuntimeError, match="invalid argument"):  # a NULL piece buffer (SEC_EINVAL)
        eng.encode_pieces_into([b"x" * 100], [(2, 3)], [0, 0, 0])
    with pytest.raises(ValueError):  # one address per piece
        eng.encode_pieces_into([b"x" * 100], [(2, 3)], [1, 2])
    lib = eng.lib
    assert lib.sec_encode_pieces(eng._ctx, None, 1, None, None, None, 1) != 0  # no descriptors
    assert lib.sec_encode_pieces(eng._ctx, None, 0, None, None, None, 0) != 0  # device mode refused


@pytest.mark.parametrize("n", [1000, 256 << 10, 512 << 10, 8 << 20])
def test_encode_chunk_host_pieces_same_as_round4_path(n):
    data = random.Random(n).randbytes(n)
    old = piece.HOST_PIECES
    try:
        piece.HOST_PIECES = False
        a = piece.encode_chunk(data, 3)
        piece.HOST_PIECES = True
        b = piece.encode_chunk(data, 3)
    finally:
        piece.HOST_PIECES = old
    assert a.model_dump() == b.model_dump()
    k, m = b.k, b.m
    assert [p.data for p in b.pieces] == cfec.easy_encode(data, k, m)
    # the validator's piece_hash right after encode_chunk (validator.py:1081): the library's ids
    assert [piece.piece_hash(p.data) for p in b.pieces] == [hashlib.sha1(p.data).hexdigest() for p in b.pieces]


@pytest.mark.parametrize("gpu_parity_ids", [False, True])
def test_encode_chunks_and_stream_host_pieces(gpu_parity_ids, monkeypatch):
    monkeypatch.setattr(piece, "GPU_PARITY_IDS", gpu_parity_ids)
    rng = random.Random(5)
    chunks = [rng.randbytes(rng.choice([3, 4096, 100_000, 300_001, 1 << 20])) for _ in range(12)]
    ecs = piece.encode_chunks(chunks, 4)
    for c, ec in zip(chunks, ecs):
        assert [p.data for p in ec.pieces] == cfec.easy_encode(c, ec.k, ec.m)
    outs = list(piece.encode_chunks_stream(chunks, 0, piece_ids=True, window_bytes=600_000))
    for c, (ec, ids) in zip(chunks, outs):
        want = cfec.easy_encode(c, ec.k, ec.m)
        assert [p.data for p in ec.pieces] == want
        assert ids == [hashlib.sha1(w).hexdigest() for w in want]


def test_native_join_decode_host_fresh_outputs_repeated():
    """The shape that once returned a wrong chunk: an all-present 8 MiB chunk
    beside 8 MiB chunks with data piece 0 lost, reassembled into fresh output objects whose lost
    rows' pages the host never touched before the GPU writes them (page-locked for the call), in
    several rounds, each against the source bytes."""
    eng = get_engine()
    rng = random.Random(21)
    n = 8 << 20
    k, m, B, padlen = piece.chunk_shape(n)
    srcs = [rng.randbytes(n) for _ in range(3)]
    blocks = [cfec.easy_encode(d, k, m) for d in srcs]
    items = []
    for i, (d, bl) in enumerate(zip(srcs, blocks)):
        lost = () if i == 0 else (0,) if i == 1 else (0, 5)
        keep = [j for j in range(m) if j not in lost][:k]
        items.append((k, m, [bl[j] for j in keep], keep, padlen))
    for _ in range(8):
        assert eng.decode_host_chunks(items) == srcs
        assert eng.decode_host(items) == b"".join(srcs)


def test_pieces_bytes_are_immutable_objects():
    """The pieces are ordinary bytes objects (filled in place before anyone sees them)."""
    ec = piece.encode_chunk(b"abc" * 50_000, 0)
    for p in ec.pieces:
        assert type(p.data) is bytes
    raw = ctypes.string_at(id(ec.pieces[0].data) + bytes.__basicsize__ - 1, 4) if piece._FILL_IN_PLACE else None
    assert raw is None or raw == ec.pieces[0].data[:4]


def test_native_join_decode_host():
    """Reassembled chunks of >= Engine.NATIVE_JOIN_MIN bytes are joined on the library's copy
    threads (sec_host_copy): every data piece present (no GPU work) and with pieces lost, per
    chunk and concatenated, against the source bytes."""
    from storb_amd._lib import COPY_DTYPE

    eng = get_engine()
    rng = random.Random(9)
    items, want = [], []
    for n in (3 << 20, (1 << 20) + 7, 5000, 8 << 20):
        data = rng.randbytes(n)
        k, m, B, padlen = piece.chunk_shape(n)
        blocks = cfec.easy_encode(data, k, m)
        for lost in ((), (0,), tuple(range(min(m - k, k)))):
            keep = [j for j in range(m) if j not in lost][:k]
            items.append((k, m, [blocks[j] for j in keep], keep, padlen))
            want.append(data)
    assert eng.decode_host_chunks(items) == want
    assert eng.decode_host(items) == b"".join(want)
    dst = np.zeros(sum(map(len, want)), np.uint8)
    assert eng.decode_host_into(items, dst) == dst.size and dst.tobytes() == b"".join(want)
    # zero-fill and a NULL destination
    buf = np.full(64, 7, np.uint8)
    jobs = np.zeros(1, dtype=COPY_DTYPE)
    jobs[0] = (buf.ctypes.data + 8, 0, 16)
    assert eng.lib.sec_host_copy(eng._ctx, jobs.ctypes.data, 1) == 0
    assert buf[8:24].sum() == 0 and buf[:8].tolist() == [7] * 8 and buf[24:].tolist() == [7] * 40
    jobs[0] = (0, buf.ctypes.data, 16)
    assert eng.lib.sec_host_copy(eng._ctx, jobs.ctypes.data, 1) != 0


@pytest.mark.parametrize("library_join", [True, False])
def test_reassembly_paths_agree(library_join, monkeypatch):
    """decode_host / _chunks / _into with the library's one-call reassembly (sec_decode_batch_ex's
    host join: present pieces copied by the task threads, the GPU on the chunks with a lost data
    piece only) and with round 4's recover-then-join form: same bytes, small and large chunks,
    padded last blocks, nothing / one / every possible primary lost, mixed shapes in one call."""
    from storb_amd.engine import Engine

    monkeypatch.setattr(Engine, "LIBRARY_JOIN", library_join)
    eng = get_engine()
    rng = random.Random(31)
    items, want = [], []
    for n in (1, 100, 70_000, (1 << 20) + 3, 3 << 20, (8 << 20) - 1):
        data = rng.randbytes(n)
        k, m, B, padlen = piece.chunk_shape(n)
        blocks = cfec.easy_encode(data, k, m)
        for lost in ((), (k - 1,), tuple(range(min(m - k, k)))):
            keep = [j for j in range(m) if j not in lost][:k]
            rng.shuffle(keep)
            items.append((k, m, [blocks[j] for j in keep], keep, padlen))
            want.append(data)
    assert eng.decode_host_chunks(items) == want
    assert eng.decode_host(items) == b"".join(want)
    dst = np.zeros(sum(map(len, want)) + 5, np.uint8)
    assert eng.decode_host_into(items, dst) == dst.size - 5
    assert dst[:-5].tobytes() == b"".join(want)


def test_reassembly_threads_concurrent():
    """Host reassembly from several threads at once, each on its own engine (the stream workers'
    form): piece objects (staged or read back from a locked output), all-present chunks copied
    without the GPU, per-call page locks of neighbouring outputs that touch one another's
    registrations.  Every result is exact however the calls interleave."""
    import threading

    from storb_amd.engine import Engine

    rng = random.Random(41)
    cases = []
    for n in (3 << 20, (1 << 20) + 11, 8 << 20, 70_000):
        data = rng.randbytes(n)
        k, m, B, padlen = piece.chunk_shape(n)
        blocks = cfec.easy_encode(data, k, m)
        for lost in ((), (0,), tuple(range(min(m - k, k)))):
            keep = [j for j in range(m) if j not in lost][:k]
            cases.append(((k, m, [blocks[j] for j in keep], keep, padlen), data))
    errors = []

    def run(seed):
        try:
            eng = Engine(0)
            try:
                r = random.Random(seed)
                for _ in range(6):
                    pick = r.sample(cases, 6)
                    items = [c for c, _ in pick]
                    if r.random() < 0.5:
                        assert eng.decode_host_chunks(items) == [d for _, d in pick]
                    else:
                        assert eng.decode_host(items) == b"".join(d for _, d in pick)
            finally:
                eng.close()
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    ts = [threading.Thread(target=run, args=(s,)) for s in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors


def test_pieces_parity_over_slab_and_empty_chunks():
    """The call's parity far above SEC_SLAB_BYTES (64 KiB here): sub-batches through two bounded
    pinned scratch buffers, a chunk whose own parity exceeds the cap alone; empty chunks' pieces
    hash as b"" (ADVICE r05)."""
    from storb_amd.engine import Engine

    rng = random.Random(5)
    cases = _shapes_and_chunks(rng)
    for k, m in ((2, 3), (4, 6)):
        cases.insert(rng.randrange(len(cases)), ((k, m, 0, 0), b""))
    eng = Engine(options={"SEC_SLAB_BYTES": 1 << 16})
    try:
        for _ in range(2):  # scratch reused across calls
            bufs, addrs = [], []
            for (k, m, B, _), _ in cases:
                row = [np.empty(max(B, 1), np.uint8) for _ in range(m)]
                bufs.append(row)
                addrs += [a.ctypes.data for a in row]
            dig = np.zeros(20 * len(addrs), np.uint8)
            eng.encode_pieces_into([c for _, c in cases], [(k, m) for (k, m, _, _), _ in cases], addrs, dig)
            j = 0
            for ((k, m, B, _), c), row in zip(cases, bufs):
                want = cfec.easy_encode(c, k, m) if c else [b""] * m
                if c:
                    assert [r.tobytes() for r in row] == want, (k, m, len(c))
                for w in want:
                    assert dig[20 * j:20 * (j + 1)].tobytes() == hashlib.sha1(w).digest(), (k, m, len(c), j)
                    j += 1
    finally:
        eng.close()


def test_library_threads_bounded_over_many_contexts():
    """32 caller threads, each with its own context (get_engine), encode pieces at once: the
    library's host threads are one shared pool sized from this process's CPUs, not a pool per
    context."""
    import os
    import threading

    def nthreads():
        return len(os.listdir("/proc/self/task"))

    get_engine()  # this thread's context and the runtime's own threads exist before the count
    base = nthreads()
    rng = random.Random(9)
    chunk = rng.randbytes(3 << 20)
    errors, ready = [], threading.Barrier(32)
    peak = [0]

    def work():
        try:
            eng = get_engine()
            ready.wait()
            k, m = 8, 12
            B = -(-len(chunk) // k)
            row = [np.empty(B, np.uint8) for _ in range(m)]
            dig = np.zeros(20 * m, np.uint8)
            for _ in range(3):
                eng.encode_pieces_into([chunk], [(k, m)], [a.ctypes.data for a in row], dig)
                peak[0] = max(peak[0], nthreads())
            assert [r.tobytes() for r in row] == cfec.easy_encode(chunk, k, m)
            eng.close()
        except BaseException as e:  # noqa: BLE001 - reported below
            errors.append(e)

    th = [threading.Thread(target=work) for _ in range(32)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors[0]
    cpus = len(os.sched_getaffinity(0))
    # the 32 callers themselves, one pool of <= 7, and a few runtime threads; a pool per
    # context would add 7 per caller
    assert peak[0] - base <= 32 + 7 + 8, (peak[0], base, cpus)

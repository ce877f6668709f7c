"""GPU parity for sec_decode_batch_ex: per-block readable lengths and recover-only decodes.

* zfec's zero-padded last data block read IN PLACE from the chunk buffer (avail = B - padlen,
  bytes past it read as zero): C4's shape (64 KiB RS(10,4), B = 6554, padlen 4) and C5's
  mixed RS(8,3) sizes decoded with block k-1 present, against the source bytes (every chunk)
  and the oracle (oracle/fec_oracle.c, a sample);
* SEC_F_RECOVER (recover-only): the e missing primaries zfec's fec_decode itself produces
  (/root/reference/storb/util/piece.py:196-197 reaches it through easyfec), B bytes each with
  block k-1's zero padding, against the oracle's padded blocks; e = 0 chunks write nothing;
* the same through the staged host path (pageable buffers, zero-filled staging) and the
  zero-copy pinned path.
"""

import random

import numpy as np
import pytest

from oracle import cfec

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from storb_amd._lib import DEC_DTYPE, ENC_DTYPE  # noqa: E402


def _dev(nbytes, seed):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    return torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device="cuda", generator=g)


def _layout(sizes, k, m):
    sizes = np.asarray(sizes, dtype=np.uint64)
    B = (sizes + k - 1) // k
    in_off = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
    par_off = np.concatenate([[0], np.cumsum(B * (m - k))[:-1]]).astype(np.uint64)
    return sizes, B, in_off, par_off


def _encode(engine, sizes, k, m, src):
    sizes, B, in_off, par_off = _layout(sizes, k, m)
    d = np.zeros(len(sizes), dtype=ENC_DTYPE)
    d["in_off"], d["n"], d["parity_off"], d["parity_stride"] = in_off, sizes, par_off, B
    d["k"], d["m"] = k, m
    par = torch.empty(int(np.sum(B)) * (m - k), dtype=torch.uint8, device="cuda")
    engine.encode_batch(d, src, par)
    return par


def _dec_inputs(sizes, k, m, keeps, data_base, par_base, recover=False):
    """Descriptors + per-slot avail reading the kept blocks in place; keeps[i] = chunk i's
    k block numbers.  An in-place block k-1 has B - padlen readable bytes."""
    sizes, B, in_off, par_off = _layout(sizes, k, m)
    n = len(sizes)
    d = np.zeros(n, dtype=DEC_DTYPE)
    d["B"], d["padlen"], d["k"], d["m"] = B, B * k - sizes, k, m
    d["slot0"] = np.arange(n, dtype=np.uint64) * k
    sn = np.zeros(n * k, np.int32)
    offs = np.zeros(n * k, np.uint64)
    avail = np.zeros(n * k, np.uint64)
    out_off, o = np.zeros(n, np.uint64), 0
    for i in range(n):
        out_off[i] = o
        keep = keeps[i]
        e = sum(1 for s in range(k) if s not in keep)
        o += (e * int(B[i])) if recover else int(sizes[i])
        for j, s in enumerate(keep):
            sn[i * k + j] = s
            if s < k:
                offs[i * k + j] = data_base + int(in_off[i]) + s * int(B[i])
                avail[i * k + j] = int(sizes[i]) - s * int(B[i]) if s == k - 1 else int(B[i])
            else:
                offs[i * k + j] = par_base + int(par_off[i]) + (s - k) * int(B[i])
                avail[i * k + j] = int(B[i])
    d["out_off"] = out_off
    return d, sn, offs, avail, o


def _check_sample(src_h, par_h, sizes, k, m, sample):
    sizes, B, in_off, par_off = _layout(sizes, k, m)
    for ci in sample:
        n, b = int(sizes[ci]), int(B[ci])
        want = cfec.easy_encode(src_h[int(in_off[ci]):int(in_off[ci]) + n].tobytes(), k, m)[k:]
        got = par_h[int(par_off[ci]):int(par_off[ci]) + (m - k) * b].tobytes()
        assert got == b"".join(want), ci


def test_c4_shape_decode_with_padded_block_in_place(engine):
    # BASELINE configs[3] shape: 64 KiB chunks, RS(10,4), B = 6554, padlen 4; block 9 (the
    # short, padded one) is PRESENT and read in place; four other data blocks erased
    nch, n, k, m = 2048, 65536, 10, 14
    src = _dev(nch * n, seed=77)
    sizes = [n] * nch
    par = _encode(engine, sizes, k, m, src)
    _check_sample(src.cpu().numpy(), par.cpu().numpy(), sizes, k, m, [0, 1, 1000, nch - 1])
    keep = [1, 3, 4, 6, 8, 9, 10, 11, 12, 13]  # erased 0, 2, 5, 7
    d, sn, offs, avail, total = _dec_inputs(sizes, k, m, [keep] * nch, src.data_ptr(), par.data_ptr())
    out = torch.empty(total, dtype=torch.uint8, device="cuda")
    engine.decode_batch(d, sn, offs, 0, out, block_avail=avail)
    assert torch.equal(out, src)


def test_c5_mixed_decode_with_padded_block_in_place(engine):
    # BASELINE configs[4] shape at reduced total: log-uniform 4 KiB..4 MiB, RS(8,3); every chunk
    # keeps block 7 in place and loses a random set of the others
    rng = np.random.default_rng(5)
    sizes = np.exp(rng.uniform(np.log(4096), np.log(4 << 20), 96)).astype(int).tolist()
    k, m = 8, 11
    src = _dev(int(np.sum(sizes)), seed=55)
    par = _encode(engine, sizes, k, m, src)
    _check_sample(src.cpu().numpy(), par.cpu().numpy(), sizes, k, m, [0, 7, 95])
    r = random.Random(5)
    keeps = [sorted([7] + r.sample([s for s in range(m) if s != 7], k - 1)) for _ in sizes]
    d, sn, offs, avail, total = _dec_inputs(sizes, k, m, keeps, src.data_ptr(), par.data_ptr())
    out = torch.empty(total, dtype=torch.uint8, device="cuda")
    engine.decode_batch(d, sn, offs, 0, out, block_avail=avail)
    assert torch.equal(out, src)


def _oracle_recovered(data, k, m, keep):
    blocks = cfec.easy_encode(data, k, m)
    return b"".join(blocks[s] for s in range(k) if s not in keep)


@pytest.mark.parametrize("k,m", [(1, 2), (2, 3), (3, 5), (4, 6), (5, 7), (8, 11), (10, 14), (16, 24), (16, 40), (32, 48)])
def test_recover_only_vs_oracle_device(k, m):
    """The copy-free decodes: k <= 4 through the small-batch kernel variant (api.cpp dec_small_kb,
    4-slot batches), wider k through the 16-slot batches."""
    from storb_amd.engine import Engine

    engine = Engine(0)
    rng = random.Random(1000 + k * m)
    sizes = [n for n in (k * k, 4096 * k - 3, 65536, 65536 + 9, 6554 * k - 1, 300007)
             if -(-n // k) * (k - 1) <= n]
    keeps = []
    for i, _ in enumerate(sizes):
        if i == 0:
            keeps.append(list(range(k)))  # e = 0: writes nothing
        elif i == 1:
            keeps.append(sorted(rng.sample(range(m), k)))
        else:  # block k-1 (padded) kept in place on odd chunks, lost on even ones
            others = [s for s in range(m) if s != k - 1]
            keeps.append(sorted(rng.sample(others, k - 1) + [k - 1]) if i % 2 else sorted(rng.sample(others, k)))
    host = [rng.randbytes(n) for n in sizes]
    src = torch.frombuffer(bytearray(b"".join(host)), dtype=torch.uint8).to("cuda")
    par = _encode(engine, sizes, k, m, src)
    d, sn, offs, avail, total = _dec_inputs(sizes, k, m, keeps, src.data_ptr(), par.data_ptr(), recover=True)
    out = torch.full((max(total, 1),), 0xA5, dtype=torch.uint8, device="cuda")
    engine.decode_batch(d, sn, offs, 0, out, block_avail=avail, recover_only=True)
    want = b"".join(_oracle_recovered(h, k, m, kp) for h, kp in zip(host, keeps))
    assert len(want) == total
    assert out.cpu().numpy()[:total].tobytes() == want
    engine.close()


def test_recover_only_c3_full_size(engine):
    # 1024 x 1 MiB RS(4,2), data shards {1,3} erased: recover-only writes e*B = 512 KiB per chunk
    nch, n, k, m = 1024, 1 << 20, 4, 6
    src = _dev(nch * n, seed=8)
    sizes = [n] * nch
    par = _encode(engine, sizes, k, m, src)
    d, sn, offs, avail, total = _dec_inputs(sizes, k, m, [[0, 2, 4, 5]] * nch, src.data_ptr(), par.data_ptr(),
                                            recover=True)
    out = torch.empty(total, dtype=torch.uint8, device="cuda")
    engine.decode_batch(d, sn, offs, 0, out, recover_only=True)
    B = n // k
    got = out.view(nch, 2, B)
    s = src.view(nch, k, B)
    assert torch.equal(got[:, 0], s[:, 1]) and torch.equal(got[:, 1], s[:, 3])


def test_host_paths_with_avail_and_recover():
    """Pageable small buffers (staged: zero-filled past avail) and pinned buffers (zero-copy),
    reassemble and recover-only, with block k-1 read in place."""
    from storb_amd.engine import Engine

    eng = Engine(0)
    try:
        rng = np.random.default_rng(9)
        k, m = 10, 14
        sizes = [65536, 65536 + 3, 40000, 6554 * 10 - 9]
        total = sum(sizes)
        for pinned in (False, True):
            hin = eng.host_empty(total) if pinned else np.empty(total, np.uint8)
            hin[:] = rng.integers(0, 256, total, dtype=np.uint8)
            szs, B, in_off, par_off = _layout(sizes, k, m)
            d = np.zeros(len(sizes), dtype=ENC_DTYPE)
            d["in_off"], d["n"], d["parity_off"], d["parity_stride"] = in_off, szs, par_off, B
            d["k"], d["m"] = k, m
            npar = int(np.sum(B)) * (m - k)
            hpar = eng.host_empty(npar) if pinned else np.empty(npar, np.uint8)
            eng.encode_batch(d, hin, hpar, host=True)
            keeps = [[1, 2, 3, 5, 6, 8, 9, 11, 12, 13]] * len(sizes)  # 9 in place; 0, 4, 7 lost
            for recover in (False, True):
                dd, sn, offs, avail, tot = _dec_inputs(sizes, k, m, keeps, hin.ctypes.data, hpar.ctypes.data,
                                                       recover=recover)
                out = eng.host_empty(tot) if pinned else np.empty(tot, np.uint8)
                out[:] = 0x5A
                eng.decode_batch(dd, sn, offs, 0, out, block_avail=avail, recover_only=recover, host=True)
                if recover:
                    want = b"".join(_oracle_recovered(hin[int(o):int(o) + int(n)].tobytes(), k, m, kp)
                                    for o, n, kp in zip(in_off, szs, keeps))
                    assert out.tobytes() == want, (pinned, recover)
                else:
                    assert np.array_equal(out, hin), (pinned, recover)
        z, r, s = eng.host_paths()
        assert z >= 3 and s >= 3, (z, r, s)  # pinned calls zero-copy, small pageable ones staged
    finally:
        eng.close()


def test_avail_is_honoured_not_read_past():
    """Bytes past a block's avail read as zero: a block whose tail holds garbage decodes as if
    that tail were zero (the contract that lets a short in-place block be used)."""
    from storb_amd.engine import get_engine

    eng = get_engine(0)
    k, m, n = 4, 6, 4 * 1000 - 3  # B = 1000, padlen 3: block 3 has 997 real bytes
    data = random.Random(3).randbytes(n)
    blocks = cfec.easy_encode(data, k, m)
    B = len(blocks[0])
    keep = [0, 3, 4, 5]  # blocks 1, 2 recovered; block 3 given with garbage in its pad
    dirty3 = blocks[3][:B - 3] + b"\xff\xfe\xfd"
    buf = np.frombuffer(b"".join([blocks[0], dirty3, blocks[4], blocks[5]]), np.uint8).copy()
    dev = torch.from_numpy(buf).to("cuda")
    dd = np.zeros(1, dtype=DEC_DTYPE)
    dd["B"], dd["padlen"], dd["k"], dd["m"], dd["slot0"], dd["out_off"] = B, 3, k, m, 0, 0
    sn = np.array(keep, np.int32)
    offs = np.array([0, B, 2 * B, 3 * B], np.uint64) + dev.data_ptr()
    out = torch.empty(n, dtype=torch.uint8, device="cuda")
    eng.decode_batch(dd, sn, offs, 0, out, block_avail=np.array([B, B - 3, B, B], np.uint64))
    assert out.cpu().numpy().tobytes() == data


def test_pure_reassembly_shapes(engine):
    """Decodes with nothing to recover (every primary present, parity ignored: the R = 0
    kernel) over tiny chunks (tail items), ragged ends with block k-1 short and read in place,
    wide k (the W instantiation), and mixed with recovering chunks in one batch; the output is
    the source bytes."""
    rng = random.Random(7)
    for k, m in [(1, 2), (2, 3), (4, 6), (10, 14), (32, 48)]:
        sizes = [1, 5, 16 * k - 3, 4096 * k, 65536, 1 << 20, 3 * 65536 + 7] + [rng.randrange(1, 200000) for _ in range(9)]
        # zfec needs a non-empty last block: n > (k - 1) * ceil(n / k)
        sizes = [s for s in sizes if s > (k - 1) * -(-s // k)]
        total = sum(sizes)
        src = _dev(total, 100 + k)
        par = _encode(engine, sizes, k, m, src)
        # every other chunk keeps its primaries (pure reassembly); the rest lose block 0
        keeps = [list(range(k)) if i % 2 == 0 else [s for s in range(1, m)][:k] for i in range(len(sizes))]
        d, sn, offs, avail, nout = _dec_inputs(sizes, k, m, keeps, src.data_ptr(), par.data_ptr())
        out = torch.zeros(nout, dtype=torch.uint8, device="cuda")
        engine.decode_batch(d, sn, offs, 0, out, block_avail=avail)
        assert torch.equal(out, src), (k, m)
        keeps = [list(range(k))] * len(sizes)  # all chunks pure reassembly
        d, sn, offs, avail, nout = _dec_inputs(sizes, k, m, keeps, src.data_ptr(), par.data_ptr())
        out.zero_()
        engine.decode_batch(d, sn, offs, 0, out, block_avail=avail)
        assert torch.equal(out, src), (k, m, "all e=0")


def test_fuzz_mixed_shapes_erasures_one_batch(engine):
    """Randomized: 160 chunks of random (k, m) (1 <= k <= 40, up to m = 2k + 3) and random
    sizes in ONE device encode and ONE device decode, each chunk with a random set of k
    surviving blocks in random order (parity-only survivors included), block k-1 read in place
    when it survives; then the recover-only decode of the same batch.  Parity and every
    recovered row against the oracle (oracle/fec_oracle.c) on a sample, reassembly against the
    source bytes everywhere."""
    rng = random.Random(2024)
    shapes, sizes = [], []
    while len(shapes) < 160:
        k = rng.choice([1, 2, 3, 4, 5, 8, 10, 13, 16, 17, 24, 32, 40])
        m = min(256, k + rng.randrange(1, k + 4))
        n = rng.randrange(1, 150000)
        if n <= (k - 1) * -(-n // k):  # zfec: the last block must be non-empty
            continue
        shapes.append((k, m))
        sizes.append(n)
    total = sum(sizes)
    src = _dev(total, 77)
    # encode: one batch of mixed shapes (per-chunk layout as _layout, but per-chunk k, m)
    B = [-(-n // k) for n, (k, m) in zip(sizes, shapes)]
    in_off = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
    pcount = [b * (m - k) for b, (k, m) in zip(B, shapes)]
    par_off = np.concatenate([[0], np.cumsum(pcount)[:-1]]).astype(np.uint64)
    ed = np.zeros(len(sizes), dtype=ENC_DTYPE)
    ed["in_off"], ed["n"], ed["parity_off"], ed["parity_stride"] = in_off, sizes, par_off, B
    ed["k"] = [k for k, _ in shapes]
    ed["m"] = [m for _, m in shapes]
    par = torch.empty(max(1, int(sum(pcount))), dtype=torch.uint8, device="cuda")
    engine.encode_batch(ed, src, par)
    src_h, par_h = src.cpu().numpy(), par.cpu().numpy()
    for i in rng.sample(range(len(sizes)), 24):
        k, m = shapes[i]
        data = src_h[int(in_off[i]):int(in_off[i]) + sizes[i]].tobytes()
        want = b"".join(cfec.easy_encode(data, k, m)[k:])
        assert par_h[int(par_off[i]):int(par_off[i]) + pcount[i]].tobytes() == want, (i, k, m, sizes[i])
    # decode: random survivors per chunk, every slot read in place
    keeps = [rng.sample(range(m), k) for (k, m) in shapes]
    nslots = sum(k for k, _ in shapes)
    for recover in (False, True):
        dd = np.zeros(len(sizes), dtype=DEC_DTYPE)
        sn = np.zeros(nslots, np.int32)
        offs = np.zeros(nslots, np.uint64)
        avail = np.zeros(nslots, np.uint64)
        o, slot, lost = 0, 0, []
        for i, ((k, m), keep) in enumerate(zip(shapes, keeps)):
            b = B[i]
            dd["out_off"][i], dd["B"][i], dd["padlen"][i] = o, b, b * k - sizes[i]
            dd["k"][i], dd["m"][i], dd["slot0"][i] = k, m, slot
            miss = sorted(s for s in range(k) if s not in keep)
            lost.append(miss)
            o += len(miss) * b if recover else sizes[i]
            for s in keep:
                sn[slot] = s
                if s < k:
                    offs[slot] = src.data_ptr() + int(in_off[i]) + s * b
                    avail[slot] = sizes[i] - s * b if s == k - 1 else b
                else:
                    offs[slot] = par.data_ptr() + int(par_off[i]) + (s - k) * b
                    avail[slot] = b
                slot += 1
        out = torch.zeros(max(o, 1), dtype=torch.uint8, device="cuda")
        engine.decode_batch(dd, sn, offs, 0, out, block_avail=avail, recover_only=recover)
        if not recover:
            assert torch.equal(out[:o], src)
            continue
        out_h = out.cpu().numpy()
        for i, miss in enumerate(lost):
            k, m = shapes[i]
            data = src_h[int(in_off[i]):int(in_off[i]) + sizes[i]].tobytes()
            blocks = cfec.easy_encode(data, k, m)
            base = int(dd["out_off"][i])
            for j, r in enumerate(miss):
                got = out_h[base + j * B[i]:base + (j + 1) * B[i]].tobytes()
                assert got == blocks[r], (i, k, m, r)


@pytest.mark.parametrize("mode", ["staged", "locked", "pinned"])
def test_fuzz_host_reassembly_join(mode):
    """Host-buffer reassembly (the host copies the present primaries, the GPU returns only the
    recovered rows) on each host path, randomized: mixed (k, m), random survivors in random
    order (parity-only ones included), block k-1 read in place with its short avail; the output
    buffer is pre-filled so every byte must be written; against the source bytes."""
    from storb_amd.engine import Engine

    # staged: never page-lock, stage through the slabs
    eng = Engine(0, options={"SEC_REGISTER_MIN": 0} if mode == "staged" else {})
    try:
        rng = random.Random(77)
        shapes, sizes = [], []
        while len(shapes) < 60:
            k = rng.choice([1, 2, 4, 5, 8, 10, 16, 24])
            m = min(256, k + rng.randrange(1, k + 3))
            n = rng.randrange(1, 400000)
            if n <= (k - 1) * -(-n // k):
                continue
            shapes.append((k, m))
            sizes.append(n)
        total = sum(sizes)
        B = [-(-n // k) for n, (k, m) in zip(sizes, shapes)]
        in_off = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
        pcount = [b * (m - k) for b, (k, m) in zip(B, shapes)]
        par_off = np.concatenate([[0], np.cumsum(pcount)[:-1]]).astype(np.uint64)
        alloc = (lambda n: eng.host_empty(n)) if mode == "pinned" else (lambda n: np.empty(n, np.uint8))
        hin = alloc(total)
        hin[:] = np.frombuffer(rng.randbytes(total), np.uint8)
        hpar = alloc(int(sum(pcount)))
        ed = np.zeros(len(sizes), dtype=ENC_DTYPE)
        ed["in_off"], ed["n"], ed["parity_off"], ed["parity_stride"] = in_off, sizes, par_off, B
        ed["k"] = [k for k, _ in shapes]
        ed["m"] = [m for _, m in shapes]
        eng.encode_batch(ed, hin, hpar, host=True)
        nslots = sum(k for k, _ in shapes)
        dd = np.zeros(len(sizes), dtype=DEC_DTYPE)
        sn = np.zeros(nslots, np.int32)
        offs = np.zeros(nslots, np.uint64)
        avail = np.zeros(nslots, np.uint64)
        slot = 0
        for i, (k, m) in enumerate(shapes):
            b = B[i]
            dd["out_off"][i], dd["B"][i], dd["padlen"][i] = int(in_off[i]), b, b * k - sizes[i]
            dd["k"][i], dd["m"][i], dd["slot0"][i] = k, m, slot
            for s in rng.sample(range(m), k):
                sn[slot] = s
                if s < k:
                    offs[slot] = hin.ctypes.data + int(in_off[i]) + s * b
                    avail[slot] = sizes[i] - s * b if s == k - 1 else b
                else:
                    offs[slot] = hpar.ctypes.data + int(par_off[i]) + (s - k) * b
                    avail[slot] = b
                slot += 1
        out = alloc(total)
        out[:] = 0xA5
        eng.decode_batch(dd, sn, offs, 0, out, block_avail=avail, host=True)
        assert np.array_equal(out, hin), mode
        z, r, st = eng.host_paths()  # (zero-copy pinned, locked per call, staged) calls
        assert {"pinned": z, "locked": r, "staged": st}[mode] >= 2, (mode, z, r, st)
    finally:
        eng.close()


@pytest.mark.parametrize("B,nch", [(256 << 10, 6), (1 << 20, 8)])
@pytest.mark.parametrize("staged_flag", [False, True])
def test_scattered_blocks_read_back_from_out(staged_flag, B, nch):
    """A host reassembly whose blocks are too scattered to page-lock (256 KiB blocks 5 MiB apart:
    the library stages them) but whose output is one large range (api.cpp join_staged): the
    present primaries are copied into `out` first and the rows-only call reads them from there
    with `out` locked (host path counts: one locked call, nothing staged).  With staged=True
    nothing may be locked: the rows-only call stages the caller's blocks while the copies run.
    Chunks with every primary present, one lost, and block k-1 lost or short in place; 12 MiB and
    64 MiB of output (the second read back in groups of chunks when SEC_JOIN_GROUPS > 1, still
    one host path per call)."""
    from storb_amd.engine import Engine

    eng = Engine(0)
    try:
        rng = random.Random(5)
        k, m, gap = 8, 12, 5 << 20
        sizes = [k * B - rng.randrange(0, 3) for _ in range(nch)]
        arena = np.empty(nch * k * gap + B, np.uint8)  # untouched pages cost nothing
        src = [rng.randbytes(n) for n in sizes]
        place = iter(range(0, arena.size - B + 1, gap))
        dd = np.zeros(nch, dtype=DEC_DTYPE)
        sn = np.zeros(nch * k, np.int32)
        offs = np.zeros(nch * k, np.uint64)
        avail = np.zeros(nch * k, np.uint64)
        lost_sets = [(), (3,), (k - 1,), (0, 5), (), (2, k - 1), (1,), (0,)][:nch]
        for i, (n, data) in enumerate(zip(sizes, src)):
            blocks = cfec.easy_encode(data, k, m)
            dd["out_off"][i], dd["B"][i], dd["padlen"][i] = i * k * B, B, k * B - n
            dd["k"][i], dd["m"][i], dd["slot0"][i] = k, m, i * k
            keep = [j for j in range(m) if j not in lost_sets[i]][:k]
            rng.shuffle(keep)
            for q, j in enumerate(keep):
                o = next(place)
                av = n - (k - 1) * B if j == k - 1 else B  # block k-1 short in place
                arena[o:o + av] = np.frombuffer(blocks[j][:av], np.uint8)
                sn[i * k + q], offs[i * k + q], avail[i * k + q] = j, arena.ctypes.data + o, av
        out = np.full(nch * k * B, 0xA5, np.uint8)
        z0, r0, s0 = eng.host_paths()
        eng.decode_batch(dd, sn, offs, 0, out, block_avail=avail, host=True, staged=staged_flag)
        z1, r1, s1 = eng.host_paths()
        for i, (n, data) in enumerate(zip(sizes, src)):
            assert out[i * k * B:i * k * B + n].tobytes() == data, i
        assert (z1 - z0, r1 - r0, s1 - s0) == ((0, 0, 1) if staged_flag else (0, 1, 0))
    finally:
        eng.close()


@pytest.mark.parametrize("opts", [{}, {"SEC_HOST_JOIN": 0}])
def test_small_chunks_reassembled(opts):
    """Chunks of at most 64 KiB with B <= 8192 and e <= 8 (the shapes round 4's LDS reassembly
    kernel took; it lost its A/B and is archived) through the row-stream tiles: against the source
    bytes and the oracle's decode, B of every residue mod 16, e = 0 .. 8, block k-1 in place with
    its short avail, device buffers; with SEC_HOST_JOIN = 0 the same blocks from host buffers
    (staged, the kernels write every byte)."""
    from storb_amd.engine import Engine

    eng = Engine(0, options=opts)
    try:
        rng = random.Random(404)
        shapes, sizes = [], []
        while len(shapes) < 96:
            k = rng.choice([1, 2, 4, 8, 10, 13, 16])
            m = k + rng.randrange(1, 9)
            n = rng.choice([65536, 16 * k + 3, rng.randrange(16 * k, 65537)])
            B = -(-n // k)
            if n <= (k - 1) * B or B > 8192 or B < 16:
                continue
            shapes.append((k, m))
            sizes.append(n)
        src_h = np.random.default_rng(404).integers(0, 256, sum(sizes), dtype=np.uint8)
        in_off = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
        host = "SEC_HOST_JOIN" in opts
        blocks_all, keeps = [], []
        for (k, m), n, o in zip(shapes, sizes, in_off):
            blocks_all.append(cfec.easy_encode(src_h[int(o):int(o) + n].tobytes(), k, m))
            keeps.append(rng.sample(range(m), k))
        par_h = np.frombuffer(b"".join(b"".join(bl[k:]) for bl, (k, m) in zip(blocks_all, shapes)), np.uint8)
        src, par = torch.from_numpy(src_h).cuda(), torch.from_numpy(par_h.copy()).cuda()
        nslots = sum(k for k, _ in shapes)
        dd = np.zeros(len(sizes), dtype=DEC_DTYPE)
        sn, offs, avail = np.zeros(nslots, np.int32), np.zeros(nslots, np.uint64), np.zeros(nslots, np.uint64)
        hostbuf, want, o, slot, po = bytearray(), [], 0, 0, 0
        for i, ((k, m), n, keep) in enumerate(zip(shapes, sizes, keeps)):
            b = -(-n // k)
            dd[i] = (o, b, b * k - n, slot, k, m)
            want.append(cfec.easy_decode([blocks_all[i][s] for s in keep], keep, b * k - n, k, m))
            o += n
            for s in keep:
                sn[slot] = s
                if host:
                    offs[slot], avail[slot] = len(hostbuf), b
                    hostbuf += blocks_all[i][s]
                elif s < k:
                    offs[slot] = src.data_ptr() + int(in_off[i]) + s * b
                    avail[slot] = n - s * b if s == k - 1 else b
                else:
                    offs[slot], avail[slot] = par.data_ptr() + po + (s - k) * b, b
                slot += 1
            po += (m - k) * b
        assert b"".join(want) == src_h.tobytes()  # the oracle's decode is the chunk
        if host:
            got = np.zeros(o, np.uint8)
            eng.decode_batch(dd, sn, offs, np.frombuffer(bytes(hostbuf), np.uint8).copy(), got, host=True)
            assert got.tobytes() == src_h.tobytes()
        else:
            out = torch.zeros(o, dtype=torch.uint8, device="cuda")
            eng.decode_batch(dd, sn, offs, 0, out, block_avail=avail)
            assert torch.equal(out, src)
    finally:
        eng.close()

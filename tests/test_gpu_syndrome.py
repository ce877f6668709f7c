"""GPU parity of the syndrome decode (wide decodes with many lost data blocks).

A chunk that lost e data blocks and holds e parity rows instead is decoded in two phases
(kernels_bs.hip sec_syndrome_bs_kernel: bit-sliced syndromes of the present parity rows, scaled
by the Cauchy solve's w, and the copies of the present primaries; then sec_solve_bs_kernel
applies the transposed parity matrix and the scaling z, gf_host.hpp cauchy_scales).  The result
must be zfec's fec_decode bytes (/root/reference/storb/util/piece.py:196-197 via easyfec).  Every
chunk's blocks are made by the CPU oracle (oracle/fec_oracle.c), and the HIP output is compared
with the oracle's own decode of exactly the blocks the kernels were given, for:

* the policy's wide shapes zfec(16,24), (32,48), (64,96) and the kernel's other shapes (C4's
  (10,14), (8,12), C5's (8,11)), e = 1 .. p lost, parity rows from one or both row groups;
* B from 16 bytes (one partial wave) to several tiles, unaligned B, padded chunks with block
  k-1 present and read in place (avail = B - padlen) or lost;
* reassemble and recover-only; device buffers, staged host buffers and pinned host buffers;
* syndrome chunks mixed with direct-path chunks and other shapes in one call;
* the path actually taken (sec_ctx_decode_paths / _methods) under SEC_SYN=1 (forced) and the
  default cost rule, with SEC_SYN=0 (the direct decode) giving the same bytes;
* zfec(64,96) with e <= 16 present parity rows in BOTH groups: the two kernels, phase 1 in
  two-wave workgroups (sec_syndrome_bs_pair_kernel).  (Round 4's one-kernel wave pair and the
  (span, row group) tile forms of both phases lost their A/Bs and are archived.)
"""

import random

import numpy as np
import pytest

from oracle import cfec

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from storb_amd._lib import DEC_DTYPE, ENC_DTYPE  # noqa: E402

SHAPES = [(16, 24), (32, 48), (64, 96), (10, 14), (8, 12), (8, 11)]


def _engine(syn=None, fused=None):
    """A fresh context with the syndrome options forced (None: the library default).  fused = 0:
    not the one-wave kernel, i.e. the two kernels, phase 2 of k >= 32 with each span's syndromes
    staged in LDS (sec_solve_bs_lds_kernel) and, for parity rows in both groups of (64,96),
    phase 1 in two-wave workgroups (sec_syndrome_bs_pair_kernel)."""
    from storb_amd.engine import Engine

    opts = {}
    if syn is not None:
        opts["SEC_SYN"] = int(syn)
    if fused is not None:
        opts["SEC_SYN_FUSED"] = int(fused)
    return Engine(0, options=opts)


def _cases(rng, k, m, sizes):
    """(size, keep) pairs: for each size several erasure patterns; keep = the k block numbers
    the decoder gets (lost data blocks replaced by parity rows)."""
    p = m - k
    out = []
    for n in sizes:
        for e in sorted({1, min(2, p), p // 2 or 1, p, rng.randint(1, p)}):
            lost = sorted(rng.sample(range(k), e))
            if p > 16 and e <= 16 and rng.random() < 0.5:  # (64,96): rows of one 16-row group
                g = rng.randrange(p // 16)
                par = sorted(rng.sample(range(k + 16 * g, k + 16 * g + 16), e))
            else:
                par = sorted(rng.sample(range(k, m), e))
            keep = [j for j in range(k) if j not in lost] + par
            rng.shuffle(keep)
            out.append((n, keep))
    return out


def _run(eng, k, m, cases, recover=False, host=None):
    """Decode chunks from ORACLE-made blocks and compare the HIP output with the oracle's decode
    of the same blocks (the syndrome kernels share gf_const.hpp with the
    encode, so GPU-made parity could hide a matrix error common to both).

    Every chunk's m blocks come from oracle/fec_oracle.c (cfec.easy_encode of seeded bytes); the
    data blocks are read in place from the source buffer (block k-1 short by padlen, avail =
    B - padlen) and the parity blocks from a buffer of the oracle's parity rows.  The expected
    bytes are cfec.easy_decode of exactly the kept blocks: the reassembled chunk, or (recover)
    the lost primaries fec_decode recovers, B bytes each in block order."""
    sizes = np.array([n for n, _ in cases], dtype=np.uint64)
    B = (sizes + k - 1) // k
    in_off = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
    par_off = np.concatenate([[0], np.cumsum(B * (m - k))[:-1]]).astype(np.uint64)
    total = int(sizes.sum())
    rng = np.random.default_rng(int(total) % 100003 + k)
    src_h = rng.integers(0, 256, total, dtype=np.uint8)
    par_h = np.zeros(max(int((B * (m - k)).sum()), 1), dtype=np.uint8)
    oracle_blocks = []
    for i, (n, _) in enumerate(cases):
        blocks = cfec.easy_encode(src_h[int(in_off[i]):int(in_off[i]) + n].tobytes(), k, m)
        oracle_blocks.append(blocks)
        b = int(B[i])
        par_h[int(par_off[i]):int(par_off[i]) + (m - k) * b] = np.frombuffer(b"".join(blocks[k:]), np.uint8)
    src = torch.from_numpy(src_h).cuda()
    par = torch.from_numpy(par_h).cuda()
    n_ch = len(cases)
    d = np.zeros(n_ch, dtype=DEC_DTYPE)
    d["B"], d["padlen"], d["k"], d["m"] = B, B * k - sizes, k, m
    d["slot0"] = np.arange(n_ch, dtype=np.uint64) * k
    sn = np.zeros(n_ch * k, np.int32)
    offs = np.zeros(n_ch * k, np.uint64)
    avail = np.zeros(n_ch * k, np.uint64)
    out_off, o, want = np.zeros(n_ch, np.uint64), 0, []
    hostbuf = bytearray()
    for i, (n, keep) in enumerate(cases):
        b = int(B[i])
        out_off[i] = o
        blocks = oracle_blocks[i]
        lost = [j for j in range(k) if j not in keep]
        if recover:
            full = cfec.easy_decode([blocks[s] for s in keep], keep, 0, k, m)
            want.append(b"".join(full[j * b:(j + 1) * b] for j in lost))
        else:
            want.append(cfec.easy_decode([blocks[s] for s in keep], keep, k * b - n, k, m))
        o += len(want[-1])
        for q, s in enumerate(keep):
            sn[i * k + q] = s
            if s < k:
                a, av = int(in_off[i]) + s * b, min(b, n - s * b)
                base = src.data_ptr()
            else:
                a, av = int(par_off[i]) + (s - k) * b, b
                base = par.data_ptr()
            if host is None:
                offs[i * k + q], avail[i * k + q] = base + a, av
            else:
                offs[i * k + q], avail[i * k + q] = len(hostbuf), b
                hostbuf += blocks[s]
    d["out_off"] = out_off
    if host is None:
        out = torch.zeros(max(o, 1), dtype=torch.uint8, device="cuda")
        eng.decode_batch(d, sn, offs, 0, out, block_avail=avail, recover_only=recover)
        got = out.cpu().numpy()
    else:
        if host == "pinned":
            hb = eng.host_empty(len(hostbuf))
            hb[:] = np.frombuffer(hostbuf, np.uint8)
            got = eng.host_empty(max(o, 1))
        else:
            hb = np.frombuffer(hostbuf, np.uint8).copy()
            got = np.zeros(max(o, 1), np.uint8)
        eng.decode_batch(d, sn, offs, hb, got, recover_only=recover, host=True)
    pos = 0
    for i, w in enumerate(want):
        assert got[pos:pos + len(w)].tobytes() == w, (k, m, cases[i][0], cases[i][1], recover, host)
        if not recover:  # and the oracle's decode is the source chunk (round trip)
            assert w == src_h[int(in_off[i]):int(in_off[i]) + cases[i][0]].tobytes()
        pos += len(w)


@pytest.mark.parametrize("k,m", SHAPES)
@pytest.mark.parametrize("recover", [False, True])
@pytest.mark.parametrize("fused", [None, 0])
def test_syndrome_decode_forced_device(k, m, recover, fused):
    """SEC_SYN=1: every chunk on the syndrome path (the one-wave kernel where it applies, or with
    SEC_SYN_FUSED=0 always the two kernels with the syndromes in HBM; both phase-2 layouts)."""
    rng = random.Random(k * 1000 + m + recover)
    sizes = [16 * k, 17 * k - 3, 2048 * k + 5 * k, 6554 * k - 4 if k == 10 else 4099 * k - 1, 65536 * k,
             rng.randrange(20000, 300000)]
    sizes = [n for n in sizes if -(-n // k) * (k - 1) < n]  # easyfec: the last block not empty
    eng = _engine(1, fused)
    try:
        cases = _cases(rng, k, m, sizes)
        _run(eng, k, m, cases, recover=recover)
        syn, direct = eng.decode_paths()
        assert syn == len(cases) and direct == 0, (syn, direct)
    finally:
        eng.close()


@pytest.mark.parametrize("k,m", [(32, 48), (64, 96), (16, 24)])
@pytest.mark.parametrize("host", ["staged", "pinned"])
def test_syndrome_decode_forced_host(k, m, host):
    rng = random.Random(7 * k + (host == "pinned"))
    eng = _engine(1)
    try:
        cases = _cases(rng, k, m, [4096 * k + 17, 1 << 20, 3 * k * 1024 - 5])
        _run(eng, k, m, cases, host=host)
        _run(eng, k, m, cases, host=host, recover=True)
        assert eng.decode_paths()[0] == 2 * len(cases)
    finally:
        eng.close()


def test_syndrome_default_rule_and_off_give_same_bytes():
    """The default choice (api.cpp syn_choice's estimate) on the verdict's case: zfec(64,96) with
    16 data blocks lost (parity rows of one group) takes the syndrome path, one lost block the
    direct path; SEC_SYN=0 decodes the same chunks directly, to the same bytes."""
    many = [(1 << 20, list(range(16, 64)) + list(range(64, 80)))]  # 16 lost, parity group 0
    one = [(1 << 20, list(range(1, 64)) + [95])]
    for syn_env, want_many, want_one in ((None, (1, 0), (0, 1)), (0, (0, 1), (0, 1))):
        eng = _engine(syn_env)
        try:
            _run(eng, 64, 96, many)
            assert eng.decode_paths() == want_many, (syn_env, eng.decode_paths())
            _run(eng, 64, 96, one)
            got = eng.decode_paths()
            assert (got[0] - want_many[0], got[1] - want_many[1]) == want_one, (syn_env, got)
        finally:
            eng.close()


def test_syndrome_mixed_batch_with_direct_chunks():
    """One call: syndrome chunks of two shapes and direct chunks (RS(4,2), and a shape without a
    bit-sliced kernel), device-resident, reassembled; every chunk against its source."""
    from storb_amd.engine import Engine

    eng = Engine(0)
    try:
        rng = random.Random(5)
        specs = []  # (k, m, n, keep)
        for _ in range(6):
            specs.append((64, 96, rng.randrange(70000, 400000), list(range(20, 64)) + list(range(70, 90))))
            specs.append((32, 48, rng.randrange(70000, 400000), list(range(12, 32)) + list(range(36, 48))))
            specs.append((4, 6, rng.randrange(4096, 100000), [0, 2, 4, 5]))
            specs.append((5, 9, rng.randrange(4096, 100000), [1, 2, 5, 7, 8]))
        sizes = np.array([n for _, _, n, _ in specs], np.uint64)
        total = int(sizes.sum())
        src = torch.randint(0, 256, (total,), dtype=torch.uint8, device="cuda")
        in_off = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
        Bs = [-(-int(n) // k) for k, m, n, _ in specs]
        par_sizes = [(m - k) * b for (k, m, _, _), b in zip(specs, Bs)]
        par_off = np.concatenate([[0], np.cumsum(par_sizes)[:-1]]).astype(np.uint64)
        par = torch.empty(int(sum(par_sizes)), dtype=torch.uint8, device="cuda")
        ed = np.zeros(len(specs), dtype=ENC_DTYPE)
        for i, ((k, m, n, _), b) in enumerate(zip(specs, Bs)):
            ed[i] = (in_off[i], n, par_off[i], b, k, m)
        eng.encode_batch(ed, src, par)
        d = np.zeros(len(specs), dtype=DEC_DTYPE)
        sn, offs, av, slot = [], [], [], 0
        for i, ((k, m, n, keep), b) in enumerate(zip(specs, Bs)):
            d[i] = (in_off[i], b, b * k - n, slot, k, m)
            for s in keep:
                sn.append(s)
                if s < k:
                    offs.append(src.data_ptr() + int(in_off[i]) + s * b)
                    av.append(min(b, n - s * b))
                else:
                    offs.append(par.data_ptr() + int(par_off[i]) + (s - k) * b)
                    av.append(b)
            slot += k
        out = torch.zeros_like(src)
        eng.decode_batch(d, np.array(sn, np.int32), np.array(offs, np.uint64), 0, out,
                         block_avail=np.array(av, np.uint64))
        assert torch.equal(out, src)
        syn, direct = eng.decode_paths()
        # the (32,48) chunks (12 lost, parity rows of one group) take the one-wave syndrome kernel;
        # the (64,96) ones (20 lost, parity rows of both groups) stay direct or take two kernels
        assert syn >= 6 and syn + direct == 24, (syn, direct)
    finally:
        eng.close()


@pytest.mark.parametrize("k,m,e,fused", [(64, 96, 32, 0), (64, 96, 24, None), (64, 96, 16, None), (64, 96, 9, None),
                                         (64, 96, 16, 0), (32, 48, 12, None), (32, 48, 16, 0), (16, 24, 6, None)])
def test_syndrome_random_patterns(k, m, e, fused):
    """Random lost data blocks and random present parity rows (both parity groups of (64,96): the
    two kernels), forced onto the syndrome path, reassembled and recover-only, against the
    sources."""
    rng = random.Random(1000 * k + e)
    eng = _engine(1, fused)
    try:
        cases = []
        for n in (rng.randrange(4096 * k, 40000 * k), 1 << 20, 64 * k - 3):
            lost = rng.sample(range(k), e)
            keep = [j for j in range(k) if j not in lost] + rng.sample(range(k, m), e)
            rng.shuffle(keep)
            cases.append((n, keep))
        _run(eng, k, m, cases)
        _run(eng, k, m, cases, recover=True)
        assert eng.decode_paths() == (2 * len(cases), 0)
    finally:
        eng.close()


@pytest.mark.parametrize("lanes", [64, 128])
def test_syndrome_lanes_option_and_replan(lanes):
    """the syndrome kernels' tile span follows the lane count the plan was
    built with.  Forced onto the syndrome path with SEC_BS_LANES = 64 / 128, then the same
    engine switched back to 256 lanes between calls (the option drops the cached plan): every
    call's bytes equal the oracle's."""
    rng = random.Random(lanes)
    eng = _engine(1)
    try:
        for k, m in [(32, 48), (64, 96)]:
            cases = _cases(rng, k, m, [2048 * k + 5 * k, 1 << 20])
            _run(eng, k, m, cases)
            eng.set_option("SEC_BS_LANES", lanes)
            _run(eng, k, m, cases)
            _run(eng, k, m, cases, recover=True)
            eng.set_option("SEC_BS_LANES", 256)
            _run(eng, k, m, cases, recover=True)
    finally:
        eng.close()


@pytest.mark.parametrize("recover", [False, True])
def test_syndrome_both_groups(recover):
    """SEC_SYN = 1: zfec(64,96), e = 1 .. 16 lost data blocks with present parity rows drawn from
    both 16-row groups (rows r and r + 16 both present included): the two kernels decode every
    both-group chunk (phase 1 in two-wave workgroups), the one-wave kernel the one-group chunks
    (decode_methods; the archived wave pair's count stays 0), equal to the oracle's decode."""
    k, m = 64, 96
    rng = random.Random(96 + recover)
    cases = []
    for n in (16 * k, 2048 * k + 5 * k, 4099 * k - 1, 1 << 20, rng.randrange(70000, 400000)):
        for e in (1, 2, 7, 12, 16):
            lost = sorted(rng.sample(range(k), e))
            g0 = rng.randrange(1, e) if e > 1 else 0
            par = sorted(rng.sample(range(k, k + 16), g0) + rng.sample(range(k + 16, m), e - g0))
            if e == 1:
                par = [k + 16 + rng.randrange(16)]  # one row, group 1 only: the one-wave kernel
            keep = [j for j in range(k) if j not in lost] + par
            rng.shuffle(keep)
            cases.append((n, keep))
    both = sum(1 for _, keep in cases if {(s - k) // 16 for s in keep if s >= k} == {0, 1})
    eng = _engine(1)
    try:
        _run(eng, k, m, cases, recover=recover)
        one, pair, two, direct = eng.decode_methods()
        assert pair == 0 and two == both and one == len(cases) - both, (one, pair, two, both)
    finally:
        eng.close()

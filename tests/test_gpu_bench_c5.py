"""GPU: bench.py --workload c5 (BASELINE configs[4], mixed 4 KiB-4 MiB RS(8,3) end to end from
pinned host memory) on the real engine, at a reduced job size.  c5_run round-trips every chunk
on every path itself (pinned zero-copy, device-resident, staged); here sampled chunks' parity —
both the pinned host parity and the device copy's — is also checked against the oracle
(oracle/fec_oracle.c), and the shares of a 4-way split cover the job once."""

from types import SimpleNamespace

import numpy as np
import pytest

from oracle import cfec

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.mark.parametrize("world,rank", [(1, 0), (4, 3)])
def test_bench_c5_share_against_oracle(world, rank):
    import bench
    from storb_amd.dist import partition
    from storb_amd.engine import Engine

    eng = Engine(0)
    try:
        ctx = SimpleNamespace(rank=rank, world=world, dmod=None, local=0, device="cuda:0",
                              sync=torch.cuda.synchronize, eng=eng, backend=None)
        total = 96 << 20
        r = bench.c5_run(ctx, steps=1, warmup=1, total=total, keep=True)
        sizes_all = bench.c5_sizes(total)
        lo, hi = partition(sizes_all, world)[rank]
        assert (r["lo"], r["hi"]) == (lo, hi) and r["sizes"] == sizes_all[lo:hi]
        k, m = bench.C5_K, bench.C5_M
        sizes = r["sizes"]
        in_off = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(int)
        Bs = [-(-n // k) for n in sizes]
        par_off = np.concatenate([[0], np.cumsum([b * (m - k) for b in Bs])[:-1]]).astype(int)
        dpar = r["par"].cpu().numpy()
        for ci in sorted({0, 1, len(sizes) // 2, len(sizes) - 1}):
            n, B = sizes[ci], Bs[ci]
            data = r["host"][in_off[ci]:in_off[ci] + n].tobytes()
            want = b"".join(cfec.easy_encode(data, k, m)[k:])
            assert r["hpar"][par_off[ci]:par_off[ci] + (m - k) * B].tobytes() == want, ci
            assert dpar[par_off[ci]:par_off[ci] + (m - k) * B].tobytes() == want, ci
        assert r["enc_launches"] >= 5 and r["dec_launches"] >= 5
        assert r["staged_encode_gibs"] > 0 and r["staged_decode_gibs"] > 0
    finally:
        eng.close()

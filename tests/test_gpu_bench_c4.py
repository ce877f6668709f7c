"""GPU: bench.py --workload c4 (BASELINE configs[3], 65536 x 64 KiB RS(10,4) split over ranks)
at N = 1 on the real engine — one GPU's 8192-chunk share of an 8-way job and the whole 65536-chunk
job.  c4_run itself round-trips every chunk (4 data blocks erased, recovered from parity, the
padded block 9 read in place); here sampled chunks' parity is also checked against the oracle
(oracle/fec_oracle.c)."""

import numpy as np
import pytest

from oracle import cfec

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.mark.parametrize("world,rank", [(8, 0), (8, 7), (1, 0)])
def test_bench_c4_share_and_full_job(world, rank):
    import bench
    from storb_amd.engine import Engine

    eng = Engine(0)
    try:
        r = bench.c4_run(eng, None, rank, world, 0, "cuda:0", torch.cuda.synchronize, steps=2, warmup=1, keep=True)
        assert r["chunks"] == 65536 // world and r["lo"] == rank * (65536 // world)
        assert r["total_chunks"] == r["chunks"] and r["enc_launches"] == 2
        n, k, m, B, ps = bench.C4_CHUNK, bench.C4_K, bench.C4_M, r["B"], r["pstride"]
        assert B == 6554 and ps == 6656  # parity rows 128-byte aligned
        for ci in (0, 1, r["chunks"] // 2, r["chunks"] - 1):
            data = r["src"][ci * n:(ci + 1) * n].cpu().numpy().tobytes()
            par = r["par"][ci * (m - k) * ps:(ci + 1) * (m - k) * ps].cpu().numpy().reshape(m - k, ps)[:, :B]
            assert par.tobytes() == b"".join(cfec.easy_encode(data, k, m)[k:]), ci
    finally:
        eng.close()

"""CPU: the N>1 path — chunk partitioning and the measurement collectives — on gloo, world 2.

The multi-GPU design has no data-path collective (chunks are independent); what needs
coverage is that ranks split the chunk list exactly once over and that the timing reduction
takes the max (and the byte count the sum) across ranks, as bench.py does."""

import os
import random
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from oracle import cfec
from storb_amd.dist import partition


def test_partition_covers_each_chunk_once():
    rng = random.Random(0)
    for world in (1, 2, 3, 4, 8):
        for n in (0, 1, 7, 1024, 999):
            sizes = [rng.randrange(4096, 4 << 20) for _ in range(n)]
            parts = partition(sizes, world)
            assert len(parts) == world
            covered = [i for lo, hi in parts for i in range(lo, hi)]
            assert covered == list(range(n))
            if n >= 64 * world:
                loads = [sum(sizes[lo:hi]) for lo, hi in parts]
                assert max(loads) <= sum(sizes) / world + max(sizes)


def test_partition_uniform_c4():
    # BASELINE configs[3]: 65536 x 64 KiB over 8 GPUs -> 8192 chunks per GPU
    parts = partition([65536] * 65536, 8)
    assert [hi - lo for lo, hi in parts] == [8192] * 8


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from storb_amd import dist as D

    d = D.init("gloo")
    rng = np.random.default_rng(5)
    sizes = np.exp(rng.uniform(np.log(4096), np.log(1 << 20), 40)).astype(int)
    lo, hi = D.partition(sizes, world)[rank]
    # each rank "encodes" its share with the CPU checker (no GPU here) and reports bytes
    local = 0
    for i in range(lo, hi):
        data = np.random.default_rng(i).integers(0, 256, sizes[i], dtype=np.uint8).tobytes()
        blocks = cfec.easy_encode(data, 8, 11)
        assert b"".join(blocks[:8])[: len(data)] == data
        local += len(data)
    D.barrier(d)
    tot = D.sum_over_ranks(d, local)
    mx = D.max_over_ranks(d, float(rank + 1))
    q.put((rank, lo, hi, tot, mx, int(sizes.sum())))
    d.destroy_process_group()


@pytest.mark.timeout(120)
def test_gloo_world2_partition_and_reductions():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=90) for _ in procs)
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    (r0, lo0, hi0, tot0, mx0, all0), (r1, lo1, hi1, tot1, mx1, _) = res
    assert lo0 == 0 and hi0 == lo1 and hi1 == 40
    assert tot0 == tot1 == all0
    assert mx0 == mx1 == 2.0


class _StubEngine:
    """Stands in for storb_amd.engine.Engine (no GPU here): bench.c4_run's partition, timing and
    reduction path runs as on the GPU ranks, with the kernels skipped."""

    def __init__(self):
        self.encoded = []

    def encode_batch(self, descs, src, par, asynchronous=False):
        self.encoded.append(int(descs["n"].sum()) if len(descs) else 0)

    def decode_batch(self, *a, **kw):
        pass

    def sync(self):
        pass

    def set_timing(self, on):
        pass

    def collect_timing(self, kind):
        return 1.0, 1


def _c4_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import bench
    from storb_amd import dist as D

    d = D.init("gloo")
    eng = _StubEngine()
    r = bench.c4_run(eng, d, rank, world, None, "cpu", lambda: None, steps=3, warmup=1, nchunks=96, verify=False)
    q.put((rank, r["lo"], r["hi"], r["total_chunks"], r["per_rank_chunks"], r["el_max"], eng.encoded))
    d.destroy_process_group()


@pytest.mark.timeout(120)
def test_gloo_world2_bench_c4_partition():
    # bench.py --workload c4 (BASELINE configs[3]) at world size 2: each rank encodes exactly its
    # contiguous half of the job, the chunk counts sum over ranks, the time is the max
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_c4_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=90) for _ in procs)
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    (_, lo0, hi0, tot0, cnt0, el0, enc0), (_, lo1, hi1, tot1, cnt1, el1, enc1) = res
    assert (lo0, hi0, lo1, hi1) == (0, 48, 48, 96)
    assert tot0 == tot1 == 96 and cnt0 == cnt1 == [48, 48]
    assert el0 == el1 > 0
    # 1 warmup + 3 timed encode calls per rank, each over the rank's 48 chunks of 64 KiB
    assert enc0 == enc1 == [48 * 65536] * 4

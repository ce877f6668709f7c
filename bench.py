#!/usr/bin/env python3
"""Benchmark: device-resident RS encode + decode of 1 MiB chunks on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--cpu-seconds S] [--workload c2c3|c4]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload (per rank; weak scaling — every rank owns its own 1024 chunks, no collective on the
data path): BASELINE configs[1]+[2] — 1024 x 1 MiB chunks, RS(k=4, m=2) (zfec Encoder(4, 6)):
one step = encode all 1024 chunks + decode/reassemble all 1024 chunks with data shards
{1, 3} erased (read from the surviving data + parity blocks in HBM).  Inputs are resident in
HBM before the timed region.  value = (chunk bytes encoded + chunk bytes decoded) by all
ranks / max-over-ranks wall time, in GiB/s (2^30 B).

--workload c4 (BASELINE configs[3]; not the headline line): 65536 x 64 KiB chunks, RS(10,4), split
over the ranks by storb_amd.dist.partition (8192 per GPU at N = 8; the whole job on one GPU at
N = 1), strong scaling: value = job bytes encoded per step / max-over-ranks time.  Decode
(blocks {0,2,5,7} erased, the padded block 9 read in place) is timed after the timed region.

Also reported on the headline line:
  roofline      the decode kernel, the dominant one by time: algorithmic bytes per launch
                (k*B read + n written = 2 MiB per chunk) / average launch time from HIP events
                on the launch stream, vs 8 TB/s HBM peak; `traffic` = rocprofv3 PMC bytes per
                launch from profiles/ (FETCH_SIZE x2 + WRITE_SIZE, gfx950 correction) when a
                matching summary is committed, else null
  encode_kernel the same for the encode kernel, the north star's target (n read + (m-k)*B
                written = 1.5 MiB per chunk)
  cpu_baseline  oracle/fec_oracle.c (C restatement of zfec's fec.c: 64 KiB LUT, 8 KiB
                strides) on a bounded sample of the same workload, rank 0 at N=1: one chunk
                per task on min(16, usable cores) threads (`value`, `cores`), and 1 thread
                (`single_thread_value`), --cpu-seconds each
  decode_recover_only_kernel  the same decode with SEC_F_RECOVER (only the 2 missing primaries
                written: k*B read + e*B written per chunk), after the timed region
  e2e           host-buffer encode+decode through the C ABI incl. PCIe: pageable buffers
                (page-locked per call, or staged through pinned slabs) and pinned buffers
                (zero-copy) — reported beside `value`, never as it
"""

from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

GIB = float(1 << 30)
PEAK_HBM_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec

N_CHUNKS = 1024
CHUNK = 1 << 20
K, M = 4, 6  # RS(k=4, m=2) == zfec Encoder(4, 6)
ERASED = (1, 3)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--workload", choices=("c2c3", "c4"), default="c2c3",
                    help="c2c3: the headline line (BASELINE configs[1]+[2], weak scaling); c4: configs[3], "
                         "65536 x 64 KiB RS(10,4) encode split over the ranks (strong scaling)")
    ap.add_argument("--c4-chunks", type=int, default=65536, help="c4: chunks in the whole job (default 65536)")
    ap.add_argument("--no-recover", action="store_true",
                    help="skip the recover-only decode measurement (it shares the decode kernel's name, so a "
                         "rocprofv3 --stats run of the headline line wants it off)")
    ap.add_argument("--no-events", action="store_true",
                    help="A/B only: no per-launch HIP events in the timed region (roofline fields then null)")
    return ap.parse_args()


def enc_descs(nchunks, n, k, m, pstride=None):
    """pstride: distance between a chunk's parity blocks (default B, i.e. packed)."""
    from storb_amd._lib import ENC_DTYPE

    B = -(-n // k)
    ps = pstride or B
    d = np.zeros(nchunks, dtype=ENC_DTYPE)
    d["in_off"] = np.arange(nchunks, dtype=np.uint64) * n
    d["n"] = n
    d["parity_off"] = np.arange(nchunks, dtype=np.uint64) * (m - k) * ps
    d["parity_stride"] = ps
    d["k"] = k
    d["m"] = m
    return d, B


def dec_descs(nchunks, n, k, m, B, data_base, par_base, erased, pstride=None, recover=False):
    """Decode descriptors whose surviving blocks are read in place from the encode buffers.

    Returns (descs, sharenums, block_offs, block_avail): an in-place data block k-1 is short
    when padlen > 0 (zfec's padded copy is not in the chunk buffer), so its avail is B - padlen
    (sec_decode_batch_ex reads the rest as zero).  recover: out_off for SEC_F_RECOVER output
    (e*B per chunk)."""
    from storb_amd._lib import DEC_DTYPE

    ps = pstride or B
    keep = [s for s in range(m) if s not in erased][:k]
    e = sum(1 for s in range(k) if s not in keep)
    d = np.zeros(nchunks, dtype=DEC_DTYPE)
    d["out_off"] = np.arange(nchunks, dtype=np.uint64) * (e * B if recover else n)
    d["B"] = B
    d["padlen"] = B * k - n
    d["slot0"] = np.arange(nchunks, dtype=np.uint64) * k
    d["k"] = k
    d["m"] = m
    sn = np.tile(np.array(keep, np.int32), nchunks)
    offs = np.zeros(nchunks * k, np.uint64)
    avail = np.full(nchunks * k, B, np.uint64)
    ci = np.arange(nchunks, dtype=np.uint64)
    for j, s in enumerate(keep):
        offs[j::k] = (data_base + ci * n + s * B) if s < k else (par_base + ci * (m - k) * ps + (s - k) * ps)
        if s == k - 1:
            avail[j::k] = n - (k - 1) * B
    return d, sn, offs, avail


def load_traffic(kind: str):
    """Per-launch HBM bytes of the encode / decode kernel from the committed rocprofv3 PMC summary
    (profiles/pmc_encode_c2.json: FETCH_SIZE x 2 + WRITE_SIZE on this workload)."""
    path = os.path.join(ROOT, "profiles", "pmc_encode_c2.json")
    try:
        with open(path) as f:
            j = json.load(f)
        if j.get("workload") == "c2" and j.get(kind, {}).get("hbm_bytes_per_launch"):
            return float(j[kind]["hbm_bytes_per_launch"])
    except (OSError, ValueError):
        pass
    return None


def _cpu_worker(seconds: float, seed: int) -> tuple[int, float]:
    """One thread of the CPU baseline: encode + decode loops over its own buffers.  ctypes
    drops the GIL inside the C calls, so threads run concurrently."""
    from oracle import cfec

    lib = cfec.lib()
    u8p = ctypes.POINTER(ctypes.c_uint8)
    rng = np.random.default_rng(seed)
    nsample = 8
    chunks = [rng.integers(0, 256, CHUNK, dtype=np.uint8).tobytes() for _ in range(nsample)]
    B = CHUNK // K
    blocks = (ctypes.c_uint8 * (M * B))()
    out = (ctypes.c_uint8 * CHUNK)()
    keep = [s for s in range(M) if s not in ERASED]
    sn = (ctypes.c_int * K)(*keep)
    base = ctypes.addressof(blocks)
    ptrs = (ctypes.c_char_p * K)(*[ctypes.c_char_p(base + s * B) for s in keep])
    done = 0
    t0 = time.perf_counter()
    while True:
        c = chunks[done % nsample]
        if lib.fo_easy_encode(K, M, c, CHUNK, ctypes.cast(blocks, u8p)) != B:
            raise RuntimeError("oracle encode failed")
        if lib.fo_easy_decode(K, M, ptrs, sn, B, 0, ctypes.cast(out, u8p)):
            raise RuntimeError("oracle decode failed")
        if done == 0 and bytes(out) != c:
            raise RuntimeError("oracle round trip mismatch")
        done += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            return done, el


def cpu_threads() -> int:
    """Threads for the multi-core baseline: the cores this process may use, at most 16 (the
    GPU box's CPU share per GPU; os.cpu_count() there reports the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def cpu_baseline(seconds: float) -> dict:
    """oracle/fec_oracle.c: encode + decode ({1,3} erased) of 1 MiB RS(4,2) chunks, one chunk
    per task; `seconds` on 1 thread, then `seconds` on cpu_threads() threads."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import cfec

    cfec.lib()  # build / load once before the threads start
    d1, e1 = _cpu_worker(seconds, 0)
    single = 2 * d1 * CHUNK / e1 / GIB
    T = cpu_threads()
    with ThreadPoolExecutor(T) as ex:
        res = list(ex.map(lambda i: _cpu_worker(seconds, i), range(T)))
    done = sum(d for d, _ in res)
    el = max(e for _, e in res)
    multi = 2 * done * CHUNK / el / GIB
    return {"value": round(multi, 4), "unit": "GiB/s", "cores": T, "kind": "port",
            "single_thread_value": round(single, 4),
            "sample": f"{T} threads x {seconds:.0f} s of (encode + decode {{1,3}} erased) of 1 MiB RS(4,2) chunks "
                      f"({done} chunks), one chunk per task; 1 thread: {d1} chunks in {e1:.1f} s; "
                      f"oracle/fec_oracle.c (zfec fec.c restatement: 64 KiB LUT, 8 KiB strides)"}


def timed_region(dmod, local, sync, steps, body):
    """The contract's timed region: barrier + device sync on both sides of exactly `steps`
    calls of body(); returns the max over ranks of the elapsed seconds."""
    from storb_amd import dist as D

    D.barrier(dmod, local)
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        body()
    sync()
    D.barrier(dmod, local)
    return D.max_over_ranks(dmod, time.perf_counter() - t0, local)


def kernel_avg_s(eng, kind):
    ms, n = eng.collect_timing(kind)
    return (ms / 1e3 / n) if n else float("nan"), n


def recover_only_rate(eng, torch, src, par, nchunks, n, k, m, B, reps=10) -> dict:
    """SEC_F_RECOVER on the same blocks as the bench decode: only the e = 2 missing primaries
    are written (zfec fec_decode's own output).  Algorithmic bytes: k*B read + e*B written."""
    e = sum(1 for s in range(k) if s in ERASED)
    dd, sn, offs, av = dec_descs(nchunks, n, k, m, B, src.data_ptr(), par.data_ptr(), ERASED, recover=True)
    rec = torch.empty(nchunks * e * B, dtype=torch.uint8, device=src.device)
    eng.decode_batch(dd, sn, offs, 0, rec, block_avail=av, recover_only=True)
    s3 = src.view(nchunks, k, B)
    r3 = rec.view(nchunks, e, B)
    for j, blk in enumerate(sorted(s for s in ERASED if s < k)):
        if not torch.equal(r3[:, j], s3[:, blk]):
            bad = (r3[:, j] != s3[:, blk]).any(dim=1).nonzero().flatten().tolist()
            raise SystemExit(f"bench: recover-only mismatch in row {j}: {len(bad)} chunks, first {bad[:8]}; "
                             f"{r3[bad[0], j, :8].tolist()} vs {s3[bad[0], blk, :8].tolist()}")
    eng.set_timing(True)
    for _ in range(reps):
        eng.decode_batch(dd, sn, offs, 0, rec, block_avail=av, recover_only=True, asynchronous=True)
    eng.sync()
    eng.set_timing(False)
    t, nl = kernel_avg_s(eng, "decode")
    alg = nchunks * (k + e) * B
    return {"achieved": round(alg / t / 1e9, 1), "unit": "GB/s", "algorithmic_bytes_per_launch": alg,
            "avg_launch_ms": round(t * 1e3, 4), "launches": nl}


def main():
    args = parse()
    if args.workload == "c4":
        return main_c4(args)
    import torch

    from storb_amd import dist as D
    from storb_amd.engine import Engine

    rank, local, world = D.rank_env()
    # rehearsal overrides (several ranks on one GPU over gloo); the driver's runs set neither
    local = int(os.environ.get("STORB_BENCH_DEVICE", local))
    torch.cuda.set_device(local)
    dmod = D.init(os.environ.get("STORB_DIST_BACKEND") or None)
    eng = Engine(local)

    n, k, m = CHUNK, K, M
    g = torch.Generator(device=f"cuda:{local}")
    g.manual_seed(1000 + rank)
    src = torch.randint(0, 256, (N_CHUNKS * n,), dtype=torch.uint8, device=f"cuda:{local}", generator=g)
    ed, B = enc_descs(N_CHUNKS, n, k, m)
    par = torch.empty(N_CHUNKS * (m - k) * B, dtype=torch.uint8, device=f"cuda:{local}")
    out = torch.empty_like(src)
    dd, sn, offs, av = dec_descs(N_CHUNKS, n, k, m, B, src.data_ptr(), par.data_ptr(), ERASED)

    def step():
        eng.encode_batch(ed, src, par, asynchronous=True)
        eng.decode_batch(dd, sn, offs, 0, out, block_avail=av, asynchronous=True)

    for _ in range(args.warmup):
        step()
    eng.sync()
    if not torch.equal(out, src):
        raise SystemExit("bench: decode round trip mismatch")

    eng.set_timing(not args.no_events)
    el_max = timed_region(dmod, local, torch.cuda.synchronize, args.steps, step)
    eng.set_timing(False)
    enc_avg_s, enc_n = kernel_avg_s(eng, "encode")
    dec_avg_s, dec_n = kernel_avg_s(eng, "decode")

    bytes_per_step = 2 * N_CHUNKS * n  # encoded + decoded chunk bytes
    value = world * args.steps * bytes_per_step / el_max / GIB

    enc_alg = N_CHUNKS * (n + (m - k) * B)  # bytes per encode launch
    dec_alg = N_CHUNKS * (k * B + n)  # reassemble: k blocks read + n written
    enc_gbs = enc_alg / enc_avg_s / 1e9
    dec_gbs = dec_alg / dec_avg_s / 1e9

    res = None
    if rank == 0:
        res = {
            "metric": "GiB/s device-resident RS encode+decode, 1 MiB chunks, 1/2/4/8 MI355X",
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (torch.randint uniform bytes, seeded per rank), HBM-resident",
            "config": {"workload": "1024 x 1 MiB chunks per GPU, RS(k=4,m=2)=zfec(4,6): encode + "
                                   "decode/reassemble with data shards {1,3} erased",
                       "chunks_per_gpu": N_CHUNKS, "chunk_bytes": n, "k": k, "m_total": m,
                       "bytes_per_step_per_gpu": bytes_per_step, "parallelism": f"chunk-partition x{world}"},
            # the dominant kernel by time is the decode (it moves 2 MiB per chunk to encode's 1.5)
            "roofline": {"bound": "hbm", "achieved": round(dec_gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": round(dec_gbs / PEAK_HBM_GBS, 4), "traffic": load_traffic("decode"),
                         "kernel": "sec_decode_kernel<2, 1, false>", "algorithmic_bytes_per_launch": dec_alg,
                         "avg_launch_ms": round(dec_avg_s * 1e3, 4), "launches": dec_n},
            # the north star's target kernel (>= 70 % of HBM roofline on C2 encode)
            "encode_kernel": {"achieved": round(enc_gbs, 1), "unit": "GB/s", "frac": round(enc_gbs / PEAK_HBM_GBS, 4),
                              "traffic": load_traffic("encode"), "kernel": "sec_encode_kernel<2, 1, false>",
                              "algorithmic_bytes_per_launch": enc_alg, "avg_launch_ms": round(enc_avg_s * 1e3, 4),
                              "launches": enc_n},
            "encode_gibs": round(N_CHUNKS * n / enc_avg_s / GIB, 2),
            "decode_gibs": round(N_CHUNKS * n / dec_avg_s / GIB, 2),
        }
        if not args.no_events and not args.no_recover:  # after the timed region; not part of `value`
            res["decode_recover_only_kernel"] = recover_only_rate(eng, torch, src, par, N_CHUNKS, n, k, m, B)

    # host-buffer (PCIe-inclusive) rate: reported, never `value`
    if rank == 0 and world == 1 and not args.no_e2e:
        res["e2e"] = e2e_rate(eng)
    if rank == 0 and world == 1 and not args.no_cpu:
        res["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
    elif rank == 0:
        res["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(res), flush=True)
    eng.close()
    if dmod is not None:
        dmod.destroy_process_group()


# ---------------------------------------------------------------- BASELINE configs[3] (C4)
C4_CHUNKS, C4_CHUNK, C4_K, C4_M = 65536, 65536, 10, 14
C4_ERASED = (0, 2, 5, 7)  # block 9 (zfec's padded last data block) survives and is read in place


def c4_share(rank: int, world: int, nchunks: int = C4_CHUNKS) -> tuple[int, int]:
    """This rank's contiguous chunk range of the C4 job (storb_amd.dist.partition by bytes)."""
    from storb_amd import dist as D

    return D.partition([C4_CHUNK] * nchunks, world)[rank]


def c4_run(eng, dmod, rank, world, local, device, sync, steps, warmup, nchunks=C4_CHUNKS, verify=True,
           keep=False):
    """C4 as BASELINE.json writes it: `nchunks` x 64 KiB RS(10,4) chunks split over the ranks
    (contiguous ranges, no data-path collective); each rank encodes its share on its device.
    Returns this rank's numbers plus the job's aggregate (max-over-ranks time, summed chunks).
    `eng` needs encode_batch / decode_batch / sync / set_timing / collect_timing (the product
    Engine; tests/test_dist.py drives it with a stand-in on CPU tensors)."""
    import torch

    from storb_amd import dist as D

    lo, hi = c4_share(rank, world, nchunks)
    nch, n, k, m = hi - lo, C4_CHUNK, C4_K, C4_M
    g = torch.Generator(device=device)
    g.manual_seed(4_000_003 + lo)  # seed 4, per share
    src = torch.randint(0, 256, (max(nch * n, 1),), dtype=torch.uint8, device=device, generator=g)
    ed, B = enc_descs(nch, n, k, m)
    par = torch.empty(max(nch * (m - k) * B, 1), dtype=torch.uint8, device=device)
    out = torch.empty_like(src)
    dd, sn, offs, av = dec_descs(nch, n, k, m, B, src.data_ptr(), par.data_ptr(), C4_ERASED)

    def step():
        eng.encode_batch(ed, src, par, asynchronous=True)

    for _ in range(warmup):
        step()
    eng.sync()
    if verify:  # every chunk: 4 data blocks erased, recovered from parity, block 9 in place
        eng.decode_batch(dd, sn, offs, 0, out, block_avail=av)
        if not torch.equal(out, src):
            raise SystemExit(f"bench c4: rank {rank} round trip mismatch")
    eng.set_timing(True)
    el_max = timed_region(dmod, local, sync, steps, step)
    eng.set_timing(False)
    enc_avg_s, enc_n = kernel_avg_s(eng, "encode")
    # decode (reassemble) of the share, after the timed region: reported beside `value`
    eng.set_timing(True)
    for _ in range(max(steps // 2, 1)):
        eng.decode_batch(dd, sn, offs, 0, out, block_avail=av, asynchronous=True)
    eng.sync()
    eng.set_timing(False)
    dec_avg_s, dec_n = kernel_avg_s(eng, "decode")
    total_chunks = int(D.sum_over_ranks(dmod, float(nch), local))
    counts = [int(D.sum_over_ranks(dmod, float(nch if r == rank else 0), local)) for r in range(world)]
    res = {"lo": lo, "hi": hi, "chunks": nch, "B": B, "el_max": el_max, "total_chunks": total_chunks,
           "per_rank_chunks": counts, "enc_avg_s": enc_avg_s, "enc_launches": enc_n, "dec_avg_s": dec_avg_s,
           "dec_launches": dec_n}
    if keep:  # the buffers, for tests that compare samples against the oracle
        res.update(src=src, par=par)
    return res


def main_c4(args):
    import torch

    from storb_amd import dist as D
    from storb_amd.engine import Engine

    rank, local, world = D.rank_env()
    local = int(os.environ.get("STORB_BENCH_DEVICE", local))
    torch.cuda.set_device(local)
    dmod = D.init(os.environ.get("STORB_DIST_BACKEND") or None)
    eng = Engine(local)
    r = c4_run(eng, dmod, rank, world, local, f"cuda:{local}", torch.cuda.synchronize, args.steps, args.warmup,
               nchunks=args.c4_chunks)
    n, k, m, B = C4_CHUNK, C4_K, C4_M, r["B"]
    job_bytes = r["total_chunks"] * n
    value = args.steps * job_bytes / r["el_max"] / GIB
    enc_alg = r["chunks"] * (n + (m - k) * B)
    dec_alg = r["chunks"] * (k * B + n)
    if rank == 0:
        enc_gbs = enc_alg / r["enc_avg_s"] / 1e9
        res = {
            "metric": "GiB/s device-resident RS(10,4) encode, 65536 x 64 KiB chunks sharded across N MI355X",
            "value": round(value, 3), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(r["el_max"] / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (torch.randint uniform bytes, seed 4 per share), HBM-resident",
            "config": {"workload": f"BASELINE configs[3]: {r['total_chunks']} x 64 KiB chunks, RS(k=10,m=4)="
                                   "zfec(10,14), B = 6554, padlen 4, encode; chunks split by "
                                   "storb_amd.dist.partition over the ranks, no data-path collective",
                       "chunks_total": r["total_chunks"], "per_rank_chunks": r["per_rank_chunks"],
                       "world_size": world,
                       "backend": dmod.get_backend() if dmod is not None else None,
                       "parallelism": f"chunk-partition x{world}"},
            "roofline": {"bound": "hbm", "achieved": round(enc_gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": round(enc_gbs / PEAK_HBM_GBS, 4), "traffic": None,
                         "kernel": ("sec_encode_kernel<4, 1, false>" if os.environ.get("SEC_BS") == "0"
                                    else "sec_encode_bs_kernel<10, 14, 0, 4, 5>"),  # api.cpp bs_shape
                         "algorithmic_bytes_per_launch": enc_alg,
                         "avg_launch_ms": round(r["enc_avg_s"] * 1e3, 4), "launches": r["enc_launches"]},
            "decode_kernel": {"achieved": round(dec_alg / r["dec_avg_s"] / 1e9, 1), "unit": "GB/s",
                              "erased": list(C4_ERASED), "block_9": "read in place, avail = B - padlen",
                              "algorithmic_bytes_per_launch": dec_alg,
                              "avg_launch_ms": round(r["dec_avg_s"] * 1e3, 4), "launches": r["dec_launches"]},
            "cpu_baseline": None,
        }
        print(json.dumps(res), flush=True)
    eng.close()
    if dmod is not None:
        dmod.destroy_process_group()


def _e2e_pass(eng, host, par, out, nchunks, steps):
    ed, B = enc_descs(nchunks, CHUNK, K, M)
    dd, sn, offs, _ = dec_descs(nchunks, CHUNK, K, M, B, host.ctypes.data, par.ctypes.data, ERASED)
    eng.encode_batch(ed, host, par, host=True)
    eng.decode_batch(dd, sn, offs, 0, out, host=True)
    if not np.array_equal(out, host):
        raise SystemExit("bench: host e2e mismatch")
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.encode_batch(ed, host, par, host=True)
    t1 = time.perf_counter()
    for _ in range(steps):
        eng.decode_batch(dd, sn, offs, 0, out, host=True)
    t2 = time.perf_counter()
    tot = nchunks * CHUNK * steps
    return round(tot / (t1 - t0) / GIB, 3), round(tot / (t2 - t1) / GIB, 3)


def e2e_rate(eng, nchunks=1024, steps=3) -> dict:
    """Encode + decode of host-resident 1 MiB chunks through SEC_F_HOST, three ways: pageable
    numpy buffers (the library page-locks them for each call and the kernels read / write them
    over PCIe), the same buffers staged through pinned slabs + DMA (SEC_REGISTER_MIN=0), and
    pinned buffers (Engine.host_empty, zero-copy)."""
    rng = np.random.default_rng(7)
    host = rng.integers(0, 256, nchunks * CHUNK, dtype=np.uint8)
    nb = nchunks * (M - K) * (CHUNK // K)
    par, out = np.empty(nb, dtype=np.uint8), np.empty_like(host)
    p0 = np.array(eng.host_paths())
    enc, dec = _e2e_pass(eng, host, par, out, nchunks, steps)
    p1 = np.array(eng.host_paths())
    os.environ["SEC_REGISTER_MIN"] = "0"
    try:
        senc, sdec = _e2e_pass(eng, host, par, out, nchunks, steps)
    finally:
        os.environ.pop("SEC_REGISTER_MIN")
    p2 = np.array(eng.host_paths())
    ph, pp, po = eng.host_empty(host.size), eng.host_empty(nb), eng.host_empty(host.size)
    ph[:] = host
    penc, pdec = _e2e_pass(eng, ph, pp, po, nchunks, steps)
    p3 = np.array(eng.host_paths())
    calls = 2 * (steps + 1)
    if (list(p1 - p0), list(p2 - p1), list(p3 - p2)) != ([0, calls, 0], [0, 0, calls], [calls, 0, 0]):
        raise SystemExit(f"bench: e2e calls did not take the expected host paths {p0} {p1} {p2} {p3}")
    del ph, pp, po
    return {"encode_gibs": enc, "decode_gibs": dec, "staged_encode_gibs": senc, "staged_decode_gibs": sdec,
            "pinned_encode_gibs": penc, "pinned_decode_gibs": pdec,
            "sample": f"{nchunks} x 1 MiB RS(4,2), {steps} calls each; *_gibs: pageable numpy buffers, page-locked "
                      f"by the library per call; staged_*: the same, staged through pinned slabs; pinned_*: "
                      f"Engine.host_empty buffers; the kernels read / write locked or pinned host memory over PCIe"}


if __name__ == "__main__":
    main()

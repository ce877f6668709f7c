#!/usr/bin/env python3
"""Benchmark: device-resident RS encode + decode of 1 MiB chunks on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--cpu-seconds S]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload (per rank; weak scaling — every rank owns its own 1024 chunks, no collective on the
data path): BASELINE configs[1]+[2] — 1024 x 1 MiB chunks, RS(k=4, m=2) (zfec Encoder(4, 6)):
one step = encode all 1024 chunks + decode/reassemble all 1024 chunks with data shards
{1, 3} erased (read from the surviving data + parity blocks in HBM).  Inputs are resident in
HBM before the timed region.  value = (chunk bytes encoded + chunk bytes decoded) by all
ranks / max-over-ranks wall time, in GiB/s (2^30 B).

Also reported on the same line:
  roofline      the encode kernel (the dominant, BASELINE-target kernel): algorithmic bytes
                per launch (n read + (m-k)*B written = 1.5 MiB per chunk) / average launch
                time from HIP events on the launch stream, vs 8 TB/s HBM peak; `traffic` =
                rocprofv3 PMC bytes per launch from profiles/ (FETCH_SIZE x2 + WRITE_SIZE,
                gfx950 correction) when a matching summary is committed, else null
  cpu_baseline  oracle/fec_oracle.c (C restatement of zfec's fec.c: 64 KiB LUT, 8 KiB
                strides) on a bounded sample of the same workload, rank 0 at N=1: one chunk
                per task on min(16, usable cores) threads (`value`, `cores`), and 1 thread
                (`single_thread_value`), --cpu-seconds each
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


def dec_descs(nchunks, n, k, m, B, data_base, par_base, erased, pstride=None):
    """Decode descriptors whose surviving blocks are read in place from the encode buffers.

    The C ABI needs B readable bytes per block; an in-place data block k-1 is short when
    padlen > 0 (zfec's padded copy is not in the chunk buffer), so it must be erased then.
    """
    from storb_amd._lib import DEC_DTYPE

    ps = pstride or B
    if B * k != n and (k - 1) not in erased:
        raise ValueError("padded last data block cannot be read in place: erase block k-1")
    keep = [s for s in range(m) if s not in erased][:k]
    d = np.zeros(nchunks, dtype=DEC_DTYPE)
    d["out_off"] = np.arange(nchunks, dtype=np.uint64) * n
    d["B"] = B
    d["padlen"] = B * k - n
    d["slot0"] = np.arange(nchunks, dtype=np.uint64) * k
    d["k"] = k
    d["m"] = m
    sn = np.tile(np.array(keep, np.int32), nchunks)
    offs = np.zeros(nchunks * k, np.uint64)
    ci = np.arange(nchunks, dtype=np.uint64)
    for j, s in enumerate(keep):
        offs[j::k] = (data_base + ci * n + s * B) if s < k else (par_base + ci * (m - k) * ps + (s - k) * ps)
    return d, sn, offs


def load_traffic():
    """Per-launch HBM bytes of the encode kernel from a committed rocprofv3 PMC summary."""
    path = os.path.join(ROOT, "profiles", "pmc_encode_c2.json")
    try:
        with open(path) as f:
            j = json.load(f)
        if j.get("workload") == "c2" and j.get("hbm_bytes_per_launch"):
            return float(j["hbm_bytes_per_launch"])
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


def main():
    args = parse()
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
    dd, sn, offs = dec_descs(N_CHUNKS, n, k, m, B, src.data_ptr(), par.data_ptr(), ERASED)

    def step():
        eng.encode_batch(ed, src, par, asynchronous=True)
        eng.decode_batch(dd, sn, offs, 0, out, asynchronous=True)

    for _ in range(args.warmup):
        step()
    eng.sync()
    if not torch.equal(out, src):
        raise SystemExit("bench: decode round trip mismatch")

    eng.set_timing(not args.no_events)
    D.barrier(dmod, local)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    eng.sync()
    torch.cuda.synchronize()
    D.barrier(dmod, local)
    el = time.perf_counter() - t0
    eng.set_timing(False)
    enc_ms, enc_n = eng.collect_timing("encode")
    dec_ms, dec_n = eng.collect_timing("decode")
    el_max = D.max_over_ranks(dmod, el, local)

    bytes_per_step = 2 * N_CHUNKS * n  # encoded + decoded chunk bytes
    value = world * args.steps * bytes_per_step / el_max / GIB

    enc_alg = N_CHUNKS * (n + (m - k) * B)  # bytes per encode launch
    dec_alg = N_CHUNKS * (k * B + n)  # reassemble: k blocks read + n written
    enc_avg_s = enc_ms / 1e3 / max(enc_n, 1) or float("nan")
    dec_avg_s = dec_ms / 1e3 / max(dec_n, 1) or float("nan")
    enc_gbs = enc_alg / enc_avg_s / 1e9
    traffic = load_traffic()

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
            "roofline": {"bound": "hbm", "achieved": round(enc_gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": round(enc_gbs / PEAK_HBM_GBS, 4),
                         "traffic": traffic,
                         "kernel": "sec_encode_kernel<2, 1, false>",
                         "algorithmic_bytes_per_launch": enc_alg,
                         "avg_launch_ms": round(enc_avg_s * 1e3, 4), "launches": enc_n},
            "decode_kernel": {"achieved": round(dec_alg / dec_avg_s / 1e9, 1), "unit": "GB/s",
                              "algorithmic_bytes_per_launch": dec_alg, "avg_launch_ms": round(dec_avg_s * 1e3, 4),
                              "launches": dec_n},
            "encode_gibs": round(N_CHUNKS * n / enc_avg_s / GIB, 2),
            "decode_gibs": round(N_CHUNKS * n / dec_avg_s / GIB, 2),
        }

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


def _e2e_pass(eng, host, par, out, nchunks, steps):
    ed, B = enc_descs(nchunks, CHUNK, K, M)
    dd, sn, offs = dec_descs(nchunks, CHUNK, K, M, B, host.ctypes.data, par.ctypes.data, ERASED)
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

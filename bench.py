#!/usr/bin/env python3
"""Benchmark: device-resident RS encode + decode of 1 MiB chunks on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--cpu-seconds S] [--workload c2c3|c4|c5]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Ranks.  One process per GPU.  Under torch.distributed.run the ranks come from RANK /
LOCAL_RANK / WORLD_SIZE, and WORLD_SIZE must equal --gpus (otherwise exit status 2).  A plain
`python bench.py --gpus N` (N > 1, WORLD_SIZE unset) launches the N ranks itself, as fresh
child processes with that environment (MASTER_ADDR 127.0.0.1), before anything touches the
GPU, and exits with the first failing rank's status.  Every line carries the world size and
backend the ranks saw.

Workload (per rank; weak scaling — every rank owns its own 1024 chunks, no collective on the
data path): BASELINE configs[1]+[2] — 1024 x 1 MiB chunks, RS(k=4, m=2) (zfec Encoder(4, 6)):
one step = encode all 1024 chunks + decode/reassemble all 1024 chunks with data shards
{1, 3} erased (read from the surviving data + parity blocks in HBM).  Inputs are resident in
HBM before the timed region.  value = (chunk bytes encoded + chunk bytes decoded) by all
ranks / max-over-ranks wall time, in GiB/s (2^30 B).

--workload c4 (BASELINE configs[3]; not the headline line): 65536 x 64 KiB chunks, RS(10,4), split
over the ranks by storb_amd.dist.partition (8192 per GPU at N = 8; the whole job on one GPU at
N = 1), strong scaling: value = job bytes encoded per step / max-over-ranks time.  Parity rows
are written at a 128-byte-aligned stride (--c4-palign; the ABI's parity_stride, the caller's
layout choice: storb keeps every piece as its own object).  Decode (blocks {0,2,5,7} erased,
the padded block 9 read in place) is timed after the timed region.

--workload c5 (BASELINE configs[4]): chunk sizes log-uniform in [4 KiB, 4 MiB] (seed 5) up to
~1 GiB, RS(8,3) = zfec(8,11), split over the ranks by bytes (strong scaling).  One step =
encode + decode ({1,3,5} erased, block 7 read in place) of the rank's share END TO END from
pinned host memory (the kernels read and write the host buffers over PCIe: the product's
zero-copy path); value = job bytes encoded + decoded per step / max-over-ranks time.  The
device-resident kernel rates and the staged (pageable -> pinned slabs -> hipMemcpyAsync) rate
are reported beside it.

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
  c4, c5        BASELINE configs[3] and [4] measured in the same run after the headline's timed
                region (the --workload c4 / c5 lines' fields, nested; --no-c4 / --no-c5 skip
                them): each with its own roofline, PMC traffic and CPU baseline
                (--sub-cpu-seconds on 1 thread, then on all threads)

`traffic` fields come from profiles/pmc_<workload>.json (tools/gpu_pmc.sh) and only when that
summary's `lib_digest` equals this build's source digest; otherwise they are null.

STORB_BENCH_ENGINE=module:Class (tests only) runs the ranks on CPU tensors with that engine
(tests/bench_stub.py: the oracle behind the Engine interface) over gloo, so the launch, the
partition and the reductions are tested without a GPU.  STORB_BENCH_DEVICE / STORB_DIST_BACKEND
(rehearsal only) put every rank on one device over another backend.
"""

from __future__ import annotations

import argparse
import ctypes
import json
import os
import signal
import socket
import subprocess
import sys
import time
from types import SimpleNamespace

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

GIB = float(1 << 30)
PEAK_HBM_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec

N_CHUNKS = 1024
CHUNK = 1 << 20
K, M = 4, 6  # RS(k=4, m=2) == zfec Encoder(4, 6)
ERASED = (1, 3)

# rocprofv3 kernel names of the headline kernels (api.cpp's plan for C2 / C3)
ENC_KERNEL_C2 = "sec_encode_kernel<2, 1, false>"
DEC_KERNEL_C3 = "sec_decode_kernel<2, 1, false, 0>"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--workload", choices=("c2c3", "c4", "c5"), default="c2c3",
                    help="c2c3: the headline line (BASELINE configs[1]+[2], weak scaling); c4: configs[3], "
                         "65536 x 64 KiB RS(10,4) encode split over the ranks (strong scaling); c5: configs[4], "
                         "mixed 4 KiB-4 MiB RS(8,3) encode + decode end to end from pinned host memory")
    ap.add_argument("--chunks", type=int, default=N_CHUNKS,
                    help="c2c3: chunks per rank (default 1024, the BASELINE config; smaller only in tests)")
    ap.add_argument("--c4-chunks", type=int, default=65536, help="c4: chunks in the whole job (default 65536)")
    ap.add_argument("--c4-palign", type=int, default=128,
                    help="c4: parity rows start at multiples of this many bytes (1 = packed, B apart)")
    ap.add_argument("--c5-bytes", type=int, default=1 << 30, help="c5: job size (default ~1 GiB)")
    ap.add_argument("--no-recover", action="store_true",
                    help="skip the recover-only decode measurement (it shares the decode kernel's name, so a "
                         "rocprofv3 --stats run of the headline line wants it off)")
    ap.add_argument("--no-c4", action="store_true", help="c2c3: skip the C4 sub-object (configs[3])")
    ap.add_argument("--no-c5", action="store_true", help="c2c3: skip the C5 sub-object (configs[4])")
    ap.add_argument("--sub-cpu-seconds", type=float, default=1.5,
                    help="c2c3: CPU-baseline seconds (1 thread, then all threads) of the c4 / c5 sub-objects")
    ap.add_argument("--c5-steps", type=int, default=10, help="c2c3: timed steps of the c5 sub-object")
    ap.add_argument("--c5-device-only", action="store_true",
                    help="c5: skip the end-to-end host steps (rocprofv3 PMC passes of the device-resident kernels)")
    ap.add_argument("--no-events", action="store_true",
                    help="A/B only: no per-launch HIP events in the timed region (roofline fields then null)")
    ap.add_argument("--in-process", action="store_true",
                    help="drive the N devices from ONE process (engine.EngineGroup: a host thread and context per "
                         "device) instead of one rank per GPU; the headline and C5 lines in that form")
    ap.add_argument("--inproc-devices", default=None,
                    help="rehearsal only: comma list of the devices the in-process form drives (default 0..N-1; "
                         "'0,0' puts two contexts on one GPU)")
    ap.add_argument("--no-in-process", action="store_true",
                    help="c2c3 under N > 1 ranks: skip the nested in-process measurement rank 0 takes after the "
                         "rank-per-GPU lines (the other ranks wait on a CPU barrier meanwhile)")
    return ap.parse_args(argv)


# ---------------------------------------------------------------- ranks
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_ranks(args, argv=None) -> int | None:
    """None when this process is a rank; otherwise launch the ranks and return the exit status.

    WORLD_SIZE set (torch.distributed.run, or our own children): it must equal --gpus.  Unset
    with --gpus N > 1: start N children of this script with RANK = LOCAL_RANK = r, WORLD_SIZE =
    N, MASTER_ADDR = 127.0.0.1 and a free MASTER_PORT.  This process never touches the GPU (it
    has imported nothing but numpy), so nothing is re-executed after GPU initialisation."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != args.gpus:
            print(f"bench: WORLD_SIZE={ws} but --gpus {args.gpus}: refusing to report a {ws}-rank line as "
                  f"{args.gpus}", file=sys.stderr, flush=True)
            return 2
        return None
    if args.gpus < 1:
        print("bench: --gpus must be >= 1", file=sys.stderr, flush=True)
        return 2
    if args.gpus == 1:
        return None
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    argv = sys.argv[1:] if argv is None else argv
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__), *argv], env=env))

    def stop(*_):
        for p in procs:
            if p.poll() is None:
                p.terminate()

    old = signal.signal(signal.SIGTERM, lambda *a: (stop(), sys.exit(143)))
    rc = 0
    try:
        pending = list(procs)
        while pending:
            for p in list(pending):
                c = p.poll()
                if c is None:
                    continue
                pending.remove(p)
                if c != 0 and rc == 0:  # first failure: stop the others (they would wait in a barrier)
                    rc = c if c > 0 else 128 - c
                    stop()
            time.sleep(0.02)
    finally:
        stop()
        for p in procs:
            try:
                p.wait(30)
            except subprocess.TimeoutExpired:
                p.kill()
        signal.signal(signal.SIGTERM, old)
    return rc


def rank_context(args) -> SimpleNamespace:
    """This rank's engine, device, sync and process group."""
    from storb_amd import dist as D

    rank, local, world = D.rank_env()
    stub = _stub_factory()
    if stub:  # tests: the oracle behind the Engine interface, CPU tensors, gloo
        eng = stub()
        device, sync, dev_idx = "cpu", (lambda: None), None
        dmod = D.init(os.environ.get("STORB_DIST_BACKEND") or "gloo")
    else:
        import torch

        from storb_amd.engine import Engine

        local = int(os.environ.get("STORB_BENCH_DEVICE", local))
        torch.cuda.set_device(local)
        dmod = D.init(os.environ.get("STORB_DIST_BACKEND") or None)
        eng = Engine(local)
        device, sync, dev_idx = f"cuda:{local}", torch.cuda.synchronize, local
    seen = dmod.get_world_size() if dmod is not None else 1
    if seen != args.gpus or seen != world:
        raise SystemExit(f"bench: rank {rank} sees world size {seen}, --gpus {args.gpus}, WORLD_SIZE {world}")
    return SimpleNamespace(rank=rank, local=dev_idx, world=world, device=device, sync=sync, dmod=dmod, eng=eng,
                           backend=dmod.get_backend() if dmod is not None else None)


def finish(ctx) -> None:
    ctx.eng.close()
    if ctx.dmod is not None:
        ctx.dmod.destroy_process_group()


# ---------------------------------------------------------------- descriptors
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


def enc_descs_var(sizes, k, m):
    """Encode descriptors of chunks of the given sizes packed back to back (parity packed too)."""
    from storb_amd._lib import ENC_DTYPE

    sizes = np.asarray(sizes, dtype=np.uint64)
    B = (sizes + k - 1) // k
    d = np.zeros(len(sizes), dtype=ENC_DTYPE)
    d["in_off"] = np.concatenate([[0], np.cumsum(sizes)[:-1]]) if len(sizes) else []
    d["n"] = sizes
    d["parity_off"] = np.concatenate([[0], np.cumsum(B * (m - k))[:-1]]) if len(sizes) else []
    d["parity_stride"] = B
    d["k"], d["m"] = k, m
    return d, B


def dec_descs_var(sizes, k, m, B, data_base, par_base, erased):
    """enc_descs_var's chunks decoded in place: descriptors, sharenums, block offsets and per-slot
    avail (an in-place block k-1 has B - padlen bytes)."""
    from storb_amd._lib import DEC_DTYPE

    keep = [s for s in range(m) if s not in erased][:k]
    n = len(sizes)
    sizes = np.asarray(sizes, dtype=np.uint64)
    in_off = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
    par_off = np.concatenate([[0], np.cumsum(B * (m - k))[:-1]]).astype(np.uint64)
    d = np.zeros(n, dtype=DEC_DTYPE)
    d["out_off"] = in_off
    d["B"] = B
    d["padlen"] = B * k - sizes
    d["slot0"] = np.arange(n, dtype=np.uint64) * k
    d["k"], d["m"] = k, m
    sn = np.tile(np.array(keep, np.int32), n)
    offs = np.zeros(n * k, np.uint64)
    avail = np.zeros(n * k, np.uint64)
    for j, s in enumerate(keep):
        offs[j::k] = (data_base + in_off + s * B) if s < k else (par_base + par_off + (s - k) * B)
        avail[j::k] = (sizes - (k - 1) * B) if s == k - 1 else B
    return d, sn, offs, avail


def lib_digest() -> str:
    """Digest of libstorbec.so's sources (storb_amd/_build.py; also its build stamp)."""
    from storb_amd import _build

    return _build._digest()


def load_traffic(kind: str, workload: str = "c2"):
    """Per-launch HBM bytes of a bench kernel from the committed rocprofv3 PMC summary of that
    workload (profiles/pmc_<workload>.json, tools/pmc_summary.py: FETCH_SIZE x 2 + WRITE_SIZE),
    or None when there is none or it was taken on other library sources than this build's
    (its `lib_digest`, VERDICT r03 weak #5: a stale summary is not this kernel's traffic)."""
    path = os.path.join(ROOT, "profiles", f"pmc_{workload}.json")
    try:
        with open(path) as f:
            j = json.load(f)
        if (j.get("workload") == workload and j.get("lib_digest") == lib_digest()
                and j.get(kind, {}).get("hbm_bytes_per_launch")):
            return float(j[kind]["hbm_bytes_per_launch"])
    except (OSError, ValueError):
        pass
    return None


# ---------------------------------------------------------------- CPU baseline (oracle)
def _cpu_worker(seconds: float, seed: int, sizes, k: int, m: int, erased, decode: bool = True) -> tuple[int, int, float]:
    """One thread of the CPU baseline: encode (+ decode with `erased` lost) of chunks of the given
    sizes in turn, each from its own buffer.  ctypes drops the GIL inside the C calls, so threads
    run concurrently.  Returns (chunks, chunk bytes processed, seconds)."""
    from oracle import cfec

    lib = cfec.lib()
    u8p = ctypes.POINTER(ctypes.c_uint8)
    rng = np.random.default_rng(seed)
    keep = [s for s in range(m) if s not in erased][:k]
    sn = (ctypes.c_int * k)(*keep)
    cases = []
    for n in sizes:
        B = -(-n // k)
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        blocks = (ctypes.c_uint8 * (m * B))()
        out = (ctypes.c_uint8 * n)()
        base = ctypes.addressof(blocks)
        ptrs = (ctypes.c_char_p * k)(*[ctypes.c_char_p(base + s * B) for s in keep])
        cases.append((n, B, data, blocks, out, ptrs))
    done = nbytes = 0
    t0 = time.perf_counter()
    while True:
        n, B, data, blocks, out, ptrs = cases[done % len(cases)]
        if lib.fo_easy_encode(k, m, data, n, ctypes.cast(blocks, u8p)) != B:
            raise RuntimeError("oracle encode failed")
        nbytes += n
        if decode:
            if lib.fo_easy_decode(k, m, ptrs, sn, B, k * B - n, ctypes.cast(out, u8p)):
                raise RuntimeError("oracle decode failed")
            if done < len(cases) and bytes(out) != data:
                raise RuntimeError("oracle round trip mismatch")
            nbytes += n
        done += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            return done, nbytes, el


def _cgroup_quota():
    """CPUs the cgroup (v2 cpu.max) grants this process, rounded up, or None when unlimited."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        return None if quota == "max" else max(1, -(-int(quota) // int(period)))
    except (OSError, ValueError):
        return None


def host_cpu_info() -> dict:
    """The box's CPUs as this process sees them: the machine's count, the affinity mask, the
    cgroup quota and the CPU model (`cores` alone is a thread count)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = None
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"os_cpu_count": os.cpu_count(), "affinity_cpus": aff, "cgroup_cpu_quota": _cgroup_quota(),
            "cpu_model": model}


def cpu_threads() -> int:
    """Threads for the multi-core baseline: the CPUs this process may use (affinity mask and
    cgroup quota), at most 16 (the GPU box's CPU share per GPU; os.cpu_count() there reports the
    whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    q = _cgroup_quota()
    return max(1, min(16, n, q or n))


def cpu_baseline(seconds: float, sizes=None, k=K, m=M, erased=ERASED, decode=True, what=None) -> dict:
    """oracle/fec_oracle.c on a bounded sample: `seconds` on 1 thread, then `seconds` on
    cpu_threads() threads, each thread cycling over its own copy of `sizes` (default: 8 chunks of
    1 MiB, RS(4,2), {1,3} erased), one chunk per task."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import cfec

    sizes = list(sizes) if sizes is not None else [CHUNK] * 8
    cfec.lib()  # build / load once before the threads start
    d1, b1, e1 = _cpu_worker(seconds, 0, sizes, k, m, erased, decode)
    T = cpu_threads()
    with ThreadPoolExecutor(T) as ex:
        res = list(ex.map(lambda i: _cpu_worker(seconds, i, sizes, k, m, erased, decode), range(T)))
    done = sum(d for d, _, _ in res)
    nb = sum(b for _, b, _ in res)
    el = max(e for _, _, e in res)
    what = what or (f"(encode + decode {{{','.join(map(str, erased))}}} erased) of 1 MiB RS({k},{m - k}) chunks")
    return {"value": round(nb / el / GIB, 4), "unit": "GiB/s", "cores": T, "kind": "port",
            "single_thread_value": round(b1 / e1 / GIB, 4), "host": host_cpu_info(),
            "sample": f"{T} threads x {seconds:.0f} s of {what} ({done} chunks), one chunk per task; 1 thread: "
                      f"{d1} chunks in {e1:.1f} s; oracle/fec_oracle.c (zfec fec.c restatement: 64 KiB LUT, "
                      f"8 KiB strides)"}


# ---------------------------------------------------------------- timing helpers
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


def _gbs(nbytes, t):
    return round(nbytes / t / 1e9, 1) if t == t and t > 0 else None


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
    return {"achieved": _gbs(alg, t), "unit": "GB/s", "algorithmic_bytes_per_launch": alg,
            "avg_launch_ms": round(t * 1e3, 4), "launches": nl}


# ---------------------------------------------------------------- BASELINE configs[1]+[2] (headline)
def c2c3_run(ctx, steps, warmup, nchunks=N_CHUNKS, events=True):
    """This rank's 1024 x 1 MiB RS(4,2) encode + {1,3}-erased decode; returns the rank's numbers
    and the job's max-over-ranks time, plus the buffers for the after-region measurements."""
    import torch

    eng = ctx.eng
    n, k, m = CHUNK, K, M
    g = torch.Generator(device=ctx.device)
    g.manual_seed(1000 + ctx.rank)
    src = torch.randint(0, 256, (nchunks * n,), dtype=torch.uint8, device=ctx.device, generator=g)
    ed, B = enc_descs(nchunks, n, k, m)
    par = torch.empty(nchunks * (m - k) * B, dtype=torch.uint8, device=ctx.device)
    out = torch.empty_like(src)
    dd, sn, offs, av = dec_descs(nchunks, n, k, m, B, src.data_ptr(), par.data_ptr(), ERASED)

    def step():
        eng.encode_batch(ed, src, par, asynchronous=True)
        eng.decode_batch(dd, sn, offs, 0, out, block_avail=av, asynchronous=True)

    for _ in range(warmup):
        step()
    eng.sync()
    if warmup and not torch.equal(out, src):
        raise SystemExit(f"bench: rank {ctx.rank} decode round trip mismatch")

    eng.set_timing(events)
    el_max = timed_region(ctx.dmod, ctx.local, ctx.sync, steps, step)
    eng.set_timing(False)
    enc_avg_s, enc_n = kernel_avg_s(eng, "encode")
    dec_avg_s, dec_n = kernel_avg_s(eng, "decode")
    from storb_amd import dist as D

    counts = D.gather_counts(ctx.dmod, nchunks, ctx.rank, ctx.world, ctx.local)
    return {"el_max": el_max, "B": B, "chunks": nchunks, "per_rank_chunks": counts, "enc_avg_s": enc_avg_s,
            "enc_launches": enc_n, "dec_avg_s": dec_avg_s, "dec_launches": dec_n, "src": src, "par": par}


def main_c2c3(args, ctx):
    import torch

    r = c2c3_run(ctx, args.steps, args.warmup, args.chunks, events=not args.no_events)
    nchunks, n, k, m, B = args.chunks, CHUNK, K, M, r["B"]
    bytes_per_step = 2 * nchunks * n  # encoded + decoded chunk bytes
    total_chunks = sum(r["per_rank_chunks"])
    value = args.steps * 2 * total_chunks * n / r["el_max"] / GIB

    enc_alg = nchunks * (n + (m - k) * B)  # bytes per encode launch
    dec_alg = nchunks * (k * B + n)  # reassemble: k blocks read + n written
    enc_avg_s, dec_avg_s = r["enc_avg_s"], r["dec_avg_s"]
    enc_gbs, dec_gbs = _gbs(enc_alg, enc_avg_s), _gbs(dec_alg, dec_avg_s)
    res = None
    if ctx.rank == 0:
        res = {
            "metric": "GiB/s device-resident RS encode+decode, 1 MiB chunks, 1/2/4/8 MI355X",
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": ctx.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(r["el_max"] / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (torch.randint uniform bytes, seeded per rank), HBM-resident",
            "config": {"workload": f"{nchunks} x 1 MiB chunks per GPU, RS(k=4,m=2)=zfec(4,6): encode + "
                                   "decode/reassemble with data shards {1,3} erased",
                       "chunks_per_gpu": nchunks, "per_rank_chunks": r["per_rank_chunks"], "chunk_bytes": n,
                       "k": k, "m_total": m, "bytes_per_step_per_gpu": bytes_per_step, "world_size": ctx.world,
                       "backend": ctx.backend, "parallelism": f"chunk-partition x{ctx.world}"},
            # the dominant kernel by time is the decode (it moves 2 MiB per chunk to encode's 1.5)
            "roofline": {"bound": "hbm", "achieved": dec_gbs, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": round(dec_gbs / PEAK_HBM_GBS, 4) if dec_gbs else None,
                         "traffic": load_traffic("decode"), "kernel": DEC_KERNEL_C3,
                         "algorithmic_bytes_per_launch": dec_alg,
                         "avg_launch_ms": round(dec_avg_s * 1e3, 4), "launches": r["dec_launches"]},
            # the north star's target kernel (>= 70 % of HBM roofline on C2 encode)
            "encode_kernel": {"achieved": enc_gbs, "unit": "GB/s",
                              "frac": round(enc_gbs / PEAK_HBM_GBS, 4) if enc_gbs else None,
                              "traffic": load_traffic("encode"), "kernel": ENC_KERNEL_C2,
                              "algorithmic_bytes_per_launch": enc_alg, "avg_launch_ms": round(enc_avg_s * 1e3, 4),
                              "launches": r["enc_launches"]},
            "lib_digest": lib_digest(),
            "encode_gibs": round(nchunks * n / enc_avg_s / GIB, 2) if enc_gbs else None,
            "decode_gibs": round(nchunks * n / dec_avg_s / GIB, 2) if dec_gbs else None,
        }
        if not args.no_events and not args.no_recover:  # after the timed region; not part of `value`
            res["decode_recover_only_kernel"] = recover_only_rate(ctx.eng, torch, r["src"], r["par"], nchunks, n, k,
                                                                  m, B)

    # BASELINE configs[3] and [4] on the same run, after the headline's timed region (VERDICT r03
    # item 1): each its own line's fields, nested; every rank takes part (its share of the job)
    r.pop("src"), r.pop("par")
    sub_cpu = 0 if args.no_cpu else args.sub_cpu_seconds
    if not args.no_c4:
        c4 = c4_result(args, ctx, sub_cpu, args.steps, args.warmup)
        if ctx.rank == 0:
            res["c4"] = c4
    if not args.no_c5:
        c5 = c5_result(args, ctx, sub_cpu, args.c5_steps, min(args.warmup, 2), staged=not args.no_e2e)
        if ctx.rank == 0:
            res["c5"] = c5
    # host-buffer (PCIe-inclusive) rate: reported, never `value`
    if ctx.rank == 0 and ctx.world == 1 and not args.no_e2e:
        res["e2e"] = e2e_rate(ctx.eng)
    if ctx.rank == 0 and ctx.world == 1 and not args.no_cpu:
        res["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
    elif ctx.rank == 0:
        res["cpu_baseline"] = None
    # N > 1 ranks: the same workloads from ONE process over all N devices (engine.EngineGroup),
    # taken by rank 0 after every rank-per-GPU measurement while the other ranks wait on a CPU
    # (gloo) barrier with their buffers freed: reported beside `value`, never as it
    if ctx.world > 1 and not args.no_in_process:
        if ctx.local is not None:  # a GPU rank (the stub's ranks hold CPU tensors)
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
        cpu_grp = ctx.dmod.new_group(backend="gloo")
        ctx.dmod.barrier(group=cpu_grp)
        if ctx.rank == 0:
            try:
                res["in_process"] = inproc_results(args, ctx.world)
            except Exception as e:  # noqa: BLE001 - the rank-per-GPU line stands on its own
                res["in_process"] = {"error": f"{type(e).__name__}: {e}"}
        ctx.dmod.barrier(group=cpu_grp)
    if ctx.rank == 0:
        print(json.dumps(res), flush=True)


# ---------------------------------------------------------------- BASELINE configs[3] (C4)
C4_CHUNKS, C4_CHUNK, C4_K, C4_M = 65536, 65536, 10, 14
C4_ERASED = (0, 2, 5, 7)  # block 9 (zfec's padded last data block) survives and is read in place


def c4_share(rank: int, world: int, nchunks: int = C4_CHUNKS) -> tuple[int, int]:
    """This rank's contiguous chunk range of the C4 job (storb_amd.dist.partition by bytes)."""
    from storb_amd import dist as D

    return D.partition([C4_CHUNK] * nchunks, world)[rank]


def c4_pstride(B: int, palign: int) -> int:
    """Parity row stride: B rounded up to a multiple of palign (1: packed)."""
    palign = max(int(palign), 1)
    return -(-B // palign) * palign


def c4_run(eng, dmod, rank, world, local, device, sync, steps, warmup, nchunks=C4_CHUNKS, verify=True,
           keep=False, palign=128):
    """C4 as BASELINE.json writes it: `nchunks` x 64 KiB RS(10,4) chunks split over the ranks
    (contiguous ranges, no data-path collective); each rank encodes its share on its device,
    parity rows `palign`-aligned (B rounded up).  Returns this rank's numbers plus the job's
    aggregate (max-over-ranks time, summed chunks).  `eng` needs encode_batch / decode_batch /
    sync / set_timing / collect_timing (the product Engine; tests drive it with the oracle)."""
    import torch

    from storb_amd import dist as D

    lo, hi = c4_share(rank, world, nchunks)
    nch, n, k, m = hi - lo, C4_CHUNK, C4_K, C4_M
    B = -(-n // k)
    ps = c4_pstride(B, palign)
    g = torch.Generator(device=device)
    g.manual_seed(4_000_003 + lo)  # seed 4, per share
    src = torch.randint(0, 256, (max(nch * n, 1),), dtype=torch.uint8, device=device, generator=g)
    ed, _ = enc_descs(nch, n, k, m, ps)
    par = torch.empty(max(nch * (m - k) * ps, 1), dtype=torch.uint8, device=device)
    out = torch.empty_like(src)
    dd, sn, offs, av = dec_descs(nch, n, k, m, B, src.data_ptr(), par.data_ptr(), C4_ERASED, ps)

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
    counts = D.gather_counts(dmod, nch, rank, world, local)
    res = {"lo": lo, "hi": hi, "chunks": nch, "B": B, "pstride": ps, "el_max": el_max, "total_chunks": sum(counts),
           "per_rank_chunks": counts, "enc_avg_s": enc_avg_s, "enc_launches": enc_n, "dec_avg_s": dec_avg_s,
           "dec_launches": dec_n}
    if keep:  # the buffers, for tests that compare samples against the oracle
        res.update(src=src, par=par)
    return res


def c4_result(args, ctx, cpu_seconds, steps, warmup):
    """BASELINE configs[3] measured on every rank; rank 0 gets the line's dict (else None)."""
    r = c4_run(ctx.eng, ctx.dmod, ctx.rank, ctx.world, ctx.local, ctx.device, ctx.sync, steps, warmup,
               nchunks=args.c4_chunks, palign=args.c4_palign)
    n, k, m, B = C4_CHUNK, C4_K, C4_M, r["B"]
    job_bytes = r["total_chunks"] * n
    value = steps * job_bytes / r["el_max"] / GIB
    enc_alg = r["chunks"] * (n + (m - k) * B)
    dec_alg = r["chunks"] * (k * B + n)
    if ctx.rank != 0:
        return None
    enc_gbs = _gbs(enc_alg, r["enc_avg_s"])
    bs_off = hasattr(ctx.eng, "option") and ctx.eng.option("SEC_BS") == 0
    kernel = "sec_encode_kernel<4, 1, false>" if bs_off else "sec_encode_bs_kernel<10, 14, 0, 4, 5>"  # api.cpp bs_shape
    # the committed PMC summary applies to the configuration it was taken on (full job, N = 1,
    # this parity alignment)
    traffic = None
    if (ctx.world, args.c4_chunks, r["pstride"]) == (1, C4_CHUNKS, c4_pstride(B, 128)):
        traffic = load_traffic("encode", "c4")
    res = {
        "metric": "GiB/s device-resident RS(10,4) encode, 65536 x 64 KiB chunks sharded across N MI355X",
        "value": round(value, 3), "unit": "GiB/s", "n_gpus": ctx.world, "steps": steps,
        "warmup": warmup, "ms_per_step": round(r["el_max"] / steps * 1e3, 4),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (torch.randint uniform bytes, seed 4 per share), HBM-resident",
        "config": {"workload": f"BASELINE configs[3]: {r['total_chunks']} x 64 KiB chunks, RS(k=10,m=4)="
                               "zfec(10,14), B = 6554, padlen 4, encode; chunks split by "
                               "storb_amd.dist.partition over the ranks, no data-path collective",
                   "chunks_total": r["total_chunks"], "per_rank_chunks": r["per_rank_chunks"],
                   "parity_stride": r["pstride"], "world_size": ctx.world, "backend": ctx.backend,
                   "parallelism": f"chunk-partition x{ctx.world}"},
        "roofline": {"bound": "hbm", "achieved": enc_gbs, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": round(enc_gbs / PEAK_HBM_GBS, 4) if enc_gbs else None, "traffic": traffic,
                     "kernel": kernel, "algorithmic_bytes_per_launch": enc_alg,
                     "avg_launch_ms": round(r["enc_avg_s"] * 1e3, 4), "launches": r["enc_launches"]},
        "decode_kernel": {"achieved": _gbs(dec_alg, r["dec_avg_s"]), "unit": "GB/s",
                          "erased": list(C4_ERASED), "block_9": "read in place, avail = B - padlen",
                          "traffic": traffic and load_traffic("decode", "c4"),
                          "algorithmic_bytes_per_launch": dec_alg,
                          "avg_launch_ms": round(r["dec_avg_s"] * 1e3, 4), "launches": r["dec_launches"]},
        "cpu_baseline": None,
    }
    if ctx.world == 1 and cpu_seconds > 0:
        res["cpu_baseline"] = cpu_baseline(cpu_seconds, [C4_CHUNK] * 16, C4_K, C4_M, C4_ERASED, decode=False,
                                           what="RS(10,4) encode of 64 KiB chunks (B = 6554, padlen 4)")
    return res


def main_c4(args, ctx):
    res = c4_result(args, ctx, 0 if args.no_cpu else args.cpu_seconds, args.steps, args.warmup)
    if res is not None:
        print(json.dumps(res), flush=True)


# ---------------------------------------------------------------- BASELINE configs[4] (C5)
C5_K, C5_M = 8, 11
C5_ERASED = (1, 3, 5)  # three data blocks lost; block 7 (zfec's padded one) read in place


def c5_sizes(total: int = 1 << 30) -> list[int]:
    """BASELINE configs[4] chunk sizes: log-uniform integers in [4 KiB, 4 MiB], seed 5, ~`total`."""
    r5 = np.random.default_rng(5)
    sizes, tot = [], 0
    while tot < total:
        s = int(np.exp(r5.uniform(np.log(4096), np.log(4 << 20))))
        sizes.append(s)
        tot += s
    return sizes


def c5_run(ctx, steps, warmup, total=1 << 30, keep=False, staged=True, device_only=False):
    """C5 on this rank's share (contiguous chunk range balanced by bytes): the timed steps are
    encode + decode END TO END from pinned host buffers (host=True on Engine.host_empty memory:
    the kernels read the chunks and write parity / reassembled chunks over PCIe); then, outside
    the timed region, the same share device-resident (kernel rates from HIP events) and, with
    `staged`, from pageable buffers through the pinned slabs (SEC_REGISTER_MIN=0: explicit
    hipMemcpyAsync both ways).  Every path's output is checked against the input."""
    import torch

    from storb_amd import dist as D

    eng = ctx.eng
    k, m = C5_K, C5_M
    sizes_all = c5_sizes(total)
    lo, hi = D.partition(sizes_all, ctx.world)[ctx.rank]
    sizes = sizes_all[lo:hi]
    nbytes = int(np.sum(sizes))
    ed, B = enc_descs_var(sizes, k, m)
    npar = int(np.sum(B)) * (m - k)
    rng = np.random.default_rng(5_000_000 + lo)
    host = eng.host_empty(nbytes)
    host[:] = rng.integers(0, 256, nbytes, dtype=np.uint8)
    hpar, hout = eng.host_empty(max(npar, 1)), eng.host_empty(max(nbytes, 1))
    dd, sn, offs, av = dec_descs_var(sizes, k, m, B, host.ctypes.data, hpar.ctypes.data, C5_ERASED)

    def step():
        eng.encode_batch(ed, host, hpar, host=True)
        eng.decode_batch(dd, sn, offs, 0, hout, block_avail=av, host=True)

    el_max = float("nan")
    if not device_only:  # (device_only: rocprofv3 PMC passes of the device-resident kernels alone)
        for _ in range(warmup):
            step()
        if warmup and not np.array_equal(hout[:nbytes], host):
            raise SystemExit(f"bench c5: rank {ctx.rank} end-to-end round trip mismatch")
        el_max = timed_region(ctx.dmod, ctx.local, ctx.sync, steps, step)
        hout[:] = 0
        step()  # the last timed step's output, checked (a fast wrong answer is not a result)
        if not np.array_equal(hout[:nbytes], host):
            raise SystemExit(f"bench c5: rank {ctx.rank} end-to-end output mismatch")

    # device-resident, after the timed region
    src = torch.from_numpy(host).to(ctx.device)
    par = torch.empty(max(npar, 1), dtype=torch.uint8, device=ctx.device)
    out = torch.empty_like(src)
    ddd, dsn, doffs, dav = dec_descs_var(sizes, k, m, B, src.data_ptr(), par.data_ptr(), C5_ERASED)
    eng.encode_batch(ed, src, par)
    eng.decode_batch(ddd, dsn, doffs, 0, out, block_avail=dav)
    if not torch.equal(out, src):
        raise SystemExit(f"bench c5: rank {ctx.rank} device round trip mismatch")
    reps = max(steps, 5)
    eng.set_timing(True)
    for _ in range(reps):
        eng.encode_batch(ed, src, par, asynchronous=True)
    for _ in range(reps):
        eng.decode_batch(ddd, dsn, doffs, 0, out, block_avail=dav, asynchronous=True)
    eng.sync()
    eng.set_timing(False)
    enc_avg_s, enc_n = kernel_avg_s(eng, "encode")
    dec_avg_s, dec_n = kernel_avg_s(eng, "decode")
    res = {"lo": lo, "hi": hi, "sizes": sizes, "bytes": nbytes, "el_max": el_max, "enc_avg_s": enc_avg_s,
           "enc_launches": enc_n, "dec_avg_s": dec_avg_s, "dec_launches": dec_n,
           "enc_alg": nbytes + npar, "dec_alg": int(np.sum(B)) * k + nbytes,
           "job_bytes": int(D.sum_over_ranks(ctx.dmod, float(nbytes), ctx.local)),
           "per_rank_chunks": D.gather_counts(ctx.dmod, hi - lo, ctx.rank, ctx.world, ctx.local)}
    if staged:  # pageable buffers staged through the pinned slabs: explicit hipMemcpyAsync both ways
        pg = np.array(host)
        ppar, pout = np.empty(max(npar, 1), np.uint8), np.empty_like(pg)
        sdd, ssn, soffs, sav = dec_descs_var(sizes, k, m, B, pg.ctypes.data, ppar.ctypes.data, C5_ERASED)
        with eng.options(SEC_REGISTER_MIN=0):  # never page-lock: stage
            eng.encode_batch(ed, pg, ppar, host=True)
            t0 = time.perf_counter()
            for _ in range(3):
                eng.encode_batch(ed, pg, ppar, host=True)
            t1 = time.perf_counter()
            for _ in range(3):
                eng.decode_batch(sdd, ssn, soffs, 0, pout, block_avail=sav, host=True)
            t2 = time.perf_counter()
        if not np.array_equal(pout, pg):
            raise SystemExit(f"bench c5: rank {ctx.rank} staged round trip mismatch")
        res["staged_encode_gibs"] = round(3 * nbytes / (t1 - t0) / GIB, 2)
        res["staged_decode_gibs"] = round(3 * nbytes / (t2 - t1) / GIB, 2)
    if keep:
        res.update(src=src, par=par, host=host, hpar=hpar)
    return res


def c5_result(args, ctx, cpu_seconds, steps, warmup, staged=True):
    """BASELINE configs[4] measured on every rank; rank 0 gets the line's dict (else None)."""
    r = c5_run(ctx, steps, warmup, total=args.c5_bytes, staged=staged, device_only=args.c5_device_only)
    value = steps * 2 * r["job_bytes"] / r["el_max"] / GIB
    if ctx.rank != 0:
        return None
    enc_gbs, dec_gbs = _gbs(r["enc_alg"], r["enc_avg_s"]), _gbs(r["dec_alg"], r["dec_avg_s"])
    dom_dec = r["dec_avg_s"] >= r["enc_avg_s"]
    full = ctx.world == 1 and args.c5_bytes == 1 << 30  # the configuration the PMC summary is taken on
    res = {
        "metric": "GiB/s end-to-end RS(8,3) encode+decode of mixed 4 KiB-4 MiB chunks from pinned host memory, "
                  "N MI355X",
        "value": round(value, 3) if value == value else None, "unit": "GiB/s", "n_gpus": ctx.world,
        "steps": steps, "warmup": warmup,
        "ms_per_step": round(r["el_max"] / steps * 1e3, 4) if value == value else None,
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (numpy uniform bytes, seed 5 per share) in pinned host memory",
        "config": {"workload": f"BASELINE configs[4]: {sum(r['per_rank_chunks'])} chunks, sizes log-uniform in "
                               f"[4 KiB, 4 MiB] (seed 5), {r['job_bytes']} B, RS(k=8,m=3)=zfec(8,11): encode + "
                               "decode with data blocks {1,3,5} erased (block 7 read in place), host buffers "
                               "(pinned, zero-copy kernels over PCIe) in and out",
                   "job_bytes": r["job_bytes"], "per_rank_chunks": r["per_rank_chunks"], "world_size": ctx.world,
                   "backend": ctx.backend, "parallelism": f"chunk-partition x{ctx.world}"},
        # the kernels on HBM-resident copies of the same share (after the timed region)
        "roofline": {"bound": "hbm", "achieved": dec_gbs if dom_dec else enc_gbs, "peak": PEAK_HBM_GBS,
                     "unit": "GB/s",
                     "frac": (round((dec_gbs if dom_dec else enc_gbs) / PEAK_HBM_GBS, 4)
                              if (dec_gbs if dom_dec else enc_gbs) else None),
                     "traffic": load_traffic("decode" if dom_dec else "encode", "c5") if full else None,
                     "kernel": "sec_decode_kernel<3, 1, false, 0> (reassemble)" if dom_dec
                               else "sec_encode_kernel<3, 1, false>",
                     "algorithmic_bytes_per_launch": r["dec_alg"] if dom_dec else r["enc_alg"],
                     "avg_launch_ms": round((r["dec_avg_s"] if dom_dec else r["enc_avg_s"]) * 1e3, 4)},
        "device_resident": {"encode_GBs": enc_gbs, "encode_gibs": round(r["bytes"] / r["enc_avg_s"] / GIB, 2),
                            "decode_GBs": dec_gbs, "decode_gibs": round(r["bytes"] / r["dec_avg_s"] / GIB, 2),
                            "encode_ms": round(r["enc_avg_s"] * 1e3, 4), "decode_ms": round(r["dec_avg_s"] * 1e3, 4),
                            "encode_traffic": load_traffic("encode", "c5") if full else None,
                            "decode_traffic": load_traffic("decode", "c5") if full else None},
        "staged": ({"encode_gibs": r["staged_encode_gibs"], "decode_gibs": r["staged_decode_gibs"],
                    "path": "pageable numpy buffers staged through the library's pinned slabs (hipMemcpyAsync)"}
                   if "staged_encode_gibs" in r else None),
        "cpu_baseline": None,
    }
    if ctx.world == 1 and cpu_seconds > 0:
        sample = c5_sizes()[:64]
        res["cpu_baseline"] = cpu_baseline(cpu_seconds, sample, C5_K, C5_M, C5_ERASED,
                                           what=f"(encode + decode {{1,3,5}} erased) of the first 64 C5 chunks "
                                                f"({sum(sample)} B), RS(8,3)")
    return res


def main_c5(args, ctx):
    res = c5_result(args, ctx, 0 if args.no_cpu else args.cpu_seconds, args.steps, args.warmup,
                    staged=not args.no_e2e)
    if res is not None:
        print(json.dumps(res), flush=True)


# ---------------------------------------------------------------- host-buffer rates (headline line)
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
    with eng.options(SEC_REGISTER_MIN=0):  # never page-lock: stage
        senc, sdec = _e2e_pass(eng, host, par, out, nchunks, steps)
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


# ---------------------------------------------------------------- in-process multi-device (EngineGroup)
def _inproc_timed(grp, prep, body, steps, done=None):
    """The timed region of the in-process form: every worker prepares (warm-up, device sync) on
    its own thread, then all start together behind a thread barrier; the clock runs from the
    barrier until the LAST device has synchronised after its `steps` bodies.  Returns (elapsed
    seconds, per-worker results of `done`)."""
    import threading

    n = len(grp)
    states = [f.result() for f in [grp.submit(i, prep, i) for i in range(n)]]
    gate = threading.Barrier(n + 1)

    def run(i, st):
        gate.wait()
        for _ in range(steps):
            body(st)
        st["eng"].sync()
        return time.perf_counter()

    futs = [grp.submit(i, run, i, st) for i, st in enumerate(states)]
    gate.wait()
    t0 = time.perf_counter()
    t1 = max(f.result() for f in futs)
    res = [f.result() for f in [grp.submit(i, done, st) for i, st in enumerate(states)]] if done else None
    return t1 - t0, res


def inproc_c2c3(grp, steps, warmup, nchunks=N_CHUNKS, cpu=False) -> dict:
    """The headline workload on every device of `grp` from ONE process and one host thread per
    device (engine.EngineGroup): each device owns its own 1024 x 1 MiB
    RS(4,2) chunks (weak scaling, as the torchrun form); value = all devices' chunk bytes
    encoded + decoded / wall time of the slowest.  cpu: the tests' stub engines on CPU tensors."""
    import torch

    from storb_amd.engine import get_engine

    def prep(i):
        d = grp.devices[i]
        dev = "cpu" if cpu else f"cuda:{d}"
        if not cpu:
            torch.cuda.set_device(d)
        eng = get_engine()
        n, k, m = CHUNK, K, M
        g = torch.Generator(device=dev)
        g.manual_seed(1000 + i)
        src = torch.randint(0, 256, (nchunks * n,), dtype=torch.uint8, device=dev, generator=g)
        ed, B = enc_descs(nchunks, n, k, m)
        par = torch.empty(nchunks * (m - k) * B, dtype=torch.uint8, device=dev)
        out = torch.empty_like(src)
        dd, sn, offs, av = dec_descs(nchunks, n, k, m, B, src.data_ptr(), par.data_ptr(), ERASED)
        st = {"eng": eng, "ed": ed, "src": src, "par": par, "out": out, "dd": dd, "sn": sn, "offs": offs, "av": av}
        for _ in range(max(warmup, 1)):
            body(st)
        eng.sync()
        if not torch.equal(out, src):
            raise SystemExit(f"bench in-process: device {d} (worker {i}) round trip mismatch")
        return st

    def body(st):
        st["eng"].encode_batch(st["ed"], st["src"], st["par"], asynchronous=True)
        st["eng"].decode_batch(st["dd"], st["sn"], st["offs"], 0, st["out"], block_avail=st["av"], asynchronous=True)

    def done(st):
        for key in ("src", "par", "out"):
            st.pop(key)
        if not cpu:
            torch.cuda.empty_cache()

    el, _ = _inproc_timed(grp, prep, body, steps, done)
    nbytes = len(grp) * nchunks * 2 * CHUNK
    return {"value": round(steps * nbytes / el / GIB, 3), "unit": "GiB/s", "n_gpus": len(grp), "steps": steps,
            "ms_per_step": round(el / steps * 1e3, 4), "scaling": "weak", "devices": list(grp.devices),
            "workload": f"{nchunks} x 1 MiB chunks per GPU, RS(4,2): encode + {{1,3}}-erased decode/reassemble",
            "launch": "one process, one host thread + libstorbec context per device (engine.EngineGroup)"}


def inproc_c5(grp, steps, warmup, total=1 << 30) -> dict:
    """BASELINE configs[4] end to end from pinned host memory over every device of `grp`, one
    process: the job's chunks split by bytes (dist.partition), each device's share in pinned
    buffers its own context allocated, encoded + decoded over PCIe by its own worker thread
    (strong scaling, as the torchrun form)."""
    from storb_amd import dist as D
    from storb_amd.engine import get_engine

    sizes_all = c5_sizes(total)
    parts = D.partition(sizes_all, len(grp))
    k, m = C5_K, C5_M

    def prep(i):
        eng = get_engine()
        lo, hi = parts[i]
        sizes = sizes_all[lo:hi]
        nbytes = int(np.sum(sizes)) if sizes else 0
        st = {"eng": eng, "n": hi - lo, "bytes": nbytes}
        if not sizes:
            return st
        ed, B = enc_descs_var(sizes, k, m)
        npar = int(np.sum(B)) * (m - k)
        host = eng.host_empty(nbytes)
        host[:] = np.random.default_rng(5_000_000 + lo).integers(0, 256, nbytes, dtype=np.uint8)
        hpar, hout = eng.host_empty(max(npar, 1)), eng.host_empty(max(nbytes, 1))
        dd, sn, offs, av = dec_descs_var(sizes, k, m, B, host.ctypes.data, hpar.ctypes.data, C5_ERASED)
        st.update(ed=ed, host=host, hpar=hpar, hout=hout, dd=dd, sn=sn, offs=offs, av=av)
        for _ in range(max(warmup, 1)):
            body(st)
        if not np.array_equal(hout[:nbytes], host):
            raise SystemExit(f"bench in-process c5: worker {i} round trip mismatch")
        return st

    def body(st):
        if st["n"]:
            st["eng"].encode_batch(st["ed"], st["host"], st["hpar"], host=True)
            st["eng"].decode_batch(st["dd"], st["sn"], st["offs"], 0, st["hout"], block_avail=st["av"], host=True)

    def done(st):
        ok = (not st["n"]) or np.array_equal(st["hout"][:st["bytes"]], st["host"])
        for key in ("host", "hpar", "hout"):
            st.pop(key, None)
        return ok

    el, oks = _inproc_timed(grp, prep, body, steps, done)
    if not all(oks):
        raise SystemExit("bench in-process c5: output mismatch after the timed steps")
    job = int(np.sum(sizes_all))
    return {"value": round(steps * 2 * job / el / GIB, 3), "unit": "GiB/s", "n_gpus": len(grp), "steps": steps,
            "ms_per_step": round(el / steps * 1e3, 4), "scaling": "strong", "devices": list(grp.devices),
            "per_device_chunks": [hi - lo for lo, hi in parts],
            "workload": f"BASELINE configs[4]: {len(sizes_all)} chunks, {job} B, RS(8,3), encode + {{1,3,5}}-erased "
                        "decode from pinned host memory (zero-copy kernels over PCIe), split by bytes",
            "launch": "one process, one host thread + libstorbec context per device (engine.EngineGroup)"}


def inproc_devices(args, ndev) -> list[int]:
    if args.inproc_devices:
        devs = [int(x) for x in args.inproc_devices.split(",")]
        if len(devs) != ndev:
            raise SystemExit(f"bench: --inproc-devices names {len(devs)} devices, the run has {ndev}")
        return devs
    return list(range(ndev))


def _stub_factory():
    """STORB_BENCH_ENGINE's class (tests: the oracle behind the Engine interface), or None."""
    stub = os.environ.get("STORB_BENCH_ENGINE")
    if not stub:
        return None
    import importlib

    mod, cls = stub.split(":")
    return getattr(importlib.import_module(mod), cls)


def inproc_results(args, ndev) -> dict:
    from storb_amd.engine import EngineGroup

    stub = _stub_factory()
    grp = EngineGroup(inproc_devices(args, ndev), engine_factory=(lambda d: stub()) if stub else None)
    try:
        res = {"c2c3": inproc_c2c3(grp, args.steps, args.warmup, args.chunks, cpu=stub is not None)}
        if not args.no_c5:
            res["c5"] = inproc_c5(grp, args.c5_steps, min(args.warmup, 2), args.c5_bytes)
    finally:
        grp.close()
    return res


def main_in_process(args) -> None:
    """`--in-process`: the N devices from this one process (no ranks); one JSON line whose value
    is the in-process headline, with the in-process C5 line nested."""
    import torch

    n = args.gpus
    if _stub_factory() is None and max(inproc_devices(args, n)) >= torch.cuda.device_count():
        raise SystemExit(f"bench --in-process: devices {inproc_devices(args, n)} asked, "
                         f"{torch.cuda.device_count()} visible")
    r = inproc_results(args, n)
    h = r["c2c3"]
    res = {"metric": "GiB/s device-resident RS encode+decode, 1 MiB chunks, 1/2/4/8 MI355X",
           "value": h["value"], "unit": "GiB/s", "n_gpus": n, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": h["ms_per_step"], "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
           "dtype": "u8", "data": "synthetic (torch.randint uniform bytes, seeded per device), HBM-resident",
           "config": {"workload": h["workload"], "chunks_per_gpu": args.chunks, "world_size": 1,
                      "parallelism": f"in-process x{n} (engine.EngineGroup)", "launch": h["launch"]},
           "lib_digest": lib_digest(), "in_process": r}
    print(json.dumps(res), flush=True)


def main(argv=None):
    args = parse(argv)
    if args.in_process:
        if os.environ.get("WORLD_SIZE", "1") != "1":
            print("bench: --in-process runs as ONE process (not under torch.distributed.run)", file=sys.stderr)
            sys.exit(2)
        main_in_process(args)
        return
    rc = spawn_ranks(args, argv)
    if rc is not None:
        sys.exit(rc)
    ctx = rank_context(args)
    try:
        {"c2c3": main_c2c3, "c4": main_c4, "c5": main_c5}[args.workload](args, ctx)
    finally:
        finish(ctx)


if __name__ == "__main__":
    main()

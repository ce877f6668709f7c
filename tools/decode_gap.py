#!/usr/bin/env python3
"""why does the headline decode (sec_decode_kernel<2,1,false,0>,
1024 x 1 MiB RS(4,2), {1,3} erased, reassemble) time 0.342-0.358 ms inside bench.py's step but
0.328 ms in tools/bench_configs.py c3_patterns?

One process, one Engine, one set of buffers allocated as bench.c2c3_run does; the schedules
below run round-robin (`--rounds` times, `--reps` steps each) and report the median per-launch
kernel times from the library's HIP events (the same timer as the bench line):

  bench        encode, decode, encode, decode ...   (bench.c2c3_run's step)
  dec_only     decode, decode, ...                  (c3_patterns: back-to-back decodes)
  enc_only     encode, encode, ...
  dec_idle     decode, sync + 2 ms host sleep, ...  (nothing of an earlier kernel left in flight)
  enc_idle_dec encode, sync + sleep, decode, sync + sleep ...  (decode with encode's writes drained)
  dec_fresh    decode into a second output buffer, alternating with the first

    python tools/decode_gap.py [--rounds 5] [--reps 10] > gpurun_out/decode_gap.json
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--chunks", type=int, default=1024)
    ap.add_argument("--only", default="", help="comma list of schedules (default: all)")
    a = ap.parse_args()

    import torch

    import bench
    from storb_amd.engine import Engine

    eng = Engine(0)
    torch.cuda.set_device(0)
    nch, n, k, m = a.chunks, bench.CHUNK, bench.K, bench.M
    g = torch.Generator(device="cuda:0")
    g.manual_seed(1000)
    src = torch.randint(0, 256, (nch * n,), dtype=torch.uint8, device="cuda:0", generator=g)
    ed, B = bench.enc_descs(nch, n, k, m)
    par = torch.empty(nch * (m - k) * B, dtype=torch.uint8, device="cuda:0")
    out = torch.empty_like(src)
    out2 = torch.empty_like(src)
    dd, sn, offs, av = bench.dec_descs(nch, n, k, m, B, src.data_ptr(), par.data_ptr(), bench.ERASED)

    def enc():
        eng.encode_batch(ed, src, par, asynchronous=True)

    def dec(o=out):
        eng.decode_batch(dd, sn, offs, 0, o, block_avail=av, asynchronous=True)

    def idle():
        eng.sync()
        time.sleep(0.002)

    flip = [0]

    def dec_fresh():
        flip[0] ^= 1
        dec(out2 if flip[0] else out)

    schedules = {
        "bench": lambda: (enc(), dec()),
        "dec_only": dec,
        "enc_only": enc,
        "dec_idle": lambda: (dec(), idle()),
        "enc_idle_dec": lambda: (enc(), idle(), dec(), idle()),
        "dec_fresh": dec_fresh,
    }
    if a.only:
        schedules = {k_: v for k_, v in schedules.items() if k_ in a.only.split(",")}
    enc()
    dec()
    eng.sync()
    assert torch.equal(out, src), "round trip"
    samples = {s: {"encode": [], "decode": []} for s in schedules}
    for _ in range(a.rounds):
        for name, fn in schedules.items():
            for _ in range(2):  # untimed lead-in: the schedule's steady state
                fn()
            eng.sync()
            eng.set_timing(True)
            for _ in range(a.reps):
                fn()
            eng.sync()
            eng.set_timing(False)
            for kind in ("encode", "decode"):
                ms, nl = eng.collect_timing(kind)
                if nl:
                    samples[name][kind].append(ms / nl)
    enc_alg = nch * (n + (m - k) * B)
    dec_alg = nch * (k * B + n)
    res = {"config": f"{nch} x 1 MiB RS(4,2), decode {{1,3}} erased reassemble; median over {a.rounds} rounds of "
                     f"{a.reps} steps; per-launch HIP events (sec_ctx_set_timing)",
           "lib_digest": bench.lib_digest()}
    for name, s in samples.items():
        r = {}
        for kind, alg in (("encode", enc_alg), ("decode", dec_alg)):
            if s[kind]:
                t = float(np.median(s[kind]))
                r[f"{kind}_ms"] = round(t, 4)
                r[f"{kind}_ms_all"] = [round(x, 4) for x in s[kind]]
                r[f"{kind}_TBs"] = round(alg / (t / 1e3) / 1e12, 3)
        res[name] = r
    print(json.dumps(res, indent=1), flush=True)
    eng.close()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Runs one device-resident shape's encode + decode `--reps` times (for rocprofv3 kernel stats /
PMC passes).  Not product code.

    python tools/prof_shape.py --workload c4 --reps 20
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c4", help="c2 | c4 | nch,n,k,m")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import torch

    from bench import dec_descs, enc_descs
    from storb_amd.engine import Engine

    if a.workload == "c2":
        nch, n, k, m, erased = 1024, 1 << 20, 4, 6, (1, 3)
    elif a.workload == "c4":
        nch, n, k, m, erased = 8192, 65536, 10, 14, (0, 2, 5, 7)  # block 9 (padded) read in place
    else:
        nch, n, k, m = map(int, a.workload.split(","))
        erased = tuple(range(0, k, 2))[: m - k]
    eng = Engine(0)
    src = torch.randint(0, 256, (nch * n,), dtype=torch.uint8, device="cuda")
    ed, B = enc_descs(nch, n, k, m)
    par = torch.empty(nch * (m - k) * B, dtype=torch.uint8, device="cuda")
    out = torch.empty_like(src)
    dd, sn, offs, av = dec_descs(nch, n, k, m, B, src.data_ptr(), par.data_ptr(), erased)
    for _ in range(a.reps):
        eng.encode_batch(ed, src, par, asynchronous=True)
    for _ in range(a.reps):
        eng.decode_batch(dd, sn, offs, 0, out, block_avail=av, asynchronous=True)
    eng.sync()
    assert torch.equal(out, src)
    print("ok", a.workload, nch, n, k, m, "enc bytes/launch", nch * (n + (m - k) * B), "dec bytes/launch", nch * (k * B + n))
    eng.close()


if __name__ == "__main__":
    main()

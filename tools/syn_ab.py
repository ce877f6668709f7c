#!/usr/bin/env python3
"""A/B of the syndrome decode against the direct decode on wide shapes (one process, fresh
engine per variant, rounds interleaved), device-resident, reassemble and recover-only.

    python tools/syn_ab.py [--rounds 3] [--reps 5] > gpurun_out/syn_ab.jsonl

Rates are TB/s of algorithmic bytes: k*B read + n written (reassemble) or k*B + e*B
(recover-only), per HIP-event kernel time of the whole decode call (both phases).  Every
variant's output is checked against the source chunks.  Not product code.
"""

from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# (name, k, m, chunk bytes, chunks, lost data blocks)
CASES = [
    ("zfec(64,96) 256MiB x4, 16 lost", 64, 96, 256 << 20, 4, 16),
    ("zfec(64,96) 256MiB x4, 32 lost (every parity row)", 64, 96, 256 << 20, 4, 32),
    ("zfec(64,96) 1MiB x1024, 16 lost", 64, 96, 1 << 20, 1024, 16),
    ("zfec(64,96) 1MiB x1024, 32 lost (every parity row)", 64, 96, 1 << 20, 1024, 32),
    ("zfec(32,48) 1MiB x1024, 16 lost (every parity row)", 32, 48, 1 << 20, 1024, 16),
    ("zfec(32,48) 32MiB x32, 8 lost", 32, 48, 32 << 20, 32, 8),
    ("zfec(16,24) 8MiB x128, 8 lost (every parity row)", 16, 24, 8 << 20, 128, 8),
    ("zfec(16,24) 8MiB x128, 4 lost", 16, 24, 8 << 20, 128, 4),
    ("C4 zfec(10,14) 64KiB x8192, 4 lost", 10, 14, 65536, 8192, 4),
    # random lost data blocks and random present parity rows (seeded): what retrievals see
    ("zfec(64,96) 1MiB x1024, 16 lost (random, parity random)", 64, 96, 1 << 20, 1024, 16, 1),
    ("zfec(64,96) 1MiB x1024, 24 lost (random, parity random)", 64, 96, 1 << 20, 1024, 24, 2),
    ("zfec(64,96) 256MiB x4, 24 lost (random, parity random)", 64, 96, 256 << 20, 4, 24, 2),
    ("zfec(32,48) 1MiB x1024, 12 lost (random, parity random)", 32, 48, 1 << 20, 1024, 12, 3),
    ("zfec(32,48) 1MiB x1024, 16 lost (random)", 32, 48, 1 << 20, 1024, 16, 4),
    # every one of the m blocks fetched, a random 10-30 % of them lost (data and parity): the decode
    # from the first k present in block order (the reference's pieces[:k], piece.py:189-191) and
    # from the k sec_decode_choose picks; e = 0 is the lost-data count then
    ("zfec(64,96) 1MiB x1024, 20 % of blocks lost, first k", 64, 96, 1 << 20, 1024, 0, 11, 0.2, "first"),
    ("zfec(64,96) 1MiB x1024, 20 % of blocks lost, chosen k", 64, 96, 1 << 20, 1024, 0, 11, 0.2, "choose"),
    ("zfec(64,96) 1MiB x1024, 15 % of blocks lost, first k", 64, 96, 1 << 20, 1024, 0, 12, 0.15, "first"),
    ("zfec(64,96) 1MiB x1024, 15 % of blocks lost, chosen k", 64, 96, 1 << 20, 1024, 0, 12, 0.15, "choose"),
    ("zfec(64,96) 1MiB x1024, 30 % of blocks lost, first k", 64, 96, 1 << 20, 1024, 0, 13, 0.3, "first"),
    ("zfec(64,96) 1MiB x1024, 30 % of blocks lost, chosen k", 64, 96, 1 << 20, 1024, 0, 13, 0.3, "choose"),
    # parity group 0's low rows lost too (the first k present then span both groups)
    ("zfec(64,96) 1MiB x1024, 14 data + parity rows 64..73 lost, first k", 64, 96, 1 << 20, 1024, 0, 21, "g0low", "first"),
    ("zfec(64,96) 1MiB x1024, 14 data + parity rows 64..73 lost, chosen k", 64, 96, 1 << 20, 1024, 0, 21, "g0low", "choose"),
    ("zfec(32,48) 1MiB x1024, 20 % of blocks lost, first k", 32, 48, 1 << 20, 1024, 0, 14, 0.2, "first"),
    ("zfec(32,48) 1MiB x1024, 20 % of blocks lost, chosen k", 32, 48, 1 << 20, 1024, 0, 14, 0.2, "choose"),
]


def lost_fraction(k, m, seed, frac, how):
    """(lost data blocks, erased block numbers) for `frac` of the m blocks lost (seeded; each
    pattern holds >= k blocks), or (frac "g0low") 14 random data blocks and parity rows k .. k+9
    lost; the decoder keeps the first k present ("first") or sec_decode_choose's k ("choose")."""
    import random

    from storb_amd.engine import choose_blocks

    rng = random.Random(seed)
    if frac == "g0low":
        gone = set(rng.sample(range(k), 14)) | set(range(k, k + 10))
    else:
        while True:
            gone = set(rng.sample(range(m), int(round(frac * m))))
            if m - len(gone) >= k:
                break
    present = [j for j in range(m) if j not in gone]
    keep = present[:k] if how == "first" else [present[i] for i in choose_blocks(k, m, present)]
    lost = tuple(j for j in range(k) if j not in keep)
    return lost, tuple(j for j in range(m) if j not in keep)


def erased_of(k, m, e, seed):
    """The erased block numbers: e data blocks and m - k - e parity rows, both random (seed), or
    (seed 0) every other data block from 0 and the last parity rows."""
    import random

    if not seed:
        lost = tuple(range(0, 2 * e, 2)) if 2 * e <= k else tuple(range(e))
        return lost, lost
    rng = random.Random(seed)
    lost = tuple(sorted(rng.sample(range(k), e)))
    keep_par = set(rng.sample(range(k, m), e))
    return lost, lost + tuple(r for r in range(k, m) if r not in keep_par)


def main():
    import torch

    import bench
    from storb_amd.engine import Engine

    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--variants", default="direct@SEC_SYN=0,syn@SEC_SYN=1,auto",
                    help="name@OPT=V+OPT2=V2[/tag]: context options per variant, optionally a prebuilt variant library "
                         "build/variants/libstorbec_<tag>.so (storb_amd._build.build(defines=..., tag=...))")
    ap.add_argument("--cases", default="")
    ap.add_argument("--modes", default="reassemble,recover_only", help="decode modes to run (PMC passes: one)")
    ap.add_argument("--no-check", default="", help="comma list of variant names whose outputs are not checked "
                    "(calibration libraries)")
    a = ap.parse_args()
    variants = []  # (name, env, lib path or None); "name@ENV=V+ENV2=V2/tag": build/variants/libstorbec_<tag>.so
    for v in a.variants.split(","):
        v, _, tag = v.partition("/")
        name, _, env = v.partition("@")
        lib = __import__("storb_amd._build", fromlist=["x"]).variant_lib(tag) if tag else None
        variants.append((name, {kv.split("=")[0]: int(kv.split("=")[1]) for kv in env.split("+")} if env else {}, lib))
    sel = [c for c in CASES if not a.cases or any(t in c[0] for t in a.cases.split(";"))]
    for name, k, m, n, nch, e, *seed in sel:
        if len(seed) == 3:  # a fraction of all m blocks lost, first or chosen k
            lost, erased = lost_fraction(k, m, *seed)
            e = len(lost)
        else:
            lost, erased = erased_of(k, m, e, seed[0] if seed else 0)
        src = torch.randint(0, 256, (nch * n,), dtype=torch.uint8, device="cuda")
        B = -(-n // k)
        ed, _ = bench.enc_descs(nch, n, k, m)
        par = torch.empty(nch * (m - k) * B, dtype=torch.uint8, device="cuda")
        eng0 = Engine(0)
        eng0.encode_batch(ed, src, par)
        eng0.close()
        dd, sn, offs, av = bench.dec_descs(nch, n, k, m, B, src.data_ptr(), par.data_ptr(), erased)
        rd, rsn, roffs, rav = bench.dec_descs(nch, n, k, m, B, src.data_ptr(), par.data_ptr(), erased, recover=True)
        out = torch.empty_like(src)
        rec = torch.empty(nch * e * B, dtype=torch.uint8, device="cuda")
        res = {v[0]: {"reassemble": [], "recover_only": []} for v in variants}
        paths = {}
        for _ in range(a.rounds):
            for vname, env, lib in variants:
                eng = Engine(0, lib_path=lib, options=env)  # the variant's options (sec_ctx_set_option)
                for mode, args in (("reassemble", (dd, sn, offs, av, out, False)),
                                   ("recover_only", (rd, rsn, roffs, rav, rec, True))):
                    if mode not in a.modes.split(","):
                        continue
                    d_, s_, o_, a_, dst, recov = args
                    dst.zero_()
                    eng.decode_batch(d_, s_, o_, 0, dst, block_avail=a_, recover_only=recov)
                    if vname in a.no_check.split(","):
                        pass  # a calibration library (SEC_PROBE_NOGF): its outputs are not the data
                    elif not recov:
                        assert torch.equal(out, src), (name, vname)
                    else:  # recovered rows against the (zero-padded) source blocks
                        r3 = rec.view(nch, e, B)
                        s3 = torch.nn.functional.pad(src.view(nch, n), (0, k * B - n)).view(nch, k, B)
                        for j, blk in enumerate(lost):
                            assert torch.equal(r3[:, j], s3[:, blk]), (name, vname, blk)
                    eng.set_timing(True)
                    for _ in range(a.reps):
                        eng.decode_batch(d_, s_, o_, 0, dst, block_avail=a_, recover_only=recov, asynchronous=True)
                    eng.sync()
                    eng.set_timing(False)
                    ms, nl = eng.collect_timing("decode")
                    alg = nch * (k * B + (e * B if recov else n))
                    res[vname][mode].append(alg / (ms / 1e3 / a.reps) / 1e12)
                paths[vname] = eng.decode_paths()
                eng.close()
        row = {"case": name, "k": k, "m": m, "chunk": n, "chunks": nch, "lost": list(lost),
               "parity_kept": [s for s in sn[:k].tolist() if s >= k]}
        for vname, r in res.items():
            row[vname] = {mode: round(float(np.median(v)), 3) for mode, v in r.items() if v}
            row[vname]["paths(syn,direct)"] = paths.get(vname)
        print(json.dumps(row), flush=True)
        del src, par, out, rec
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

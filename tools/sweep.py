#!/usr/bin/env python3
"""Interleaved A/B sweep of kernel build variants x tile sizes, in ONE process on one GPU
(cdna_hip_programming.md §5.4 rule 24).  Not product code.

    python tools/sweep.py [--build] [--rounds 5] [--variants base,nt,...] [--us 1,2,4]
                          [--workload c2|c4]

Each variant is libstorbec_<tag>.so built with the -D knobs in VARIANTS; each (variant, U)
gets its own Engine (fresh plan).  Prints one JSON line per config: median / min encode and
decode kernel time (HIP events) and GB/s of algorithmic bytes.
"""

from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

VARIANTS = {
    # build knobs of kernels.hip / api.cpp that remain (each a measured design parameter; the
    # A/B-only knobs and their kernels are archived, tools/archive/README.md)
    "base": {},  # defaults: nontemporal loads + stores, 16-vector load batches
    "tmp": {"SEC_NT_LOAD": 0, "SEC_NT_STORE": 0},  # temporal (cached) loads and stores
    "decb8": {"SEC_DEC_BATCH": 8},  # default is 16: all slot loads up front for k * U <= 16
    # store cache policy (kernels.hip SEC_ENC_ST / SEC_DEC_ST: 0 plain, 1 nt, 2 nt sc1, 3 sc0 sc1)
    "dst2": {"SEC_DEC_ST": 2},
    "dst0": {"SEC_DEC_ST": 0},
    "est2": {"SEC_ENC_ST": 2},
    "est3": {"SEC_ENC_ST": 3},
    "est0": {"SEC_ENC_ST": 0},
    "est2dst2": {"SEC_ENC_ST": 2, "SEC_DEC_ST": 2},
    "dst3": {"SEC_DEC_ST": 3},
    # calibration: the product kernels' traffic with no GF arithmetic (outputs are not parity)
    "nogf": {"SEC_PROBE_NOGF": 1},
    "xcd": {"SEC_XCD_ORDER": 1},  # api.cpp: XCD order for every tile group (default off)
    "eb4": {"SEC_ENC_BATCH": 4},
    "eb8": {"SEC_ENC_BATCH": 8},
    "db8": {"SEC_DEC_BATCH": 8},  # decode KB = 8 / U (valid only for k * U <= 8)
    "db8eb8": {"SEC_DEC_BATCH": 8, "SEC_ENC_BATCH": 8},
    "b4": {"SEC_DEC_BATCH": 4, "SEC_ENC_BATCH": 4},  # KB = 4 / U: valid for k * U <= 4 only
    "decearly": {"SEC_DEC_LATE": 0},  # decode: copies stored as each slot arrives
    # wide k (W kernels): the earlier 16-vector batches without block pairs for 8-row groups;
    # 4-vector batches; pairs for 8-row groups in the k <= 16 kernels too
    "prevwide": {"SEC_WIDE_BATCH": 16, "SEC_WIDE_PAIR_ROWS": 4},
    "wb4": {"SEC_WIDE_BATCH": 4},
    "pair8": {"SEC_PAIR_ROWS": 8},
    "sha1nopf": {"SEC_SHA1_PF": 0},  # SHA-1 next-block prefetch off (default on)
    "sha1d1": {"SEC_SHA1_DEPTH": 1},  # prefetch depth in blocks (default 2)
    "sha1d3": {"SEC_SHA1_DEPTH": 3},
    # table dwords 1 and 3 from a per-wave LDS copy instead of v_mov from SGPRs (SEC_LDS_TAB)
    # (default 2: encode kernels of 8-row groups only; 1: every tile kernel; 0: none)
    "ldstab": {"SEC_LDS_TAB": 1},
    "noldstab": {"SEC_LDS_TAB": 0},
    # syndrome decode ring depths: phase 1 of the 16-row groups, phase 2 (solve), the fused kernel
    "synr4": {"SEC_SYN_RING": 4, "SEC_SOLVE_RING": 4},
    "fr2": {"SEC_FUSED_RING": 2},
    "fr4": {"SEC_FUSED_RING": 4},
    "lds6": {"SEC_FUSED_LDS_RING": 6},
}


def build(tags):
    """tag -> library; a tag "prev" is build/variants/libstorbec_prev.so as it lies (an earlier
    build kept for an A/B against the current sources), never rebuilt."""
    from storb_amd import _build

    libs = {t: _build.build(defines=VARIANTS[t], tag=t) for t in tags if t != "prev"}
    if "prev" in tags:
        libs["prev"] = _build.variant_lib("prev")
    return libs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--variants", default="base,tmp")
    ap.add_argument("--us", default="1,2,4")
    ap.add_argument("--palign", type=int, default=1, help="parity stride rounded up to this many bytes")
    ap.add_argument("--workload", default="c2", help="c2 | c4 | nch,n,k,m (custom shape)")
    ap.add_argument("--recover", action="store_true", help="also time recover-only decodes (not c5)")
    ap.add_argument("--erased", default="", help="erased block numbers, e.g. 1,3 (not c5; default per workload)")
    a = ap.parse_args()
    # a variant is TAG or TAG@OPT=VALUE[+OPT2=V2]: the TAG build, with those context options
    # (sec_ctx_set_option) on its engine
    specs = a.variants.split(",")
    tags = sorted({v.split("@")[0] for v in specs})
    libs = build(tags)
    if a.build:
        return
    import torch

    from bench import dec_descs, enc_descs
    from storb_amd.engine import Engine

    if a.workload == "c5":  # BASELINE configs[4]: mixed sizes, as tools/bench_configs.py
        from tools.bench_configs import c5_sizes, dec_descs_var, enc_descs_var

        sizes, k, m, erased = c5_sizes(), 8, 11, (1, 3, 5)
        total = int(np.sum(sizes))
        src = torch.randint(0, 256, (total,), dtype=torch.uint8, device="cuda")
        ed, Bs = enc_descs_var(sizes, k, m)
        par = torch.empty(int(np.sum(Bs)) * (m - k), dtype=torch.uint8, device="cuda")
        out = torch.empty_like(src)
        dd, sn, offs, av = dec_descs_var(sizes, k, m, Bs, src.data_ptr(), par.data_ptr(), erased)
        enc_bytes = total + int(np.sum(Bs)) * (m - k)
        dec_bytes = int(np.sum(Bs)) * k + total
    else:
        if a.workload == "c2":
            nch, n, k, m, erased = 1024, 1 << 20, 4, 6, (1, 3)
        elif a.workload == "c4":  # per-GPU share: 8192 x 64 KiB RS(10,4)
            nch, n, k, m, erased = 8192, 65536, 10, 14, (0, 2, 5, 7)  # block 9 (padded) in place
        else:
            nch, n, k, m = map(int, a.workload.split(","))
            erased = tuple(range(0, k, 2))[: m - k]
        if a.erased:
            erased = tuple(int(x) for x in a.erased.split(","))
        src = torch.randint(0, 256, (nch * n,), dtype=torch.uint8, device="cuda")
        B = -(-n // k)
        ps = -(-B // a.palign) * a.palign
        ed, B = enc_descs(nch, n, k, m, ps)
        par = torch.zeros(nch * (m - k) * ps, dtype=torch.uint8, device="cuda")
        out = torch.empty_like(src)
        dd, sn, offs, av = dec_descs(nch, n, k, m, B, src.data_ptr(), par.data_ptr(), erased, ps)
        enc_bytes = nch * (n + (m - k) * B)
        dec_bytes = nch * (k * B + n)
        if a.recover:  # SEC_F_RECOVER: the e missing primaries only, e * B per chunk
            ne = sum(1 for s in erased if s < k)
            rd, rsn, roffs, rav = dec_descs(nch, n, k, m, B, src.data_ptr(), par.data_ptr(), erased, ps, recover=True)
            rec = torch.empty(nch * ne * B, dtype=torch.uint8, device="cuda")
            rec_bytes = nch * (k + ne) * B
    recov = a.recover and a.workload != "c5"

    configs = [(v, int(u)) for v in specs for u in a.us.split(",")]
    engines = {}
    for v, u in configs:
        t, _, env = v.partition("@")
        # the variant's options hold on its own engine (sec_ctx_set_option) for every call
        opts = {"SEC_TILE_U": u}
        for kv in filter(None, env.split("+")):
            opts[kv.split("=")[0]] = int(kv.split("=")[1])
        e = Engine(0, lib_path=libs[t], options=opts)
        out.zero_()
        e.encode_batch(ed, src, par, asynchronous=True)
        e.decode_batch(dd, sn, offs, 0, out, block_avail=av, asynchronous=True)
        if recov:
            e.decode_batch(rd, rsn, roffs, 0, rec, block_avail=rav, recover_only=True, asynchronous=True)
        e.sync()
        assert torch.equal(out, src), (v, u)
        engines[(v, u)] = e
    samples = {c: ([], [], []) for c in configs}

    for _ in range(a.rounds):
        for c in configs:
            e = engines[c]
            e.set_timing(True)
            for _ in range(a.reps):
                e.encode_batch(ed, src, par, asynchronous=True)
            for _ in range(a.reps):
                e.decode_batch(dd, sn, offs, 0, out, block_avail=av, asynchronous=True)
            e.sync()
            e.set_timing(False)
            ms, nl = e.collect_timing("encode")
            samples[c][0].append(ms / nl)
            ms, nl = e.collect_timing("decode")
            samples[c][1].append(ms / nl)
            if recov:
                e.set_timing(True)
                for _ in range(a.reps):
                    e.decode_batch(rd, rsn, roffs, 0, rec, block_avail=rav, recover_only=True, asynchronous=True)
                e.sync()
                e.set_timing(False)
                ms, nl = e.collect_timing("decode")
                samples[c][2].append(ms / nl)
    # the timed calls must have produced the same bytes (a fast wrong kernel is not a result)
    ref_par = par.clone()
    engines[configs[0]].encode_batch(ed, src, ref_par, asynchronous=True)
    engines[configs[0]].sync()
    bad = set()
    if recov:
        ref_rec = rec.clone()
    for c in configs:
        if recov:
            rec.zero_()
            engines[c].decode_batch(rd, rsn, roffs, 0, rec, block_avail=rav, recover_only=True, asynchronous=True)
            engines[c].sync()
            if not torch.equal(rec, ref_rec):
                bad.add(c)
        out.zero_()
        par.zero_()
        engines[c].encode_batch(ed, src, par, asynchronous=True)
        engines[c].decode_batch(dd, sn, offs, 0, out, block_avail=av, asynchronous=True)
        engines[c].sync()
        if not (torch.equal(par, ref_par) and torch.equal(out, src)):
            bad.add(c)
    for c in configs:
        enc, dec = np.array(samples[c][0]), np.array(samples[c][1])
        extra = {}
        if recov:
            rv = np.array(samples[c][2])
            extra = {"rec_ms_med": round(float(np.median(rv)), 4), "rec_GBs": round(rec_bytes / np.median(rv) / 1e6, 1)}
        print(json.dumps({"variant": c[0], "U": c[1], "workload": a.workload, "palign": a.palign,
                          **({"erased": a.erased} if a.erased else {}),
                          "enc_ms_med": round(float(np.median(enc)), 4), "enc_GBs": round(enc_bytes / np.median(enc) / 1e6, 1),
                          "enc_GBs_best": round(enc_bytes / enc.min() / 1e6, 1),
                          "dec_ms_med": round(float(np.median(dec)), 4), "dec_GBs": round(dec_bytes / np.median(dec) / 1e6, 1),
                          "dec_GBs_best": round(dec_bytes / dec.min() / 1e6, 1),
                          **extra, "verified": c not in bad}), flush=True)


if __name__ == "__main__":
    main()

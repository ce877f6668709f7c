#!/usr/bin/env python3
"""Instruction counts of XOR schedules for the bit-sliced zfec(k, m) encode.

The bit-sliced kernel (storb_amd/csrc/kernels_bs.hip, sec_encode_bs2_kernel) computes, per wave
and 16-row group, 128 output planes (16 parity rows x 8 bits) from 512 input planes (64 blocks x
8 bits): output plane (r, i) is the XOR of the input planes (j, s) where bit i of c[r][j] * alpha^s
is set.  Its schedule is a "four Russians" one: per block the XORs of every subset of planes 0-3
(lo) and 4-7 (hi) (only the subsets some row reads: <= 11 + 11 XOR2), then per output plane one
v_bitop3 XOR3 `acc ^= lo[mask & 15] ^ hi[mask >> 4]` (an XOR2 when one half is empty).

This tool counts that schedule's VALU per group, and the two common-subexpression schedules the
verdict asked to try, all in instructions of gfx950's VALU (XOR2 or XOR3 = 1 instruction):

  terms : greedy pair sharing (Paar) over the (block, half, nibble-subset) terms the four-Russians
          schedule XORs into each output, i.e. CSE on top of the current schedule;
  bits  : greedy Paar over the raw 512 x 128 GF(2) matrix, outputs then folded into XOR3 chains.

Each greedy step takes the pair of variables present in the most outputs (ties: lowest index),
adds their XOR as a new variable (1 instruction) and substitutes it; it stops when no pair is
shared by two outputs.  An output with t remaining variables then costs ceil((t - 1) / 2) XOR3s.
The counts exclude the 8x8 transposes (48 VALU per block in, 48 per parity row out) that every
schedule shares.  Not product code; nothing here runs on the GPU.

    python tools/xor_schedule.py [--k 64 --m 96] [--rows 16] [--json out.json]
"""

from __future__ import annotations

import argparse
import json
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import zfec_ref  # noqa: E402  (test infrastructure: the matrix zfec builds)


def bit_matrix(coefs: np.ndarray) -> np.ndarray:
    """coefs (R x K) GF(2^8) -> (8R x 8K) GF(2) matrix: row 8r + i, column 8j + s is bit i of
    coefs[r][j] * alpha^s (alpha = 2 in zfec's field)."""
    R, K = coefs.shape
    out = np.zeros((8 * R, 8 * K), dtype=np.uint8)
    for r in range(R):
        for j in range(K):
            c = int(coefs[r, j])
            for s in range(8):
                v = zfec_ref.gf_mul(c, 1 << s)
                for i in range(8):
                    out[8 * r + i, 8 * j + s] = (v >> i) & 1
    return out


def four_russians(mat: np.ndarray) -> dict:
    """The current kernel's schedule: per block the live lo / hi subsets, then one XOR3 (or XOR2)
    per (output, block) with a nonzero mask."""
    n_out, n_in = mat.shape
    K = n_in // 8
    sub = acc = 0
    for j in range(K):
        cols = mat[:, 8 * j:8 * j + 8]
        lo = cols[:, :4] @ (1 << np.arange(4))
        hi = cols[:, 4:] @ (1 << np.arange(4))
        for half in (lo, hi):
            live = {int(v) for v in half if v}
            # s[1], s[2], s[4], s[8] are the planes; every other live subset is one XOR2 (its
            # prefix subset is live or computed on the way: count the closure)
            need = set()
            for v in live:
                while bin(v).count("1") > 1:
                    need.add(v)
                    v &= v - 1  # drop the lowest bit: s[v] = s[v & (v-1)] ^ plane
            sub += len(need)
        both = (lo != 0) & (hi != 0)
        one = (lo != 0) ^ (hi != 0)
        acc += int(both.sum()) + int(one.sum())
    # the first block of a row initialises acc (no XOR with 0): 1 fewer per output, roughly
    return {"subsets": sub, "accumulate": acc, "total": sub + acc}


MIN_SHARE = 2


def paar(rows: list[set], n_vars: int, max_steps: int = 1 << 20) -> tuple[int, list[set]]:
    """Greedy pair sharing over outputs given as sets of variable ids; returns (new XOR2s,
    remaining rows).  A pair is taken while it is shared by >= MIN_SHARE outputs (2: Paar's XOR2
    rule; with XOR3 accumulation a pair saves about half an instruction per use, so 3 or more is
    the break-even)."""
    rows = [set(r) for r in rows]
    n = n_vars
    steps = 0
    # incidence as a dense 0/1 matrix over the variables in use; recomputed counts per step
    while steps < max_steps:
        used = sorted(set().union(*rows))
        idx = {v: i for i, v in enumerate(used)}
        M = np.zeros((len(rows), len(used)), dtype=np.float32)
        for r, s in enumerate(rows):
            for v in s:
                M[r, idx[v]] = 1.0
        C = M.T @ M
        np.fill_diagonal(C, 0)
        best = float(C.max())
        if best < MIN_SHARE:
            break
        a, b = np.unravel_index(int(np.argmax(C)), C.shape)
        va, vb = used[a], used[b]
        new = n
        n += 1
        for s in rows:
            if va in s and vb in s:
                s.discard(va)
                s.discard(vb)
                s.add(new)
        steps += 1
    return steps, rows


def xor3_fold(rows: list[set]) -> int:
    return sum(math.ceil(max(len(s) - 1, 0) / 2) for s in rows)


def terms_schedule(mat: np.ndarray) -> dict:
    """Paar over the four-Russians terms: variable (j, half, v) for v != 0."""
    n_out, n_in = mat.shape
    K = n_in // 8
    ids = {}
    rows = [set() for _ in range(n_out)]
    for j in range(K):
        cols = mat[:, 8 * j:8 * j + 8]
        lo = cols[:, :4] @ (1 << np.arange(4))
        hi = cols[:, 4:] @ (1 << np.arange(4))
        for h, half in enumerate((lo, hi)):
            for o, v in enumerate(half):
                if v:
                    rows[o].add(ids.setdefault((j, h, int(v)), len(ids)))
    base = four_russians(mat)["subsets"]
    before = xor3_fold(rows)
    shared, rest = paar(rows, len(ids))
    after = xor3_fold(rest)
    return {"subsets": base, "accumulate_before": before, "shared_xor2": shared, "accumulate_after": after,
            "total_before": base + before, "total_after": base + shared + after}


def window_schedule(mat: np.ndarray, window: int) -> dict:
    """Paar over the terms of `window` consecutive blocks at a time (the sharing a kernel that holds
    that many blocks' subsets in registers could use), each output accumulated per window as
    ceil(t_w / 2) XOR3s (acc ^ a ^ b; no term carried across windows)."""
    n_out, n_in = mat.shape
    K = n_in // 8
    before = shared = after = 0
    for w0 in range(0, K, window):
        ids = {}
        rows = [set() for _ in range(n_out)]
        for j in range(w0, min(K, w0 + window)):
            cols = mat[:, 8 * j:8 * j + 8]
            lo = cols[:, :4] @ (1 << np.arange(4))
            hi = cols[:, 4:] @ (1 << np.arange(4))
            for h, half in enumerate((lo, hi)):
                for o, v in enumerate(half):
                    if v:
                        rows[o].add(ids.setdefault((j, h, int(v)), len(ids)))
        before += sum(math.ceil(len(r) / 2) for r in rows)
        n, rest = paar(rows, len(ids))
        shared += n
        after += sum(math.ceil(len(r) / 2) for r in rest)
    base = four_russians(mat)["subsets"]
    return {"window": window, "accumulate_before": before, "shared_xor2": shared, "accumulate_after": after,
            "total_before": base + before, "total_after": base + shared + after}


def bits_schedule(mat: np.ndarray) -> dict:
    rows = [set(np.nonzero(mat[o])[0].tolist()) for o in range(mat.shape[0])]
    naive = xor3_fold(rows)
    shared, rest = paar(rows, mat.shape[1])
    return {"naive_xor3": naive, "shared_xor2": shared, "fold_after": xor3_fold(rest),
            "total_after": shared + xor3_fold(rest)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=64)
    ap.add_argument("--m", type=int, default=96)
    ap.add_argument("--rows", type=int, default=16, help="parity rows per group (one wave's outputs)")
    ap.add_argument("--groups", default="", help="comma list of groups (default all)")
    ap.add_argument("--bits", action="store_true", help="also the raw-bit Paar (slow: minutes per group)")
    ap.add_argument("--windows", default="2,4,8", help="block windows for window_schedule")
    ap.add_argument("--no-global", action="store_true", help="skip the global terms Paar (minutes per group)")
    ap.add_argument("--min-share", type=int, default=2)
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    global MIN_SHARE
    MIN_SHARE = a.min_share
    par = zfec_ref.parity_rows(a.k, a.m)
    P = a.m - a.k
    groups = [int(g) for g in a.groups.split(",")] if a.groups else list(range(P // a.rows))
    res = {"k": a.k, "m": a.m, "rows_per_group": a.rows, "groups": []}
    for g in groups:
        mat = bit_matrix(par[g * a.rows:(g + 1) * a.rows])
        row = {"group": g, "density": round(float(mat.mean()), 4), "four_russians": four_russians(mat)}
        for w in (int(x) for x in a.windows.split(",") if x):
            row[f"window_{w}"] = window_schedule(mat, w)
        if not a.no_global:
            row["terms_paar"] = terms_schedule(mat)
        if a.bits:
            row["bits_paar"] = bits_schedule(mat)
        res["groups"].append(row)
        print(json.dumps(row), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()

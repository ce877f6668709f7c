#!/usr/bin/env python3
"""F4: APDP throughput on one MI355X (bignum.hip) beside the reference's arithmetic restated
on one CPU core (oracle/apdp_ref.py, CPython pow — gmpy2 is absent from this image).

    python tools/bench_apdp.py [--pieces 4096] [--piece-bytes 262144] > gpurun_out/apdp.json

Cases (all with one RSA-2048 key, device-resident inputs unless noted):
  reduce       piece mod n over `pieces` pieces                  (GB/s of piece bytes)
  modexp       base^e mod n, 2048-bit exponents                  (modexps/s)
  crt_modexp   the same powers by CRT over p, q (the key owner)  (modexps/s)
  gpow         g^e from the fixed-base table (challenges' g^s)   (pows/s)
  tag          generate_tag fused: reduce + table g^X + d power, without / with CRT (tags/s)
  proofs / verifies through storb_amd.apdp.ChallengeSystem from host memory (items/s)
`mad_frac` = algorithmic 32x32->64 multiply-adds (8192 per 2048-bit Montgomery product)
over the measured v_mad_u64_u32 ceiling.
"""

from __future__ import annotations

import argparse
import json
import os
import random
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


MAD_PEAK = 3.367e13  # measured v_mad_u64_u32 lane-ops/s per MI355X (tools/mad_ceiling.hip)


def kernel_ms(eng, fn, reps):
    fn()
    eng.sync()
    eng.collect_timing("bignum")
    eng.set_timing(True)
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    eng.sync()
    wall = (time.perf_counter() - t0) / reps
    eng.set_timing(False)
    ms, n = eng.collect_timing("bignum")
    return ms / max(n, 1), wall


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pieces", type=int, default=4096)
    ap.add_argument("--piece-bytes", type=int, default=262144)
    ap.add_argument("--modexps", type=int, default=16384)
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--quick", action="store_true", help="kernels only (no CPU baseline / API legs)")
    args = ap.parse_args()

    import torch

    from oracle import apdp_ref
    from storb_amd import apdp, bn
    from storb_amd._lib import MSG_DTYPE
    from storb_amd.engine import get_engine

    eng = get_engine(0)
    n, e, d, p, q = apdp_ref.test_key(21)
    g = pow(7, 2, n)
    prf_key = b"bench-prf-key"
    fdh = apdp_ref.full_domain_hash(n, apdp_ref.prf(prf_key, 0))
    mk = bn.ModKey(n, eng)  # public key only: no CRT
    mk.set_tag(g, fdh, d)
    mc = bn.ModKey(n, eng)  # key owner: CRT over p, q
    mc.set_crt(p, q)
    mc.set_tag(g, fdh, d)
    res = {"key_bits": 2048, "pieces": args.pieces, "piece_bytes": args.piece_bytes}

    P, L = args.pieces, args.piece_bytes
    src = torch.randint(0, 256, (P * L,), dtype=torch.uint8, device="cuda")
    msgs = np.zeros(P, dtype=MSG_DTYPE)
    msgs["addr"] = src.data_ptr() + np.arange(P, dtype=np.uint64) * L
    msgs["len"] = L
    msgs["avail"] = L
    out = torch.empty(P * 256, dtype=torch.uint8, device="cuda")
    host = src[:L].cpu().numpy().tobytes()

    ms, wall = kernel_ms(eng, lambda: mk.reduce_batch(msgs, out, asynchronous=True), 5)
    res["reduce"] = {"kernel_ms": round(ms, 3), "GBs": round(P * L / ms / 1e6, 1),
                     "mont_mul_per_s": round(P * (L // 256) / ms * 1e3, 0),
                     "mad_frac": round(P * (L // 256) * 8192 / ms * 1e3 / MAD_PEAK, 3)}
    assert bn.from_be(out[:256].cpu().numpy())[0] == int.from_bytes(host, "big") % n

    M = args.modexps
    rng = np.random.default_rng(1)
    bases = torch.from_numpy(rng.integers(0, 256, (M, 256), dtype=np.uint8)).cuda()
    exps = torch.from_numpy(rng.integers(0, 256, (M, 256), dtype=np.uint8)).cuda()
    exps[:, 0] |= 0x80
    mo = torch.empty(M * 256, dtype=torch.uint8, device="cuda")
    ms, wall = kernel_ms(eng, lambda: mk.modexp_batch(bases, exps, 256, M, mo, asynchronous=True), 3)
    b0 = int.from_bytes(bases[0].cpu().numpy().tobytes(), "big")
    e0 = int.from_bytes(exps[0].cpu().numpy().tobytes(), "big")
    assert bn.from_be(mo[:256].cpu().numpy())[0] == pow(b0, e0, n)
    mm = M * (2048 + 512 + 16)  # Montgomery products of a 4-bit-window 2048-bit power
    res["modexp_2048bit_exp"] = {"count": M, "kernel_ms": round(ms, 3), "modexps_per_s": round(M / ms * 1e3, 0),
                                 "mad_frac": round(mm * 8192 / ms * 1e3 / MAD_PEAK, 3)}

    # the same powers by CRT (exponents reduced per factor on the host)
    hexps = [int.from_bytes(exps[i].cpu().numpy().tobytes(), "big") for i in range(M)]
    ep = torch.from_numpy(bn.to_be([bn.ModKey._half_exp(x, p - 1) for x in hexps], 128)).cuda()
    eq = torch.from_numpy(bn.to_be([bn.ModKey._half_exp(x, q - 1) for x in hexps], 128)).cuda()
    ms, wall = kernel_ms(eng, lambda: mc.crt_modexp_batch(bases, ep, eq, 128, M, mo, asynchronous=True), 3)
    assert bn.from_be(mo[:256].cpu().numpy())[0] == pow(b0, e0, n)
    res["crt_modexp_2048bit_exp"] = {"count": M, "kernel_ms": round(ms, 3), "modexps_per_s": round(M / ms * 1e3, 0)}

    ms, wall = kernel_ms(eng, lambda: mc.gpow_batch(exps, 256, M, mo, asynchronous=True), 3)
    assert bn.from_be(mo[:256].cpu().numpy())[0] == pow(g, e0, n)
    res["gpow_fixed_base_2048bit_exp"] = {"count": M, "kernel_ms": round(ms, 3),
                                          "pows_per_s": round(M / ms * 1e3, 0)}

    expect_tag = apdp_ref.tag_value(n, g, d, prf_key, host)
    for label, key in (("tag_fused", mk), ("tag_fused_crt", mc)):
        ms, wall = kernel_ms(eng, lambda: key.tag_batch(msgs, out, asynchronous=True), 2)
        assert bn.from_be(out[:256].cpu().numpy())[0] == expect_tag
        res[label] = {"kernel_ms": round(ms, 3), "tags_per_s": round(P / ms * 1e3, 1),
                      "piece_GBs": round(P * L / ms / 1e6, 2)}

    if args.quick:
        print(json.dumps(res))
        return
    # CPU: the reference's generate_tag arithmetic restated (CPython pow), one core
    cpu_rng = random.Random(3)
    cnt, t_start = 0, time.perf_counter()
    while time.perf_counter() - t_start < args.cpu_seconds:
        apdp_ref.tag_value(n, g, d, prf_key, cpu_rng.randbytes(L))
        cnt += 1
    cpu_t = (time.perf_counter() - t_start) / cnt
    res["cpu_baseline_tag"] = {"tags_per_s": round(1 / cpu_t, 2), "cores": 1, "kind": "port",
                               "sample": f"{cnt} tags of {L} B pieces, CPython pow (gmpy2 absent)"}
    res["tag_speedup_vs_cpu_core"] = round(res["tag_fused_crt"]["tags_per_s"] * cpu_t, 1)

    # end-to-end through the drop-in API, host memory
    cs = apdp.ChallengeSystem()
    cs.key.rsa = apdp.RSAPrivateKey(p, q, e)
    cs.key.g = g
    cs.key.prf_key = prf_key
    K = min(P, 1024)
    datas = [os.urandom(L) for _ in range(K)]
    # the first call of a key also derives it on the device (Montgomery constants, CRT halves,
    # g's 16 MiB fixed-base table); a validator pays that once per key, so the steady state is
    # timed separately (second call, same key)
    t = time.perf_counter()
    tags = cs.generate_tags(datas)
    t_first = time.perf_counter() - t
    t = time.perf_counter()
    tags = cs.generate_tags(datas)
    t_tag = time.perf_counter() - t
    t = time.perf_counter()
    chs = cs.issue_challenges(tags)
    t_ch = time.perf_counter() - t
    pr_items = list(zip(datas, tags, chs))
    cs.generate_proofs(pr_items[:8])  # the challenge moduli's keys are derived per call thread
    t = time.perf_counter()
    proofs = cs.generate_proofs(pr_items)
    t_pr = time.perf_counter() - t
    t = time.perf_counter()
    ok = cs.verify_proofs(list(zip(proofs, chs, tags)))
    t_ver = time.perf_counter() - t
    assert all(ok)
    res["api_host"] = {"items": K, "piece_bytes": L, "generate_tags_first_call_per_s": round(K / t_first, 1),
                       "generate_tags_per_s": round(K / t_tag, 1), "issue_challenges_per_s": round(K / t_ch, 1),
                       "generate_proofs_per_s": round(K / t_pr, 1), "verify_proofs_per_s": round(K / t_ver, 1)}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()

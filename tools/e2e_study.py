#!/usr/bin/env python3
"""Where the PCIe-inclusive (host-buffer) path loses time, and what a pinned caller buffer buys.

Not product code: a measurement tool for DESIGN.md's end-to-end numbers.  Prints one JSON object:
  link_*          torch pinned <-> device copies of 1 GiB (H2D, D2H, both directions at once on two
                  streams): the PCIe ceiling the e2e path is measured against
  staged_*        the library's SEC_F_HOST path from pageable numpy buffers (copy pool -> pinned
                  slabs -> H2D -> kernels -> D2H -> copy pool), C2 encode / C3 decode
  zerocopy_*      the device-mode kernels pointed straight at pinned host memory (sec_host_alloc):
                  the kernels read and write the host buffers over PCIe, no copies at all
All rates are GiB/s of chunk bytes (1024 x 1 MiB RS(4,2), data shards {1,3} erased for decode).
"""

from __future__ import annotations

import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

GIB = float(1 << 30)


def timed(fn, reps=3):
    fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t0) / reps


def link_rates():
    import torch

    n = 1 << 30
    h1 = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    h2 = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    d1 = torch.empty(n, dtype=torch.uint8, device="cuda")
    d2 = torch.empty(n, dtype=torch.uint8, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def h2d():
        d1.copy_(h1, non_blocking=True)
        torch.cuda.synchronize()

    def d2h():
        h2.copy_(d2, non_blocking=True)
        torch.cuda.synchronize()

    def both():
        with torch.cuda.stream(s1):
            d1.copy_(h1, non_blocking=True)
        with torch.cuda.stream(s2):
            h2.copy_(d2, non_blocking=True)
        torch.cuda.synchronize()

    return {"link_h2d_gibs": round(n / timed(h2d) / GIB, 2), "link_d2h_gibs": round(n / timed(d2h) / GIB, 2),
            "link_bidir_gibs_each_way": round(n / timed(both) / GIB, 2)}


def host_buf(eng, nbytes):
    """Pinned host memory from the library (hipHostMalloc), as a numpy array."""
    p = ctypes.c_void_p()
    rc = eng.lib.sec_host_alloc(eng._ctx, nbytes, ctypes.byref(p))
    assert rc == 0, rc
    arr = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(p.value))
    return arr, p


def main():
    import torch

    from bench import CHUNK, ERASED, K, M, N_CHUNKS, dec_descs, enc_descs
    from storb_amd.engine import Engine

    eng = Engine(0)
    res = link_rates()
    n = N_CHUNKS * CHUNK
    ed, B = enc_descs(N_CHUNKS, CHUNK, K, M)
    rng = np.random.default_rng(7)

    # staged (pageable caller memory)
    host = rng.integers(0, 256, n, dtype=np.uint8)
    par = np.empty(N_CHUNKS * (M - K) * B, dtype=np.uint8)
    out = np.empty_like(host)
    dd, sn, offs, _av = dec_descs(N_CHUNKS, CHUNK, K, M, B, host.ctypes.data, par.ctypes.data, ERASED)
    te = timed(lambda: eng.encode_batch(ed, host, par, host=True))
    td = timed(lambda: eng.decode_batch(dd, sn, offs, 0, out, host=True))
    assert np.array_equal(out, host)
    res["staged_encode_gibs"] = round(n / te / GIB, 2)
    res["staged_decode_gibs"] = round(n / td / GIB, 2)
    ref_par = par.copy()

    # zero-copy: kernels on pinned host memory
    hin, pin_in = host_buf(eng, n)
    hpar, pin_par = host_buf(eng, par.size)
    hout, pin_out = host_buf(eng, n)
    hin[:] = host
    dd2, sn2, offs2, _av2 = dec_descs(N_CHUNKS, CHUNK, K, M, B, pin_in.value, pin_par.value, ERASED)
    te = timed(lambda: eng.encode_batch(ed, pin_in.value, pin_par.value))
    res["zerocopy_encode_gibs"] = round(n / te / GIB, 2)
    res["zerocopy_encode_ok"] = bool(np.array_equal(hpar, ref_par))
    td = timed(lambda: eng.decode_batch(dd2, sn2, offs2, 0, pin_out.value))
    res["zerocopy_decode_gibs"] = round(n / td / GIB, 2)
    res["zerocopy_decode_ok"] = bool(np.array_equal(hout, host))
    for p in (pin_in, pin_par, pin_out):
        eng.lib.sec_host_free(eng._ctx, p)

    # page-locking pageable buffers on the fly: what one register + unregister of the C2
    # input (1 GiB) costs, and the zero-copy rate on registered memory
    t0 = time.perf_counter()
    eng.register(host)
    t1 = time.perf_counter()
    eng.register(par)
    eng.register(out)
    res["register_1GiB_ms"] = round((t1 - t0) * 1e3, 2)
    te = timed(lambda: eng.encode_batch(ed, host, par, host=True))
    td = timed(lambda: eng.decode_batch(dd, sn, offs, 0, out, host=True))
    res["registered_encode_gibs"] = round(n / te / GIB, 2)
    res["registered_decode_gibs"] = round(n / td / GIB, 2)
    res["registered_ok"] = bool(np.array_equal(out, host))
    res["registered_paths"] = eng.host_paths()
    t0 = time.perf_counter()
    eng.unregister(host)
    res["unregister_1GiB_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
    eng.unregister(par)
    eng.unregister(out)
    torch.cuda.synchronize()
    print(json.dumps(res), flush=True)
    eng.close()


if __name__ == "__main__":
    main()

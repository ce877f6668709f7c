"""Builds libstorbec.so in-tree with hipcc for gfx950 (no JIT cache, no pip install).

The .so lands in storb_amd/lib/ (git-ignored) so it travels with the repo snapshot to the
GPU box.  A stamp of the source hashes skips rebuilds when nothing changed.
"""

from __future__ import annotations

import hashlib
import os
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIBDIR = os.path.join(PKG, "lib")
LIB = os.path.join(LIBDIR, "libstorbec.so")
INCLUDE = os.path.join(ROOT, "include")
SOURCES = ["kernels.hip", "kernels_bs.hip", "bignum.hip", "api.cpp"]
HEADERS = ["kernels.hpp", "bignum.hpp", "gf_host.hpp", "gf_const.hpp", "copy_pool.hpp"]
# gfx950 (MI355X) only: the kernels use gfx950 instructions (16-byte global_load_lds, v_bitop3)
# and up to 160 KiB of LDS per workgroup; kernels_bs.hip stops any other target with #error
ARCH = "gfx950"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _digest() -> str:
    h = hashlib.sha256()
    for name in SOURCES + HEADERS:
        with open(os.path.join(CSRC, name), "rb") as f:
            h.update(name.encode() + f.read())
    with open(os.path.join(INCLUDE, "storb_ec.h"), "rb") as f:
        h.update(f.read())
    h.update(ARCH.encode())
    return h.hexdigest()


def build(force: bool = False, verbose: bool = False, defines: dict | None = None, tag: str | None = None) -> str:
    """Compile libstorbec.so (or, with `tag`, an A/B variant libstorbec_<tag>.so built with
    extra -D `defines`, used by tools/sweep.py)."""
    os.makedirs(LIBDIR, exist_ok=True)
    lib = LIB if not tag else os.path.join(LIBDIR, f"libstorbec_{tag}.so")
    defs = [f"-D{k}={v}" for k, v in sorted((defines or {}).items())]
    stamp = lib + ".stamp"
    dig = _digest() + " ".join(defs)
    if not force and os.path.exists(lib) and os.path.exists(stamp):
        with open(stamp) as f:
            if f.read().strip() == dig:
                return lib
    tmp = lib + ".tmp"
    # one hipcc per source, in parallel (the device code of each file is compiled on its own
    # anyway), then one link
    objdir = os.path.join(LIBDIR, "obj_" + (tag or "lib"))
    os.makedirs(objdir, exist_ok=True)
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function",
             f"-I{INCLUDE}", *defs]
    objs, procs = [], []
    for src in SOURCES:
        obj = os.path.join(objdir, src + ".o")
        objs.append(obj)
        cmd = [HIPCC, *flags, "-c", os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd))
        procs.append((src, subprocess.Popen(cmd)))
    failed = [src for src, p in procs if p.wait() != 0]
    if failed:
        raise RuntimeError(f"hipcc failed on {', '.join(failed)}")
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-fPIC", "-shared", "-o", tmp, *objs]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(tmp, lib)
    with open(stamp, "w") as f:
        f.write(dig)
    return lib


if __name__ == "__main__":
    print(build(force=True, verbose=True))

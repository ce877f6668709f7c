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
# A/B and calibration builds (tools/sweep.py): outside the package, so the product's lib/ holds
# only the library the product loads
VARIANT_DIR = os.path.join(ROOT, "build", "variants")
INCLUDE = os.path.join(ROOT, "include")
SOURCES = ["kernels.hip", "kernels_bs.hip", "bignum.hip", "api.cpp"]
HEADERS = ["kernels.hpp", "bignum.hpp", "gf_host.hpp", "gf_const.hpp", "task_pool.hpp"]
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


def _read(path: str) -> str | None:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def _includes(path: str, seen: set) -> None:
    """The local headers `path` includes, transitively (csrc/ and include/)."""
    with open(path, encoding="utf-8", errors="replace") as f:
        for line in f:
            line = line.strip()
            if line.startswith("#include \""):
                name = line.split("\"")[1]
                for d in (CSRC, INCLUDE):
                    h = os.path.join(d, name)
                    if os.path.exists(h) and h not in seen:
                        seen.add(h)
                        _includes(h, seen)


_COMPILER_ID: str | None = None


def _compiler_id() -> str:
    """The compiler an object was built with (HIPCC and its --version), part of the object key:
    a ROCm upgrade or another HIPCC must not link old objects into a new library."""
    global _COMPILER_ID
    if _COMPILER_ID is None:
        try:
            out = subprocess.run([HIPCC, "--version"], capture_output=True, text=True, timeout=60).stdout
        except (OSError, subprocess.SubprocessError) as e:
            out = f"unavailable: {e}"
        _COMPILER_ID = HIPCC + "\n" + out
    return _COMPILER_ID


def _obj_key(src: str, flags: list) -> str:
    path = os.path.join(CSRC, src)
    deps: set = set()
    _includes(path, deps)
    h = hashlib.sha256(_compiler_id().encode() + b"\0" + " ".join(flags).encode())
    for p in [path, *sorted(deps)]:
        with open(p, "rb") as f:
            h.update(p.encode() + f.read())
    return h.hexdigest()


def variant_lib(tag: str) -> str:
    """Where the A/B variant `tag` (build(defines=..., tag=tag)) lies."""
    return os.path.join(VARIANT_DIR, f"libstorbec_{tag}.so")


def build(force: bool = False, verbose: bool = False, defines: dict | None = None, tag: str | None = None) -> str:
    """Compile libstorbec.so (or, with `tag`, an A/B variant libstorbec_<tag>.so built with
    extra -D `defines`, used by tools/sweep.py)."""
    lib = LIB if not tag else variant_lib(tag)
    os.makedirs(os.path.dirname(lib), exist_ok=True)
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
    objdir = os.path.join(os.path.dirname(lib), "obj_" + (tag or "lib"))
    os.makedirs(objdir, exist_ok=True)
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function",
             f"-I{INCLUDE}", *defs]
    objs, procs = [], []
    for src in SOURCES:
        obj = os.path.join(objdir, src + ".o")
        objs.append(obj)
        # an object is rebuilt only when its source, a header it includes or the flags changed
        # (kernels_bs.hip alone takes minutes; an api.cpp edit should not recompile it)
        key = _obj_key(src, flags)
        if not force and os.path.exists(obj) and _read(obj + ".key") == key:
            continue
        for stale in (obj, obj + ".key"):  # a failed compile must leave no object its key matches
            if os.path.exists(stale):
                os.remove(stale)
        cmd = [HIPCC, *flags, "-c", os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd))
        procs.append((src, obj, key, subprocess.Popen(cmd)))
    failed = [src for src, _, _, p in procs if p.wait() != 0]
    if failed:
        raise RuntimeError(f"hipcc failed on {', '.join(failed)}")
    for _, obj, key, _ in procs:
        with open(obj + ".key", "w") as f:
            f.write(key)
    # libcrypto: OpenSSL's SHA-1 for the host piece ids of sec_encode_pieces (task_pool.hpp)
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-fPIC", "-shared", "-o", tmp, *objs, "-lcrypto"]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(tmp, lib)
    with open(stamp, "w") as f:
        f.write(dig)
    return lib


if __name__ == "__main__":
    print(build(force=True, verbose=True))

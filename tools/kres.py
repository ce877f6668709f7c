#!/usr/bin/env python3
"""Static resource usage and instruction mix of the tile kernels for build-knob variants
(cross-compiled here, no GPU).  Not product code.

    python tools/kres.py [-DKNOB=V ...] [--filter REGEX] [--mix]

Prints per kernel: VGPRs, SGPRs, occupancy (waves/SIMD), static LDS, spills; with --mix the
top VALU / LDS / scalar-memory instruction counts of each matching kernel's body.
"""

from __future__ import annotations

import argparse
import collections
import os
import re
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "storb_amd", "csrc", "kernels.hip")


def demangle(n: str) -> str:
    m = re.search(r"(sec_\w+?kernel)ILi(\d+)ELi(\d+)ELb(\d)E", n)
    if m:
        return f"{m.group(1)}<{m.group(2)},{m.group(3)},{'true' if m.group(4) == '1' else 'false'}>"
    m = re.search(r"(sec_\w+)", n)
    return m.group(1) if m else n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("defs", nargs="*")
    ap.add_argument("--filter", default=r"encode_kernel|decode_kernel")
    ap.add_argument("--mix", action="store_true")
    ap.add_argument("--src", default=SRC, help="kernel source (default storb_amd/csrc/kernels.hip)")
    a, extra = ap.parse_known_args()
    a.defs += extra
    with tempfile.TemporaryDirectory() as td:
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", f"-I{ROOT}/include",
               "--save-temps", "-c", os.path.abspath(a.src), "-o", os.path.join(td, "k.o"),
               "-Rpass-analysis=kernel-resource-usage", *a.defs]
        p = subprocess.run(cmd, cwd=td, capture_output=True, text=True, check=True)
        rows, cur = [], None
        for line in p.stderr.splitlines():
            m = re.search(r"remark: (.*?) \[-Rpass", line)
            if not m:
                continue
            t = re.sub(r"^\S+:\d+:\d+:\s*", "", m.group(1))
            if t.startswith("Function Name:"):
                cur = {"name": t.split(":", 1)[1].strip()}
                rows.append(cur)
            elif cur is not None and ":" in t:
                k, v = t.split(":", 1)
                cur[k.strip()] = v.strip()
        stem = os.path.splitext(os.path.basename(a.src))[0]
        asm = open(os.path.join(td, f"{stem}-hip-amdgcn-amd-amdhsa-gfx950.s")).read()
    for r in rows:
        nm = demangle(r["name"])
        if not re.search(a.filter, nm):
            continue
        print(f"{nm:40s} vgpr {r.get('VGPRs', '?'):>4s} sgpr {r.get('SGPRs', '?'):>4s} "
              f"occ {r.get('Occupancy [waves/SIMD]', '?'):>2s} lds {r.get('LDS Size [bytes/block]', '?'):>5s} "
              f"vspill {r.get('VGPRs Spill', '?')} sspill {r.get('SGPRs Spill', '?')}")
        if a.mix:
            i = asm.find(r["name"] + ":")
            j = asm.find(".Lfunc_end", i)
            c = collections.Counter()
            for ln in asm[i:j].splitlines():
                ln = ln.strip()
                if ln and not ln.startswith((".", ";", "_")):
                    c[ln.split()[0]] += 1
            print("   ", ", ".join(f"{k} {v}" for k, v in c.most_common(14)))


if __name__ == "__main__":
    main()

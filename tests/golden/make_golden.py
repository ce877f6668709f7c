"""Generates tests/golden/golden.json from the CPU oracle (oracle/zfec_ref.py, cross-checked
against oracle/fec_oracle.c before anything is written).

    python tests/golden/make_golden.py

Label: "restatement-derived; UNPINNED against real zfec 1.6.0.0 bytes" — zfec is not
available in this environment and the reference (/root/reference/storb/util/piece_test.py)
holds no known-answer vectors.  What the fixture pins is this repo's oracle at the time it
was generated, so later changes to either oracle or the kernels cannot drift silently.

Inputs are ``random.Random(seed).randbytes(n)`` — the reference's own tests draw their data
with ``random.randbytes`` (piece_test.py:19,49,84), here seeded.
"""

from __future__ import annotations

import hashlib
import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import cfec, zfec_ref  # noqa: E402

SHAPES = [(1, 2), (2, 3), (3, 5), (4, 6), (8, 11), (8, 12), (10, 14), (16, 24), (32, 48), (64, 96), (5, 256)]
SIZES = [1, 63, 1000, 4096, 6554 * 10 - 4, 65536, 100003, 262144 + 17]
POLICY_SIZES = [1, 1000, 4096, 16384, 65536, 131072, 262144, 524288, 1 << 20, 4 << 20, 16 << 20, 64 << 20,
                256 << 20, 1 << 30, 16 << 30, 1 << 40]
DECODE_CASES = [  # (k, m, sharenums)
    (2, 3, [0, 2]), (2, 3, [2, 1]), (4, 6, [0, 2, 4, 5]), (4, 6, [5, 4, 3, 1]), (4, 6, [4, 1, 5, 3]),
    (8, 11, [10, 1, 2, 3, 9, 5, 6, 8]), (10, 14, [0, 1, 2, 3, 4, 5, 10, 11, 12, 13]),
    (10, 14, [13, 12, 11, 10, 9, 8, 7, 6, 5, 4]), (16, 24, list(range(8, 24))),
]


def sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


def valid(n: int, k: int) -> bool:
    B = -(-n // k)
    return k == 1 or (k - 1) * B <= n


def main() -> None:
    out = {"label": "restatement-derived; UNPINNED against real zfec 1.6.0.0 bytes",
           "generator": "tests/golden/make_golden.py", "matrices": {}, "encode": [], "decode": [], "policy": []}
    for k, m in SHAPES:
        rows = zfec_ref.parity_rows(k, m)
        c = cfec.encode_matrix(k, m)[k * k:]
        assert rows.tobytes() == c, (k, m)
        out["matrices"][f"{k},{m}"] = [bytes(r).hex() for r in rows]
    for k, m in SHAPES:
        for n in SIZES:
            if not valid(n, k) or (k >= 32 and n > 70000):
                continue
            seed = n * 1000 + k * 7 + m
            data = random.Random(seed).randbytes(n)
            blocks = zfec_ref.easy_encode(data, k, m)
            assert blocks == cfec.easy_encode(data, k, m), (k, m, n)
            ent = {"k": k, "m": m, "n": n, "seed": seed, "B": len(blocks[0]),
                   "blocks_sha256": [sha(b) for b in blocks]}
            if n <= 1000:
                ent["parity_hex"] = [b.hex() for b in blocks[k:]]
            out["encode"].append(ent)
    for k, m, sn in DECODE_CASES:
        dm, idx = None, None
        slots, idx = zfec_ref.normalise([b"x"] * k, sn, k, m)
        dm = zfec_ref.decode_matrix(k, m, idx)
        n = 4096 * k - 3
        seed = 77 + k + m
        data = random.Random(seed).randbytes(n)
        blocks = zfec_ref.easy_encode(data, k, m)
        B = len(blocks[0])
        pad = B * k - n
        got = zfec_ref.easy_decode([blocks[s] for s in sn], sn, pad, k, m)
        assert got == data and cfec.easy_decode([blocks[s] for s in sn], sn, pad, k, m) == data
        out["decode"].append({"k": k, "m": m, "sharenums": sn, "normalised": idx,
                              "decode_matrix": [bytes(r).hex() for r in dm], "n": n, "seed": seed,
                              "out_sha256": sha(data)})
    for size in POLICY_SIZES:
        chunk = zfec_ref.piece_length(size)
        nch = -(-size // chunk)
        k, m, B, pad = zfec_ref.chunk_shape(min(chunk, size))
        out["policy"].append({"file_size": size, "chunk": chunk, "chunks": nch, "k": k, "m": m, "B": B,
                              "padlen": pad, "piece": zfec_ref.piece_length(min(chunk, size))})
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(f"wrote {path}: {len(out['encode'])} encode, {len(out['decode'])} decode vectors")


if __name__ == "__main__":
    main()

"""Python/numpy restatement of zfec 1.6.0.0 (easyfec + _fec) — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker.  The product (``storb_amd``) never does.

PARITY STATUS: "parity unpinned" against real zfec bytes.  zfec (pinned
``zfec==1.6.0.0`` at /root/reference/uv.lock:1088-1091, imported at
/root/reference/storb/util/piece.py:8) is not vendored or installed here and the
reference tests hold no known-answer vectors (storb/util/piece_test.py:48-125 only
assert round-trip identity).  This twin builds the encode matrix by a route
independent of ``oracle/fec_oracle.c``:

* here:  ``tmp[k:] @ inv(tmp[:k])`` with a generic Gauss–Jordan inverse — the
  construction zfec's ``fec_new`` performs (seed Vandermonde on points 0, 1, a, a^2, ...)
* C:     closed-form Lagrange basis ``L_j(x_r)``

and ``tests/test_oracle.py`` asserts the two agree for every shape in the configs.

Reference call sites restated:
  easyfec.Encoder(k, m).encode(data)          storb/util/piece.py:129-130
  easyfec.Decoder(k, m).decode(b, s, padlen)  storb/util/piece.py:196-197
"""

from __future__ import annotations

import numpy as np

POLY = 0x11D  # x^8+x^4+x^3+x^2+1, zfec Pp="101110001"


def _tables():
    exp = np.zeros(510, dtype=np.uint8)
    log = np.zeros(256, dtype=np.int32)
    v = 1
    for e in range(255):
        exp[e] = v
        exp[e + 255] = v
        log[v] = e
        v <<= 1
        if v & 0x100:
            v ^= POLY
    log[0] = 255
    a = np.arange(256)
    mul = exp[(log[a][:, None] + log[a][None, :]) % 255].astype(np.uint8)
    mul[0, :] = 0
    mul[:, 0] = 0
    inv = np.zeros(256, dtype=np.uint8)
    inv[1:] = exp[255 - log[1:]]
    return exp, log, mul, inv


EXP, LOG, MUL, INV = _tables()


def gf_mul(a: int, b: int) -> int:
    return int(MUL[a, b])


def gf_matmul(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """GF(2^8) matrix product (uint8)."""
    out = np.zeros((a.shape[0], b.shape[1]), dtype=np.uint8)
    for t in range(a.shape[1]):
        out ^= MUL[a[:, t][:, None], b[t, :][None, :]]
    return out


def gf_invert(a: np.ndarray) -> np.ndarray:
    """Gauss–Jordan inverse over GF(2^8); raises ValueError if singular."""
    k = a.shape[0]
    w = np.concatenate([a.astype(np.uint8), np.eye(k, dtype=np.uint8)], axis=1)
    for c in range(k):
        nz = np.nonzero(w[c:, c])[0]
        if nz.size == 0:
            raise ValueError("singular matrix")
        piv = c + int(nz[0])
        if piv != c:
            w[[c, piv]] = w[[piv, c]]
        w[c] = MUL[INV[w[c, c]], w[c]]
        for r in range(k):
            f = w[r, c]
            if r != c and f:
                w[r] ^= MUL[f, w[c]]
    return w[:, k:].copy()


def seed_matrix(k: int, m: int) -> np.ndarray:
    """zfec fec_new's seed: row 0 = [1,0..0], row r>=1 = alpha^((r-1)*c mod 255)."""
    tmp = np.zeros((m, k), dtype=np.uint8)
    tmp[0, 0] = 1
    for r in range(1, m):
        for c in range(k):
            tmp[r, c] = EXP[((r - 1) * c) % 255]
    return tmp


def encode_matrix(k: int, m: int) -> np.ndarray:
    """Full m x k systematic encode matrix (identity on top)."""
    if not (1 <= k <= m <= 256):
        raise ValueError(f"bad (k, m) = ({k}, {m})")
    tmp = seed_matrix(k, m)
    enc = np.zeros((m, k), dtype=np.uint8)
    enc[:k] = np.eye(k, dtype=np.uint8)
    if m > k:
        enc[k:] = gf_matmul(tmp[k:], gf_invert(tmp[:k]))
    return enc


def parity_rows(k: int, m: int) -> np.ndarray:
    return encode_matrix(k, m)[k:]


def _addmul_rows(coef: np.ndarray, blocks: np.ndarray) -> np.ndarray:
    """out[r] = XOR_j coef[r, j] * blocks[j]   (zfec addmul over whole blocks)."""
    out = np.zeros((coef.shape[0], blocks.shape[1]), dtype=np.uint8)
    for r in range(coef.shape[0]):
        for j in range(coef.shape[1]):
            c = coef[r, j]
            if c:
                out[r] ^= MUL[c][blocks[j]]
    return out


def split_blocks(data: bytes, k: int) -> tuple[np.ndarray, int]:
    """easyfec split: k slices of B = ceil(n/k), the last zero-padded."""
    n = len(data)
    B = -(-n // k)
    if k > 1 and (k - 1) * B > n:
        raise ValueError("Precondition violation: Input blocks are required to be all the same length.")
    buf = np.zeros(k * B, dtype=np.uint8)
    buf[:n] = np.frombuffer(bytes(data), dtype=np.uint8)
    return buf.reshape(k, B), k * B - n


def easy_encode(data: bytes, k: int, m: int) -> list[bytes]:
    """zfec.easyfec.Encoder(k, m).encode(data) -> m blocks."""
    enc = encode_matrix(k, m)
    blocks, _ = split_blocks(data, k)
    par = _addmul_rows(enc[k:], blocks) if m > k else np.zeros((0, blocks.shape[1]), np.uint8)
    return [bytes(b) for b in blocks] + [bytes(p) for p in par]


def normalise(blocks, sharenums, k: int, m: int):
    """_fecmodule Decoder_decode checks + move primaries into their own slot."""
    if len(blocks) != k or len(sharenums) != k:
        raise ValueError("Precondition violation: exactly k blocks and sharenums required")
    if len({len(b) for b in blocks}) > 1:
        raise ValueError("Precondition violation: Input blocks are required to be all the same length.")
    idx = [int(s) for s in sharenums]
    for s in idx:
        if s < 0 or s >= m:
            raise ValueError("Precondition violation: sharenum out of range")
    if len(set(idx)) != k:
        raise ValueError("Precondition violation: duplicate sharenum")
    slots = list(blocks)
    i = 0
    while i < k:
        if idx[i] >= k or idx[i] == i:
            i += 1
        else:
            c = idx[i]
            idx[i], idx[c] = idx[c], idx[i]
            slots[i], slots[c] = slots[c], slots[i]
    return slots, idx


def decode_matrix(k: int, m: int, idx) -> np.ndarray:
    enc = encode_matrix(k, m)
    dm = np.zeros((k, k), dtype=np.uint8)
    for i, s in enumerate(idx):
        if s < k:
            dm[i, i] = 1
        else:
            dm[i] = enc[s]
    return gf_invert(dm)


def easy_decode(blocks, sharenums, padlen: int, k: int, m: int) -> bytes:
    """zfec.easyfec.Decoder(k, m).decode(blocks, sharenums, padlen) -> bytes."""
    slots, idx = normalise(blocks, sharenums, k, m)
    B = len(slots[0])
    missing = [i for i in range(k) if idx[i] >= k]
    out = [np.frombuffer(bytes(s), dtype=np.uint8) for s in slots]
    if missing:
        minv = decode_matrix(k, m, idx)
        arr = np.stack(out)
        rec = _addmul_rows(minv[missing], arr)
        for t, i in enumerate(missing):
            out[i] = rec[t]
    data = b"".join(bytes(o) for o in out)
    return data[:-padlen] if padlen else data
    # NB: B unused beyond the equal-length check, as in easyfec


# ---- storb/util/piece.py policy restatement (piece.py:71-100, 116-134) ----
import math  # noqa: E402

MIN_PIECE_SIZE = 16 * 1024  # storb/constants.py:11
MAX_PIECE_SIZE = 256 * 1024 * 1024  # storb/constants.py:12
PIECE_LENGTH_SCALING = 0.5  # storb/constants.py:13
PIECE_LENGTH_OFFSET = 8.39  # storb/constants.py:14


def piece_length(content_length: int, min_size: int = MIN_PIECE_SIZE, max_size: int = MAX_PIECE_SIZE) -> int:
    exponent = int((math.log2(content_length) * PIECE_LENGTH_SCALING) + PIECE_LENGTH_OFFSET)
    length = 1 << exponent
    return min(max(length, min_size), max_size)


def chunk_shape(n: int) -> tuple[int, int, int, int]:
    """(k, m, B, padlen) that encode_chunk picks for an n-byte chunk (piece.py:116-134)."""
    piece = piece_length(n)
    k = math.ceil(n / piece)
    m = k + math.ceil(k / 2)
    B = (n + (k - 1)) // k
    return k, m, B, B * k - n

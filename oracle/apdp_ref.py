"""Python-int restatement of storb's APDP arithmetic — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py`` / ``tools/`` CPU baselines may
import this module, and only as the checker.  The product (``storb_amd``) never does.

Restates, with Python's built-in ``pow`` in place of ``gmpy2.powmod``:
  generate_tag     /root/reference/storb/challenge/__init__.py:304-350
  generate_proof   /root/reference/storb/challenge/__init__.py:401-463
  verify_proof     /root/reference/storb/challenge/__init__.py:465-528
  full_domain_hash, prf                                   :52-104

PARITY STATUS: the reference itself cannot run here (gmpy2 2.2.1 and cryptography, both
pinned in /root/reference/uv.lock, are absent from this image) and its tests
(storb/challenge/challenge_test.py) use fresh random keys, so they hold no known-answer
vectors.  Parity of the GPU path is therefore pinned against this restatement, whose
only arithmetic primitive is CPython's arbitrary-precision ``pow`` / ``%`` — an
implementation independent of both gmpy2 and bignum.hip computing the same functions.
"""

from __future__ import annotations

import base64
import hashlib
import hmac
import math
import random


def int_to_bytes(x: int, length: int | None = None) -> bytes:
    return x.to_bytes(length or (x.bit_length() + 7) // 8 or 1, "big")


def prf(key: bytes, i: int, out_len: int = 16) -> bytes:
    return hmac.digest(key, int_to_bytes(i, out_len), hashlib.sha256)


def full_domain_hash(n: int, data: bytes) -> int:
    return int.from_bytes(hashlib.sha256(data).digest(), "big") % n


def tag_value(n: int, g: int, d: int, prf_key: bytes, data: bytes) -> int:
    """generate_tag (challenge/__init__.py:322-346)."""
    x = int.from_bytes(data, "big") % n
    fdh = full_domain_hash(n, prf(prf_key, 0))
    return pow(fdh * pow(g, x, n) % n, d, n)


def proof(n: int, data: bytes, tag: int, ch_prf_key: bytes, g_s: int) -> tuple[int, int, str]:
    """generate_proof (challenge/__init__.py:424-457): (aggregated tag, aggregated blocks,
    base64 SHA-256 of rho)."""
    x = int.from_bytes(data, "big") % n
    c = int.from_bytes(prf(ch_prf_key, 0), "big") % n
    agg_tag = pow(tag, c, n)
    agg_blocks = c * x
    rho = pow(g_s, agg_blocks, n)
    return agg_tag, agg_blocks, base64.b64encode(hashlib.sha256(int_to_bytes(rho)).digest()).decode()


def verify(n: int, e: int, proof_tag: int, hashed_result: str, ch_prf_key: bytes, tag_prf_value: bytes,
           s: int) -> bool:
    """verify_proof (challenge/__init__.py:497-528)."""
    tau = pow(proof_tag, e, n)
    c = int.from_bytes(prf(ch_prf_key, 0), "big") % n
    den = pow(full_domain_hash(n, tag_prf_value), c, n) % n
    tau = tau * pow(den, -1, n) % n
    tau_s = pow(tau, s, n)
    return base64.b64encode(hashlib.sha256(int_to_bytes(tau_s)).digest()).decode() == hashed_result


def _is_prime(c: int, rng: random.Random) -> bool:
    for p in (3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37):
        if c % p == 0:
            return c == p
    d, r = c - 1, 0
    while d % 2 == 0:
        d, r = d // 2, r + 1
    for _ in range(24):
        x = pow(rng.randrange(2, c - 1), d, c)
        if x in (1, c - 1):
            continue
        for _ in range(r - 1):
            x = x * x % c
            if x == c - 1:
                break
        else:
            return False
    return True


def test_key(seed: int, bits: int = 2048, e: int = 65537) -> tuple[int, int, int, int, int]:
    """Deterministic RSA key (n, e, d, p, q) for tests, `bits`-bit modulus."""
    rng = random.Random(seed)

    def prime():
        while True:
            c = rng.getrandbits(bits // 2) | (3 << (bits // 2 - 2)) | 1
            if math.gcd(c - 1, e) == 1 and _is_prime(c, rng):
                return c

    p = prime()
    q = prime()
    while q == p:
        q = prime()
    lam = (p - 1) * (q - 1) // math.gcd(p - 1, q - 1)
    return p * q, e, pow(e, -1, lam), p, q

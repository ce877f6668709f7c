"""Drop-in for storb's APDP challenge system (/root/reference/storb/challenge/__init__.py)
with the 2048-bit modular arithmetic on the MI355X.

Same classes, fields, serialisation and error behaviour as the reference module
(``APDPError``, ``CryptoUtils``, ``APDPKey``, ``APDPTag``, ``Challenge``, ``Proof``,
``ChallengeSystem``).  Every gmpy2 ``powmod`` / ``% n`` of a piece runs in bignum.hip through
:class:`storb_amd.bn.ModKey`; batched entry points (``generate_tags``, ``issue_challenges``,
``generate_proofs``, ``verify_proofs``) hand many pieces to the GPU in one call.

Deliberate differences:

* RSA keys are generated here (Miller-Rabin over ``secrets`` randomness, e = 65537,
  d = e^-1 mod lcm(p-1, q-1), as OpenSSL does) because ``cryptography`` is not a dependency
  of this package; :class:`RSAPrivateKey` exposes the accessors the reference uses
  (``public_key().public_numbers().n/.e``, ``private_numbers().d``, ``key_size``).
* only 2048-bit keys (the reference's ``DEFAULT_RSA_KEY_SIZE``): the kernels are
  one-wave-per-2048-bit-integer; ``initialize_keys(rsa_bits=other)`` raises APDPError.
* ``g`` and ``s`` come from ``secrets`` rather than ``random`` (same ranges).
* the validator holds p and q, so its exponentiations (the d power of ``generate_tag``,
  everything in ``verify_proof``) run by CRT as two 1024-bit halves, and g's powers
  (``g^X`` in tags, ``g^s`` in challenges) come from a per-key fixed-base table; the
  results are the same integers.  The modular inverse in ``verify_proof`` is
  ``den^(p-2)`` / ``den^(q-2)`` per factor, checked by ``den * inv == 1``; a
  non-invertible denominator raises APDPError as gmpy2's ``powmod(x, -1, n)`` does.
* ``generate_proof`` / ``verify_proof`` take ``n`` (and ``e``) as optional: they default to
  the system's own key, which is how the reference's own tests call them
  (challenge_test.py:79,82).  A modulus other than the key's makes ``verify_proof`` return
  False (the reference would compute a tau that cannot match).
"""

from __future__ import annotations

import base64
import hashlib
import hmac
import math
import os
import secrets
import threading
from typing import Optional

from pydantic import BaseModel, ConfigDict, field_serializer, field_validator

from .bn import NBYTES, ModKey
from .constants import DEFAULT_RSA_KEY_SIZE, G_CANDIDATE_RETRY, S_CANDIDATE_RETRY
from .engine import get_engine

__all__ = ["APDPError", "CryptoUtils", "APDPKey", "APDPTag", "Challenge", "Proof", "ChallengeSystem",
           "RSAPrivateKey", "generate_private_key", "int_to_bytes"]

_TOP = 1 << (8 * NBYTES)


class APDPError(Exception):
    """Custom exception for APDP-related errors (challenge/__init__.py:25-28)."""


def int_to_bytes(integer: int, length: Optional[int] = None) -> bytes:
    """Big-endian bytes of a non-negative int, minimal length unless given
    (cryptography.utils.int_to_bytes, used at challenge/__init__.py:104,444,517)."""
    return integer.to_bytes(length or (integer.bit_length() + 7) // 8 or 1, "big")


# ---------------------------------------------------------------- RSA keys
class RSAPublicNumbers:
    def __init__(self, e: int, n: int):
        self.e, self.n = e, n


class RSAPublicKey:
    def __init__(self, numbers: RSAPublicNumbers):
        self._numbers = numbers
        self.key_size = numbers.n.bit_length()

    def public_numbers(self) -> RSAPublicNumbers:
        return self._numbers


class RSAPrivateNumbers:
    def __init__(self, p: int, q: int, d: int, public_numbers: RSAPublicNumbers):
        self.p, self.q, self.d, self.public_numbers = p, q, d, public_numbers


class RSAPrivateKey:
    """The subset of cryptography's RSAPrivateKey the challenge system reads."""

    def __init__(self, p: int, q: int, e: int = 65537):
        n = p * q
        lam = (p - 1) * (q - 1) // math.gcd(p - 1, q - 1)
        self._priv = RSAPrivateNumbers(p, q, pow(e, -1, lam), RSAPublicNumbers(e, n))
        self.key_size = n.bit_length()

    def public_key(self) -> RSAPublicKey:
        return RSAPublicKey(self._priv.public_numbers)

    def private_numbers(self) -> RSAPrivateNumbers:
        return self._priv


_SMALL_PRIMES = [p for p in range(3, 2000) if all(p % q for q in range(2, int(p ** 0.5) + 1))]


def _probable_prime(c: int, rounds: int = 40) -> bool:
    for p in _SMALL_PRIMES:
        if c % p == 0:
            return c == p
    d, r = c - 1, 0
    while d % 2 == 0:
        d //= 2
        r += 1
    for _ in range(rounds):
        a = secrets.randbelow(c - 3) + 2
        x = pow(a, d, c)
        if x in (1, c - 1):
            continue
        for _ in range(r - 1):
            x = x * x % c
            if x == c - 1:
                break
        else:
            return False
    return True


def _prime(bits: int, e: int) -> int:
    while True:
        c = secrets.randbits(bits) | (3 << (bits - 2)) | 1  # top two bits set: p*q has 2*bits bits
        if math.gcd(c - 1, e) == 1 and _probable_prime(c):
            return c


def generate_private_key(public_exponent: int = 65537, key_size: int = DEFAULT_RSA_KEY_SIZE) -> RSAPrivateKey:
    """An RSA key with an exactly `key_size`-bit modulus (key generation runs on the host)."""
    if key_size < 16 or key_size % 2:
        raise APDPError("Invalid RSA key size.")
    while True:
        p = _prime(key_size // 2, public_exponent)
        q = _prime(key_size // 2, public_exponent)
        if p != q:
            return RSAPrivateKey(p, q, public_exponent)


def _fernet_key() -> bytes:
    """Fernet.generate_key(): url-safe base64 of 32 random bytes."""
    return base64.urlsafe_b64encode(os.urandom(32))


class CryptoUtils:
    """Utility class for cryptographic operations (challenge/__init__.py:31-104)."""

    @staticmethod
    def generate_rsa_private_key(key_size: int) -> RSAPrivateKey:
        return generate_private_key(public_exponent=65537, key_size=key_size)

    @staticmethod
    def full_domain_hash(rsa_key: RSAPrivateKey, data: bytes) -> int:
        """int(SHA-256(data)) mod n (challenge/__init__.py:52-78)."""
        if rsa_key is None or data is None:
            raise APDPError("Invalid parameters for full_domain_hash. RSA key or data is None.")
        hashed = hashlib.sha256(data).digest()
        return int.from_bytes(hashed, "big") % rsa_key.public_key().public_numbers().n

    @staticmethod
    def prf(key: bytes, input_int: int, out_len=16) -> bytes:
        """HMAC-SHA256(key, input_int as out_len big-endian bytes) (challenge/__init__.py:80-104)."""
        if not key or len(key) == 0:
            raise APDPError("Invalid key for PRF")
        block = int_to_bytes(input_int, out_len)
        return hmac.digest(key, block, hashlib.sha256)


def _b64decode_field(value, what: str):
    if isinstance(value, str):
        try:
            return base64.b64decode(value)
        except Exception:
            raise ValueError(f"Invalid base64 for {what}")
    return value


# ---------------------------------------------------------------- models
class APDPKey(BaseModel):
    """RSA key, generator g and PRF key (challenge/__init__.py:107-171)."""

    model_config = ConfigDict(arbitrary_types_allowed=True)

    rsa: Optional[RSAPrivateKey] = None
    g: Optional[int] = None
    prf_key: Optional[bytes] = None

    def generate(self, rsa_bits=DEFAULT_RSA_KEY_SIZE):
        if rsa_bits <= 0:
            raise APDPError("Invalid RSA key size.")
        if rsa_bits != 8 * NBYTES:
            raise APDPError(f"storb_amd supports {8 * NBYTES}-bit RSA keys only (got {rsa_bits}).")
        self.rsa = generate_private_key(public_exponent=65537, key_size=rsa_bits)
        if self.rsa is None:
            raise APDPError("Failed to generate RSA key.")
        n = self.rsa.public_key().public_numbers().n
        mk = ModKey(n)
        g_candidate = None
        for _ in range(G_CANDIDATE_RETRY):
            candidate = 2 + secrets.randbelow(n - 3)  # randint(2, n - 2)
            temp_val = mk.powmod([candidate], [2])[0]
            if temp_val not in (0, 1):  # g = candidate^2 mod n, not in {0, 1}
                g_candidate = temp_val
                break
        if g_candidate is None:
            raise APDPError("Failed to find suitable generator g.")
        self.g = g_candidate
        self.prf_key = _fernet_key()
        if not self.prf_key:
            raise APDPError("Failed to generate PRF key")

    def clear(self):
        self.rsa = None
        self.g = None
        self.prf_key = None


class APDPTag(BaseModel):
    """challenge/__init__.py:174-205; prf_value travels as base64."""

    index: int
    tag_value: int
    prf_value: bytes

    @field_serializer("prf_value")
    def _ser_prf_value(self, prf_value: bytes) -> str:
        return base64.b64encode(prf_value).decode("utf-8")

    @field_validator("prf_value", mode="before")
    @classmethod
    def _de_prf_value(cls, value):
        return _b64decode_field(value, "prf_value")


class Challenge(BaseModel):
    """challenge/__init__.py:208-278; prp_key / prf_key travel as base64."""

    tag: APDPTag
    prp_key: bytes
    prf_key: bytes
    s: int
    g_s: int

    @field_serializer("prp_key", "prf_key")
    def _ser_keys(self, value: bytes) -> str:
        return base64.b64encode(value).decode("utf-8") if isinstance(value, bytes) else value

    @field_validator("prf_key", mode="before")
    @classmethod
    def _de_prf_key(cls, value):
        return _b64decode_field(value, "prf_key")

    @field_validator("prp_key", mode="before")
    @classmethod
    def _de_prp_key(cls, value):
        return _b64decode_field(value, "prp_key")


class Proof(BaseModel):
    """challenge/__init__.py:281-286."""

    tag_value: int
    block_value: int
    hashed_result: str


# ---------------------------------------------------------------- the system
def _fit(x: int, n: int) -> int:
    """An operand the kernels take (< 2^2048), congruent to x mod n."""
    return x if 0 <= x < _TOP else x % n


class ChallengeSystem:
    """Main class for the APDP challenge system (challenge/__init__.py:289-528)."""

    def __init__(self):
        self.key = APDPKey()
        self._local = threading.local()

    # ModKeys live on the calling thread's engine, one per modulus.  The system's own key
    # also gets its factors (CRT) and, for tags / challenges, g's fixed-base table.
    def _modkey(self, n: int, tag: bool = False) -> ModKey:
        cache = getattr(self._local, "keys", None)
        if cache is None or getattr(self._local, "engine", None) is not get_engine():
            cache = self._local.keys = {}
            self._local.engine = get_engine()
        mk = cache.get(n)
        if mk is None:
            if not (n.bit_length() == 8 * NBYTES and n & 1):
                raise APDPError(f"storb_amd supports odd {8 * NBYTES}-bit moduli only.")
            mk = cache[n] = ModKey(n)
        rsa = self.key.rsa
        if rsa is not None and rsa.public_key().public_numbers().n == n and mk.p is None:
            priv = rsa.private_numbers()
            mk.set_crt(priv.p, priv.q)
        if tag:
            sig = (self.key.g, self.key.prf_key, rsa.private_numbers().d)
            if getattr(mk, "_tag_sig", None) != sig:
                fdh = CryptoUtils.full_domain_hash(rsa, CryptoUtils.prf(self.key.prf_key, 0))
                mk.set_tag(self.key.g, fdh, rsa.private_numbers().d)
                mk._tag_sig = sig
        return mk

    def _n(self) -> int:
        return self.key.rsa.public_key().public_numbers().n

    def initialize_keys(self, rsa_bits=DEFAULT_RSA_KEY_SIZE):
        assert self.key is not None
        if rsa_bits <= 0:
            raise APDPError("Invalid RSA key size.")
        self.key.generate(rsa_bits)

    # -- tags (validator, validator.py:945-947) ------------------------------------
    def generate_tag(self, data: bytes) -> APDPTag:
        """tag = (FDH(prf(key, 0)) * g^(data mod n))^d mod n (challenge/__init__.py:304-350)."""
        return self.generate_tags([data])[0]

    def generate_tags(self, datas) -> list[APDPTag]:
        """``generate_tag`` for many pieces in one GPU call."""
        if self.key.rsa is None or self.key.g is None or self.key.prf_key is None:
            raise APDPError("Key values are not initialized. Call initialize_keys first.")
        for data in datas:
            if not data:
                raise APDPError("No data to generate tag.")
        if not datas:
            return []
        prf_value = CryptoUtils.prf(self.key.prf_key, 0)
        tags = self._modkey(self._n(), tag=True).tags(list(datas))
        return [APDPTag(index=0, tag_value=t, prf_value=prf_value) for t in tags]

    # -- challenges (validator.py:644) --------------------------------------------
    def issue_challenge(self, tag: APDPTag) -> Challenge:
        """Random s in Z*_n, g_s = g^s mod n, fresh PRP / PRF keys (challenge/__init__.py:352-399)."""
        return self.issue_challenges([tag])[0]

    def issue_challenges(self, tags) -> list[Challenge]:
        if self.key.rsa is None or self.key.g is None:
            raise APDPError("Key values are not initialized. Call initialize_keys first.")
        parsed = []
        for tag in tags:
            if isinstance(tag, str):
                try:
                    tag = APDPTag.model_validate_json(tag)
                except Exception:
                    raise APDPError("Failed to parse tag JSON.")
            parsed.append(tag)
        n = self._n()
        ss = []
        for _ in parsed:
            s = 2 + secrets.randbelow(n - 2)  # randint(2, n - 1)
            attempt = 0
            while math.gcd(s, n) != 1:
                s = 2 + secrets.randbelow(n - 2)
                attempt += 1
                if attempt > S_CANDIDATE_RETRY:
                    raise APDPError("Failed to find suitable s in Z*_n")
            ss.append(s)
        g_ss = self._modkey(n, tag=True).gpow(ss) if ss else []
        out = []
        for tag, s, g_s in zip(parsed, ss, g_ss):
            try:
                tag_obj = APDPTag.model_validate_json(tag.model_dump_json())
            except Exception:
                raise APDPError("Failed to validate tag.")
            out.append(Challenge(s=s, g_s=g_s, prf_key=_fernet_key(), prp_key=_fernet_key(), tag=tag_obj))
        return out

    # -- proofs (miner, miner.py:284-289) -----------------------------------------
    def generate_proof(self, data: bytes, tag: APDPTag, challenge: Challenge, n: Optional[int] = None) -> Proof:
        """(tag^c mod n, c * (data mod n), b64 SHA-256 of g_s^(c * X) mod n), c = prf(challenge
        key, 0) mod n (challenge/__init__.py:401-463)."""
        return self.generate_proofs([(data, tag, challenge)], n)[0]

    def generate_proofs(self, items, n: Optional[int] = None) -> list[Proof]:
        """``generate_proof`` over [(data, tag, challenge)] sharing one modulus, on the GPU."""
        for _data, tag, challenge in items:
            if not tag or not challenge:
                raise APDPError("Invalid tag or challenge for proof generation.")
        if self.key.rsa is None:
            raise APDPError("Keys not initialized.")
        if not items:
            return []
        n = self._n() if n is None else n
        mk = self._modkey(n)
        xs = mk.reduce([d for d, _, _ in items])
        coefs = [int.from_bytes(CryptoUtils.prf(ch.prf_key, 0), "big") % n for _, _, ch in items]
        aggs = [c * x for c, x in zip(coefs, xs)]
        res = mk.powmod([_fit(t.tag_value, n) for _, t, _ in items] + [_fit(ch.g_s, n) for _, _, ch in items],
                        coefs + aggs)
        k = len(items)
        out = []
        for i in range(k):
            digest = hashlib.sha256(int_to_bytes(res[k + i])).digest()
            out.append(Proof(tag_value=res[i], block_value=aggs[i],
                             hashed_result=base64.b64encode(digest).decode("utf-8")))
        return out

    # -- verification (validator) ---------------------------------------------------
    def verify_proof(self, proof: Proof, challenge: Challenge, tag: APDPTag, n: Optional[int] = None,
                     e: Optional[int] = None) -> bool:
        """SHA-256((tag^e / FDH(prf_value)^c)^s mod n) == proof.hashed_result
        (challenge/__init__.py:465-528)."""
        return self.verify_proofs([(proof, challenge, tag)], n, e)[0]

    def verify_proofs(self, items, n: Optional[int] = None, e: Optional[int] = None) -> list[bool]:
        """``verify_proof`` over [(proof, challenge, tag)] in four GPU launches."""
        for proof, challenge, tag in items:
            if proof is None or challenge is None or tag is None:
                raise APDPError("Invalid proof, challenge, or tag.")
        if self.key.rsa is None:
            raise APDPError("Keys not initialized.")
        if not items:
            return []
        rsa_key = self.key.rsa
        pub = rsa_key.public_key().public_numbers()
        n = pub.n if n is None else n
        e = pub.e if e is None else e
        if n != pub.n:
            return [False] * len(items)
        priv = rsa_key.private_numbers()
        mk = self._modkey(n)  # the system's own key: CRT over p, q
        k = len(items)
        coefs = [int.from_bytes(CryptoUtils.prf(ch.prf_key, 0), "big") % n for _, ch, _ in items]
        fdhs = [CryptoUtils.full_domain_hash(rsa_key, t.prf_value) for _, _, t in items]
        r1 = mk.crt_powmod([_fit(p.tag_value, n) for p, _, _ in items] + fdhs, [e] * k + coefs)
        taus, dens = r1[:k], r1[k:]
        # den^-1: den^(p-2) mod p and den^(q-2) mod q (Fermat per factor), checked below
        invs = mk.crt_powmod_pq(dens, [priv.p - 2] * k, [priv.q - 2] * k)
        r2 = mk.mulmod(dens + taus, invs + invs)
        if any(v != 1 for v in r2[:k]):
            raise APDPError("Failed to invert denominator modulo n.")
        tau_s = mk.crt_powmod(r2[k:], [ch.s for _, ch, _ in items])
        out = []
        for (proof, _, _), v in zip(items, tau_s):
            expected = base64.b64encode(hashlib.sha256(int_to_bytes(v)).digest()).decode("utf-8")
            out.append(expected == proof.hashed_result)
        return out

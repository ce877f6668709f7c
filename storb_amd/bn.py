"""2048-bit modular arithmetic on the MI355X (sec_bn_* in include/storb_ec.h).

The GPU replacement for the gmpy2 calls of storb's APDP challenge system
(/root/reference/storb/challenge/__init__.py:304-350, 401-463, 465-528): reduction of a
whole piece modulo n, modular exponentiation and modular multiplication, batched over many
pieces / challenges.  One 64-lane wave holds one 2048-bit integer (bignum.hip).

Integers cross the boundary as 256-byte big-endian strings.  :class:`ModKey` keeps one RSA
modulus (and optionally generate_tag's constants) resident on an engine's device.
"""

from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import MSG_DTYPE, SEC_F_ASYNC, SEC_F_HOST
from .engine import ECRuntimeError, Engine, addr, get_engine

NBYTES = 256  # RSA-2048, DEFAULT_RSA_KEY_SIZE (storb/constants.py:26)


def to_be(values, width: int = NBYTES) -> np.ndarray:
    """Python ints -> (len, width) uint8 big-endian rows."""
    buf = b"".join(int(v).to_bytes(width, "big") for v in values)
    return np.frombuffer(buf, dtype=np.uint8).reshape(len(values), width).copy() if values else \
        np.zeros((0, width), np.uint8)


def from_be(rows: np.ndarray) -> list[int]:
    rows = np.asarray(rows, dtype=np.uint8).reshape(-1, NBYTES)
    return [int.from_bytes(r.tobytes(), "big") for r in rows]


def _flags(host: bool, asynchronous: bool) -> int:
    return (SEC_F_HOST if host else 0) | (SEC_F_ASYNC if asynchronous else 0)


class ModKey:
    """An odd 2048-bit modulus resident on one engine's device (``sec_bn_key``)."""

    def __init__(self, n: int, engine: Engine | None = None):
        if not (isinstance(n, int) and n.bit_length() == 8 * NBYTES and n & 1):
            raise ValueError("modulus must be an odd 2048-bit integer")
        self.engine = engine or get_engine()
        self.lib = self.engine.lib
        self.n = n
        h = ctypes.c_void_p()
        nb = n.to_bytes(NBYTES, "big")
        self._check(self.lib.sec_bn_key_create(self.engine._ctx, nb, ctypes.byref(h)))
        self._key = h
        self.has_tag = False
        self.p = self.q = None

    def _check(self, rc: int) -> None:
        self.engine._check(rc)

    def close(self) -> None:
        if getattr(self, "_key", None):
            self.lib.sec_bn_key_destroy(self._key)
            self._key = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_crt(self, p: int, q: int) -> None:
        """The key owner's factors (n = p*q, both 1024-bit): enables CRT exponentiation."""
        if p * q != self.n or p.bit_length() != 1024 or q.bit_length() != 1024:
            raise ValueError("p, q must be the 1024-bit factors of n")
        cp = q * pow(q, -1, p) % self.n
        cq = p * pow(p, -1, q) % self.n
        self._check(self.lib.sec_bn_key_set_crt(self.engine._ctx, self._key, p.to_bytes(128, "big"),
                                                q.to_bytes(128, "big"), cp.to_bytes(NBYTES, "big"),
                                                cq.to_bytes(NBYTES, "big")))
        self.p, self.q = p, q

    @staticmethod
    def _half_exp(e: int, m: int) -> int:
        """An exponent congruent to e mod m and nonzero when e is: exact for every base."""
        return 0 if e == 0 else (e - 1) % m + 1

    def set_tag(self, g: int, fdh: int, d: int) -> None:
        """generate_tag's per-key constants: generator g, FDH of the PRF value, private d.
        With set_crt done first, tags raise to d as two 1024-bit halves."""
        n = self.n
        dp = dq = None
        if self.p is not None:
            dp = self._half_exp(d, self.p - 1).to_bytes(128, "big")
            dq = self._half_exp(d, self.q - 1).to_bytes(128, "big")
        self._check(self.lib.sec_bn_key_set_tag(self.engine._ctx, self._key, (g % n).to_bytes(NBYTES, "big"),
                                                (fdh % n).to_bytes(NBYTES, "big"), d.to_bytes(NBYTES, "big"),
                                                dp, dq))
        self.has_tag = True

    # -- raw batches: device pointers (or host with host=True) ----------------------
    def reduce_batch(self, msgs: np.ndarray, out, *, host: bool = False, asynchronous: bool = False) -> None:
        msgs = np.ascontiguousarray(msgs, dtype=MSG_DTYPE)
        o, _ko = addr(out)
        self._check(self.lib.sec_bn_reduce_batch(self.engine._ctx, self._key, int(msgs.ctypes.data) if len(msgs)
                                                 else None, len(msgs), o or None, _flags(host, asynchronous)))

    def tag_batch(self, msgs: np.ndarray, tags, *, host: bool = False, asynchronous: bool = False) -> None:
        msgs = np.ascontiguousarray(msgs, dtype=MSG_DTYPE)
        o, _ko = addr(tags)
        self._check(self.lib.sec_apdp_tag_batch(self.engine._ctx, self._key, int(msgs.ctypes.data) if len(msgs)
                                                else None, len(msgs), o or None, _flags(host, asynchronous)))

    def modexp_batch(self, bases, exps, exp_bytes: int, count: int, out, *, host: bool = False,
                     asynchronous: bool = False) -> None:
        b, _kb = addr(bases)
        e, _ke = addr(exps)
        o, _ko = addr(out)
        self._check(self.lib.sec_bn_modexp_batch(self.engine._ctx, self._key, b or None, e or None, exp_bytes,
                                                 count, o or None, _flags(host, asynchronous)))

    def crt_modexp_batch(self, bases, exps_p, exps_q, exp_bytes: int, count: int, out, *, host: bool = False,
                         asynchronous: bool = False) -> None:
        b, _kb = addr(bases)
        ep, _kp = addr(exps_p)
        eq, _kq = addr(exps_q)
        o, _ko = addr(out)
        self._check(self.lib.sec_bn_crt_modexp_batch(self.engine._ctx, self._key, b or None, ep or None, eq or None,
                                                     exp_bytes, count, o or None, _flags(host, asynchronous)))

    def gpow_batch(self, exps, exp_bytes: int, count: int, out, *, host: bool = False,
                   asynchronous: bool = False) -> None:
        e, _ke = addr(exps)
        o, _ko = addr(out)
        self._check(self.lib.sec_apdp_gpow_batch(self.engine._ctx, self._key, e or None, exp_bytes, count,
                                                 o or None, _flags(host, asynchronous)))

    def mulmod_batch(self, a, b, count: int, out, *, host: bool = False, asynchronous: bool = False) -> None:
        pa, _ka = addr(a)
        pb, _kb = addr(b)
        o, _ko = addr(out)
        self._check(self.lib.sec_bn_mulmod_batch(self.engine._ctx, self._key, pa or None, pb or None, count,
                                                 o or None, _flags(host, asynchronous)))

    # -- Python-int conveniences (host memory) --------------------------------------
    @staticmethod
    def _msgs(datas) -> tuple[np.ndarray, list]:
        msgs = np.zeros(len(datas), dtype=MSG_DTYPE)
        keep = []
        for i, d in enumerate(datas):
            a, kp = addr(d)
            keep.append(kp)
            ln = len(kp) if isinstance(kp, np.ndarray) else len(d)
            msgs[i] = (a, ln, ln)
        return msgs, keep

    def reduce(self, datas) -> list[int]:
        """``[int.from_bytes(d, "big") % n for d in datas]``."""
        if not datas:
            return []
        msgs, _keep = self._msgs(datas)
        out = np.empty((len(datas), NBYTES), dtype=np.uint8)
        self.reduce_batch(msgs, out, host=True)
        return from_be(out)

    def tags(self, datas) -> list[int]:
        """generate_tag's tag_value per piece: ``pow(fdh * pow(g, X, n), d, n)``, X = piece mod n."""
        if not self.has_tag:
            raise ECRuntimeError("ModKey.tags needs set_tag(g, fdh, d) first")
        if not datas:
            return []
        msgs, _keep = self._msgs(datas)
        out = np.empty((len(datas), NBYTES), dtype=np.uint8)
        self.tag_batch(msgs, out, host=True)
        return from_be(out)

    def powmod(self, bases, exps) -> list[int]:
        """``[pow(b, e, n) for b, e in zip(bases, exps)]`` for 0 <= b < 2^2048, e >= 0."""
        if len(bases) != len(exps):
            raise ValueError("bases and exps differ in length")
        if not bases:
            return []
        if any(e < 0 for e in exps):
            raise ValueError("negative exponent")
        width = max(1, max((int(e).bit_length() + 7) // 8 for e in exps))
        if width > 4096:
            raise ValueError("exponent wider than 32768 bits")
        out = np.empty((len(bases), NBYTES), dtype=np.uint8)
        self.modexp_batch(to_be(bases), to_be(exps, width), width, len(bases), out, host=True)
        return from_be(out)

    def crt_powmod_pq(self, bases, exps_p, exps_q) -> list[int]:
        """x with x = b^ep mod p and x = b^eq mod q, per item (needs set_crt)."""
        if not (len(bases) == len(exps_p) == len(exps_q)):
            raise ValueError("operands differ in length")
        if not bases:
            return []
        width = max(1, max((int(e).bit_length() + 7) // 8 for e in list(exps_p) + list(exps_q)))
        if width > 4096:
            raise ValueError("exponent wider than 32768 bits")
        out = np.empty((len(bases), NBYTES), dtype=np.uint8)
        self.crt_modexp_batch(to_be(bases), to_be(exps_p, width), to_be(exps_q, width), width, len(bases), out,
                              host=True)
        return from_be(out)

    def crt_powmod(self, bases, exps) -> list[int]:
        """``[pow(b, e, n) ...]`` by CRT over the key's factors (needs set_crt)."""
        if self.p is None:
            raise ECRuntimeError("ModKey.crt_powmod needs set_crt(p, q) first")
        if any(e < 0 for e in exps):
            raise ValueError("negative exponent")
        return self.crt_powmod_pq(bases, [self._half_exp(e, self.p - 1) for e in exps],
                                  [self._half_exp(e, self.q - 1) for e in exps])

    def gpow(self, exps) -> list[int]:
        """``[pow(g, e, n) ...]`` from the key's fixed-base table of g (needs set_tag), e < 2^2048."""
        if not self.has_tag:
            raise ECRuntimeError("ModKey.gpow needs set_tag(g, fdh, d) first")
        if not exps:
            return []
        if any(e < 0 or e >= 1 << (8 * NBYTES) for e in exps):
            raise ValueError("exponent outside [0, 2^2048)")
        width = max(1, max((int(e).bit_length() + 7) // 8 for e in exps))
        out = np.empty((len(exps), NBYTES), dtype=np.uint8)
        self.gpow_batch(to_be(exps, width), width, len(exps), out, host=True)
        return from_be(out)

    def mulmod(self, a, b) -> list[int]:
        """``[x * y % n for x, y in zip(a, b)]`` for 0 <= x, y < 2^2048."""
        if len(a) != len(b):
            raise ValueError("operands differ in length")
        if not a:
            return []
        out = np.empty((len(a), NBYTES), dtype=np.uint8)
        self.mulmod_batch(to_be(a), to_be(b), len(a), out, host=True)
        return from_be(out)

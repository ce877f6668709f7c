"""ctypes binding of libstorbec.so (include/storb_ec.h).

This is the binding a storb maintainer would add in place of ``from zfec.easyfec import
Decoder, Encoder`` (/root/reference/storb/util/piece.py:8).  It fails loudly: if the
library is missing or cannot be loaded there is no CPU fallback, the import raises.
"""

from __future__ import annotations

import ctypes
import os
import sys

import numpy as np

from ._build import LIB

SEC_OK = 0
SEC_EINVAL = -1
SEC_EKM = -2
SEC_EBLOCKLEN = -3
SEC_ENBLOCKS = -4
SEC_ESHARENUM = -5
SEC_EDUPSHARE = -6
SEC_EPADLEN = -7
SEC_ESIZE = -8
SEC_ENODEV = -9
SEC_EHIP = -10
SEC_ENOMEM = -11
SEC_ESINGULAR = -12
SEC_EMODULUS = -13
SEC_ENOTAG = -14
SEC_ENOCRT = -15

SEC_F_HOST = 1
SEC_F_ASYNC = 2
SEC_F_RECOVER = 4
SEC_F_STAGED = 8
SEC_F_GPU_PARITY_IDS = 16

# zfec precondition failures (raised by zfec as zfec.Error)
PRECONDITION_CODES = {SEC_EKM, SEC_EBLOCKLEN, SEC_ENBLOCKS, SEC_ESHARENUM, SEC_EDUPSHARE, SEC_EPADLEN, SEC_ESIZE}


class sec_enc_chunk(ctypes.Structure):
    _fields_ = [("in_off", ctypes.c_uint64), ("n", ctypes.c_uint64), ("parity_off", ctypes.c_uint64),
                ("parity_stride", ctypes.c_uint64), ("k", ctypes.c_int32), ("m", ctypes.c_int32)]


class sec_dec_chunk(ctypes.Structure):
    _fields_ = [("out_off", ctypes.c_uint64), ("B", ctypes.c_uint64), ("padlen", ctypes.c_uint64),
                ("slot0", ctypes.c_uint64), ("k", ctypes.c_int32), ("m", ctypes.c_int32)]


# numpy mirrors of the descriptor structs (same layout: 4 x u64 + 2 x i32 = 40 B)
ENC_DTYPE = np.dtype([("in_off", "<u8"), ("n", "<u8"), ("parity_off", "<u8"), ("parity_stride", "<u8"),
                      ("k", "<i4"), ("m", "<i4")], align=True)
DEC_DTYPE = np.dtype([("out_off", "<u8"), ("B", "<u8"), ("padlen", "<u8"), ("slot0", "<u8"),
                      ("k", "<i4"), ("m", "<i4")], align=True)
MSG_DTYPE = np.dtype([("addr", "<u8"), ("len", "<u8"), ("avail", "<u8")], align=True)
COPY_DTYPE = np.dtype([("dst", "<u8"), ("src", "<u8"), ("len", "<u8")], align=True)  # sec_copy


class sec_msg(ctypes.Structure):
    _fields_ = [("addr", ctypes.c_uint64), ("len", ctypes.c_uint64), ("avail", ctypes.c_uint64)]


assert ENC_DTYPE.itemsize == ctypes.sizeof(sec_enc_chunk) == 40
assert MSG_DTYPE.itemsize == ctypes.sizeof(sec_msg) == 24
assert DEC_DTYPE.itemsize == ctypes.sizeof(sec_dec_chunk) == 40

# every symbol include/storb_ec.h declares: name -> (restype, argtypes)
_vp = ctypes.c_void_p
_SIGS = {
    "sec_abi_version": (ctypes.c_int, []),
    "sec_strerror": (ctypes.c_char_p, [ctypes.c_int]),
    "sec_last_hip_error": (ctypes.c_char_p, []),
    "sec_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    "sec_ctx_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_vp)]),
    "sec_ctx_destroy": (None, [_vp]),
    "sec_ctx_set_stream": (ctypes.c_int, [_vp, _vp]),
    "sec_sync": (ctypes.c_int, [_vp]),
    "sec_ctx_set_timing": (ctypes.c_int, [_vp, ctypes.c_int]),
    "sec_timing_collect": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                          ctypes.POINTER(ctypes.c_int64)]),
    "sec_ctx_set_option": (ctypes.c_int, [_vp, ctypes.c_char_p, ctypes.c_int64]),
    "sec_ctx_get_option": (ctypes.c_int, [_vp, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int64)]),
    "sec_option_name": (ctypes.c_char_p, [ctypes.c_int]),
    "sec_decode_choose": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int64, _vp, _vp]),
    "sec_encode_matrix": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _vp]),
    "sec_decode_matrix": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _vp, _vp, _vp]),
    "sec_encode_batch": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, _vp, _vp, ctypes.c_uint]),
    "sec_decode_batch": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, _vp, _vp, _vp, _vp, ctypes.c_uint]),
    "sec_decode_batch_ex": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, _vp, _vp, _vp, _vp, _vp, ctypes.c_uint]),
    "sec_sha1_batch": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, _vp, ctypes.c_uint]),
    "sec_encode_digest_batch": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, _vp, _vp, _vp, ctypes.c_uint]),
    "sec_encode_pieces": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, _vp, _vp, _vp, ctypes.c_uint]),
    "sec_bn_key_create": (ctypes.c_int, [_vp, _vp, ctypes.POINTER(_vp)]),
    "sec_bn_key_destroy": (None, [_vp]),
    "sec_bn_key_set_crt": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp]),
    "sec_bn_key_set_tag": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "sec_bn_reduce_batch": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_int64, _vp, ctypes.c_uint]),
    "sec_bn_modexp_batch": (ctypes.c_int, [_vp, _vp, _vp, _vp, ctypes.c_uint32, ctypes.c_int64, _vp,
                                           ctypes.c_uint]),
    "sec_bn_crt_modexp_batch": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, ctypes.c_uint32, ctypes.c_int64, _vp,
                                               ctypes.c_uint]),
    "sec_apdp_gpow_batch": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_uint32, ctypes.c_int64, _vp, ctypes.c_uint]),
    "sec_bn_mulmod_batch": (ctypes.c_int, [_vp, _vp, _vp, _vp, ctypes.c_int64, _vp, ctypes.c_uint]),
    "sec_apdp_tag_batch": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_int64, _vp, ctypes.c_uint]),
    "sec_malloc": (ctypes.c_int, [_vp, ctypes.c_size_t, ctypes.POINTER(_vp)]),
    "sec_free": (ctypes.c_int, [_vp, _vp]),
    "sec_host_alloc": (ctypes.c_int, [_vp, ctypes.c_size_t, ctypes.POINTER(_vp)]),
    "sec_host_free": (ctypes.c_int, [_vp, _vp]),
    "sec_host_register": (ctypes.c_int, [_vp, _vp, ctypes.c_size_t]),
    "sec_host_unregister": (ctypes.c_int, [_vp, _vp]),
    "sec_ctx_host_paths": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64),
                                          ctypes.POINTER(ctypes.c_int64)]),
    "sec_host_pinned_bytes": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]),
    "sec_ctx_decode_paths": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]),
    "sec_ctx_decode_methods": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64),
                                              ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]),
    "sec_memcpy": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_size_t, ctypes.c_int]),
    "sec_memset": (ctypes.c_int, [_vp, _vp, ctypes.c_int, ctypes.c_size_t]),
    "sec_host_copy": (ctypes.c_int, [_vp, _vp, ctypes.c_int64]),
}
SYMBOLS = tuple(_SIGS)

_libs: dict = {}


def load(path: str | None = None) -> ctypes.CDLL:
    """Load libstorbec.so from the package tree; raise if it is absent (no fallback).

    `path` selects an A/B build variant (tools/sweep.py); default: $STORB_EC_LIB or the
    in-tree storb_amd/lib/libstorbec.so."""
    path = path or os.environ.get("STORB_EC_LIB", LIB)
    if path in _libs:
        return _libs[path]
    _share_torch_runtime()
    if not os.path.exists(path):
        raise ImportError(
            f"libstorbec.so not found at {path}: build it with `python -m storb_amd._build` "
            "(or __graft_entry__.build()); storb_amd has no CPU fallback")
    lib = ctypes.CDLL(path)
    for name, (res, args) in _SIGS.items():
        try:
            fn = getattr(lib, name)
        except AttributeError:
            # an A/B variant built from an earlier round's sources (build/variants/) may predate
            # an entry point; the product library must export every one
            if os.path.abspath(path) == os.path.abspath(LIB):
                raise
            continue
        fn.restype = res
        fn.argtypes = args
    if lib.sec_abi_version() != 1:
        raise ImportError("libstorbec.so ABI version mismatch")
    _libs[path] = lib
    return lib


def _share_torch_runtime() -> None:
    """Load torch's bundled HIP runtime before libstorbec.so when torch is installed.

    ROCm torch wheels ship their own libamdhip64.so / libhsa-runtime64.so.  If libstorbec
    pulled /opt/rocm's runtime in first, a later `import torch` would start a second HIP
    runtime in the process that sees no GPU ("No HIP GPUs are available").  Loaded after
    torch, libstorbec's NEEDED libamdhip64.so.7 resolves to torch's copy: one runtime, and
    torch tensors / streams interoperate.  STORB_EC_PRELOAD_TORCH=0 skips this.
    """
    if "torch" in sys.modules or os.environ.get("STORB_EC_PRELOAD_TORCH", "1") == "0":
        return
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def strerror(code: int, lib: ctypes.CDLL | None = None) -> str:
    """Message for a status code; pass the library that returned it (its HIP error text is
    thread-local per loaded library)."""
    lib = lib or load()
    msg = lib.sec_strerror(code).decode()
    if code == SEC_EHIP:
        msg += ": " + lib.sec_last_hip_error().decode()
    return msg

"""CPU: libstorbec.so loads, exports every symbol include/storb_ec.h declares, and its host
arithmetic (matrices, validation) agrees with the oracle.  No compute call needs a GPU here;
the product path must fail loudly (no CPU fallback) when no device is present."""

import ctypes
import json
import os
import re

import numpy as np
import pytest

from oracle import zfec_ref
from storb_amd import _lib, engine, easyfec

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))


def header_functions():
    txt = open(os.path.join(ROOT, "include", "storb_ec.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(sec_[a-z0-9_]+)\s*\(", txt)))


def test_header_and_binding_agree():
    declared = header_functions()
    assert declared == sorted(_lib.SYMBOLS)
    assert len(declared) >= 15


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    for name in header_functions():
        assert hasattr(lib, name), name
    assert lib.sec_abi_version() == 1


def test_struct_layouts():
    assert ctypes.sizeof(_lib.sec_enc_chunk) == 40
    assert ctypes.sizeof(_lib.sec_dec_chunk) == 40
    assert _lib.ENC_DTYPE.names == tuple(f for f, _ in _lib.sec_enc_chunk._fields_)
    assert _lib.DEC_DTYPE.names == tuple(f for f, _ in _lib.sec_dec_chunk._fields_)


@pytest.mark.parametrize("km", list(GOLDEN["matrices"]))
def test_product_encode_matrix_matches_oracle(km):
    k, m = map(int, km.split(","))
    assert engine.encode_matrix(k, m) == zfec_ref.parity_rows(k, m).tobytes()


@pytest.mark.parametrize("ent", GOLDEN["decode"], ids=lambda e: f"k{e['k']}m{e['m']}")
def test_product_decode_matrix_matches_oracle(ent):
    dm, idx = engine.decode_matrix(ent["k"], ent["m"], ent["sharenums"])
    assert idx == ent["normalised"]
    assert [dm[i * ent["k"]:(i + 1) * ent["k"]].hex() for i in range(ent["k"])] == ent["decode_matrix"]


def test_error_codes():
    lib = _lib.load()
    out = np.zeros(64, np.uint8)
    assert lib.sec_encode_matrix(0, 1, out.ctypes.data) == _lib.SEC_EKM
    assert lib.sec_encode_matrix(5, 4, out.ctypes.data) == _lib.SEC_EKM
    assert lib.sec_encode_matrix(4, 257, out.ctypes.data) == _lib.SEC_EKM
    sn = np.array([0, 1, 1, 2], np.int32)
    assert lib.sec_decode_matrix(4, 6, sn.ctypes.data, out.ctypes.data, None) == _lib.SEC_EDUPSHARE
    sn = np.array([0, 1, 2, 6], np.int32)
    assert lib.sec_decode_matrix(4, 6, sn.ctypes.data, out.ctypes.data, None) == _lib.SEC_ESHARENUM
    assert "same length" in _lib.strerror(_lib.SEC_EBLOCKLEN)
    assert lib.sec_encode_batch(None, None, 0, None, None, 0) == _lib.SEC_EINVAL


def test_no_cpu_fallback_without_gpu():
    if engine.device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(engine.ECRuntimeError):
        engine.Engine(0)
    with pytest.raises(engine.ECRuntimeError):
        easyfec.Encoder(4, 6).encode(b"x" * 4096)


def test_easyfec_preconditions_host_side():
    # validated before any device work, same cases zfec raises zfec.Error for
    for k, m in [(0, 1), (5, 4), (1, 257)]:
        with pytest.raises(easyfec.Error):
            easyfec.Encoder(k, m)
        with pytest.raises(easyfec.Error):
            easyfec.Decoder(k, m)
    with pytest.raises(easyfec.Error):
        easyfec.Encoder(4, 6).encode(b"12345")  # B=2, middle slice short
    with pytest.raises(easyfec.Error):
        easyfec.Decoder(4, 6).decode([b"ab"] * 3, [0, 1, 2], 0)
    assert issubclass(easyfec.Error, Exception) and not issubclass(easyfec.Error, engine.ECRuntimeError)


def test_options_listed_with_defaults_and_no_environment_reads():
    """plan choices are context options (sec_ctx_set_option), not environment
    variables read by the library.  Every option is listed with its default; an unknown name or an
    out-of-range value is SEC_EINVAL; the product sources call no getenv."""
    from storb_amd._build import CSRC, HEADERS, SOURCES

    names = engine.option_names()
    assert {"SEC_SYN", "SEC_BS", "SEC_BS_LANES", "SEC_REGISTER_MIN", "SEC_HOST_JOIN"} <= set(names)
    assert engine.option_default("SEC_SYN") == -1 and engine.option_default("SEC_BS_LANES") == 256
    assert engine.option_default("SEC_REGISTER_MIN") == 4 << 20
    # round 5 archived the A/B-only options with their kernels: at most 12
    # remain, each forcing a shipped path or sizing the host pipeline
    assert len(names) <= 12, names
    for gone in ("SEC_BS_LDS", "SEC_DEC_LDS", "SEC_BS_PAIR", "SEC_SYN_PAIR", "SEC_SOLVE_LDS", "SEC_SYN_WG2",
                 "SEC_TILE_U", "SEC_STAGE_DMA", "SEC_EXACT_LANES", "SEC_RAGGED_KERNEL"):
        assert gone not in names, gone
    lib = _lib.load()
    v = ctypes.c_int64(0)
    assert lib.sec_ctx_get_option(None, b"SEC_NOPE", ctypes.byref(v)) == _lib.SEC_EINVAL
    assert lib.sec_ctx_set_option(None, b"SEC_SYN", 1) == _lib.SEC_EINVAL  # no context
    for name in SOURCES + HEADERS:
        with open(os.path.join(CSRC, name)) as f:
            assert not re.search(r"\bgetenv\s*\(", f.read()), name

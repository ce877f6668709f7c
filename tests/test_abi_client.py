"""The C ABI from a plain C caller (tests/native/abi_client.c): what a cgo / JNI / FFI binding
of the path does, with no Python or HIP in the caller.  The client links the
CPU oracle as its checker (test infrastructure) and checks host and device encode / decode /
recover-only batches over the policy shapes, C4 and C5, bit-exact, plus zfec's precondition
codes.  Built by __graft_entry__.build() (make -C tests/native); the GPU test only runs it."""

import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "tests", "native")
CLIENT = os.path.join(NATIVE, "build", "abi_client")


def build_client() -> str:
    subprocess.run(["make", "-s", "-C", NATIVE], check=True, capture_output=True, text=True)
    return CLIENT


def test_client_builds_against_header_and_library():
    """No GPU needed: the header compiles as C11 and the library resolves every symbol the
    client uses (the link would fail otherwise)."""
    from storb_amd import _build

    _build.build()
    assert os.access(build_client(), os.X_OK)


@pytest.mark.gpu
def test_client_runs_bit_exact_on_gpu():
    assert os.access(CLIENT, os.X_OK), "tests/native/build/abi_client missing: run __graft_entry__.build() first"
    p = subprocess.run([CLIENT], capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "abi_client ok" in p.stdout, p.stdout

"""CPU: libstorbec's host C++ (GF matrix code, staging copy pool, task pool + OpenSSL SHA-1)
under sanitizers.

The GPU kernels cannot run under a sanitizer on this pool; the host code around them can:
g++ -fsanitize=address,undefined and -fsanitize=thread builds of tests/native/test_host.cpp."""

import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "native", "test_host.cpp")
CSRC = os.path.join(ROOT, "storb_amd", "csrc")


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ missing")
@pytest.mark.parametrize("san", ["address,undefined", "thread"])
def test_native_host_sanitized(tmp_path, san):
    exe = tmp_path / "test_host"
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", f"-fsanitize={san}", "-fno-omit-frame-pointer", "-pthread",
                    f"-I{CSRC}", SRC, "-o", str(exe), "-lcrypto"], check=True)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1", ASAN_OPTIONS="detect_leaks=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "native host tests ok" in r.stdout

cat /sys/fs/cgroup/cpu.max 2>/dev/null; cat /sys/fs/cgroup/cpu.stat 2>/dev/null | head -6; nproc
python3 - <<'PY'
import hashlib, time, os, numpy as np
from concurrent.futures import ThreadPoolExecutor
b = os.urandom(512 << 10)
t = time.perf_counter(); [hashlib.sha1(b).digest() for _ in range(200)]; dt = time.perf_counter() - t
print("sha1 1 thread GB/s", round(200 * len(b) / dt / 1e9, 3))
for n in (4, 8, 16, 32):
    with ThreadPoolExecutor(n) as ex:
        t = time.perf_counter(); list(ex.map(lambda _: hashlib.sha1(b).digest(), range(1600))); dt = time.perf_counter() - t
    print("sha1", n, "threads GB/s", round(1600 * len(b) / dt / 1e9, 3))
PY
cat /sys/fs/cgroup/cpu.stat 2>/dev/null | head -6

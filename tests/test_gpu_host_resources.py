"""GPU: the library's host resources when every caller thread has its own context (VERDICT r05
next #5; a validator's request handlers run on a thread pool, /root/reference/storb/validator/
validator.py:188-193,1301).  32 threads each take engine.get_engine() (one context per thread)
and encode through the host paths at once: the library's threads stay one shared task pool
sized from the CPU quota (task_pool.hpp shared_pool / default_pool_threads), and its pinned
staging memory is borrowed per call from one process pool, so none is held once the calls
return and at most 512 MiB stays idle (sec_host_pinned_bytes).  Pieces are checked against
the oracle."""

import os
import threading

import numpy as np
import pytest

from oracle import cfec

pytestmark = pytest.mark.gpu

from storb_amd import engine, piece  # noqa: E402

N_THREADS = 32


def _threads() -> int:
    return len(os.listdir("/proc/self/task"))


def test_32_caller_threads_share_threads_and_pinned_memory():
    rng = np.random.default_rng(9)
    chunks = [rng.integers(0, 256, (8 << 20) + 777 * i, dtype=np.uint8).tobytes() for i in range(4)]
    shapes = [piece.chunk_shape(len(c)) for c in chunks]
    want = [cfec.easy_encode(c, k, m) for c, (k, m, _, _) in zip(chunks, shapes)]
    engine.get_engine()  # the main thread's context (the runtime's own threads start here)
    before = _threads()
    done, release = threading.Barrier(N_THREADS + 1), threading.Barrier(N_THREADS + 1)
    errs, loaned_peak = [], [0]

    def work(t):
        try:
            eng = engine.get_engine()
            c, (k, m, _, _) = chunks[t % 4], shapes[t % 4]
            par = eng.encode_host([c], [(k, m)])  # the staged slab pipeline
            assert [bytes(x) for x in par[0]] == want[t % 4][k:]
            ec = piece.encode_chunk(c, t)  # sec_encode_pieces: pieces + ids on the shared pool
            assert [p.data for p in ec.pieces] == want[t % 4]
            loaned_peak[0] = max(loaned_peak[0], engine.pinned_bytes()[0])
        except Exception as e:  # noqa: BLE001 - reported on the main thread
            errs.append(e)
        finally:
            done.wait(timeout=60)
            release.wait(timeout=60)

    ts = [threading.Thread(target=work, args=(t,)) for t in range(N_THREADS)]
    for th in ts:
        th.start()
    done.wait(timeout=60)
    # every worker alive, each with its own context: what the library added beyond the workers
    added = _threads() - before - N_THREADS
    loaned, idle = engine.pinned_bytes()
    release.wait(timeout=60)
    for th in ts:
        th.join(timeout=60)
    assert not errs, errs[0]
    quota = piece._usable_cpus()
    print(f"threads added by {N_THREADS} contexts: {added} (usable CPUs {quota}); pinned loaned {loaned} "
          f"idle {idle} peak-seen {loaned_peak[0]}")
    assert added <= quota + 8, added
    assert loaned == 0  # no context holds pinned staging between calls
    assert idle <= 512 << 20

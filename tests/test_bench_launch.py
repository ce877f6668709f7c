"""CPU: `python bench.py --gpus N` launches and checks its own ranks.

Each case runs the real bench.py as a child process, with STORB_BENCH_ENGINE pointing at
tests/bench_stub.py (oracle/fec_oracle.c behind the Engine interface, CPU tensors, gloo): the
parent spawns the ranks, every rank builds its share's descriptors, runs (and round-trip
checks) its steps, and rank 0 prints the line.  Rank 1 sleeps in every encode call, so the
line's time is the max over ranks, not rank 0's own."""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, extra_env=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_PORT")}
    env.update(STORB_BENCH_ENGINE="tests.bench_stub:OracleEngine", PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    env.update(extra_env or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p, lines


@pytest.mark.timeout(300)
def test_bench_gpus2_c2c3_spawns_two_ranks():
    p, lines = _run(["--gpus", "2", "--steps", "2", "--warmup", "1", "--chunks", "3", "--no-cpu", "--no-e2e",
                     "--c4-chunks", "12", "--c5-bytes", str(6 << 20), "--c5-steps", "1"],
                    {"STORB_STUB_SLOW_RANK": "1"})
    assert p.returncode == 0, p.stderr[-3000:]
    assert len(lines) == 1, p.stdout  # rank 0 only
    j = json.loads(lines[0])
    assert j["n_gpus"] == 2 and j["config"]["world_size"] == 2 and j["config"]["backend"] == "gloo"
    assert j["config"]["per_rank_chunks"] == [3, 3]
    # rank 1 sleeps 50 ms per encode: the reported step time is at least that (max over ranks)
    assert j["ms_per_step"] >= 50
    assert j["value"] == pytest.approx(2 * 2 * 2 * 3 * (1 << 20) / (j["ms_per_step"] * 2 / 1e3) / (1 << 30), rel=0.02)
    assert j["decode_recover_only_kernel"]["launches"] == 10
    # configs[3] and [4] ride on the same line, split over the same two ranks
    assert j["c4"]["config"]["per_rank_chunks"] == [6, 6] and j["c4"]["n_gpus"] == 2
    assert j["c4"]["roofline"]["traffic"] is None  # a PMC summary applies to the full job at N = 1 only
    assert sum(j["c5"]["config"]["per_rank_chunks"]) == len(__import__("bench").c5_sizes(6 << 20))
    assert j["c4"]["cpu_baseline"] is None and j["c5"]["cpu_baseline"] is None  # N > 1


@pytest.mark.timeout(300)
def test_bench_gpus2_c4_partition_and_max():
    p, lines = _run(["--gpus", "2", "--workload", "c4", "--steps", "2", "--warmup", "1", "--c4-chunks", "40",
                     "--no-cpu"], {"STORB_STUB_SLOW_RANK": "1"})
    assert p.returncode == 0, p.stderr[-3000:]
    j = json.loads(lines[0])
    assert j["n_gpus"] == 2 and j["config"]["per_rank_chunks"] == [20, 20]
    assert j["config"]["chunks_total"] == 40 and j["config"]["parity_stride"] == 6656
    assert j["ms_per_step"] >= 50


@pytest.mark.timeout(300)
def test_bench_gpus3_c5_partition_by_bytes():
    p, lines = _run(["--gpus", "3", "--workload", "c5", "--steps", "1", "--warmup", "1",
                     "--c5-bytes", str(24 << 20), "--no-cpu", "--no-e2e"])
    assert p.returncode == 0, p.stderr[-3000:]
    j = json.loads(lines[0])
    sys.path.insert(0, ROOT)
    import bench
    from storb_amd.dist import partition

    sizes = bench.c5_sizes(24 << 20)
    want = [hi - lo for lo, hi in partition(sizes, 3)]
    assert j["n_gpus"] == 3 and j["config"]["per_rank_chunks"] == want and sum(want) == len(sizes)
    assert j["config"]["job_bytes"] == sum(sizes)


@pytest.mark.timeout(120)
def test_bench_world_size_mismatch_exits_nonzero():
    p, lines = _run(["--gpus", "2", "--steps", "1", "--warmup", "0", "--chunks", "1", "--no-cpu", "--no-e2e"],
                    {"WORLD_SIZE": "1", "RANK": "0"})
    assert p.returncode == 2 and not lines
    assert "WORLD_SIZE=1 but --gpus 2" in p.stderr


@pytest.mark.timeout(300)
def test_bench_gpus1_c4_cpu_baseline_line():
    # N = 1: no children; the c4 line carries its CPU baseline (the oracle's RS(10,4) encode)
    p, lines = _run(["--workload", "c4", "--steps", "1", "--warmup", "1", "--c4-chunks", "8",
                     "--cpu-seconds", "0.3"])
    assert p.returncode == 0, p.stderr[-3000:]
    j = json.loads(lines[0])
    assert j["n_gpus"] == 1 and j["config"]["backend"] is None
    cb = j["cpu_baseline"]
    assert cb["kind"] == "port" and cb["value"] > 0 and cb["cores"] >= 1 and "RS(10,4)" in cb["sample"]
    host = cb["host"]  # the box, beside the thread count
    assert host["os_cpu_count"] >= 1 and host["affinity_cpus"] >= cb["cores"] and "cgroup_cpu_quota" in host


@pytest.mark.timeout(300)
def test_bench_gpus1_c2c3_nests_c4_c5_with_cpu_baselines():
    """N = 1 headline line: configs[3] and [4] measured in the same run, each with its roofline and
    its own CPU baseline."""
    p, lines = _run(["--steps", "1", "--warmup", "1", "--chunks", "2", "--no-e2e", "--cpu-seconds", "0.2",
                     "--sub-cpu-seconds", "0.2", "--c4-chunks", "8", "--c5-bytes", str(4 << 20), "--c5-steps", "1"])
    assert p.returncode == 0, p.stderr[-3000:]
    j = json.loads(lines[0])
    assert j["cpu_baseline"]["kind"] == "port"
    for sub, what in (("c4", "RS(10,4)"), ("c5", "RS(8,3)")):
        s = j[sub]
        assert s["n_gpus"] == 1 and s["roofline"]["bound"] == "hbm" and s["roofline"]["achieved"] > 0
        assert s["cpu_baseline"]["value"] > 0 and what in s["cpu_baseline"]["sample"]
    assert len(j["lib_digest"]) == 64

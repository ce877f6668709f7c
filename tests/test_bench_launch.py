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


# ---- the N > 1 lines exactly as the driver's 8-GPU node will parse them ----
def _check_in_process(ip, n, c5_bytes):
    sys.path.insert(0, ROOT)
    import bench
    from storb_amd.dist import partition

    h = ip["c2c3"]
    assert h["n_gpus"] == n and h["devices"] == list(range(n)) and h["scaling"] == "weak"
    assert h["value"] > 0 and h["ms_per_step"] > 0 and "EngineGroup" in h["launch"]
    c5 = ip["c5"]
    sizes = bench.c5_sizes(c5_bytes)
    assert c5["n_gpus"] == n and c5["scaling"] == "strong" and c5["value"] > 0
    assert c5["per_device_chunks"] == [hi - lo for lo, hi in partition(sizes, n)]
    assert sum(c5["per_device_chunks"]) == len(sizes)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("n", [2, 8])
def test_bench_gpus_n_headline_line_with_in_process(n):
    """`bench.py --gpus N`: the headline line with c4 / c5 nested and, after them, the in-process
    form (EngineGroup over N stub engines) nested as `in_process`."""
    c5_bytes = 8 << 20
    p, lines = _run(["--gpus", str(n), "--steps", "1", "--warmup", "1", "--chunks", "2", "--no-cpu", "--no-e2e",
                     "--c4-chunks", str(2 * n), "--c5-bytes", str(c5_bytes), "--c5-steps", "1"], timeout=540)
    assert p.returncode == 0, p.stderr[-3000:]
    assert len(lines) == 1, p.stdout
    j = json.loads(lines[0])
    assert j["metric"] == "GiB/s device-resident RS encode+decode, 1 MiB chunks, 1/2/4/8 MI355X"
    assert j["n_gpus"] == n and j["config"]["world_size"] == n and j["config"]["backend"] == "gloo"
    assert j["config"]["per_rank_chunks"] == [2] * n and j["scaling"] == "weak"
    assert j["value"] == pytest.approx(2 * 2 * n * (1 << 20) / (j["ms_per_step"] / 1e3) / (1 << 30), rel=0.02)
    assert j["c4"]["n_gpus"] == n and j["c4"]["config"]["per_rank_chunks"] == [2] * n
    assert j["c5"]["n_gpus"] == n and j["cpu_baseline"] is None
    sys.path.insert(0, ROOT)
    import bench
    from storb_amd.dist import partition

    sizes = bench.c5_sizes(c5_bytes)
    parts = partition(sizes, n)
    assert j["c5"]["config"]["per_rank_chunks"] == [hi - lo for lo, hi in parts]
    # C5's split balances bytes: no rank holds more than the average plus one chunk
    per = [sum(sizes[lo:hi]) for lo, hi in parts]
    assert sum(per) == sum(sizes) and max(per) <= sum(sizes) / n + max(sizes)
    assert "error" not in j["in_process"], j["in_process"]
    _check_in_process(j["in_process"], n, c5_bytes)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("workload", ["c4", "c5"])
def test_bench_gpus8_c4_c5_lines(workload):
    args = ["--gpus", "8", "--workload", workload, "--steps", "1", "--warmup", "1", "--no-cpu", "--no-e2e"]
    args += ["--c4-chunks", "64"] if workload == "c4" else ["--c5-bytes", str(16 << 20)]
    p, lines = _run(args, timeout=540)
    assert p.returncode == 0, p.stderr[-3000:]
    j = json.loads(lines[0])
    assert j["n_gpus"] == 8 and j["config"]["world_size"] == 8
    if workload == "c4":
        assert j["config"]["per_rank_chunks"] == [8] * 8 and j["config"]["chunks_total"] == 64
    else:
        sys.path.insert(0, ROOT)
        import bench
        from storb_amd.dist import partition

        sizes = bench.c5_sizes(16 << 20)
        assert j["config"]["per_rank_chunks"] == [hi - lo for lo, hi in partition(sizes, 8)]


def test_c4_default_job_splits_8_x_8192():
    sys.path.insert(0, ROOT)
    import bench

    shares = [bench.c4_share(r, 8) for r in range(8)]
    assert [hi - lo for lo, hi in shares] == [8192] * 8
    assert shares[0][0] == 0 and shares[-1][1] == 65536
    assert all(shares[i][1] == shares[i + 1][0] for i in range(7))


@pytest.mark.timeout(300)
def test_bench_in_process_mode_stub():
    """`bench.py --gpus 4 --in-process`: one process, the line's value is the in-process headline."""
    c5_bytes = 8 << 20
    p, lines = _run(["--gpus", "4", "--in-process", "--steps", "1", "--warmup", "1", "--chunks", "2",
                     "--c5-bytes", str(c5_bytes), "--c5-steps", "1"])
    assert p.returncode == 0, p.stderr[-3000:]
    j = json.loads(lines[0])
    assert j["n_gpus"] == 4 and j["config"]["world_size"] == 1 and "in-process x4" in j["config"]["parallelism"]
    assert j["value"] == j["in_process"]["c2c3"]["value"]
    _check_in_process(j["in_process"], 4, c5_bytes)

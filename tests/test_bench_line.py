"""bench.py's contract on CPU: the ONE stdout line stays compact (the driver keeps only the last 8000 characters of
stdout) and carries roofline + cpu_baseline; `--gpus N` reaches the world size (one rank process per GPU, or the
in-process node), and fewer visible GPUs than asked is an error."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def canned_record(name, big=True):
    """A full per-workload record shaped like run_workload's, with every verbose field filled."""
    return {
        "value": 3.3e12, "ms_per_step": 0.3037, "steps": 20, "n_gpus": 1,
        "config": {"workload": name, "description": "x" * 200, "query": "SELECT " + "y" * 300,
                   "segments_per_gpu": 30, "docs_per_segment": 1 << 25, "rows_per_gpu": 30 << 25,
                   "total_rows": 30 << 25, "queries_in_flight": 3, "parallelism": "z" * 120},
        "roofline": {"bound": "hbm", "achieved": 5319.4, "peak": 8000.0, "unit": "GB/s", "frac": 0.6649,
                     "traffic": 1.763e9, "traffic_source": "profiles/pmc_adanalytics.json @ d282974",
                     "kernel": "query_kernel_rdirect", "algorithmic_bytes_per_launch": 1512985088,
                     "kernel_ms_avg": 0.2844, "kernel_ms_definition": "d" * 200,
                     "bytes_breakdown": {k: 123456789 for k in "abcdef"}, "bytes_definition": "e" * 100,
                     "bytes_read_model": 1669053696, "bytes_read_breakdown": {k: 1 for k in "abcde"}},
        "cpu_baseline": {"value": 6.8e9, "unit": "rows/s", "cores": 10, "kind": "port", "sample": "s" * 400,
                         "sample_short": "40 run(s) x 10 seg x 33554432 docs, oracle/pinot_cpu.c, 10 threads",
                         "seconds": 10.0, "all_cores": {"value": 1.1e10, "cores": 16, "available_cores": 16,
                                                        "segments": 16, "runs": 22, "seconds": 5.0}},
        "result": {"matched_docs_per_gpu": 5, "groups": 4, "rows": [[17853, 1716617.0, 1424020.0]] * 3},
        "parity_check": {"docs": 1 << 20, "matched": [0, 4105], "groups": [0, 8], "ok": True,
                         "full_size": True, "full_size_detail": {"k" * 20: "v" * 50 for _ in range(1)}},
        "hbm": {"resident_bytes_per_gpu": 11770064040, "by_kind": {k: 10 ** 10 for k in "abcdefgh"}},
        "setup_s": 1.3,
    }


def test_compact_line_fits_the_driver_tail():
    args = bench.parse_args([])
    head = canned_record("adanalytics")
    workloads = {name: canned_record(name) for name, *_ in bench.SECONDARY}
    workloads["broken"] = {"error": "RuntimeError(" + "m" * 1000 + ")"}
    line = bench.compact_line(head, workloads, args, 1)
    text = json.dumps(line, default=float, separators=(",", ":"))
    assert len(text) < bench.LINE_LIMIT < 8000
    back = json.loads(text)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in back, k
    assert back["config"]["workload"] == "adanalytics"
    assert set(back["roofline"]) == set(bench.ROOFLINE_KEYS)
    assert back["roofline"]["frac"] == pytest.approx(0.6649)
    assert back["cpu_baseline"]["kind"] == "port" and back["cpu_baseline"]["cores"] == 10
    assert set(back["cpu_baseline"]["all_cores"]) == {"value", "cores"}
    w = back["workloads"]["groupby1m"]
    assert set(w) == {"ms_per_step", "kernel_ms", "frac", "traffic_ratio", "parity_ok", "cpu_rows_s"}
    assert w["traffic_ratio"] == pytest.approx(1.763e9 / 1512985088, rel=1e-3)
    assert back["workloads"]["broken"]["error"].startswith("RuntimeError(")


def test_gpus_spawns_one_rank_per_gpu(monkeypatch):
    """`bench.py --gpus 4` without a launcher starts four rank processes with the torch.distributed environment
    (WORLD_SIZE = 4, ranks 0..3, one port, 127.0.0.1), before touching the GPU."""
    import subprocess

    import torch

    started = []

    class FakeProc:
        def __init__(self, cmd, env):
            started.append((cmd, env))

        def wait(self, timeout=None):
            return 0

        def poll(self):
            return 0

    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    monkeypatch.setattr(subprocess, "Popen", lambda cmd, env: FakeProc(cmd, env))
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "3"])
    assert bench.main(["--gpus", "4", "--steps", "3"]) == 0
    assert len(started) == 4
    envs = [e for _, e in started]
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert {e["WORLD_SIZE"] for e in envs} == {"4"}
    assert {e["MASTER_ADDR"] for e in envs} == {"127.0.0.1"}
    assert len({e["MASTER_PORT"] for e in envs}) == 1
    assert all(cmd[-4:] == ["--gpus", "4", "--steps", "3"] for cmd, _ in started)


def test_gpus_more_than_visible_fails(monkeypatch):
    import torch
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert bench.main(["--gpus", "8"]) == 2


def test_node_mode_is_not_spawned(monkeypatch):
    """--node keeps every device in this process (the in-library RCCL combine), so no rank is spawned."""
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    called = []
    monkeypatch.setattr(bench, "spawn_ranks", lambda a: called.append(a) or 0)
    import torch
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 0)
    with pytest.raises(Exception):  # no GPU here: the node cannot start, but nothing was spawned
        bench.main(["--gpus", "2", "--node"])
    assert not called

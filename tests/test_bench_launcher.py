"""bench.py's launcher and timing harness on the CPU (--stub: gloo, a trivial step instead of the encode).

`python bench.py --gpus N` without a torchrun environment must start N ranks itself (one process per GPU, before
the parent touches the GPU), each seeing RANK / LOCAL_RANK / WORLD_SIZE, and rank 0 must print one JSON line with
n_gpus = N (--gpus was parsed and ignored)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*extra, env=None):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--stub", "--steps", "3", "--warmup", "1",
           "--values", "4096", *extra]
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=e, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [2, 3])
def test_bench_self_launches_n_ranks(n):
    d = _run("--gpus", str(n))
    assert d["n_gpus"] == n
    assert sorted(tuple(r[:3]) for r in d["ranks"]) == [(i, i, n) for i in range(n)]
    assert all(r[3] == "self" for r in d["ranks"])
    # one rendezvous on the loopback address, at the port torchrun's own store bound (not one picked beforehand)
    assert len({(r[4], r[5]) for r in d["ranks"]}) == 1 and d["ranks"][0][4] == "127.0.0.1"
    assert d["steps"] == 3 and d["warmup"] == 1 and d["ms_per_step"] > 0


def test_bench_single_rank():
    d = _run("--gpus", "1")
    assert d["n_gpus"] == 1 and d["ranks"][0][:4] == [0, 0, 1, "torchrun"]


def test_bench_programmatic_argv_reaches_ranks():
    """main(argv) launches its ranks with `argv`, not with the parent's sys.argv."""
    code = ("import sys; sys.argv = ['bench.py', '--steps', '999']; import bench; "
            "bench.main(['--stub', '--gpus', '2', '--steps', '2', '--warmup', '1', '--values', '4096'])")
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240, env=e, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 2


@pytest.mark.parametrize("n", [1, 2])
def test_bench_fails_loudly_on_oracle_mismatch(n):
    """a `*_matches_oracle` false in the line (a stitch or shard-offset bug on the driver's N-rank run) must
    end the run with rc != 0 after the line is printed, not only show up as a boolean in it."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--stub", "--stub-mismatch", "--gpus", str(n), "--steps",
           "2", "--warmup", "1", "--values", "4096"]
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=e, cwd=ROOT)
    assert r.returncode != 0
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1 and json.loads(lines[0])["stub_check"]["stream_matches_oracle"] is False
    assert "ORACLE CHECK FAILED" in r.stderr


def test_parity_failures_scan():
    sys.path.insert(0, ROOT)
    import bench
    line = {"a": {"gathered_stream_matches_oracle": True}, "c5_sharded": {"stitched_stream_matches_oracle": False},
            "legs": [{"x_matches_oracle": None}, {"y_matches_oracle": False}]}
    assert bench.parity_failures(line) == ["c5_sharded.stitched_stream_matches_oracle", "legs.1.y_matches_oracle"]


def test_launcher_lets_torchrun_pick_the_port():
    """the N > 1 launcher used to bind port 0, read the port, close it and pass it as --master-port, a
    window in which another job could take it. It now asks torchrun for a standalone rendezvous on 127.0.0.1."""
    sys.path.insert(0, ROOT)
    import bench
    cmd = bench.launcher_cmd(8, ["--gpus", "8"])
    assert "--standalone" in cmd and "--local-addr=127.0.0.1" in cmd and "--nproc-per-node=8" in cmd
    assert not any(a.startswith("--master-port") for a in cmd)
    assert cmd[-2:] == ["--gpus", "8"]

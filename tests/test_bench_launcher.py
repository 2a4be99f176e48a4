"""CPU: bench.py's own rank launcher (`--gpus N` with no outer torchrun) and
its world-size check — the wiring the driver's 1/2/4/8-GPU scaling runs use.
`--launch-check` makes every rank join a gloo group and report what it saw,
without touching a GPU."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(kw)
    return env


@pytest.mark.parametrize("n", [2, 3, 8])
def test_gpus_n_starts_n_ranks(n):
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--launch-check"], env=_env(),
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    out = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(out) == 1, r.stdout  # rank 0's line only (gloo's connection lines go to stderr)
    lines = [json.loads(out[0])]
    seen = lines[0]["launch_check"]
    assert sorted(s["rank"] for s in seen) == list(range(n))
    assert sorted(s["local_rank"] for s in seen) == list(range(n))
    assert {s["world_size"] for s in seen} == {n}
    assert {s["master_addr"] for s in seen} == {"127.0.0.1"}
    assert len({s["pid"] for s in seen}) == n  # one process per rank


def test_driver_style_outer_launcher():
    """The driver's own form: torch.distributed.run starts the ranks and each
    runs `bench.py --gpus N`; bench.py must not launch again."""
    import socket

    n = 4
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), BENCH, "--gpus", str(n),
                        "--launch-check"], env=_env(), capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    out = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(out) == 1, r.stdout  # the driver reads exactly one line
    seen = json.loads(out[0])["launch_check"]
    assert sorted(s["rank"] for s in seen) == list(range(n)) and {s["world_size"] for s in seen} == {n}
    assert len({s["pid"] for s in seen}) == n


def test_world_size_must_match_gpus():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1", "--launch-check"],
                       env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2
    assert "WORLD_SIZE=2 but --gpus 1" in r.stderr


def test_cpu_share_reports_usable_cpus():
    sys.path.insert(0, ROOT)
    import bench

    n, how = bench.cpu_share()
    assert 1 <= n <= (os.cpu_count() or 1)
    assert "host CPUs" in how

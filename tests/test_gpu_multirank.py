"""GPU: the N > 1 path through the ENGINE (not the oracle stand-in of
tests/test_multirank.py): W processes on one card (gloo), each checksumming
its shard of a BASELINE configuration through libicsum.so; the rank-ordered
concatenation of their outputs must equal the reference's SHA-256 digest of
the whole batch (tests/golden/configs.json).

  config 0 (1 M x 1500 B) in 2 and 3 contiguous shards;
  config 5 (8 M x 9000 B, 75.5 GB) in 8 contiguous shards of ~9.4 GB — the
    8-way split BASELINE names, eight engine processes on one card;
  config 4 (1 M mixed 64 B-64 KiB) in 2 and 3 byte-balanced shards of its
    packed offsets (cut by the prefix sum of L_i), each rank's
    byte count within one segment of an equal share."""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT, golden

WORKER = os.path.join(ROOT, "tests", "mr_engine_worker.py")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(config, world, timeout):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), ICSUM_MR_CONFIG=config)
        procs.append(subprocess.Popen([sys.executable, WORKER], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = []
    try:
        for p in procs:
            o, e = p.communicate(timeout=timeout)
            outs.append((p.returncode, o, e))
    except subprocess.TimeoutExpired:
        for q in procs:
            q.kill()
        raise
    assert all(rc == 0 for rc, _, _ in outs), [e[-1500:] for _, _, e in outs]
    return json.loads([l for l in outs[0][1].splitlines() if l.startswith("{")][-1])


@pytest.mark.gpu
@pytest.mark.parametrize("config,world", [("0", 2), ("0", 3), ("5", 8), ("4", 2), ("4", 3)])
def test_engine_shards_concatenate_to_reference_digest(config, world):
    g = golden("configs.json")[config]
    line = _run(config, world, timeout=110)
    assert line["n"] == g["n"]
    shards = line["shards"]
    assert len(shards) == world and shards[0][0] == 0
    assert all(a[0] + a[1] == b[0] for a, b in zip(shards, shards[1:]))  # contiguous, in order
    assert line["sha256"] == g["out_sha256"]
    if config == "4":
        nb = [s[2] for s in shards]
        ideal = sum(nb) / world
        assert all(abs(b - ideal) < 65536 for b in nb), nb  # each within one segment (< 64 KiB) of an equal share


@pytest.mark.gpu
def test_bench_two_ranks_one_line():
    """The driver's N > 1 bench as a one-card rehearsal: `bench.py --gpus 2`
    starts its two ranks itself (torch.distributed.run on 127.0.0.1, gloo for
    the timing barrier and the max over ranks), and stdout is exactly ONE
    JSON line — gloo's connection messages kept off it — carrying the NS
    weak-scaling value over 2 x 1 M segments and the config-5 strong-scaling
    view (8 M x 9000 B, 4 M segments per rank)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
                        "--settle-ms", "10", "--config5-steps", "2", "--no-pmc", "--cpu-seconds", "0"],
                       capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    out = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(out) == 1, r.stdout
    d = json.loads(out[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["value"] > 0
    assert d["config"]["segments_total"] == 2 << 20 and d["config"]["segments_per_gpu"] == 1 << 20
    c5 = d["config5"]
    assert c5["segments_total"] == 8 << 20 and c5["segments_per_gpu"] == 4 << 20 and c5["value"] > 0
    assert d["cpu_baseline"] is None and d["host_inclusive"] is None  # N = 1 only
    # the timed outputs checked against the reference digests: EVERY rank's
    # NS shard against its own shard digest (rank r = global segments
    # [r 2^20, (r+1) 2^20)), both ranks' config-5 outputs gathered = config 5
    assert d["bit_exact"] is True and c5["bit_exact"] is True
    assert [r["rank"] for r in d["per_rank"]] == [0, 1] and [r["rank"] for r in c5["per_rank"]] == [0, 1]
    assert all(r["bit_exact"] is True for r in d["per_rank"])
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "configs.json")))["0"]["shard_sha256"]
    assert [r["out_sha256"] for r in d["per_rank"]] == gold[:2]
    assert [r["index0"] for r in d["per_rank"]] == [0, 1 << 20]
    assert all(r["kernel_ms"] > 0 for r in d["per_rank"] + c5["per_rank"])
    # device identity measured, not inferred: both ranks on this box's one card
    assert all(r["pci"] and ":" in r["pci"] for r in d["per_rank"])
    assert d["config"]["devices"] == 1 and d["config"]["ranks_per_gpu"] == 2

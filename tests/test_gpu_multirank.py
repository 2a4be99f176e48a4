"""GPU: the N > 1 path through the ENGINE (not the oracle stand-in of
tests/test_multirank.py): two processes on one card (gloo), each
checksumming its shard.fixed_stride_shard of BASELINE config 0 through
libicsum.so; the rank-ordered concatenation of their outputs must equal the
reference's SHA-256 digest of the whole batch (tests/golden/configs.json["0"])."""
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


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_engine_shards_concatenate_to_reference_digest(world):
    g = golden("configs.json")["0"]
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, WORKER], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        try:
            o, e = p.communicate(timeout=100)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append((p.returncode, o, e))
    assert all(rc == 0 for rc, _, _ in outs), [e[-1500:] for _, _, e in outs]
    line = json.loads([l for l in outs[0][1].splitlines() if l.startswith("{")][-1])
    assert line["n"] == g["n"]
    assert line["shards"][0][0] == 0 and sum(s[1] for s in line["shards"]) == g["n"]
    assert line["sha256"] == g["out_sha256"]

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through libicsum.so)")
    config.addinivalue_line("markers", "slow: long CPU oracle runs (set ICSUM_FULL_ORACLE=1)")


def golden(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def orc():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    from oracle import oracle

    return oracle


@pytest.fixture(scope="session")
def engine():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("gpu-marked test without a visible GPU (run with -m 'not gpu' on CPU hosts)")
    from tcpip_network_protocol_stack_amd.engine import Engine

    eng = Engine(0)
    yield eng
    torch.cuda.synchronize()
    eng.close()

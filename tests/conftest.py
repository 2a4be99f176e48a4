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


def engine_with(force=None, debug=False):
    """Generator: an Engine created with the ICSUM_FORCE test hook set to
    `force` ({key: value}: lps, unroll, mode, segs, bin, bin_min, bin_plan,
    bin_blocks, last_bin_lps, last_bin_blocks, dense_segs, twoclass,
    wrap_passes, xcd_remap, zero_copy_max, tile, span_segs, span_blocks,
    tick_inline, tick_server, srv_pollers, srv_blocks, srv_vram, slot_prio, poison_ticket —
    INTEGRATION.md §6), read once at
    ics_create."""
    import torch

    from tcpip_network_protocol_stack_amd.engine import Engine

    old = os.environ.pop("ICSUM_FORCE", None)
    if force:
        os.environ["ICSUM_FORCE"] = ",".join(f"{k}={v}" for k, v in force.items())
    try:
        eng = Engine(0, debug=debug)
    finally:
        os.environ.pop("ICSUM_FORCE", None)
        if old is not None:
            os.environ["ICSUM_FORCE"] = old
    eng.forced = dict(force or {})
    yield eng
    torch.cuda.synchronize()
    eng.close()


def force_id(force):
    return "-".join(f"{k}{v}" for k, v in force.items()) or "auto"


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


@pytest.fixture(scope="session", autouse=True)
def _sentinel_outputs():
    """GPU runs: every output array the Engine allocates starts as a 0x5A byte
    pattern, so an output no kernel writes cannot pass on an earlier call's
    results left in a block the caching allocator hands out again."""
    try:
        import torch
    except ImportError:  # pragma: no cover
        yield
        return
    if not torch.cuda.is_available():
        yield
        return
    import tcpip_network_protocol_stack_amd.engine as em

    real = em.torch

    class _Torch:
        def __getattr__(self, name):
            return getattr(real, name)

        @staticmethod
        def empty(*args, **kw):
            t = real.empty(*args, **kw)
            if t.is_cuda and t.numel():
                if t.dtype.is_floating_point:
                    t.fill_(float("nan"))
                else:
                    t.fill_(int.from_bytes(b"\x5a" * t.element_size(), "little", signed=t.dtype != real.uint8))
            return t

    em.torch = _Torch()
    try:
        yield
    finally:
        em.torch = real

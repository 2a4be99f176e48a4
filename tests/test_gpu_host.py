"""GPU: icsum::BatchEngine (the C++ drop-in batch API over libicsum.so) against
the per-object CPU calls of the same types, and the reference stack running
over the GPU batch path end to end (binary built where /root/reference exists)."""
import os
import subprocess

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

BIN = os.path.join(ROOT, "tcpip_network_protocol_stack_amd", "csrc", "host", "build")


def test_batch_engine_matches_per_object_calls():
    exe = os.path.join(BIN, "host_gpu_test")
    assert os.path.exists(exe), "build() did not produce host_gpu_test"
    out = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr[-3000:]
    assert out.stdout.startswith("OK:")


def test_reference_stack_over_gpu_batches():
    exe = os.path.join(BIN, "dropin_stack")
    if not os.path.exists(exe):
        pytest.skip("dropin_stack is only built where the reference sources exist")
    out = subprocess.run([exe, "--gpu"], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout[-2000:]
    assert out.stdout.startswith("OK: GPU batch path, 1048576 + 300000 bytes")


def test_batch_engine_under_asan():
    """The same checks with the host layer built with ASan+UBSan (`make asan`;
    SURVEY §5): the batch API, the threaded unwrap, the rings and their
    threads against the real engine.  Host code only — the HIP kernels and
    runtime are not instrumented (GPU sanitizers are not available)."""
    exe = os.path.join(os.path.dirname(BIN), "build-asan", "host_gpu_test")
    assert os.path.exists(exe), "build() did not produce build-asan/host_gpu_test"
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    out = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    assert out.returncode == 0, out.stdout + out.stderr[-3000:]
    assert out.stdout.startswith("OK:")
    assert "ERROR: AddressSanitizer" not in out.stderr and "runtime error:" not in out.stderr

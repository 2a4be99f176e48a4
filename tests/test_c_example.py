"""CPU: examples/c_abi_example.c — the C-ABI from plain C, as INTEGRATION.md
§3 documents it — compiles as strict C11 and C17 against include/icsum.h and
links against libicsum.so (the header is C, not C++-only; every documented
call type-checks), and without a GPU it fails loudly (ICS_ERR_NODEVICE and
the message), never silently computing on the CPU."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "tcpip_network_protocol_stack_amd")
SRC = os.path.join(ROOT, "examples", "c_abi_example.c")


def _compile(std, out):
    subprocess.check_call(["gcc", f"-std={std}", "-O2", "-Wall", "-Wextra", "-pedantic", "-Werror",
                           "-I", os.path.join(ROOT, "include"), SRC, "-L", LIB, "-licsum",
                           f"-Wl,-rpath,{LIB}", "-Wl,-rpath-link,/opt/rocm/lib", "-o", out])


@pytest.mark.parametrize("std", ["c11", "c17"])
def test_c_example_compiles_strict(tmp_path, std):
    _compile(std, str(tmp_path / "c_abi_example"))


def test_c_example_fails_loudly_without_gpu(tmp_path):
    import torch

    if torch.cuda.device_count() > 0:
        pytest.skip("a GPU is visible: tests/test_gpu_c_example.py runs the example")
    exe = str(tmp_path / "c_abi_example")
    _compile("c11", exe)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1
    assert "ics_create" in r.stderr and "-4" in r.stderr and "no GPU" in r.stderr, r.stderr
    assert r.stdout == ""

"""CPU: the C-ABI library loads, exports every symbol include/*.h declares, and
fails loudly (no fallback) when there is no GPU."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT


def declared_symbols():
    syms = set()
    for h in ("icsum.h", "icsum_workload.h"):
        text = open(os.path.join(ROOT, "include", h)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        syms |= set(re.findall(r"\b(ics[w]?_[a-z0-9_]+)\s*\(", text))
    return syms


@pytest.mark.parametrize("debug", [False, True])
def test_library_exports_every_declared_symbol(debug):
    """libicsum.so and its bounds-checked build libicsum_debug.so export the
    same declared surface."""
    from tcpip_network_protocol_stack_amd import _lib

    path = _lib.DEBUG_LIB_PATH if debug else _lib.LIB_PATH
    lib = _lib.load(path)
    syms = declared_symbols()
    assert len(syms) >= 24
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    # and the ctypes binding covers exactly that surface
    assert syms == set(_lib.SIGNATURES), syms ^ set(_lib.SIGNATURES)
    out = subprocess.check_output(["nm", "-D", "--defined-only", path], text=True)
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    assert syms <= exported


def test_version_and_abi():
    from tcpip_network_protocol_stack_amd import _lib

    lib = _lib.load()
    assert lib.ics_abi_version() == 2
    assert b"gfx950" in lib.ics_version()


def test_struct_layouts_match_the_header(tmp_path):
    """The ctypes mirrors of include/icsum.h's structs have the C compiler's
    size and field offsets (a field added on one side only would make the
    library write past the caller's struct)."""
    from tcpip_network_protocol_stack_amd import _lib

    structs = {"ics_dispatch_info_t": _lib.DispatchInfo, "ics_seg_batch": _lib.SegBatch,
               "ics_dgram_batch": _lib.DgramBatch}
    lines = ['#include <stddef.h>', '#include <stdio.h>', '#include "icsum.h"', "int main(void) {"]
    for c, py in structs.items():
        t = c if c.endswith("_t") else "struct " + c
        lines.append(f'  printf("{c} size %zu\\n", sizeof({t}));')
        for f, _ in py._fields_:
            lines.append(f'  printf("{c} {f} %zu\\n", offsetof({t}, {f}));')
    lines += ["  return 0;", "}"]
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines) + "\n")
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)])
    got = dict(l.rsplit(" ", 1) for l in subprocess.check_output([str(exe)], text=True).splitlines())
    for c, py in structs.items():
        assert int(got[f"{c} size"]) == ctypes.sizeof(py), c
        for f, _ in py._fields_:
            assert int(got[f"{c} {f}"]) == getattr(py, f).offset, (c, f)


def test_no_gpu_fails_loudly():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from tcpip_network_protocol_stack_amd import _lib

    lib = _lib.load()
    n = ctypes.c_int(-1)
    assert lib.ics_device_count(ctypes.byref(n)) == 0 and n.value == 0
    ctx = ctypes.c_void_p()
    rc = lib.ics_create(0, ctypes.byref(ctx))
    assert rc == -4 and not ctx.value
    assert b"no GPU" in lib.ics_last_error()
    with pytest.raises(_lib.IcsumError):
        from tcpip_network_protocol_stack_amd.engine import Engine

        Engine(0)


def test_null_context_is_an_error_not_a_crash():
    from tcpip_network_protocol_stack_amd import _lib

    lib = _lib.load()
    assert lib.ics_checksum_batch(None, None, None, 0, 0, None, None, 0, None) == -1
    assert b"null context" in lib.ics_last_error()

"""MI355X-native Internet-checksum engine for the qmmzzdx/tcpip_network_protocol_stack path.

The product is libicsum.so (HIP kernels for gfx950 behind the C-ABI in
include/icsum.h) plus the C++ drop-in types in csrc/host/.  This Python
package is the binding used by tests/ and bench.py.
"""
from ._lib import LIB_PATH, IcsumError, load  # noqa: F401

__all__ = ["LIB_PATH", "IcsumError", "load", "Engine"]


def __getattr__(name):
    # torch is imported lazily so that `import tcpip_network_protocol_stack_amd`
    # stays cheap for the C-ABI-only users (symbol checks, FFI stubs)
    if name in ("Engine", "engine"):
        from . import engine

        return engine.Engine if name == "Engine" else engine
    raise AttributeError(name)

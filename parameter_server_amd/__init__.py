"""parameter_server_amd -- MI355X-native server-side push aggregation for
the wakensky/parameter_server push/pull KV surface.

The product is libpsg.so (HIP kernels for gfx950 + host runtime) behind the
C ABI in include/psg.h; this package holds its ctypes binding, a Python
mirror of KVVector for tests and tools, and synthetic workload generators.
"""
from ._lib import PSGError, lib  # noqa: F401

__all__ = ["PSGError", "lib"]

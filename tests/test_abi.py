"""CPU: the C-ABI library loads and exports every symbol include/psg.h
declares (no device calls)."""
import ctypes as C
import os
import re

from parameter_server_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "psg.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(psg_[a-z_0-9]+)\s*\(", src)))


def test_header_and_binding_agree():
    decl = declared_symbols()
    assert len(decl) >= 25
    assert sorted(_lib.SIGNATURES) == decl


def test_library_exports_every_declared_symbol():
    L = _lib.lib()
    for name in declared_symbols():
        assert hasattr(L, name), name
    raw = C.CDLL(_lib.LIB_PATH)
    for name in declared_symbols():
        assert C.cast(getattr(raw, name), C.c_void_p).value


def test_host_only_entry_points():
    L = _lib.lib()
    assert L.psg_abi_version() == 1
    assert L.psg_status_string(_lib.PSG_ERR_UNMATCHED) == b"pushed key not matched"
    assert L.psg_plan_max_push() == 4096
    # shard bounds is pure host arithmetic (range.h:85-98)
    import numpy as np
    from parameter_server_amd.kv_vector import shard_bounds
    b = shard_bounds(8)
    assert int(b[1]) == 2305843009213693951 and int(b[8]) == (1 << 64) - 1
    # argument validation needs no device
    assert L.psg_create(0, 7, 0, C.byref(C.c_void_p())) == _lib.PSG_ERR_ARG
    assert L.psg_shard_bounds(0, None) == _lib.PSG_ERR_ARG


def test_no_cpu_fallback_when_library_missing(tmp_path, monkeypatch):
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "libpsg.so"))
    monkeypatch.setattr(_lib, "_LIB", None)
    import pytest
    with pytest.raises(ImportError):
        _lib.lib()

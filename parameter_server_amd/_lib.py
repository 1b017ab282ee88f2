"""ctypes binding of the native C ABI (include/psg.h) in libpsg.so.

The library is built in-tree by ``__graft_entry__.build()`` (or
``make -C parameter_server_amd/csrc``).  There is no fallback: if the
shared object is missing, :func:`lib` raises, so nothing silently runs a CPU
path in its place.

``torch`` is imported before the library is loaded whenever it is
available, so that the process holds ONE HIP runtime (torch's bundled
``libamdhip64.so.7``, which then also satisfies libpsg's dependency by
soname) and device pointers / streams from torch are valid here.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# PSG_LIB_PATH: benchmarking aid (an A/B build of the same sources)
LIB_PATH = os.environ.get("PSG_LIB_PATH") or os.path.join(_HERE, "libpsg.so")

PSG_OK = 0
PSG_ERR_ARG = -1
PSG_ERR_UNMATCHED = -2
PSG_ERR_RANGE = -3
PSG_ERR_NO_TIME = -4
PSG_ERR_OOM = -5
PSG_ERR_DEVICE = -6
PSG_ERR_UNSORTED = -7
PSG_ERR_SIZE = -8
PSG_ERR_CHANNEL = -9
PSG_ERR_EMPTY_KEYS = -10
PSG_ERR_SIGNATURE = -11
PSG_KC_SIG = 1
PSG_KC_KEYS = 2
PSG_KC_ERASE = 4
PSG_MAX_SIG_LEN = 2048

PSG_F32 = 0
PSG_F64 = 1
PSG_SERIAL_MATCH = 0
PSG_PARALLEL_MATCH = 1
PSG_HOLD_BUFFERS = 0x100
# kernel-form overrides (include/psg.h): tests and A/B measurements only
PSG_FORM_PACKED = 0x1000
PSG_FORM_UNIFORM = 0x2000
PSG_PART_SEARCH = 0x4000
PSG_PART_STREAM = 0x8000
PSG_GROUP32 = 0x10000
PSG_GROUP64 = 0x20000
PSG_NO_DENSE = 0x40000
PSG_NO_ZERO_COPY = 0x80000
PSG_NO_INDEX = 0x100000
# plan option: push keys fixed for the plan's lifetime (enables the dense kernel)
PSG_STATIC_KEYS = 0x200000
PSG_FORM_CURSOR = 0x400000
PSG_NO_CURSOR = 0x800000
# psg_plan_form: the aggregate kernel a plan runs
(PSG_KERNEL_TILE, PSG_KERNEL_TILE64, PSG_KERNEL_PACKED, PSG_KERNEL_DENSE, PSG_KERNEL_CURSOR,
 PSG_KERNEL_PACKED_CURSOR) = range(6)
MAX_VALUE_ARRAYS = 4

# Every symbol include/psg.h declares, with its ctypes signature.
_u64 = C.c_uint64
_sz = C.c_size_t
_p = C.c_void_p
_pu64 = C.POINTER(C.c_uint64)
_psz = C.POINTER(C.c_size_t)


class MergeJob(C.Structure):
    """psg_merge_job (include/psg.h)."""

    _fields_ = [
        ("keys", _p),
        ("nslots", _u64),
        ("npush", C.c_int),
        ("push_keys", C.POINTER(_p)),
        ("push_vals", C.POINTER(_p)),
        ("push_n", _pu64),
        ("out", C.POINTER(_p)),
    ]


SIGNATURES = {
    "psg_abi_version": (C.c_int, []),
    "psg_status_string": (C.c_char_p, [C.c_int]),
    "psg_last_error": (C.c_char_p, []),
    "psg_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "psg_create": (C.c_int, [C.c_int, C.c_int, C.c_uint, C.POINTER(_p)]),
    "psg_destroy": (C.c_int, [_p]),
    "psg_set_flush_pushes": (C.c_int, [_p, C.c_int]),
    "psg_set_match_flags": (C.c_int, [_p, C.c_uint]),
    "psg_key_union": (C.c_int, [_p, C.c_int, _p, _sz]),
    "psg_key_size": (C.c_int, [_p, C.c_int, _psz]),
    "psg_key_copy": (C.c_int, [_p, C.c_int, _sz, _sz, _p]),
    "psg_find_range": (C.c_int, [_p, C.c_int, _u64, _u64, _psz, _psz]),
    "psg_value_assign": (C.c_int, [_p, C.c_int, _p, _sz]),
    "psg_value_size": (C.c_int, [_p, C.c_int, _psz]),
    "psg_value_copy": (C.c_int, [_p, C.c_int, _sz, _sz, _p]),
    "psg_push": (C.c_int, [_p, C.c_int, C.c_int, _u64, _u64, _p, _sz, C.c_int,
                           C.POINTER(_p)]),
    "psg_push_cached": (C.c_int, [_p, C.c_int, C.c_int, C.c_int, _u64, _u64, C.c_uint,
                                  C.c_uint32, _p, _sz, C.c_int, _p, _sz]),
    "psg_key_cache_clear": (C.c_int, [_p, C.c_int]),
    "psg_push_compressed": (C.c_int, [_p, C.c_int, C.c_int, _u64, _u64, _p, _sz, C.c_int,
                                      _p, _p]),
    "psg_key_cache_bytes": (C.c_int, [_p, C.c_int, _psz]),
    "psg_received_shape": (C.c_int, [_p, C.c_int, C.POINTER(C.c_int), _psz, _psz]),
    "psg_received": (C.c_int, [_p, C.c_int, C.c_int, C.POINTER(_p)]),
    "psg_gather": (C.c_int, [_p, C.c_int, _p, _sz, _p, _psz]),
    "psg_plan_create": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_uint,
                                  C.POINTER(MergeJob), C.c_int, C.POINTER(_p)]),
    "psg_plan_max_push": (C.c_int, []),
    "psg_plan_run": (C.c_int, [_p, _p]),
    "psg_plan_run_stage": (C.c_int, [_p, C.c_int, _p]),
    "psg_plan_matched": (C.c_int, [_p, _pu64]),
    "psg_plan_bytes": (C.c_int, [_p, _pu64, _pu64]),
    "psg_plan_form": (C.c_int, [_p, C.POINTER(C.c_int)]),
    "psg_plan_destroy": (C.c_int, [_p]),
    "psg_gather_dev": (C.c_int, [C.c_int, _p, _u64, _p, _p, _u64, _p, _p, _p]),
    "psg_key_union_dev": (C.c_int, [_p, _u64, _p, _u64, _p, _pu64, _p]),
    "psg_shard_bounds": (C.c_int, [_sz, _pu64]),
    "psg_slice_dev": (C.c_int, [_p, _u64, _u64, _u64, _p, C.c_int, _p, _p]),
    "psg_crc32c_dev": (C.c_int, [_p, _p, _u64, _u64, _p, _p, _p]),
    "psg_snappy_uncompress_dev": (C.c_int, [_p, _p, _u64, _p, _p, _p, _p]),
    "psg_snappy_uncompressed_length": (C.c_int, [_p, _sz, _psz]),
    "psg_freq_resize": (C.c_int, [_p, C.c_int, C.c_int, C.c_int]),
    "psg_freq_clear": (C.c_int, [_p, C.c_int]),
    "psg_freq_empty": (C.c_int, [_p, C.c_int, C.POINTER(C.c_int)]),
    "psg_freq_insert": (C.c_int, [_p, C.c_int, _p, _p, _sz]),
    "psg_freq_query": (C.c_int, [_p, C.c_int, _p, _sz, C.c_int, _p, _psz]),
    "psg_freq_insert_dev": (C.c_int, [_p, C.c_int, _p, _p, _sz, _p]),
    "psg_freq_query_scratch_bytes": (_sz, [_sz]),
    "psg_freq_query_dev": (C.c_int, [_p, C.c_int, _p, _sz, C.c_int, _p, _p, _p, _p]),
    "psg_freq_table": (C.c_int, [_p, C.c_int, _p, _sz]),
    "psg_comm_unique_id": (C.c_int, [_p]),
    "psg_comm_init": (C.c_int, [C.c_int, C.c_int, _p, C.c_int, C.POINTER(_p)]),
    "psg_comm_destroy": (C.c_int, [_p]),
    "psg_comm_init_loopback": (C.c_int, [C.c_int, C.c_int, C.POINTER(_p)]),
    "psg_exchange_create": (C.c_int, [_p, C.c_int, C.c_int, C.c_int, _p, _p, _p,
                                      C.POINTER(_p)]),
    "psg_exchange_run": (C.c_int, [_p, _p]),
    "psg_exchange_recv": (C.c_int, [_p, C.POINTER(_p), _p, _pu64, _p, _pu64]),
    "psg_exchange_destroy": (C.c_int, [_p]),
    "psg_exchange_status": (C.c_int, [_p, _pu64]),
    "psg_exchange_create_local": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, _p,
                                            _p, _p, C.POINTER(_p)]),
    "psg_exchange_set_direct": (C.c_int, [_p, C.c_int]),
    "psg_exchange_send_layout": (C.c_int, [_p, C.POINTER(_p), _p, _p]),
    "psg_key_union_batch": (C.c_int, [_p, C.c_int, _p, _p, C.c_int]),
    "psg_nway_max_push": (C.c_int, []),
    "psg_nway_create": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_uint, C.c_int, _p, _p, _p, _p,
                                  _p, C.POINTER(_p)]),
    "psg_nway_create_batch": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_uint, C.c_int, _p, _p, _p,
                                         _p, _p, _p, C.POINTER(_p)]),
    "psg_nway_run": (C.c_int, [_p, _p]),
    "psg_nway_count_dev": (C.c_int, [_p, C.POINTER(_p)]),
    "psg_nway_result": (C.c_int, [_p, _pu64]),
    "psg_nway_bytes": (C.c_int, [_p, _pu64, _pu64]),
    "psg_nway_destroy": (C.c_int, [_p]),
    "psg_darling_init": (C.c_int, [_p, C.c_int, C.c_double]),
    "psg_darling_reset_active": (C.c_int, [_p, C.c_int]),
    "psg_darling_update": (C.c_int, [_p, C.c_int, C.c_int, _p, C.POINTER(C.c_double)]),
    "psg_darling_state": (C.c_int, [_p, C.c_int, _sz, _sz, _p, _p, _psz]),
}

_LIB = None


class PSGError(RuntimeError):
    """A negative psg_status from the native library."""

    def __init__(self, status: int, msg: str):
        super().__init__(f"psg status {status}: {msg}")
        self.status = status


def lib() -> C.CDLL:
    """Load libpsg.so (raises if it has not been built)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` "
            "(no CPU fallback exists for this path)")
    try:  # one HIP runtime per process: let torch load it first
        import torch  # noqa: F401
    except Exception:  # pragma: no cover - torch is optional for the ABI
        pass
    L = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    if L.psg_abi_version() != 1:
        raise ImportError("libpsg ABI version mismatch")
    _LIB = L
    return L


def check(rc: int) -> None:
    if rc != PSG_OK:
        L = lib()
        raise PSGError(rc, L.psg_last_error().decode(errors="replace"))


def ptr_array(ptrs) -> "C.Array":
    arr = (_p * max(1, len(ptrs)))()
    for i, v in enumerate(ptrs):
        arr[i] = v
    return arr

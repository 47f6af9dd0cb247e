"""ctypes binding of libkbz_hip.so (include/kbz_triage.h).

There is no fallback: if the HIP library is missing or cannot be loaded this module raises,
so nothing can silently run a CPU path in its place.
"""
from __future__ import annotations

import ctypes as C
import os
import re

from . import build as _build

_LIB = None
ABI_VERSION = 3

# (name, restype, argtypes) for every function declared in include/kbz_triage.h
_vp, _sz, _i, _u32, _u64 = C.c_void_p, C.c_size_t, C.c_int, C.c_uint32, C.c_uint64
SIGNATURES = [
    ("kbz_abi_version", _i, []),
    ("kbz_last_error", C.c_char_p, []),
    ("kbz_build_flags", C.c_char_p, []),
    ("kbz_ctx_create", _vp, [_sz, _i, _sz]),
    ("kbz_ctx_destroy", None, [_vp]),
    ("kbz_set_ignore", _i, [_vp, _vp]),
    ("kbz_get_virgin", _i, [_vp, _vp]),
    ("kbz_set_virgin", _i, [_vp, _vp]),
    ("kbz_reset_virgin", _i, [_vp, _vp]),
    ("kbz_get_last_hash", _i, [_vp, C.POINTER(_u32)]),
    ("kbz_set_last_hash", _i, [_vp, _u32]),
    ("kbz_virgin_device", _vp, [_vp]),
    ("kbz_ctx_set_pass1", _i, [_vp, _i]),
    ("kbz_ctx_stats", _i, [_vp, _vp]),
    ("kbz_ctx_time_pass1", _i, [_vp, _i, C.POINTER(C.c_double), C.POINTER(_u32)]),
    ("kbz_ctx_time_pass1_every", _i, [_vp, _u32]),
    ("kbz_ctx_time_stages", _i, [_vp, _i, _vp, C.POINTER(_u32)]),
    ("kbz_triage_batch_device", _i, [_vp, _vp, _sz, _sz, _vp, _vp, _vp, _vp, _i, _vp]),
    ("kbz_triage_batch_host", _i, [_vp, _vp, _sz, _sz, _vp, _vp, _vp, _vp, _i]),
    ("kbz_ring_acquire", _i, [_vp, C.POINTER(_vp), C.POINTER(_vp), C.POINTER(_sz)]),
    ("kbz_ring_submit", _i, [_vp, _sz, _i, _vp, _vp, _vp, _i]),
    ("kbz_ring_flush", _i, [_vp]),
    ("kbz_ring_release", _i, [_vp]),
    ("kbz_ring_commit", _i, [_vp, _sz]),
    ("kbz_shard_begin", _i, [_vp, _vp, _sz, _sz, _vp, _vp, _vp, _i, _vp]),
    ("kbz_shard_last_hash", _i, [_vp, _vp, _vp]),
    ("kbz_shard_last_row", _i, [_vp, _vp, _vp]),
    ("kbz_shard_link", _i, [_vp, _vp, _vp, _i, _vp, _vp, _vp]),
    ("kbz_shard_reduce", _i, [_vp, _vp]),
    ("kbz_shard_aggregate", _i, [_vp, _vp, _vp]),
    ("kbz_shard_aggregate_bytes", _sz, [_vp]),
    ("kbz_shard_finish", _i, [_vp, _vp, _vp, _vp, _vp]),
    ("kbz_shard_exchange_row", _i, [_vp, _vp, _vp]),
    ("kbz_shard_reduce_into", _i, [_vp, _vp, _vp]),
    ("kbz_shard_finish_gathered", _i, [_vp, _vp, _sz, _sz, _vp, _vp]),
    ("kbz_or_reduce", _i, [_vp, _vp, _sz, _sz, _sz, _vp]),
    ("kbz_or_prefix_total", _i, [_vp, _vp, _vp, _sz, _sz, _sz, _vp]),
    ("kbz_merge_and_device", _i, [_vp, _vp, _sz, _sz, _vp]),
    ("kbz_merge_and_host", _i, [_vp, _vp, _sz, _sz]),
    ("kbz_merge_and_fill", _i, [_vp, _sz, _sz, _vp, _vp]),
    ("kbz_merge_and_fill_device", _i, [_vp, _sz, _sz, _vp, _vp, _vp]),
    ("kbz_merge_and_fill_devices", _i, [_vp, _sz, _sz, _vp, _vp, _vp, _sz, _i, C.POINTER(_i)]),
    ("kbz_mctx_create", _vp, [_sz, _i, _sz, _vp, _sz]),
    ("kbz_mctx_destroy", None, [_vp]),
    ("kbz_mctx_workers", _i, [_vp]),
    ("kbz_mctx_worker", _vp, [_vp, _sz]),
    ("kbz_triage_batch_devices", _i, [_vp, _vp, _sz, _sz, _vp, _vp, _vp, _i]),
    ("kbz_triage_batch_devices_resident", _i, [_vp, _vp, _vp, _sz, _vp, _vp, _vp, _i]),
    ("kbz_mctx_peer_pairs", _i, [_vp]),
    ("kbz_mctx_get_virgin", _i, [_vp, _vp]),
    ("kbz_mctx_set_virgin", _i, [_vp, _vp]),
    ("kbz_mctx_get_last_hash", _i, [_vp, C.POINTER(_u32)]),
    ("kbz_triage_modules_device", _i, [_vp, _sz, _vp, _sz, _sz, _vp, _vp, _vp, _vp, _vp, _vp]),
    ("kbz_triage_modules_host", _i, [_vp, _sz, _vp, _sz, _sz, _vp, _vp, _vp, _vp, _vp]),
    ("kbz_transform_rows_device", _i, [_vp, _sz, _sz, _sz, _i, _vp, _sz, _vp]),
    ("kbz_transform_rows_host", _i, [_vp, _sz, _sz, _sz, _i, _vp, _sz]),
    ("kbz_picker_ignore_device", _i, [_vp, _sz, _sz, _sz, _vp, _vp, _vp, _vp]),
    ("kbz_hash32_device", _i, [_vp, _sz, _sz, _sz, _u32, _vp, _vp]),
    ("kbz_xxh64_device", _i, [_vp, _sz, _sz, _sz, _u64, _vp, _vp]),
    ("kbz_sync", _i, [_vp, _vp]),
    ("kbz_set_create", _vp, [_sz]),
    ("kbz_set_destroy", None, [_vp]),
    ("kbz_set_last_error", C.c_char_p, []),
    ("kbz_set_insert_device", _i, [_vp, _vp, _vp, _sz, _vp, _vp]),
    ("kbz_set_size", _i, [_vp, C.POINTER(_sz)]),
    ("kbz_set_keys", _i, [_vp, _vp, _sz, C.POINTER(_sz)]),
    ("kbz_set_merge", _vp, [_vp, _vp, _vp]),
    ("kbz_set_insert_host", _i, [_vp, _vp, _sz, _vp]),
    ("kbz_ipt_batch_create", _vp, []),
    ("kbz_ipt_batch_destroy", None, [_vp]),
    ("kbz_ipt_last_error", C.c_char_p, []),
    ("kbz_ipt_set_ranges", _i, [_vp, _sz, _vp, _vp, _vp, _u64, _u64]),
    ("kbz_ipt_add_tnt", _i, [_vp, _vp, _i]),
    ("kbz_ipt_add_tip", _i, [_vp, _u64]),
    ("kbz_ipt_end_exec", _i, [_vp]),
    ("kbz_ipt_execs", _sz, [_vp]),
    ("kbz_ipt_hash_device", _i, [_vp, _vp, _vp]),
    ("kbz_ipt_triage", _i, [_vp, _vp, _vp, _vp]),
]


def header_functions(header: str | None = None) -> list[str]:
    """Names of the functions declared in include/kbz_triage.h."""
    header = header or os.path.join(_build.INC, "kbz_triage.h")
    text = open(header).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(kbz_[a-z0-9_]+)\s*\(", text)))


class KbzError(RuntimeError):
    pass


def lib(build_if_missing: bool = True):
    """Load libkbz_hip.so (building it first if needed and allowed)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    # KBZ_HIP_LIB: load an alternative in-tree build (A/B timing of kernel variants)
    path = os.environ.get("KBZ_HIP_LIB") or _build.HIP_LIB
    if not os.path.exists(path):
        if not build_if_missing:
            raise KbzError(f"{path} not built (run killerbeez_amd.build.build_all())")
        _build.build_hip()
    L = C.CDLL(path)
    for name, res, args in SIGNATURES:
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    if L.kbz_abi_version() != ABI_VERSION:
        raise KbzError("ABI version mismatch")
    _LIB = L
    return L


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = lib().kbz_last_error()
        raise KbzError(f"{what}: {msg.decode() if msg else 'error'}")

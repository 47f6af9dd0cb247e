"""ctypes handle on libkbz_plugin.so (include/kbz_plugin.h): the afl_gpu / dynamorio_gpu
instrumentation plugins, driven the way the reference's fuzzer and merger drive a plugin
(instrumentation/instrumentation.h:40-62).  Used by the tests; a C caller links the library
directly.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import _lib
from . import build as _build

_PLUGIN = None

_vp, _sz, _i, _l = C.c_void_p, C.c_size_t, C.c_int, C.c_long
_FN = {
    "create": (_vp, [C.c_char_p, C.c_char_p]),
    "cleanup": (None, [_vp]),
    "merge": (_vp, [_vp, _vp]),
    "merge_many": (_vp, [C.POINTER(_vp), _sz]),
    "merge_files": (_vp, [C.c_char_p, C.POINTER(C.c_char_p), _sz]),
    "get_state": (C.c_void_p, [_vp]),
    "free_state": (None, [C.c_void_p]),
    "set_state": (_i, [_vp, C.c_char_p]),
    "enable": (_i, [_vp, _vp, C.c_char_p, C.c_char_p, _sz]),
    "is_new_path": (_i, [_vp]),
    "get_fuzz_result": (_i, [_vp]),
    "is_process_done": (_i, [_vp]),
    "triage_batch": (_i, [_vp, _vp, _sz, _sz, _vp, _vp, _vp, _vp]),
    "help": (_i, [C.POINTER(C.c_char_p)]),
    "record": (_l, [_vp, _vp, _i]),
    "result": (_i, [_vp, _l]),
    "flush": (_i, [_vp]),
}
PLUGINS = ("afl_gpu", "dynamorio_gpu")
FUZZ_NONE, FUZZ_HANG, FUZZ_CRASH, FUZZ_ERROR = 0, 1, 2, -1


class VTable(C.Structure):
    """kbz_instrumentation_t: struct instrumentation's members in order + 2 appended."""
    _fields_ = [(n, C.c_void_p) for n in (
        "create", "cleanup", "merge", "get_state", "free_state", "set_state", "enable",
        "is_new_path", "get_fuzz_result", "get_module_info", "get_edges", "is_process_done",
        "triage_batch", "merge_many")]


def lib():
    global _PLUGIN
    if _PLUGIN is None:
        _lib.lib()  # the HIP library first (the plugin links it)
        # KBZ_PLUGIN_LIB: an alternative build of the same sources (scripts/sanitize.sh loads
        # its ASan + UBSan build this way)
        path = os.environ.get("KBZ_PLUGIN_LIB") or _build.PLUGIN_LIB
        if not os.path.exists(path):
            _build.build_plugin()
        L = C.CDLL(path)
        for name in PLUGINS:
            for fn, (res, args) in _FN.items():
                f = getattr(L, f"kbz_{name}_{fn}")
                f.restype, f.argtypes = res, args
        L.kbz_dynamorio_gpu_get_module_info.restype = _i
        L.kbz_dynamorio_gpu_get_module_info.argtypes = [_vp, _i, C.POINTER(_i),
                                                        C.POINTER(C.c_char_p),
                                                        C.POINTER(C.c_void_p), C.POINTER(_i)]
        L.kbz_dynamorio_gpu_get_edges.restype = _vp
        L.kbz_dynamorio_gpu_get_edges.argtypes = [_vp, _i]
        L.kbz_instrumentation_factory.restype = C.POINTER(VTable)
        L.kbz_instrumentation_factory.argtypes = [C.c_char_p]
        L.kbz_plugin_last_error.restype = C.c_char_p
        _PLUGIN = L
    return _PLUGIN


def last_error() -> str:
    e = lib().kbz_plugin_last_error()
    return e.decode() if e else ""


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


class Plugin:
    """One instrumentation state of plugin `name` ("afl_gpu" or "dynamorio_gpu")."""

    def __init__(self, name: str, options: str | None = None, state: str | None = None,
                 _handle=None):
        self.name = name
        self._f = lambda fn: getattr(lib(), f"kbz_{name}_{fn}")
        if _handle is not None:
            self.h = _handle
        else:
            self.h = self._f("create")(options.encode() if options else None,
                                       state.encode() if state else None)
        if not self.h:
            raise RuntimeError(f"{name}_create: {last_error()}")

    def close(self):
        if getattr(self, "h", None):
            self._f("cleanup")(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # per-exec API
    def record(self, trace: np.ndarray, fuzz_result: int) -> int:
        t = np.ascontiguousarray(trace, dtype=np.uint8)
        return int(self._f("record")(self.h, _p(t), int(fuzz_result)))

    def result(self, ticket: int) -> int:
        return int(self._f("result")(self.h, int(ticket)))

    def flush(self) -> int:
        return int(self._f("flush")(self.h))

    def is_new_path(self) -> int:
        return int(self._f("is_new_path")(self.h))

    def get_fuzz_result(self) -> int:
        return int(self._f("get_fuzz_result")(self.h))

    def enable(self) -> int:
        return int(self._f("enable")(self.h, None, b"", b"", 0))

    def is_process_done(self) -> int:
        return int(self._f("is_process_done")(self.h))

    def get_module_info(self, index: int, want_info: bool = True):
        """dynamorio_gpu get_module_info (dynamorio_instrumentation.c:1541-1573) as the picker
        calls it (picker/main.c:187): -> (rc, is_new, name, info uint8[size] copy or None)."""
        is_new, name, info, size = C.c_int(-1), C.c_char_p(), C.c_void_p(), C.c_int(0)
        rc = lib().kbz_dynamorio_gpu_get_module_info(
            self.h, int(index), C.byref(is_new), C.byref(name),
            C.byref(info) if want_info else None, C.byref(size))
        if rc:
            return rc, None, None, None
        arr = None
        if want_info and info.value:
            arr = np.ctypeslib.as_array(C.cast(info, C.POINTER(C.c_uint8)),
                                        shape=(size.value,)).copy()
        return rc, is_new.value, name.value.decode(), arr

    def get_edges(self, index: int = 0):
        return lib().kbz_dynamorio_gpu_get_edges(self.h, int(index))

    # batched API
    def triage_batch(self, traces: np.ndarray, outcome=None, hashes: bool = True):
        t = np.ascontiguousarray(traces, dtype=np.uint8)
        n = t.shape[0]
        oc = None if outcome is None else np.ascontiguousarray(outcome, dtype=np.int8)
        hnb = np.zeros(n, np.uint8)
        h32 = np.zeros(n, np.uint32) if hashes else None
        x64 = np.zeros(n, np.uint64) if hashes else None
        rc = self._f("triage_batch")(self.h, _p(t), n, t.shape[1] if n else 0, _p(oc), _p(hnb),
                                     _p(h32), _p(x64))
        if rc:
            raise RuntimeError(f"{self.name}_triage_batch: {last_error()}")
        return {"hnb": hnb, "h32": h32, "x64": x64}

    # state
    def get_state(self) -> str:
        p = self._f("get_state")(self.h)
        if not p:
            raise RuntimeError(f"{self.name}_get_state: {last_error()}")
        s = C.string_at(p).decode()
        self._f("free_state")(p)
        return s

    def set_state(self, state: str) -> int:
        return int(self._f("set_state")(self.h, state.encode()))

    def merge(self, other: "Plugin") -> "Plugin":
        h = self._f("merge")(self.h, other.h)
        if not h:
            raise RuntimeError(f"{self.name}_merge: {last_error()}")
        return Plugin(self.name, _handle=h)

    @staticmethod
    def merge_many(states: list["Plugin"]) -> "Plugin":
        arr = (C.c_void_p * len(states))(*[s.h for s in states])
        h = getattr(lib(), f"kbz_{states[0].name}_merge_many")(arr, len(states))
        if not h:
            raise RuntimeError(f"merge_many: {last_error()}")
        return Plugin(states[0].name, _handle=h)


    @staticmethod
    def merge_files(name: str, options: str | None, paths: list[str]) -> "Plugin":
        """The merger's loop over state files (merger/merger.c:79-99) as one GPU fold: the
        files are decoded straight into pinned staging memory by worker threads."""
        arr = (C.c_char_p * max(1, len(paths)))(*[os.fsencode(x) for x in paths])
        h = getattr(lib(), f"kbz_{name}_merge_files")(options.encode() if options else None, arr,
                                                       len(paths))
        if not h:
            raise RuntimeError(f"merge_files: {last_error()}")
        return Plugin(name, _handle=h)


def state_maps(state_json: str, map_size: int) -> dict:
    """Decode the hex maps of a state string: {"virgin_bits": uint8[map_size], ...}."""
    import json

    d = json.loads(state_json)
    out = {}
    for k in ("virgin_bits", "virgin_tmout", "virgin_crash"):
        if k in d:
            out[k] = np.frombuffer(bytes.fromhex(d[k]), np.uint8)
            assert out[k].size == map_size
    for k in ("last_shm_hash", "last_path_was_new", "last_process_status"):
        if k in d:
            out[k] = int(d[k])
    if "modules" in d:  # dynamorio per_module_coverage: {name: {virgin_bits, last_shm_hash, ...}}
        out["modules"] = {m["name"]: {"virgin_bits": np.frombuffer(bytes.fromhex(m["virgin_bits"]),
                                                                   np.uint8),
                                      "last_shm_hash": int(m["last_shm_hash"]),
                                      "last_path_was_new": int(m["last_path_was_new"])}
                          for m in d["modules"]}
    return out


def state_json(maps: dict, map_size: int) -> str:
    import json

    d = {"map_size": map_size}
    for k, v in maps.items():
        if k == "modules":
            d[k] = [{"name": name, "virgin_bits": bytes(np.asarray(m["virgin_bits"], np.uint8)).hex(),
                     "last_shm_hash": int(m.get("last_shm_hash", 0)),
                     "last_path_was_new": int(m.get("last_path_was_new", 0))}
                    for name, m in v.items()]
        elif k in ("last_shm_hash", "last_path_was_new", "last_process_status"):
            d[k] = int(v)
        else:
            d[k] = bytes(np.asarray(v, np.uint8)).hex()
    return json.dumps(d)

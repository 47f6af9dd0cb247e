"""Host-side handle on the gfx950 triage engine (over include/kbz_triage.h via ctypes).

Device memory and streams come from PyTorch (``torch.cuda`` tensors and their
``data_ptr()``; ``torch.cuda.current_stream().cuda_stream``); all arithmetic runs in the HIP
kernels of libkbz_hip.so.  See include/kbz_triage.h for the reference functions each call
replaces.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import KbzError, check, lib

MODE_AFL, MODE_DYNAMORIO, MODE_AFL_CLASSIFY = 0, 1, 2
FUZZ_NONE, FUZZ_HANG, FUZZ_CRASH = 0, 1, 2
WANT_H32, WANT_X64 = 1, 2
MODES = {"afl": MODE_AFL, "dynamorio": MODE_DYNAMORIO, "afl_classify": MODE_AFL_CLASSIFY}
PASS1_AUTO, PASS1_NARROW, PASS1_WIDE = 0, 1, 2
XF_RAW, XF_CLASSIFY, XF_SIMPLIFY = 0, 1, 2
PASS1 = {"auto": PASS1_AUTO, "narrow": PASS1_NARROW, "wide": PASS1_WIDE}


def _np_ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def _stream_handle(stream):
    import torch

    if stream is None:
        stream = torch.cuda.current_stream()
    return C.c_void_p(stream.cuda_stream)


def _host_batch(traces, outcome, map_size):
    """A host batch as the C side reads it: uint8 rows of exactly map_size bytes (stride =
    map_size) and, if given, one int8 outcome per row -- checked here, since a narrower array or
    a short outcome would make the C copies read past the caller's buffers."""
    t = np.ascontiguousarray(traces, dtype=np.uint8)
    if t.ndim != 2 or t.shape[1] != map_size:
        raise ValueError(f"traces must be 2-D [n, {map_size}], got shape {t.shape}")
    oc = None
    if outcome is not None:
        oc = np.ascontiguousarray(outcome, dtype=np.int8)
        if oc.ndim != 1 or oc.shape[0] != t.shape[0]:
            raise ValueError(f"outcome must hold one entry per trace ({t.shape[0]}), got shape "
                             f"{oc.shape}")
    return t, oc


def nclass(mode: int) -> int:
    return 1 if mode == MODE_DYNAMORIO else 3


class TriageContext:
    """One virgin-map state (3 maps) + workspace on the current GPU.

    Mirrors the bitmap half of the AFL/DynamoRIO instrumentation state
    (instrumentation/afl_instrumentation.h:12-34): virgin_bits/tmout/crash, last hash."""

    def __init__(self, map_size: int = 65536, mode: int | str = MODE_AFL,
                 max_batch: int = 65536, pass1: int | str | None = None):
        if isinstance(mode, str):
            mode = MODES[mode]
        self.map_size, self.mode, self.max_batch = int(map_size), int(mode), int(max_batch)
        L = lib()
        self._h = L.kbz_ctx_create(self.map_size, self.mode, self.max_batch)
        if not self._h:
            raise KbzError("kbz_ctx_create: " + (L.kbz_last_error() or b"").decode())
        if pass1 is not None:
            self.set_pass1(pass1)

    def set_pass1(self, choice: int | str) -> None:
        """Force the pass-1 kernel ("auto" / "narrow" / "wide"; results are identical)."""
        if isinstance(choice, str):
            choice = PASS1[choice]
        check(lib().kbz_ctx_set_pass1(self._h, int(choice)), "kbz_ctx_set_pass1")

    def stats(self) -> dict:
        """Work counters of the last finished batch (kbz_ctx_stats).  "claims" counts the claim
        items appended for k_resolve (window items); claimed bytes k_scan resolves itself are not
        in it."""
        out = np.zeros(3, np.uint32)
        check(lib().kbz_ctx_stats(self._h, _np_ptr(out)), "kbz_ctx_stats")
        return {"claims": int(out[0]), "fixed_chunks": int(out[1]), "bad_rows": int(out[2])}

    def time_pass1(self, enable: bool = True):
        """-> (summed ms, launches) of the pass-1 launches timed since the last call (HIP events
        around each launch); then times later launches iff `enable`."""
        ms, k = C.c_double(), C.c_uint32()
        check(lib().kbz_ctx_time_pass1(self._h, int(bool(enable)), C.byref(ms), C.byref(k)),
              "kbz_ctx_time_pass1")
        return ms.value, k.value

    def time_pass1_every(self, every: int) -> None:
        """While pass-1 timing is on, time one launch in `every` (events on a dispatch leave ~5 us
        of idle GPU behind it: a benchmark samples the launches).  No sync."""
        check(lib().kbz_ctx_time_pass1_every(self._h, int(every)), "kbz_ctx_time_pass1_every")

    STAGES = ("pass1", "skip", "link", "reduce", "scan", "resolve", "pack")

    def time_stages(self, enable: bool = True):
        """-> ({stage: summed ms}, batches) of the stages after pass 1 (k_skip ... k_pack) timed
        since the last call; then times later batches iff `enable`."""
        ms = np.zeros(len(self.STAGES), np.float64)
        nb = C.c_uint32()
        check(lib().kbz_ctx_time_stages(self._h, int(bool(enable)), _np_ptr(ms), C.byref(nb)),
              "kbz_ctx_time_stages")
        return {k: float(v) for k, v in zip(self.STAGES[1:], ms[1:])}, nb.value

    # -- lifetime --------------------------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None):
            lib().kbz_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def handle(self):
        return self._h

    # -- state -----------------------------------------------------------------------------
    def get_virgin(self) -> np.ndarray:
        out = np.empty((3, self.map_size), np.uint8)
        check(lib().kbz_get_virgin(self._h, _np_ptr(out)), "kbz_get_virgin")
        return out

    def set_virgin(self, v: np.ndarray) -> None:
        v = np.ascontiguousarray(v, dtype=np.uint8).reshape(3, self.map_size)
        check(lib().kbz_set_virgin(self._h, _np_ptr(v)), "kbz_set_virgin")

    def reset_virgin(self, stream=None) -> None:
        """All-0xff virgin maps for the next batch on `stream`, stream-ordered (no host sync)."""
        check(lib().kbz_reset_virgin(self._h, _stream_handle(stream)), "kbz_reset_virgin")

    @property
    def last_hash(self) -> int:
        x = C.c_uint32()
        check(lib().kbz_get_last_hash(self._h, C.byref(x)), "kbz_get_last_hash")
        return x.value

    @last_hash.setter
    def last_hash(self, v: int) -> None:
        check(lib().kbz_set_last_hash(self._h, int(v) & 0xFFFFFFFF), "kbz_set_last_hash")

    def set_ignore(self, ignore) -> None:
        if ignore is None:
            check(lib().kbz_set_ignore(self._h, None), "kbz_set_ignore")
            return
        ig = np.ascontiguousarray(ignore, dtype=np.uint8).reshape(self.map_size)
        check(lib().kbz_set_ignore(self._h, _np_ptr(ig)), "kbz_set_ignore")

    def sync(self, stream=None) -> None:
        check(lib().kbz_sync(self._h, _stream_handle(stream)), "kbz_sync")

    # -- triage ----------------------------------------------------------------------------
    def triage(self, traces, outcome=None, want: int = WANT_H32, out=None, stream=None):
        """Device-resident batch: traces is a CUDA uint8 tensor [n, map_size] (rows may be
        strided).  Returns dict of CUDA tensors hnb (uint8), h32 (int32 view of uint32),
        x64 (int64 view of uint64; only with WANT_X64)."""
        import torch

        assert traces.is_cuda and traces.dtype == torch.uint8 and traces.dim() == 2
        n = traces.shape[0]
        if n and traces.shape[1] != self.map_size:
            raise ValueError("trace rows must be map_size bytes")
        stride = traces.stride(0) if n else self.map_size
        if n and traces.stride(1) != 1:
            raise ValueError("trace rows must be contiguous")
        dev = traces.device
        if out is None:
            out = {"hnb": torch.empty(n, dtype=torch.uint8, device=dev)}
            if want & WANT_H32:
                out["h32"] = torch.empty(n, dtype=torch.int32, device=dev)
            if want & WANT_X64:
                out["x64"] = torch.empty(n, dtype=torch.int64, device=dev)
        oc = None
        if outcome is not None:
            oc = outcome.to(device=dev, dtype=torch.int8).contiguous()
            if stream is not None:  # the kernels read it on `stream` after this returns
                oc.record_stream(stream)
        rc = lib().kbz_triage_batch_device(
            self._h, C.c_void_p(traces.data_ptr()), n, stride,
            None if oc is None else C.c_void_p(oc.data_ptr()),
            C.c_void_p(out["hnb"].data_ptr()),
            C.c_void_p(out["h32"].data_ptr()) if "h32" in out else None,
            C.c_void_p(out["x64"].data_ptr()) if "x64" in out else None,
            want, _stream_handle(stream))
        check(rc, "kbz_triage_batch_device")
        return out

    def triage_host(self, traces: np.ndarray, outcome=None, want: int = WANT_H32):
        """Host-memory batch (numpy uint8 [n, map_size]); streamed through pinned slots."""
        t, oc = _host_batch(traces, outcome, self.map_size)
        n = t.shape[0]
        hnb = np.zeros(n, np.uint8)
        h32 = np.zeros(n, np.uint32) if want & WANT_H32 else None
        x64 = np.zeros(n, np.uint64) if want & WANT_X64 else None
        rc = lib().kbz_triage_batch_host(self._h, _np_ptr(t), n, self.map_size, _np_ptr(oc),
                                         _np_ptr(hnb), _np_ptr(h32), _np_ptr(x64), want)
        check(rc, "kbz_triage_batch_host")
        res = {"hnb": hnb}
        if h32 is not None:
            res["h32"] = h32
        if x64 is not None:
            res["x64"] = x64
        return res

    # -- pinned ingest ring (zero-copy producer path; include/kbz_triage.h kbz_ring_*) ------
    def ring_acquire(self):
        """-> (rows, outcome): numpy views of the next pinned slot, uint8 [cap, map_size] and
        int8 [cap].  Blocks until that slot's previous batch is done."""
        rows, oc, cap = C.c_void_p(), C.c_void_p(), C.c_size_t()
        check(lib().kbz_ring_acquire(self._h, C.byref(rows), C.byref(oc), C.byref(cap)),
              "kbz_ring_acquire")
        n = cap.value
        r = np.ctypeslib.as_array(C.cast(rows, C.POINTER(C.c_uint8)), shape=(n, self.map_size))
        o = np.ctypeslib.as_array(C.cast(oc, C.POINTER(C.c_int8)), shape=(n,))
        return r, o

    def ring_submit(self, n, have_outcome=True, hnb_out=None, h32_out=None, x64_out=None,
                    want: int = WANT_H32):
        """Queue the slot's first n rows; the numpy result buffers are filled when the slot is
        acquired again or at ring_flush (keep them alive until then)."""
        check(lib().kbz_ring_submit(self._h, n, int(bool(have_outcome)), _np_ptr(hnb_out),
                                    _np_ptr(h32_out), _np_ptr(x64_out), want), "kbz_ring_submit")

    def ring_commit(self, n_ready):
        """Rows [0, n_ready) of the acquired slot are written: start their copy to the GPU."""
        check(lib().kbz_ring_commit(self._h, n_ready), "kbz_ring_commit")

    def ring_flush(self):
        check(lib().kbz_ring_flush(self._h), "kbz_ring_flush")

    # -- sharded triage (one rank's part; see killerbeez_amd.dist) --------------------------
    def shard_begin(self, traces, outcome=None, want=WANT_H32, out=None, stream=None):
        import torch

        n = traces.shape[0]
        stride = traces.stride(0) if n else self.map_size
        dev = traces.device
        if out is None:
            out = {"hnb": torch.empty(n, dtype=torch.uint8, device=dev)}
            if want & WANT_H32:
                out["h32"] = torch.empty(n, dtype=torch.int32, device=dev)
            if want & WANT_X64:
                out["x64"] = torch.empty(n, dtype=torch.int64, device=dev)
        self._oc = None if outcome is None else outcome.to(device=dev, dtype=torch.int8).contiguous()
        if self._oc is not None and stream is not None:
            self._oc.record_stream(stream)
        self._out = out
        rc = lib().kbz_shard_begin(
            self._h, C.c_void_p(traces.data_ptr()) if n else None, n, stride,
            None if self._oc is None else C.c_void_p(self._oc.data_ptr()),
            C.c_void_p(out["h32"].data_ptr()) if "h32" in out else None,
            C.c_void_p(out["x64"].data_ptr()) if "x64" in out else None,
            want, _stream_handle(stream))
        check(rc, "kbz_shard_begin")
        return out

    def shard_last_hash(self, out, stream=None):
        """Copy {h32 of this shard's last trace, nonempty} into CUDA int32 tensor out[2]."""
        check(lib().kbz_shard_last_hash(self._h, C.c_void_p(out.data_ptr()),
                                        _stream_handle(stream)), "kbz_shard_last_hash")
        return out

    def shard_last_row(self, out, stream=None):
        """Copy this shard's last raw trace into CUDA uint8 tensor out[map_size]."""
        check(lib().kbz_shard_last_row(self._h, C.c_void_p(out.data_ptr()),
                                       _stream_handle(stream)), "kbz_shard_last_row")
        return out

    def shard_link(self, prev_last, prev_row, is_first, global_last, global_row, stream=None):
        """prev_last / global_last: CUDA int32 tensors [2] (or None); prev_row / global_row:
        CUDA uint8 [map_size] last raw traces of those ranks (or None)."""
        ptr = lambda t: None if t is None else C.c_void_p(t.data_ptr())
        check(lib().kbz_shard_link(self._h, ptr(prev_last), ptr(prev_row), int(bool(is_first)),
                                   ptr(global_last), ptr(global_row), _stream_handle(stream)),
              "kbz_shard_link")

    def shard_reduce(self, stream=None):
        check(lib().kbz_shard_reduce(self._h, _stream_handle(stream)), "kbz_shard_reduce")

    def shard_aggregate(self, out, stream=None):
        """Copy this shard's OR aggregate into CUDA uint8 tensor out[nclass*map_size]."""
        check(lib().kbz_shard_aggregate(self._h, C.c_void_p(out.data_ptr()),
                                        _stream_handle(stream)), "kbz_shard_aggregate")
        return out

    def shard_aggregate_bytes(self) -> int:
        return lib().kbz_shard_aggregate_bytes(self._h)

    def shard_finish(self, prefix, total, stream=None):
        out = self._out
        ptr = lambda t: None if t is None else C.c_void_p(t.data_ptr())
        check(lib().kbz_shard_finish(self._h, ptr(prefix), ptr(total), ptr(out["hnb"]),
                                     _stream_handle(stream)), "kbz_shard_finish")
        return out

    # the protocol with fewer launches per step (include/kbz_triage.h, round 6)
    def shard_exchange_row(self, out, stream=None):
        """This shard's last raw trace and hash pair into CUDA uint8 out[map_size + 8 ...]: the
        row at [0, map_size), the int32 pair at [map_size, map_size + 8); one launch."""
        check(lib().kbz_shard_exchange_row(self._h, C.c_void_p(out.data_ptr()),
                                           _stream_handle(stream)), "kbz_shard_exchange_row")
        return out

    def shard_reduce_into(self, out, stream=None):
        """Fix path + this shard's OR aggregate straight into CUDA uint8 out[nclass*map_size]
        (e.g. this rank's slot of the all-gather buffer)."""
        check(lib().kbz_shard_reduce_into(self._h, C.c_void_p(out.data_ptr()),
                                          _stream_handle(stream)), "kbz_shard_reduce_into")
        return out

    def shard_finish_gathered(self, gathered, rank, world, stream=None):
        """Resolve with the prefix / total of the all-gathered aggregates
        (CUDA uint8 [world, nclass*map_size]) inside the fused tail."""
        out = self._out
        check(lib().kbz_shard_finish_gathered(self._h, C.c_void_p(gathered.data_ptr()), rank,
                                              world, C.c_void_p(out["hnb"].data_ptr()),
                                              _stream_handle(stream)),
              "kbz_shard_finish_gathered")
        return out

    @staticmethod
    def or_reduce(out, stacked, r_lo, r_hi, nbytes, stream=None):
        return or_reduce(out, stacked, r_lo, r_hi, nbytes, stream)

    @staticmethod
    def or_prefix_total(prefix, total, stacked, rank, world, nbytes, stream=None):
        """prefix = OR of rows [0, rank) (None: skipped), total = OR of all rows, one launch."""
        check(lib().kbz_or_prefix_total(None if prefix is None else C.c_void_p(prefix.data_ptr()),
                                        C.c_void_p(total.data_ptr()),
                                        C.c_void_p(stacked.data_ptr()), rank, world, nbytes,
                                        _stream_handle(stream)), "kbz_or_prefix_total")
        return prefix, total


# ---- stateless device helpers ------------------------------------------------------------------

def merge_and(states, out=None, stream=None):
    """AND-fold of CUDA uint8 states [n, state_bytes] (merger/merger.c:79-99)."""
    import torch

    n = states.shape[0]
    nbytes = states.shape[1] if states.dim() == 2 else (states[0].numel() if n else 0)
    if out is None:
        out = torch.empty(nbytes, dtype=torch.uint8, device=states.device)
    check(lib().kbz_merge_and_device(C.c_void_p(out.data_ptr()),
                                     C.c_void_p(states.data_ptr()) if n else None, n, nbytes,
                                     _stream_handle(stream)), "kbz_merge_and_device")
    return out


def merge_and_host(states: np.ndarray) -> np.ndarray:
    s = np.ascontiguousarray(states, dtype=np.uint8)
    n = s.shape[0]
    nbytes = s[0].size if n else 0
    out = np.empty(nbytes, np.uint8)
    check(lib().kbz_merge_and_host(_np_ptr(out), _np_ptr(s), n, nbytes), "kbz_merge_and_host")
    return out


EXCHANGE_AUTO, EXCHANGE_COPY, EXCHANGE_RCCL = 0, 1, 2
_FILL_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t)


def merge_and_devices(states: np.ndarray, devices=None, exchange: int = EXCHANGE_AUTO):
    """The merger fold sharded over GPUs from C (kbz_merge_and_fill_devices): host states
    [n, state_bytes] are handed to the workers through the fill callback (called from the
    library's worker threads).  devices: ordinals (a device may repeat) or None = every visible
    GPU.  Returns (merged state, exchange used)."""
    s = np.ascontiguousarray(states, dtype=np.uint8)
    n = s.shape[0]
    nbytes = s[0].size if n else (s.shape[1] if s.ndim == 2 else 0)
    flat = s.reshape(n, nbytes)

    def fill(_user, dst, first, count):
        try:
            C.memmove(dst, flat[first:first + count].ctypes.data, count * nbytes)
            return 0
        except Exception:  # noqa: BLE001 - reported to the library as a failed fill
            return 1

    cb = _FILL_FN(fill)
    out = np.empty(nbytes, np.uint8)
    used = C.c_int(-1)
    if devices is None:
        dev_arr, ndev = None, 0
    else:
        dev_arr = (C.c_int * len(devices))(*devices)
        ndev = len(devices)
    check(lib().kbz_merge_and_fill_devices(_np_ptr(out), n, nbytes, C.cast(cb, C.c_void_p), None,
                                           C.cast(dev_arr, C.c_void_p) if dev_arr is not None
                                           else None, ndev, exchange, C.byref(used)),
          "kbz_merge_and_fill_devices")
    return out, used.value


class MultiTriageContext:
    """Sharded triage over several GPUs of one node from C (kbz_mctx_*,
    kbz_triage_batch_devices): worker w is a context on devices[w] (a device may repeat); a host
    batch is split into contiguous shards, one per worker, and the results are those of one
    sequential pass over the whole batch (the reference's per-exec has_new_bits)."""

    def __init__(self, map_size: int = 65536, mode: int | str = MODE_AFL,
                 max_batch: int = 65536, devices=(0,)):
        if isinstance(mode, str):
            mode = MODES[mode]
        self.map_size, self.mode = map_size, mode
        arr = (C.c_int * len(devices))(*devices)
        self._h = lib().kbz_mctx_create(map_size, mode, max_batch, C.cast(arr, C.c_void_p),
                                        len(devices))
        if not self._h:
            raise KbzError((lib().kbz_last_error() or b"kbz_mctx_create failed").decode())

    def close(self):
        if getattr(self, "_h", None):
            lib().kbz_mctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def workers(self) -> int:
        return lib().kbz_mctx_workers(self._h)

    def triage_host(self, traces: np.ndarray, outcome=None, want: int = WANT_H32):
        t, oc = _host_batch(traces, outcome, self.map_size)
        n = t.shape[0]
        hnb = np.zeros(n, np.uint8)
        h32 = np.zeros(n, np.uint32)
        check(lib().kbz_triage_batch_devices(self._h, _np_ptr(t) if n else None, n, self.map_size,
                                             None if oc is None else _np_ptr(oc), _np_ptr(hnb),
                                             _np_ptr(h32), want), "kbz_triage_batch_devices")
        return {"hnb": hnb, "h32": h32}

    def peer_pairs(self) -> int:
        """Ordered pairs of the workers' distinct devices with peer access enabled."""
        return lib().kbz_mctx_peer_pairs(self._h)

    def triage_resident(self, shards, outcomes=None, want: int = WANT_H32):
        """A batch already on the devices: shards[w] is worker w's uint8 [n_w, map_size] tensor
        on its device (the batch is shard 0's rows, then shard 1's, ...), outcomes[w] its int8
        [n_w] tensor (or None).  Returns per-worker device tensors {"hnb": [...], "h32": [...]}."""
        import torch

        W = self.workers()
        if len(shards) != W or (outcomes is not None and len(outcomes) != W):
            raise ValueError(f"one shard (and outcome) per worker ({W})")
        ptrs = (C.c_void_p * W)()
        ops = (C.c_void_p * W)()
        hp = (C.c_void_p * W)()
        h3 = (C.c_void_p * W)()
        ns = (C.c_size_t * W)()
        hnb, h32 = [], []
        for w, t in enumerate(shards):
            if t.dim() != 2 or t.shape[1] != self.map_size or t.dtype != torch.uint8 or \
                    not t.is_contiguous():
                raise ValueError("each shard: a contiguous uint8 [n, map_size] tensor")
            ns[w] = t.shape[0]
            ptrs[w] = t.data_ptr() if t.shape[0] else None
            if outcomes is not None:
                o = outcomes[w]
                if o.dtype != torch.int8 or o.shape[0] != t.shape[0]:
                    raise ValueError("each outcome: int8 [n] on its shard's device")
                ops[w] = o.data_ptr() if t.shape[0] else None
            hnb.append(torch.empty(max(1, t.shape[0]), dtype=torch.uint8, device=t.device))
            h32.append(torch.empty(max(1, t.shape[0]), dtype=torch.int32, device=t.device))
            hp[w], h3[w] = hnb[-1].data_ptr(), h32[-1].data_ptr()
        check(lib().kbz_triage_batch_devices_resident(
            self._h, C.cast(ptrs, C.c_void_p), C.cast(ns, C.c_void_p), self.map_size,
            None if outcomes is None else C.cast(ops, C.c_void_p), C.cast(hp, C.c_void_p),
            C.cast(h3, C.c_void_p), want), "kbz_triage_batch_devices_resident")
        return {"hnb": [h[:shards[w].shape[0]] for w, h in enumerate(hnb)],
                "h32": [h[:shards[w].shape[0]] for w, h in enumerate(h32)]}

    def get_virgin(self) -> np.ndarray:
        v = np.empty((3, self.map_size), np.uint8)
        check(lib().kbz_mctx_get_virgin(self._h, _np_ptr(v)), "kbz_mctx_get_virgin")
        return v

    def set_virgin(self, v: np.ndarray) -> None:
        v = np.ascontiguousarray(v, dtype=np.uint8)
        check(lib().kbz_mctx_set_virgin(self._h, _np_ptr(v)), "kbz_mctx_set_virgin")

    @property
    def last_hash(self) -> int:
        out = C.c_uint32()
        check(lib().kbz_mctx_get_last_hash(self._h, C.byref(out)), "kbz_mctx_get_last_hash")
        return out.value

    @last_hash.setter
    def last_hash(self, v: int) -> None:
        """Every worker's context: a worker whose earlier workers hold no rows links its row 0
        to its own context's last hash."""
        for w in range(self.workers()):
            check(lib().kbz_set_last_hash(lib().kbz_mctx_worker(self._h, w), int(v) & 0xFFFFFFFF),
                  "kbz_set_last_hash")

    def set_ignore(self, ignore) -> None:
        """DynamoRIO ignore bytes (has_new_bits_with_ignore) on every worker; None clears them."""
        ig = None if ignore is None else np.ascontiguousarray(ignore, dtype=np.uint8).reshape(
            self.map_size)
        for w in range(self.workers()):
            check(lib().kbz_set_ignore(lib().kbz_mctx_worker(self._h, w),
                                       None if ig is None else _np_ptr(ig)), "kbz_set_ignore")


def triage_modules(ctxs, traces, offsets, outcome=None, stream=None, hashes=False):
    """DynamoRIO per-module coverage (has_new_coverage_per_module,
    dynamorio_instrumentation.c:1477-1493) over an ordered batch.  ctxs: one TriageContext per
    module; traces: CUDA uint8 [n, row_bytes] holding every module's map at offsets[m].
    Returns (hnb [k, n] uint8 per module, any [n] uint8: OR over modules), plus h32 [k, n] int32
    (each module's hash32 per exec) when `hashes`."""
    import torch

    n, k = traces.shape[0], len(ctxs)
    hs = (C.c_void_p * max(k, 1))(*[c.handle for c in ctxs])
    offs = (C.c_size_t * max(k, 1))(*offsets)
    hnb = torch.empty((k, n), dtype=torch.uint8, device=traces.device)
    anyv = torch.empty(n, dtype=torch.uint8, device=traces.device)
    h32 = torch.empty((k, n), dtype=torch.int32, device=traces.device) if hashes else None
    oct = None
    if outcome is not None:  # device int8, alive until the kernels on `stream` have read it
        oct = outcome.to(device=traces.device, dtype=torch.int8).contiguous()
        if stream is not None:
            oct.record_stream(stream)
    oc = None if oct is None else C.c_void_p(oct.data_ptr())
    check(lib().kbz_triage_modules_device(hs, k, C.c_void_p(traces.data_ptr()) if n else None,
                                          n, traces.stride(0), offs, oc,
                                          C.c_void_p(hnb.data_ptr()) if n else None,
                                          C.c_void_p(anyv.data_ptr()) if n else None,
                                          C.c_void_p(h32.data_ptr()) if (hashes and n) else None,
                                          _stream_handle(stream)), "kbz_triage_modules_device")
    return (hnb, anyv, h32) if hashes else (hnb, anyv)


def transform_rows(rows, xf, out=None, stream=None):
    """classify_counts (xf=XF_CLASSIFY, dynamorio_instrumentation.c:265-292) or simplify_trace
    (XF_SIMPLIFY, afl_instrumentation.c:674-706) of every row of a CUDA uint8 [n, len] tensor
    (len % 16 == 0) into out (default: a new tensor)."""
    import torch

    n, ln = rows.shape
    if out is None:
        out = torch.empty((n, ln), dtype=torch.uint8, device=rows.device)
    check(lib().kbz_transform_rows_device(C.c_void_p(rows.data_ptr()) if n else None, n,
                                          rows.stride(0) if n else ln, ln, int(xf),
                                          C.c_void_p(out.data_ptr()) if n else None,
                                          out.stride(0) if n else ln, _stream_handle(stream)),
          "kbz_transform_rows_device")
    return out


def picker_ignore(runs, stream=None):
    """The picker's ignore-bytes diff (picker/main.c:240-262) for one module.  runs: CUDA uint8
    [files, iters, size] (size % 16 == 0).  Returns (ignore [size] uint8: 0x00 = noisy byte,
    0xff = keep; pair_counts [files, iters-1] int32: differing bytes per consecutive pair;
    total: 0-d int64 tensor, the number of noisy bytes), all on the device."""
    import torch

    files, iters, size = runs.shape
    runs = runs.contiguous()
    ign = torch.empty(size, dtype=torch.uint8, device=runs.device)
    pc = torch.empty((files, max(iters - 1, 0)), dtype=torch.int32, device=runs.device)
    tot = torch.empty((), dtype=torch.int64, device=runs.device)
    check(lib().kbz_picker_ignore_device(C.c_void_p(runs.data_ptr()) if runs.numel() else None,
                                         files, iters, size, C.c_void_p(ign.data_ptr()),
                                         C.c_void_p(pc.data_ptr()) if pc.numel() else None,
                                         C.c_void_p(tot.data_ptr()), _stream_handle(stream)),
          "kbz_picker_ignore_device")
    return ign, pc, tot


def or_reduce(out, stacked, r_lo, r_hi, nbytes, stream=None):
    check(lib().kbz_or_reduce(C.c_void_p(out.data_ptr()), C.c_void_p(stacked.data_ptr()), r_lo,
                              r_hi, nbytes, _stream_handle(stream)), "kbz_or_reduce")
    return out


def hash32_rows(rows, length=None, seed=0xA5B35705, stream=None):
    import torch

    n = rows.shape[0]
    length = rows.shape[1] if length is None else length
    out = torch.empty(n, dtype=torch.int32, device=rows.device)
    check(lib().kbz_hash32_device(C.c_void_p(rows.data_ptr()), n, rows.stride(0), length, seed,
                                  C.c_void_p(out.data_ptr()), _stream_handle(stream)),
          "kbz_hash32_device")
    return out


def xxh64_rows(rows, length=None, seed=0, stream=None):
    import torch

    n = rows.shape[0]
    length = rows.shape[1] if length is None else length
    out = torch.empty(n, dtype=torch.int64, device=rows.device)
    check(lib().kbz_xxh64_device(C.c_void_p(rows.data_ptr()), n, rows.stride(0), length, seed,
                                 C.c_void_p(out.data_ptr()), _stream_handle(stream)),
          "kbz_xxh64_device")
    return out


class UniqueSet:
    """Insert-if-absent set of 16-byte keys on the GPU (kbz_set_*; the reference's hash-set
    novelty, linux_ipt_instrumentation.c:412-424): the unique crash/hang table."""

    def __init__(self, capacity: int):
        L = lib()
        self._h = L.kbz_set_create(int(capacity))
        if not self._h:
            raise KbzError("kbz_set_create: " + (L.kbz_set_last_error() or b"").decode())

    def close(self):
        if getattr(self, "_h", None):
            lib().kbz_set_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc != 0:
            raise KbzError(f"{what}: {(lib().kbz_set_last_error() or b'').decode()}")

    def insert(self, keys, mask=None, stream=None):
        """keys: CUDA int64 tensor [n, 2]; mask: CUDA bool/uint8 [n] or None.  Returns CUDA uint8
        [n]: 1 where the key was new (and is now in the set)."""
        import torch

        keys = keys.contiguous()
        n = keys.shape[0]
        out = torch.empty(n, dtype=torch.uint8, device=keys.device)
        m = None if mask is None else mask.to(torch.uint8).contiguous()
        self._check(lib().kbz_set_insert_device(
            self._h, C.c_void_p(keys.data_ptr()) if n else None,
            None if m is None else C.c_void_p(m.data_ptr()), n,
            C.c_void_p(out.data_ptr()) if n else None, _stream_handle(stream)),
            "kbz_set_insert_device")
        return out

    def size(self) -> int:
        x = C.c_size_t()
        self._check(lib().kbz_set_size(self._h, C.byref(x)), "kbz_set_size")
        return x.value

    def keys(self) -> np.ndarray:
        """All keys in insertion order, uint64 [size, 2]."""
        n = self.size()
        out = np.zeros((max(n, 1), 2), np.uint64)
        got = C.c_size_t()
        self._check(lib().kbz_set_keys(self._h, _np_ptr(out), n, C.byref(got)), "kbz_set_keys")
        return out[:got.value]

    def insert_host(self, keys: np.ndarray) -> np.ndarray:
        """Insert host keys uint64 [n, 2] in order (a state's key list being loaded); -> is_new."""
        k = np.ascontiguousarray(keys, dtype=np.uint64).reshape(-1, 2)
        out = np.zeros(max(k.shape[0], 1), np.uint8)
        self._check(lib().kbz_set_insert_host(self._h, _np_ptr(k), k.shape[0], _np_ptr(out)),
                    "kbz_set_insert_host")
        return out[:k.shape[0]]

    def merge(self, other: "UniqueSet", stream=None) -> "UniqueSet":
        """A new set: the union of self and other, self's keys first (linux_ipt_merge,
        linux_ipt_instrumentation.c:944-978).  Neither input changes."""
        L = lib()
        h = L.kbz_set_merge(self._h, other._h, _stream_handle(stream))
        if not h:
            raise KbzError("kbz_set_merge: " + (L.kbz_set_last_error() or b"").decode())
        m = UniqueSet.__new__(UniqueSet)
        m._h = h
        return m


def dedup_keys(x64, outcome):
    """Keys {XXH64 of the transformed trace, outcome class} for UniqueSet (CUDA int64 [n, 2])."""
    import torch

    return torch.stack([x64.to(torch.int64), outcome.to(torch.int64)], dim=1)


class IptBatch:
    """Intel-PT path keys for a batch of execs (kbz_ipt_*; linux_ipt_instrumentation.c
    analyze_ipt :212-425): the host parser feeds TNT bits / TIP addresses per exec, the GPU
    hashes every exec's two streams; novelty = UniqueSet insert-if-absent."""

    def __init__(self, libraries=(), target=(0, 0)):
        """libraries: [(start, end, hash32)] coverage libraries; target: (start, end) of the
        executable (used when there are no libraries): add_tip_to_hash's ASLR adjustment."""
        L = lib()
        self._h = L.kbz_ipt_batch_create()
        starts = np.array([l[0] for l in libraries], np.uint64)
        ends = np.array([l[1] for l in libraries], np.uint64)
        hashes = np.array([l[2] for l in libraries], np.uint32)
        self._chk(L.kbz_ipt_set_ranges(self._h, len(libraries), _np_ptr(starts), _np_ptr(ends),
                                       _np_ptr(hashes), int(target[0]), int(target[1])),
                  "kbz_ipt_set_ranges")

    @staticmethod
    def _chk(rc, what):
        if rc != 0:
            raise KbzError(f"{what}: {(lib().kbz_ipt_last_error() or b'').decode()}")

    def close(self):
        if getattr(self, "_h", None):
            lib().kbz_ipt_batch_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def add_tnt(self, bits: bytes, num_bits: int):
        b = np.frombuffer(bytes(bits) + b"\0" * 8, np.uint8)
        self._chk(lib().kbz_ipt_add_tnt(self._h, _np_ptr(b), int(num_bits)), "kbz_ipt_add_tnt")

    def add_tip(self, tip: int):
        self._chk(lib().kbz_ipt_add_tip(self._h, int(tip)), "kbz_ipt_add_tip")

    def end_exec(self):
        self._chk(lib().kbz_ipt_end_exec(self._h), "kbz_ipt_end_exec")

    def feed(self, events):
        """events uint64 [k, 3]: (0, bit bytes little endian, num_bits) / (1, tip, -) / (2, -, -)
        = end of exec."""
        for kind, a, b in np.asarray(events, np.uint64).reshape(-1, 3).tolist():
            if kind == 0:
                self.add_tnt(int(a).to_bytes(8, "little"), int(b))
            elif kind == 1:
                self.add_tip(int(a))
            else:
                self.end_exec()

    def execs(self) -> int:
        return lib().kbz_ipt_execs(self._h)

    def hash_device(self, stream=None):
        """-> CUDA int64 [n, 2] keys {tip, tnt} of the completed execs (the batch empties)."""
        import torch

        n = self.execs()
        out = torch.empty((n, 2), dtype=torch.int64, device="cuda")
        self._chk(lib().kbz_ipt_hash_device(self._h, C.c_void_p(out.data_ptr()) if n else None,
                                            _stream_handle(stream)), "kbz_ipt_hash_device")
        return out

    def triage(self, table: "UniqueSet"):
        """-> (keys uint64 [n, 2], is_new uint8 [n]) on the host; the batch empties."""
        n = self.execs()
        keys = np.zeros((max(n, 1), 2), np.uint64)
        isnew = np.zeros(max(n, 1), np.uint8)
        self._chk(lib().kbz_ipt_triage(self._h, table._h, _np_ptr(keys), _np_ptr(isnew)),
                  "kbz_ipt_triage")
        return keys[:n], isnew[:n]

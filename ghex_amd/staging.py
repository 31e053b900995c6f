"""staging — device <-> pinned host copies of the host-staged exchange on SDMA engines chosen by
measurement (libghx ghx_copier_*). The reference leaves this staging to its
transport (oomph device/host buffers, include/ghex/arch_traits.hpp:51-75; the non-stream-aware
branch of include/ghex/communication_object.hpp:611-637, 715-729).

hipMemcpyAsync lets the runtime pick the copy engine; on the MI355X boxes both directions of an
exchange often share one engine (they serialise) or one lands on a slow engine. A Copier probes
engines 0-3 once per process and device (a few ms), keeps the (D2H, H2D) pair with the best
concurrent rate, and issues the copies there. Tickets order copies: an H2D copy can be made to
start after a D2H copy on the engines themselves (chunked round trips overlap both directions).
Copies are invisible to the HIP runtime: kernels that read what an H2D copy wrote are enqueued
after `acquire(stream)`, which invalidates the L2 caches on that stream first."""
from __future__ import annotations

import ctypes
import sys
import threading

from . import _ghx

_copiers = {}
_lock = threading.Lock()


class Copier:
    def __init__(self, device, probe_bytes: int = 4 << 20, timeout: float = 30.0):
        import torch
        self.device = torch.device(device)
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _ghx.call("ghx_copier_create", probe_bytes, float(timeout), ctypes.byref(h))
        self.h = h
        self._lock = threading.Lock()  # the native copier is not thread-safe

    @classmethod
    def for_device(cls, device) -> "Copier":
        """The process's copier for `device` (probed at the first request)."""
        import torch
        key = torch.device(device).index or 0
        with _lock:
            c = _copiers.get(key)
            if c is None:
                c = _copiers[key] = cls(torch.device("cuda", key))
        return c

    def info(self) -> dict:
        e = [ctypes.c_int32() for _ in range(2)]
        r = [ctypes.c_float() for _ in range(3)]
        _ghx.call("ghx_copier_info", self.h, *(ctypes.byref(x) for x in e + r))
        return {"d2h_engine": e[0].value, "h2d_engine": e[1].value,
                "d2h_GBps": round(r[0].value, 2), "h2d_GBps": round(r[1].value, 2),
                "both_GBps": round(r[2].value, 2)}

    def _submit(self, dst, src, nbytes, direction, after):
        t = ctypes.c_uint64()
        with self._lock:
            _ghx.call("ghx_copier_submit", self.h, ctypes.c_void_p(dst), ctypes.c_void_p(src),
                      int(nbytes), direction, -1 if after is None else int(after), ctypes.byref(t))
        return t.value

    def d2h(self, host_ptr, dev_ptr, nbytes, after=None) -> int:
        """Device -> pinned host copy; returns its ticket. The device bytes must be complete
        (e.g. the producing kernel's event waited for on the host)."""
        return self._submit(host_ptr, dev_ptr, nbytes, 0, after)

    def h2d(self, dev_ptr, host_ptr, nbytes, after=None) -> int:
        """Pinned host -> device copy; `after`: a ticket the copy engine waits for first."""
        return self._submit(dev_ptr, host_ptr, nbytes, 1, after)

    def wait(self, ticket: int):
        with self._lock:
            _ghx.call("ghx_copier_wait", self.h, int(ticket))

    def acquire(self, stream):
        """Enqueue the L2 invalidation kernels reading H2D-copied bytes need before them."""
        _ghx.call("ghx_copier_acquire", self.h, stream.cuda_stream)

    def __del__(self):
        if sys is None or sys.is_finalizing():
            return  # process teardown releases the engines' signals itself
        try:
            if self.h:
                _ghx.lib().ghx_copier_destroy(self.h)
                self.h = None
        except Exception:
            pass

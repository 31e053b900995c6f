"""context: rank/size and the setup-time all-gather (ghex::context, include/ghex/context.hpp;
Python: bindings/python/src/ghex/context.py make_context)."""
from __future__ import annotations

import ctypes
import sys


class Context:
    """Wraps a torch.distributed process group (or a single process when none is initialised).

    The reference context wraps an MPI communicator and an oomph transport context; here the
    transport is torch.distributed (RCCL for device buffers, gloo for host tests)."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self._dist = dist if dist.is_available() and dist.is_initialized() else None
        self.group = group
        if self._dist is not None:
            self._rank = self._dist.get_rank(group)
            self._size = self._dist.get_world_size(group)
        else:
            self._rank, self._size = 0, 1
        # pipelined exchanges: one 2-rank RCCL communicator per peer pair, created on first use
        # and shared by every communication object of this context (destroyed with it)
        self._pair_comms = {}

    def rank(self) -> int:
        return self._rank

    def size(self) -> int:
        return self._size

    @property
    def distributed(self):
        return self._dist

    def all_gather_object(self, obj):
        """Setup-time all-gather (the reference's mpi::communicator::all_gather,
        include/ghex/mpi/communicator.hpp:63-160)."""
        if self._dist is None or self._size == 1:
            return [obj]
        out = [None] * self._size
        self._dist.all_gather_object(out, obj, group=self.group)
        return out

    def pair_communicators(self, peers, order):
        """One 2-rank RCCL communicator per peer (a 1-rank one for this rank itself), created at
        the first request (setup time, collective over the context: every rank reaches it
        together) and reused by every later pipelined exchange of this context. The lower rank of
        a pair draws the unique id; ids travel by the setup all-gather; communicators are
        created in `order` (the global round order: each ncclCommInitRank blocks until both ends
        have called it). Returns [(comm handle, this rank's rank in it)] in `peers` order."""
        import os

        import torch

        from . import _ghx
        me = self.rank()
        want = [p for p in peers if p not in self._pair_comms]
        if want:
            _ghx.call("ghx_rccl_open", os.path.join(os.path.dirname(torch.__file__), "lib",
                                                    "librccl.so").encode())
        mine = {}
        for p in want:
            if p == me or me < p:
                buf = (ctypes.c_ubyte * 128)()
                _ghx.call("ghx_rccl_unique_id", buf)
                mine[(me, p)] = bytes(buf)
        # collective on every call, also when this rank needs no new communicator: another rank
        # may (the call happens at the same point of every rank's program)
        every = self.all_gather_object(mine)
        for p in order(want):
            a, b = min(me, p), max(me, p)
            uid = every[a].get((a, b))  # drawn by the lower rank of the pair
            if uid is None:
                raise RuntimeError(f"no RCCL id for pair {(a, b)}: ranks disagree on peers")
            comm = ctypes.c_void_p()
            n = 1 if p == me else 2
            _ghx.call("ghx_rccl_comm_init", (ctypes.c_ubyte * 128).from_buffer_copy(uid), n,
                      0 if me <= p else 1, ctypes.byref(comm))
            self._pair_comms[p] = (comm, 0 if p == me else (1 if me < p else 0))
        return [self._pair_comms[p] for p in peers]

    def close(self):
        """Destroy the pair communicators (every pipeline that uses them must be gone)."""
        comms, self._pair_comms = self.__dict__.get("_pair_comms", {}), {}
        if comms:
            from . import _ghx
            for comm, _ in comms.values():
                _ghx.lib().ghx_rccl_comm_destroy(comm)

    def __del__(self):
        if sys is None or sys.is_finalizing():
            return  # process teardown: leave the communicators to it (RCCL's own exit path)
        try:
            self.close()
        except Exception:
            pass

    def global_rank(self, group_rank: int) -> int:
        if self._dist is None or self.group is None:
            return group_rank
        return self._dist.get_global_rank(self.group, group_rank)


def make_context(comm=None, thread_safe: bool = False) -> Context:
    """make_context(comm, thread_safe) — comm is a torch.distributed group (None = WORLD)."""
    return Context(comm)

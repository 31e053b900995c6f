"""context: rank/size and the setup-time all-gather (ghex::context, include/ghex/context.hpp;
Python: bindings/python/src/ghex/context.py make_context)."""
from __future__ import annotations


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

    def global_rank(self, group_rank: int) -> int:
        if self._dist is None or self.group is None:
            return group_rank
        return self._dist.get_global_rank(self.group, group_rank)


def make_context(comm=None, thread_safe: bool = False) -> Context:
    """make_context(comm, thread_safe) — comm is a torch.distributed group (None = WORLD)."""
    return Context(comm)

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

    def _collective_device(self):
        import torch
        if self._dist.get_backend(self.group) == "nccl":
            return torch.device("cuda", torch.cuda.current_device())
        return torch.device("cpu")

    def all_gather_array(self, arr):
        """Setup-time all-gather of one int64 array per rank (sizes may differ), as tensors (no
        pickling): the reduced halos of make_pattern<unstructured> (the reference moves them
        around its distributed_for_each ring, include/ghex/mpi/communicator.hpp:233-345)."""
        import numpy as np
        arr = np.ascontiguousarray(arr, dtype=np.int64)
        if self._dist is None or self._size == 1:
            return [arr]
        import torch
        dev = self._collective_device()
        n = torch.tensor([arr.size], dtype=torch.int64, device=dev)
        ns = [torch.empty_like(n) for _ in range(self._size)]
        self._dist.all_gather(ns, n, group=self.group)
        sizes = [int(x.item()) for x in ns]
        m = max(1, max(sizes))
        t = torch.zeros(m, dtype=torch.int64, device=dev)
        t[:arr.size] = torch.from_numpy(arr).to(dev)
        outs = [torch.empty(m, dtype=torch.int64, device=dev) for _ in range(self._size)]
        self._dist.all_gather(outs, t, group=self.group)
        return [o[:k].cpu().numpy() for o, k in zip(outs, sizes)]

    def ring_arrays(self, arr):
        """The reference's distributed_for_each (include/ghex/mpi/communicator.hpp:233-345):
        yields (rank, that rank's int64 array) for every rank, this rank's first, then passing
        the arrays around a ring (send to rank-1, receive from rank+1), so at most two arrays are
        held at a time (every rank must consume the whole generator)."""
        import numpy as np
        arr = np.ascontiguousarray(arr, dtype=np.int64)
        me, w = self.rank(), self.size()
        if self._dist is None or w == 1:
            yield me, arr
            return
        import torch
        dist, dev = self._dist, self._collective_device()
        m = torch.tensor([arr.size], dtype=torch.int64, device=dev)
        dist.all_reduce(m, op=dist.ReduceOp.MAX, group=self.group)
        cap = int(m.item()) + 1
        buf = torch.zeros(cap, dtype=torch.int64, device=dev)
        buf[0] = arr.size
        buf[1:1 + arr.size] = torch.from_numpy(arr).to(dev)
        left, right = self.global_rank((me - 1) % w), self.global_rank((me + 1) % w)
        for step in range(w):
            n = int(buf[0].item())
            yield (me + step) % w, buf[1:1 + n].cpu().numpy()
            if step < w - 1:
                nxt = torch.empty(cap, dtype=torch.int64, device=dev)
                ops = [dist.P2POp(dist.isend, buf, left, self.group),
                       dist.P2POp(dist.irecv, nxt, right, self.group)]
                for wk in dist.batch_isend_irecv(ops):
                    wk.wait()
                buf = nxt

    def exchange_arrays(self, sends, recvs):
        """Setup-time point-to-point: sends = [(dst rank, int64 array)], recvs = [(src rank,
        length)]; returns the received arrays in `recvs` order. Messages of one (src, dst) pair
        are matched in order (the reference's isend/recv of gid lists,
        include/ghex/unstructured/pattern.hpp:321, 352)."""
        import numpy as np
        me = self.rank()
        out = [None] * len(recvs)
        own = [np.ascontiguousarray(a, dtype=np.int64) for d, a in sends if d == me]
        for k, (src, n) in enumerate(recvs):
            if src == me:
                out[k] = own.pop(0)
        if self._dist is None or self._size == 1:
            return out
        import torch
        dist, dev = self._dist, self._collective_device()
        ops, keep = [], []
        for d, a in sends:
            if d != me:
                t = torch.from_numpy(np.ascontiguousarray(a, dtype=np.int64)).to(dev)
                keep.append(t)
                ops.append(dist.P2POp(dist.isend, t, self.global_rank(d), self.group))
        slots = []
        for k, (src, n) in enumerate(recvs):
            if src != me:
                t = torch.empty(int(n), dtype=torch.int64, device=dev)
                slots.append((k, t))
                ops.append(dist.P2POp(dist.irecv, t, self.global_rank(src), self.group))
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        for k, t in slots:
            out[k] = t.cpu().numpy()
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


class LoopbackWorld:
    """Several ranks as threads of one process, for the setup collectives only (patterns): the
    Python side of the C++ loopback_hub (include/ghex_amd/transport.hpp). run(fn) calls fn(ctx) on
    one thread per rank and returns the results in rank order; the native work inside
    (ghx_udomain_*, ghx_upattern_*) releases the GIL, so the ranks' setups run in parallel."""

    def __init__(self, n: int):
        import threading
        if n < 1:
            raise ValueError("LoopbackWorld needs at least one rank")
        self.n = n
        self._bar = threading.Barrier(n)
        self._slots = [None] * n
        self._mail = {}
        self._lock = threading.Lock()

    def context(self, rank: int) -> "LoopbackContext":
        return LoopbackContext(self, rank)

    def run(self, fn):
        import threading
        res, err = [None] * self.n, []
        # a fresh rendezvous per run: an earlier run's failure leaves its barrier broken and
        # possibly undelivered mail
        self._bar = threading.Barrier(self.n)
        self._slots = [None] * self.n
        self._mail = {}

        def body(r):
            try:
                res[r] = fn(self.context(r))
            except BaseException as e:  # noqa: BLE001 - re-raised below
                with self._lock:
                    err.append((r, e))
                self._bar.abort()

        ts = [threading.Thread(target=body, args=(r,), daemon=True) for r in range(self.n)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        if err:
            import threading as _t
            first = sorted(((r, e) for r, e in err
                            if not isinstance(e, _t.BrokenBarrierError)), key=lambda x: x[0])
            raise (first or err)[0][1]
        return res


class LoopbackContext:
    """One rank of a LoopbackWorld (rank, size and the setup collectives of Context)."""

    distributed = None
    group = None

    def __init__(self, world: LoopbackWorld, rank: int):
        self._w, self._r = world, rank

    def rank(self) -> int:
        return self._r

    def size(self) -> int:
        return self._w.n

    def global_rank(self, r: int) -> int:
        return r

    def all_gather_object(self, obj):
        w = self._w
        w._slots[self._r] = obj
        w._bar.wait()
        out = list(w._slots)
        w._bar.wait()
        return out

    def all_gather_array(self, arr):
        import numpy as np
        return self.all_gather_object(np.ascontiguousarray(arr, dtype=np.int64))

    def ring_arrays(self, arr):
        every = self.all_gather_array(arr)
        for step in range(self._w.n):
            r = (self._r + step) % self._w.n
            yield r, every[r]

    def exchange_arrays(self, sends, recvs):
        import numpy as np
        w, me = self._w, self._r
        with w._lock:
            for d, a in sends:
                w._mail.setdefault((me, d), []).append(np.ascontiguousarray(a, dtype=np.int64))
        w._bar.wait()
        out = []
        with w._lock:
            for src, n in recvs:
                a = w._mail[(src, me)].pop(0)
                if a.size != n:
                    raise RuntimeError(f"loopback exchange_arrays: {a.size} != {n} from {src}")
                out.append(a)
        w._bar.wait()
        return out

"""Helpers for the GPU parity tests: device fields in logical (x, y, z) order over memory laid
out by a layout map, an in-process multi-rank router, and a fake per-rank context."""
from __future__ import annotations

import numpy as np


def device_field(a_mem: np.ndarray, layout, has_components=False):
    """a_mem is the numpy array in MEMORY order (slowest dim first, as helpers.* build them).
    Returns (base, logical): base = contiguous device copy in memory order, logical = a view of
    it indexed (x, y, z[, c]) whose strides realise `layout`."""
    import os

    import torch
    how = os.environ.get("GHX_TEST_FIELD_ALLOC", "numpy")
    host = torch.from_numpy(np.ascontiguousarray(a_mem))
    if how == "pinned":  # H2D from page-locked host memory
        base = host.pin_memory().cuda()
    elif how == "device":  # allocated on the device first, then filled
        base = torch.empty(host.shape, dtype=host.dtype, device="cuda")
        base.copy_(host.pin_memory())
    else:  # H2D from pageable host memory
        base = host.cuda()
    nsp = len(layout) - (1 if has_components else 0)
    order = sorted(range(nsp), key=lambda d: layout[d])  # memory axis -> logical dim
    perm = [order.index(d) for d in range(nsp)]
    if has_components:
        perm.append(nsp)
    return base, base.permute(*perm)


class FakeContext:
    """A per-rank context for emulating R ranks inside one process (one GPU): all_gather returns
    every rank's setup data from a shared table filled beforehand."""

    def __init__(self, rank, size, table):
        self._r, self._n, self._t = rank, size, table

    def rank(self):
        return self._r

    def size(self):
        return self._n

    def all_gather_object(self, obj):
        return [self._t[r] for r in range(self._n)]

    distributed = None
    group = None

    def global_rank(self, r):
        return r


def unstructured_patterns(per_rank_domains, halo_gids=None):
    """Every emulated rank's unstructured DomainDescriptors and its make_pattern<unstructured>:
    per_rank_domains[r] = [(id, gids, outer_lids)], halo_gids[r] = that rank's halo generator
    list (None: all outer gids). The ranks run as threads of this process (LoopbackWorld), each
    passing only its own domains, as the reference's make_pattern does over MPI. Returns
    [(dds, pattern_container)] in rank order."""
    from ghex_amd import unstructured as U
    from ghex_amd.context import LoopbackWorld

    def rank_fn(ctx):
        r = ctx.rank()
        dds = [U.DomainDescriptor(i, g, o) for i, g, o in per_rank_domains[r]]
        hg = U.HaloGenerator(None if halo_gids is None else halo_gids[r])
        return dds, U.make_pattern(ctx, hg, dds)

    return LoopbackWorld(len(per_rank_domains)).run(rank_fn)


def emulated_exchange(cos, bis_per_rank, mixed=False):
    """Pack on every emulated rank, route send buffers to the matching recv buffers by
    (sender rank, domain pair, tag), unpack on every rank (all on one stream). mixed=True: the
    product's path for exchanges with self AND peer messages (ghx_exchange_pack_self, then
    ghx_exchange_unpack_peers) on every rank whose plan has one."""
    import torch
    plans, bufs, used = [], [], []
    for r, (co, bis) in enumerate(zip(cos, bis_per_rank)):
        m = mixed and co.mixed(co.plan(bis))
        plan, send, recv = co.pack_self_only(bis) if m else co.pack_only(bis)
        plans.append(plan)
        bufs.append((send, recv))
        used.append(m)
    for r, plan in enumerate(plans):
        send_r, recv_r = bufs[r]
        for i, x in enumerate(plan.recv):
            if x["rank"] == r:
                continue  # self message: recv buffer aliases the send buffer
            src = x["rank"]
            j = next(j for j, s in enumerate(plans[src].send)
                     if s["pair"] == x["pair"] and s["rank"] == r)
            assert plans[src].send[j]["tag"] == x["tag"]
            assert plans[src].send[j]["size"] == x["size"]
            recv_r[i][:x["size"]].copy_(bufs[src][0][j][:x["size"]])
    for co, bis, m in zip(cos, bis_per_rank, used):
        if m:
            co.unpack_peers_only(bis)
        else:
            co.unpack_only(bis)
    torch.cuda.synchronize()
    if mixed:
        emulated_exchange.mixed_ranks = sum(used)
    return plans, bufs


def _dbl(n):
    """Offset of the odd-parity copy of a double-buffered receive buffer (as the product's)."""
    return max(256, (int(n) + 255) // 256 * 256)


class EmulatedDirect:
    """The direct exchange's launches for emulated ranks (one process, one stream): every peer
    message is packed straight into its receiver's buffer, which exists twice (sentinel 0xA5
    until written); the copy is chosen on the device from an epoch word through
    ghx_exchange_set_parity, as around the one-launch close: pack with the word at e - 1 and
    add 1, unpack with it at e and add 0, so exchange e uses copy e & 1. Self messages keep one
    copy (their receive buffer is their send buffer). mixed=True: ranks whose plans hold self
    AND peer messages run ghx_exchange_pack_self / ghx_exchange_unpack_peers."""

    def __init__(self, cos, bis_all, mixed=False):
        import ctypes

        import torch
        from ghex_amd import _ghx
        self.cos, self.bis_all = cos, bis_all
        self.word = torch.zeros(1, dtype=torch.int64, device="cuda")
        wp = ctypes.c_void_p(self.word.data_ptr())
        self.plans = [co.plan(bis) for co, bis in zip(cos, bis_all)]
        self.mixed = [mixed and co.mixed(p) for co, p in zip(cos, self.plans)]
        own = [[torch.full((max(1, b["size"]),), 0x5A, dtype=torch.uint8, device="cuda")
                for b in p.send] for p in self.plans]
        self.recv = []
        for r, p in enumerate(self.plans):
            rr = []
            for b in p.recv:
                j = next((i for i, sb in enumerate(p.send)
                          if sb["pair"] == b["pair"] and b["rank"] == r), None)
                rr.append(own[r][j] if j is not None else
                          torch.full((2 * _dbl(b["size"]),), 0xA5, dtype=torch.uint8,
                                     device="cuda"))
            self.recv.append(rr)
        self.sptr, self.rptr, self.fptr = [], [], []
        for r, p in enumerate(self.plans):
            ptrs, offs = [], []
            for i, b in enumerate(p.send):
                if b["rank"] == r:
                    ptrs.append(own[r][i].data_ptr())
                    offs.append(0)
                    continue
                q = b["rank"]
                k = next(k for k, rb in enumerate(self.plans[q].recv)
                         if rb["pair"] == b["pair"] and rb["rank"] == r)
                rb = self.plans[q].recv[k]
                assert rb["size"] == b["size"] and rb["tag"] == b["tag"]
                ptrs.append(self.recv[q][k].data_ptr())
                offs.append(_dbl(b["size"]))
            roff = [_dbl(b["size"]) if b["rank"] != r else 0 for b in p.recv]
            for direction, add, o in ((0, 1, offs), (1, 0, roff)):
                _ghx.call("ghx_exchange_set_parity", p.h, direction, wp, add,
                          (ctypes.c_int64 * max(1, len(o)))(*o), len(o))
            self.sptr.append(_ghx.ptr_array(ptrs))
            self.rptr.append(_ghx.ptr_array([t.data_ptr() for t in self.recv[r]]))
            self.fptr.append(_ghx.ptr_array([bi.field.data_ptr() for bi in bis_all[r]]))
        self.own = own

    def exchange(self, e):
        """Exchange e (>= 1) on the current stream, then synchronise."""
        import torch
        from ghex_amd import _ghx
        L = _ghx.lib()
        s = torch.cuda.current_stream().cuda_stream
        self.word.fill_(e - 1)
        for r, p in enumerate(self.plans):
            fn = L.ghx_exchange_pack_self if self.mixed[r] else L.ghx_exchange_pack
            _ghx.check(fn(p.h, self.fptr[r], len(self.bis_all[r]), self.sptr[r], len(p.send), s),
                       "pack")
        self.word.fill_(e)
        for r, p in enumerate(self.plans):
            fn = L.ghx_exchange_unpack_peers if self.mixed[r] else L.ghx_exchange_unpack
            _ghx.check(fn(p.h, self.fptr[r], len(self.bis_all[r]), self.rptr[r], len(p.recv), s),
                       "unpack")
        torch.cuda.synchronize()

    def peer_messages(self):
        """[(receiver r, recv index i, sender q, the sender's send dict, odd-copy offset)]."""
        out = []
        for r, p in enumerate(self.plans):
            for i, b in enumerate(p.recv):
                if b["rank"] == r:
                    continue
                q = b["rank"]
                x = next(x for x in self.plans[q].send if x["pair"] == b["pair"] and x["rank"] == r)
                out.append((r, i, q, x, _dbl(b["size"])))
        return out

"""Helpers for the GPU parity tests: device fields in logical (x, y, z) order over memory laid
out by a layout map, an in-process multi-rank router, and a fake per-rank context."""
from __future__ import annotations

import numpy as np


def device_field(a_mem: np.ndarray, layout, has_components=False):
    """a_mem is the numpy array in MEMORY order (slowest dim first, as helpers.* build them).
    Returns (base, logical): base = contiguous device copy in memory order, logical = a view of
    it indexed (x, y, z[, c]) whose strides realise `layout`."""
    import torch
    base = torch.from_numpy(np.ascontiguousarray(a_mem)).cuda()
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

"""Field layouts for MI355X (no reference counterpart: the reference takes whatever storage the
caller wraps). The x-normal halo faces move one 128-B cache line per row boundary, and how fast
those lines move depends on the field's row pitch (at 512^3 H=2 a field
allocated 518 cells wide in x instead of 516 runs the pack+unpack step 11 % faster, with the same
cells and bytes). These helpers allocate fields with a wider x row and pick the width by timing
the exchange on the device.

    x_alloc = suggest_x_alloc((516, 516, 516), halo=2)            # a few ms per candidate
    f = allocate((516, 516, 516), torch.float64, x_alloc=x_alloc)  # logical (x, y, z) view
    fd = make_field_descriptor(dd, f, (2, 2, 2), (516, 516, 516))
"""
from __future__ import annotations

from typing import Iterable, Optional, Sequence


def allocate(extents: Sequence[int], dtype, x_alloc: Optional[int] = None, device="cuda",
             fill=None):
    """A logical (x, y, z) tensor of `extents` with x contiguous (layout_map<2,1,0>) whose rows
    are allocated `x_alloc` >= extents[0] elements wide (the pad is never read or written by an
    exchange). fill: initial value (None: uninitialised)."""
    import torch
    ex, ey, ez = (int(e) for e in extents)
    xa = ex if x_alloc is None else int(x_alloc)
    if xa < ex:
        raise ValueError(f"x_alloc {xa} < x extent {ex}")
    store = (torch.empty if fill is None else torch.full)
    args = ((ez, ey, xa),) if fill is None else ((ez, ey, xa), fill)
    mem = store(*args, dtype=dtype, device=device)
    return mem[:, :, :ex].permute(2, 1, 0)


class _LocalContext:
    """A one-rank context: the trial exchanges are self exchanges of this process only."""
    distributed = None
    group = None

    def rank(self):
        return 0

    def size(self):
        return 1

    def all_gather_object(self, obj):
        return [obj]

    def global_rank(self, r):
        return r


def suggest_x_alloc(extents: Sequence[int], halo: int, dtype=None,
                    candidates: Optional[Iterable[int]] = None, reps: int = 20,
                    device="cuda", return_times: bool = False):
    """The x allocation (row width in elements) among `candidates` (default: the extent itself
    and the 16-B aligned widths up to 16 bytes' worth of elements beyond it) for which the pack+unpack of a single periodic
    domain of these extents and halo width runs fastest on this device: each candidate is planned
    through the product path and timed from a hipGraph of `reps` steps. Runs at setup time.
    return_times: also return {x_alloc: microseconds per step}."""
    import torch

    from ghex_amd import _ghx
    from ghex_amd.structured import regular as R
    dtype = torch.float64 if dtype is None else dtype
    ex, ey, ez = (int(e) for e in extents)
    h = int(halo)
    first, last = (0, 0, 0), (ex - 2 * h - 1, ey - 2 * h - 1, ez - 2 * h - 1)
    if min(last) < 0:
        raise ValueError("extents must exceed twice the halo in every dimension")
    es = torch.empty((), dtype=dtype).element_size()
    step = max(1, 16 // es)
    if candidates is None:
        base = -(-ex // step) * step  # smallest 16-B aligned width >= ex
        candidates = [base + k * step for k in range(0, max(1, 16 // step) + 1)]
        candidates = sorted({ex, *candidates})
    ctx = _LocalContext()  # this process alone, even under torch.distributed (no collective)
    dd = R.DomainDescriptor(0, first, last)
    pc = R.make_pattern(ctx, R.HaloGenerator(first, last, (h,) * 6, (True,) * 3), [dd])
    L = _ghx.lib()
    dev = torch.device(device)
    stream = torch.cuda.current_stream(dev)
    best, best_t, times = None, None, {}
    for xa in candidates:
        f = allocate(extents, dtype, xa, device)
        f.random_(0, 1 << 20)  # varied data: an all-zero field moves measurably faster
        fd = R.make_field_descriptor(dd, f, (h,) * 3, (ex, ey, ez))
        co = R.make_communication_object(ctx)
        bis = [pc(fd)]
        plan = co.plan(bis)
        send, recv = co.buffers(plan, dev)
        fp = _ghx.ptr_array([fd.data_ptr()])
        sp = _ghx.ptr_array([t.data_ptr() for t in send])
        rp = _ghx.ptr_array([t.data_ptr() for t in recv])

        def one(s):
            _ghx.check(L.ghx_exchange_pack(plan.h, fp, 1, sp, len(send), s), "pack")
            _ghx.check(L.ghx_exchange_unpack(plan.h, fp, 1, rp, len(recv), s), "unpack")
        side = torch.cuda.Stream(dev)
        side.wait_stream(stream)
        with torch.cuda.stream(side):
            one(side.cuda_stream)
        stream.wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(reps):
                one(torch.cuda.current_stream(dev).cuda_stream)
        g.replay()
        ts = []
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            g.replay()
            e1.record(stream)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        t = sorted(ts)[1]
        times[xa] = round(t * 1e3 / reps, 2)
        if best_t is None or t < best_t * 0.98:  # ties go to the narrower allocation
            best, best_t = xa, t
        del g, co, plan, send, recv, fd, f
        torch.cuda.empty_cache()
    return (best, times) if return_times else best

#!/usr/bin/env python3
"""Developer measurement (not product): the 512^3 H=2 two-launch step in four cache states, as
plain eager launches so that a rocprofv3 --pmc pass attributes counters per dispatch.

  warm         pack, unpack back to back (the bench's steady state)
  cold_step    1 GiB read-only flush, then pack, unpack (an application after a stencil sweep)
  cold_pack    flush, pack
  cold_unpack  flush, unpack

Without a profiler (--time) it prints per-kernel begin/end durations (libghx launch events,
medians) for every mode in one JSON line; under rocprofv3 run one --mode per pass and parse
with tools/parse_cold_pmc.py. --tune passes ghx_tune knobs; --x-alloc pads the field's rows."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

MODES = ("warm", "cold_step", "cold_pack", "cold_unpack")


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--mode", default="all", choices=MODES + ("all",))
    p.add_argument("--iters", type=int, default=8)
    p.add_argument("--N", type=int, default=512)
    p.add_argument("--halo", type=int, default=2)
    p.add_argument("--x-alloc", type=int, default=0)
    p.add_argument("--tune", default="")
    p.add_argument("--time", action="store_true", help="print launch durations per mode")
    a = p.parse_args()
    import ctypes

    import torch

    import ghex_amd
    from ghex_amd import _ghx
    from ghex_amd.structured import regular as R
    for kv in filter(None, a.tune.split(",")):
        k, v = kv.split("=")
        _ghx.call("ghx_tune", k.encode(), int(v))
    L = _ghx.lib()
    dev = torch.device("cuda", 0)
    N, H = a.N, a.halo
    E = N + 2 * H
    alloc = torch.full((E, E, a.x_alloc or E), -1.0, dtype=torch.float64, device=dev)
    base = alloc[:, :, :E]
    ar = torch.arange(N, device=dev, dtype=torch.float64)
    base[H:H + N, H:H + N, H:H + N] = ar.view(1, 1, N) + N * (ar.view(1, N, 1) + N * ar.view(N, 1, 1))
    ctx = ghex_amd.make_context()
    dd = R.DomainDescriptor(0, (0, 0, 0), (N - 1,) * 3)
    pc = R.make_pattern(ctx, R.HaloGenerator((0, 0, 0), (N - 1,) * 3, (H,) * 6, (True,) * 3), [dd])
    fd = R.make_field_descriptor(dd, base.permute(2, 1, 0), (H,) * 3, (E,) * 3)
    co = R.make_communication_object(ctx)
    bis = [pc(fd)]
    co.exchange(bis).wait()
    plan = co.plan(bis)
    send, recv = co.buffers(plan, dev)
    fptr = _ghx.ptr_array([fd.data_ptr()])
    sptr = _ghx.ptr_array([t.data_ptr() for t in send])
    rptr = _ghx.ptr_array([t.data_ptr() for t in recv])
    s = torch.cuda.current_stream(dev).cuda_stream
    fl = torch.zeros(1 << 27, dtype=torch.float64, device=dev)
    acc = torch.empty((), dtype=torch.float64, device=dev)

    def pack():
        _ghx.check(L.ghx_exchange_pack(plan.h, fptr, 1, sptr, len(send), s), "pack")

    def unpack():
        _ghx.check(L.ghx_exchange_unpack(plan.h, fptr, 1, rptr, len(recv), s), "unpack")

    def flush():
        torch.sum(fl, dim=(0,), out=acc)

    seq = {"warm": [pack, unpack], "cold_step": [flush, pack, unpack],
           "cold_pack": [flush, pack], "cold_unpack": [flush, unpack]}
    modes = MODES if a.mode == "all" else (a.mode,)
    res = {}
    for m in modes:
        for _ in range(3):
            for f in seq[m]:
                f()
        torch.cuda.synchronize(dev)
        if not a.time:
            for _ in range(a.iters):
                for f in seq[m]:
                    f()
            torch.cuda.synchronize(dev)
            continue
        kern = [f for f in seq[m] if f is not flush]
        n = a.iters * len(kern)
        ms = (ctypes.c_float * n)()
        got = ctypes.c_int32()
        durs = []
        for _ in range(a.iters):
            # events around the whole sequence on the stream (device time incl. boundaries) ...
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            if m != "warm":
                flush()
            e0.record()
            _ghx.call("ghx_launch_timing", 1)
            for f in kern:
                f()
            e1.record()
            _ghx.call("ghx_launch_timing_read", ms, n, ctypes.byref(got))
            _ghx.call("ghx_launch_timing", 0)
            e1.synchronize()
            durs.append((e0.elapsed_time(e1) * 1e3, [ms[i] * 1e3 for i in range(got.value)]))
        seqt = sorted(d for d, _ in durs)
        per = [sorted(k[i] for _, k in durs if len(k) == len(kern)) for i in range(len(kern))]
        names = [f.__name__ for f in kern]
        res[m] = {"seq_us": round(seqt[len(seqt) // 2], 2),
                  **{f"{nm}_us": round(p_[len(p_) // 2], 2) for nm, p_ in zip(names, per) if p_}}
    if a.time:
        print(json.dumps({"N": N, "H": H, "x_alloc": a.x_alloc or E, "tune": a.tune,
                          "iters": a.iters, "modes": res}), flush=True)


if __name__ == "__main__":
    main()

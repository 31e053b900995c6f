#!/usr/bin/env python3
"""Developer benchmark: the host-staged exchange step at N=1 (512^3 fp64, H=2): pack -> D2H into
pinned memory -> H2D -> unpack, in several forms, to find what overlaps on this box's PCIe link.

  raw_d2h / raw_h2d / raw_both   the 25.4 MB buffer alone one way, and both ways at once on two
                                 streams (is the link used full duplex?)
  serial                         pack, D2H, H2D, unpack on one stream (bench's host_staged form)
  chunked_C                      pack; then chunk i: D2H on the d2h stream, H2D of chunk i on the
                                 h2d stream behind its own D2H only; unpack behind the last H2D
Copies are hipMemcpyAsync through torch (non_blocking copy_ of pinned tensors). One JSON line
per form with ms per step and the algorithmic rate (4*n*8 bytes per step)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--N", type=int, default=512)
    p.add_argument("--halo", type=int, default=2)
    p.add_argument("--iters", type=int, default=20)
    a = p.parse_args()
    import torch
    import ghex_amd
    from ghex_amd import _ghx
    from ghex_amd.structured import regular as R
    L = _ghx.lib()
    N, H = a.N, a.halo
    E = N + 2 * H
    dev = torch.device("cuda", 0)
    base = torch.randn((E, E, E), dtype=torch.float64, device=dev)
    ctx = ghex_amd.make_context()
    dd = R.DomainDescriptor(0, (0, 0, 0), (N - 1,) * 3)
    pc = R.make_pattern(ctx, R.HaloGenerator((0, 0, 0), (N - 1,) * 3, (H,) * 6, (True,) * 3), [dd])
    fd = R.make_field_descriptor(dd, base.permute(2, 1, 0), (H,) * 3, (E,) * 3)
    co = R.make_communication_object(ctx)
    bis = [pc(fd)]
    plan = co.plan(bis)
    n = plan.send[0]["size"]
    sbuf = torch.empty(n, dtype=torch.uint8, device=dev)
    rbuf = torch.empty(n, dtype=torch.uint8, device=dev)
    hsend = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    fp = _ghx.ptr_array([fd.data_ptr()])
    sp = _ghx.ptr_array([sbuf.data_ptr()])
    rp = _ghx.ptr_array([rbuf.data_ptr()])
    main_s = torch.cuda.current_stream()
    d2h = torch.cuda.Stream()
    h2d = torch.cuda.Stream()
    step_bytes = 4 * n

    def pack():
        _ghx.check(L.ghx_exchange_pack(plan.h, fp, 1, sp, 1, main_s.cuda_stream), "pack")

    def unpack():
        _ghx.check(L.ghx_exchange_unpack(plan.h, fp, 1, rp, 1, main_s.cuda_stream), "unpack")

    def timeit(fn, k=a.iters):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / k

    out = []

    def rec(name, t, nbytes=step_bytes, **kw):
        out.append(dict(form=name, ms=round(t * 1e3, 4), GBps=round(nbytes / t / 1e9, 2), **kw))
        print(json.dumps(out[-1]), flush=True)

    hrecv = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    rec("raw_d2h", timeit(lambda: hsend.copy_(sbuf, non_blocking=True)), n)
    rec("raw_h2d", timeit(lambda: rbuf.copy_(hrecv, non_blocking=True)), n)

    def both():
        d2h.wait_stream(main_s)
        h2d.wait_stream(main_s)
        with torch.cuda.stream(d2h):
            hsend.copy_(sbuf, non_blocking=True)
        with torch.cuda.stream(h2d):
            rbuf.copy_(hrecv, non_blocking=True)
        main_s.wait_stream(d2h)
        main_s.wait_stream(h2d)
    rec("raw_both_directions", timeit(both), 2 * n)

    def serial():
        pack()
        hsend.copy_(sbuf, non_blocking=True)
        rbuf.copy_(hsend, non_blocking=True)
        unpack()
    rec("serial", timeit(serial))

    for mib in (1, 2, 4, 8):
        C = mib << 20
        cuts = [(o, min(o + C, n)) for o in range(0, n, C)]
        evs = [torch.cuda.Event() for _ in cuts]

        def chunked():
            pack()
            d2h.wait_stream(main_s)
            for (o, e), ev in zip(cuts, evs):
                with torch.cuda.stream(d2h):
                    hsend[o:e].copy_(sbuf[o:e], non_blocking=True)
                    ev.record(d2h)
                h2d.wait_event(ev)
                with torch.cuda.stream(h2d):
                    rbuf[o:e].copy_(hsend[o:e], non_blocking=True)
            main_s.wait_stream(h2d)
            unpack()
        rec(f"chunked_{mib}MiB", timeit(chunked), chunks=len(cuts))
    print(json.dumps({"summary": out, "env_HSA_ENABLE_SDMA": os.environ.get("HSA_ENABLE_SDMA")}))


if __name__ == "__main__":
    main()
